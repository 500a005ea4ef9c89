"""Forward line search (hop_forward_linesearch_f64) and the whole device outer
loop (solver.ilqr_timeopt_batch) on one GPU.

    python tools/bench_forward.py [--system quadrotor] [--batch 4096] [--N 100]
                                  [--iters 4] [--cpu-seconds 10] [--no-loop]

Line 1 per system: forward line searches per second (5 step sizes, T* = N)
with X, U, K, k resident in HBM; the kernel time is HIP events on the launch
stream; the HBM roofline uses the algorithmic bytes (X, U, K, k read once,
X', U' written once, J read/written) -- the rollout is a sequential chain per
(problem, alpha) lane, so the kernel is latency-bound and the fraction is low
by construction.  The CPU leg runs the oracle's scalar line search
(oracle/ilqr_oracle.forward_linesearch, one F call per step as the reference
does) on a bounded sample.

Line 2 (quadrotor, --loop): ilqr_timeopt_batch(method=each of --methods) for a
batch of problems around the maker's x0 (random offsets), fixed
``--loop-iters`` iterations (max_iter, the stop rule active): problem-iterations
per second and the per-stage device time, next to the oracle's scalar outer
loop on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
SYS = {"di": 0, "cartpole": 1, "quadrotor": 2, "pointmass": 3, "segway": 4}


def algorithmic_bytes(Bn, N, n, m):
    """per launch: X, U, K, k read once, X', U' written once, J / accepted out"""
    return 8 * Bn * (2 * ((N + 1) * n + N * m) + N * m * n + N * m + 3)


def problem(sid, Bn, N, seed=3):
    from time_opt_ilqr_amd import systems
    from oracle import ilqr_oracle as io
    mk = list(systems.MAKERS.values())[sid]
    F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap, extra = mk(N=N)
    n, m = F.n, F.m
    rng = np.random.default_rng(seed)
    U = u_ref + 0.05 * rng.standard_normal((Bn, N, m))
    X = np.stack([io.rollout(sid, F.dt, x0, U[b]) for b in range(min(Bn, 64))])
    X = np.concatenate([X] * ((Bn + 63) // 64))[:Bn]
    U = np.concatenate([U[:64]] * ((Bn + 63) // 64))[:Bn]
    K = -0.05 * rng.standard_normal((Bn, N, m, n))
    k = 0.1 * rng.standard_normal((Bn, N, m))
    Qf = io.orc.terminal_weight(alpha, n)
    obs = None
    if extra:
        obs = np.array([[o[0], o[1], r, wt] for o, r, wt in systems.OBSTACLES])
    return F, (X, U, K, k), (x0, xg, u_ref, Q, R, Qf, w, wrap, obs)


def bench_linesearch(sid, name, Bn, N, rounds, iters, cpu_seconds):
    import torch
    from time_opt_ilqr_amd import engine
    from oracle import ilqr_oracle as io
    dev = torch.device("cuda", 0)
    F, (X, U, K, k), (x0, xg, u_ref, Q, R, Qf, w, wrap, obs) = problem(sid, Bn, N)
    t = lambda a: torch.as_tensor(a, dtype=torch.float64, device=dev)  # noqa: E731
    cost = engine.CostParams(t(xg), t(u_ref), t(Q), t(R), t(Qf), w,
                             None if obs is None else t(obs), wrap)
    Xt, Ut, Kt, kt = t(X), t(U), t(K), t(k)
    T = torch.full((Bn,), N, dtype=torch.int32, device=dev)
    for _ in range(3):
        r = engine.forward_linesearch(sid, Xt, Ut, T, Kt, kt, cost, F.dt)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    samples = []
    for _ in range(rounds):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(iters):
            engine.forward_linesearch(sid, Xt, Ut, T, Kt, kt, cost, F.dt)
        e1.record(stream)
        torch.cuda.synchronize()
        samples.append(e0.elapsed_time(e1) / iters)
    samples.sort()
    ms = samples[len(samples) // 2]
    acc = np.bincount(r.accepted.cpu().numpy() + 2, minlength=7)
    byts = algorithmic_bytes(Bn, N, F.n, F.m)
    gbs = byts / (ms * 1e-3) / 1e9
    cpu = None
    if cpu_seconds > 0:
        t0 = time.perf_counter()
        cnt = 0
        while cnt < Bn and time.perf_counter() - t0 < cpu_seconds:
            io.forward_linesearch(sid, F.dt, X[cnt], U[cnt], xg, u_ref, Q, R, Qf, w, N, k[cnt],
                                  K[cnt], wrap_idx=wrap, obstacles=obs)
            cnt += 1
        el = time.perf_counter() - t0
        cpu = {"value": cnt / el, "unit": "line searches/s", "cores": 1, "kind": "port",
               "sample": f"{cnt} line searches (N={N}) of oracle/ilqr_oracle.py, {el:.1f} s"}
    print(json.dumps({
        "metric": "batched forward line searches/s", "system": name, "batch": Bn, "N": N,
        "n_alpha": 5, "value": Bn / (ms * 1e-3), "unit": "line searches/s", "kernel_ms": ms,
        "kernel_ms_min": samples[0], "dtype": "f64", "data": "synthetic",
        "accepted_hist": {"inactive": int(acc[0]), "none": int(acc[1]),
                          **{f"alpha{i}": int(acc[i + 2]) for i in range(5)}},
        "roofline": {"bound": "latency (sequential rollout per lane)", "achieved": gbs,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                     "bytes_per_launch": byts},
        "cpu_baseline": cpu}), flush=True)


def bench_loop(Bn, N, iters, cpu_seconds, loop_rounds=5, method="propagator"):
    import torch
    from time_opt_ilqr_amd import solver, systems
    from oracle import ilqr_oracle as io
    F, x0, xg, u_ref, Q, R, alpha, w, _, T_min, T_max, wrap, _ = systems.make_quadrotor(N=N)
    T_min, T_max = max(1, N // 5), N
    rng = np.random.default_rng(9)
    X0 = x0 + 0.2 * rng.standard_normal((Bn, F.n))
    Qf = io.orc.terminal_weight(alpha, F.n)
    kw = dict(dt=F.dt, max_iter=iters, wrap_idx=wrap, use_central_diff=False, method=method)
    # warm-up on the same batch: the first use of torch's gather / scatter kernels
    # (active-set compaction) loads them lazily
    solver.ilqr_timeopt_batch(2, X0, xg, u_ref, Q, R, Qf, w, N, T_min, T_max, **kw)
    torch.cuda.synchronize()
    walls = []
    for _ in range(loop_rounds):  # median of several whole runs (allocator / clocks warm)
        t0 = time.perf_counter()
        solver.ilqr_timeopt_batch(2, X0, xg, u_ref, Q, R, Qf, w, N, T_min, T_max, **kw,
                                  stage_timers=False)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
    el = sorted(walls)[len(walls) // 2]
    # a third run, each stage synchronised, for the per-stage breakdown
    res = solver.ilqr_timeopt_batch(2, X0, xg, u_ref, Q, R, Qf, w, N, T_min, T_max, **kw)
    its = res["iterations"] + 1  # + the warm start
    cpu = None
    if cpu_seconds > 0:
        t0 = time.perf_counter()
        cnt = 0
        done_its = 0
        while cnt < Bn and time.perf_counter() - t0 < cpu_seconds:
            o = io.ilqr_timeopt(2, F.dt, X0[cnt], xg, u_ref, Q, R, Qf, w, N, T_min, T_max,
                                max_iter=iters, wrap_idx=wrap, central=False, method=method)
            done_its += len(o["J_hist"])
            cnt += 1
        cel = time.perf_counter() - t0
        cpu = {"value": cnt / cel, "unit": "problems/s", "cores": 1, "kind": "port",
               "sample": f"{cnt} outer loops (max_iter={iters}) of oracle/ilqr_oracle.py, "
                         f"{cel:.1f} s"}
    print(json.dumps({
        "metric": f"batched iLQR outer loop ({method}), quadrotor", "batch": Bn, "N": N,
        "T_min": T_min, "T_max": T_max, "max_iter": iters, "iterations_run": its,
        "value": Bn / el, "unit": "problems/s", "problem_iterations_per_s": Bn * its / el,
        "wall_s": el, "wall_runs": len(walls), "stage_s": {k: round(v, 6) for k, v in res["timers"].items()},
        "accepted_mean": float((res["n_hist"].float().mean()).item()),
        "crashed": int(res["crashed"].sum().item()), "dtype": "f64", "data": "synthetic",
        "cpu_baseline": cpu}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--system", default="all", choices=sorted(SYS) + ["all"])
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--N", type=int, default=100)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--loop-iters", type=int, default=4)
    ap.add_argument("--no-loop", action="store_true")
    ap.add_argument("--methods", default="propagator",
                    help="comma list of outer-loop select methods (propagator, bruteforce)")
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    args = ap.parse_args()
    names = sorted(SYS, key=SYS.get) if args.system == "all" else [args.system]
    for name in names:
        bench_linesearch(SYS[name], name, args.batch, args.N, args.rounds, args.iters,
                         args.cpu_seconds)
    if not args.no_loop:
        for meth in args.methods.split(","):
            bench_loop(args.batch, args.N, args.loop_iters, args.cpu_seconds, method=meth)


if __name__ == "__main__":
    main()
