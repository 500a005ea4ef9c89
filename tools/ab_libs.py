"""Same-process interleaved A/B of two (or more) builds of libhop_amd.so on the bench
workloads (config 3 tile64 fp32, config 2 fp64, config 4 shard, Riccati mode 0/1):

    python tools/ab_libs.py time_opt_ilqr_amd/libhop_amd.so <other.so> [--rounds 7]

Each round times every (workload, library) pair once (10 launches, HIP events; the
library order alternates between rounds),
so clock drift hits both alike (cdna_hip_programming.md 5.4 rule 24); prints the
median ms per launch and checks the outputs are bitwise equal.
"""
import argparse
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--only", default="", help="comma list of workloads")
    # even: each library is timed first after the warm-up in half the rounds (round 6:
    # the library timed second ran 3-6 % faster on config 2, so an odd count biased the
    # median ratio; the geometric mean of the per-round ratios is reported too)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warm", type=int, default=10, help="untimed launches after a workload switch")
    args = ap.parse_args()
    import torch
    from time_opt_ilqr_amd import _lib, engine, synth
    dev = torch.device("cuda", 0)
    libs = [_lib.load(p) for p in args.libs]
    work = {}
    A, Bm, Q, Ri, z0, QT = synth.device_batch(65536, 5, 1, 200, seed=3, device=dev,
                                              dtype=torch.float32)
    At, Bt, Qt, QTt = (engine.to_tile64(x) for x in (A, Bm, Q, QT))
    del A, Bm, Q, QT
    work["config3_tile64"] = lambda: engine.propagate(At, Bt, Qt, Ri, z0, QTt, t_min=20,
                                                      t_max=200).J
    c2 = synth.device_batch(4096, 13, 4, 100, seed=4, device=dev)
    work["config2"] = lambda: engine.propagate(*c2, t_min=40, t_max=100).J
    if "config4_shard" in args.only.split(","):  # 15 GB of blocks: only on request
        c4 = synth.device_batch(32768, 13, 4, 100, seed=5, device=dev)
        work["config4_shard"] = lambda: engine.propagate(*c4, t_min=40, t_max=100).J
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    n, m, N, Bn = 12, 4, 100, 4096
    kw = dict(device=dev, dtype=torch.float64, generator=g)
    rA = torch.eye(n, device=dev, dtype=torch.float64) + 0.05 * torch.randn((Bn, N, n, n), **kw)
    rB = 0.1 * torch.randn((Bn, N, n, m), **kw)
    rX = 0.5 * torch.randn((Bn, N + 1, n), **kw)
    rU = 0.1 * torch.randn((Bn, N, m), **kw)
    M = torch.randn((n, n), **kw)
    rQ = M @ M.T / n + 0.5 * torch.eye(n, device=dev, dtype=torch.float64)
    rR = torch.diag(0.5 + 1.5 * torch.rand((m,), **kw))
    rQf = 10.0 * torch.eye(n, device=dev, dtype=torch.float64)
    xg = torch.zeros(n, device=dev, dtype=torch.float64)
    ur = torch.zeros(m, device=dev, dtype=torch.float64)
    for md in (0, 1):
        work[f"riccati_mode{md}"] = (lambda md=md: engine.riccati(
            rA, rB, rX, rU, xg, ur, rQ, rR, rQf, N, 1e-3, mode=md).K)
    # the brute-force J curve (bench --workload bruteforce shape) and the select
    # block's closed-form trajectory kernel (bench --workload select_gains)
    jX = 0.5 * torch.randn((Bn, N + 1, n), **kw)
    jU = 0.3 * torch.randn((Bn, N, m), **kw)
    jxg, jur = 0.2 * torch.randn((n,), **kw), 0.1 * torch.randn((m,), **kw)
    work["bruteforce_jcurve"] = lambda: engine.bruteforce_jcurve(
        rA, rB, jX, jU, jxg, jur, rQ, rR, rQf, N, lm_lambda=1e-6, w_stage=0.5)[0]
    ares = 0.02 * torch.randn((Bn, N, n), **kw)
    rRi = torch.linalg.inv(rR).contiguous()
    work["select_traj_cf"] = lambda: engine.propagate_traj(
        rA, rB, ares, jX, jU, jxg, jur, rQ, rRi, rQf, 0.5, t_min=40, t_max=N, rho_reg=1.0).J
    from time_opt_ilqr_amd import systems
    F, x0, xg_q, ur_q, *_ = systems.make_quadrotor(N=100)
    Uq = torch.as_tensor(ur_q, device=dev) + 0.05 * torch.randn((4096, 100, 4), **kw)
    Xq = engine.rollout(2, torch.as_tensor(x0, device=dev) + 0.1 * torch.randn((4096, 12), **kw),
                        Uq, F.dt)
    for cen in (False, True):
        work[f"linearize_quad_{'central' if cen else 'forward'}"] = (
            lambda cen=cen: engine.linearize(2, Xq, Uq, F.dt, central=cen).A)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import bench_forward as bf
    Fq, (lX, lU, lK, lk), (_, lxg, lur, lQ, lR, lQf, lw, lwrap, _) = bf.problem(2, 4096, 100)
    tt = lambda a: torch.as_tensor(a, dtype=torch.float64, device=dev)  # noqa: E731
    lcost = engine.CostParams(tt(lxg), tt(lur), tt(lQ), tt(lR), tt(lQf), lw, None, lwrap)
    lXt, lUt, lKt, lkt = tt(lX), tt(lU), tt(lK), tt(lk)
    lT = torch.full((4096,), 100, dtype=torch.int32, device=dev)
    work["linesearch_quad"] = lambda: engine.forward_linesearch(2, lXt, lUt, lT, lKt, lkt, lcost,
                                                                Fq.dt).X
    lin = engine.linearize(2, Xq, Uq, F.dt)
    P = tt(lQf)
    work["augment_quad"] = lambda: engine.augment(lin.A, lin.B, lin.a_res, Xq, Uq, tt(lxg),
                                                  tt(lur), tt(lQ), P, lw).Q
    # fp64 s = 5 blocks at B = 4,096 (round 6: the row-group kernel against the lane
    # kernel of the libraries before it); synthetic SPD blocks, N = 200
    s5 = synth.device_batch(4096, 5, 1, 200, seed=6, device=dev)
    work["small_s5_f64_4096"] = lambda: engine.propagate(*s5, t_min=40, t_max=200).J
    if args.only:
        work = {w: f for w, f in work.items() if w in args.only.split(",")}
    L = len(libs)
    times = {(w, i): [] for w in work for i in range(L)}
    outs = {}
    for i in range(L):  # warm-up + outputs
        _lib._lib = libs[i]
        for w, f in work.items():
            outs[(w, i)] = f().clone()
    torch.cuda.synchronize()
    for rnd in range(args.rounds):
        for w, f in work.items():
            # a workload switch changes the clocks: run it untimed first (round 5: the
            # first library timed after a switch came out up to 12 % off either way)
            _lib._lib = libs[0]
            for _ in range(args.warm):
                f()
            # alternate the order every round as well
            for i in (range(L) if rnd % 2 == 0 else reversed(range(L))):
                _lib._lib = libs[i]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    f()
                e1.record()
                torch.cuda.synchronize()
                times[(w, i)].append(e0.elapsed_time(e1) / args.iters)
    for w in work:
        r = {os.path.basename(args.libs[i]): round(statistics.median(times[(w, i)]), 4)
             for i in range(L)}
        same = all(torch.equal(outs[(w, 0)].nan_to_num(7.0), outs[(w, i)].nan_to_num(7.0))
                   for i in range(1, L))
        lo = {os.path.basename(args.libs[i]): round(min(times[(w, i)]), 4) for i in range(L)}
        # per-round ratios to the first library: clock drift between rounds cancels
        ratio = {os.path.basename(args.libs[i]): round(statistics.median(
            [a / b for a, b in zip(times[(w, i)], times[(w, 0)])]), 4) for i in range(L)}
        rounds = {os.path.basename(args.libs[i]): [round(x, 4) for x in times[(w, i)]]
                  for i in range(L)}
        geo = {os.path.basename(args.libs[i]): round(math.exp(statistics.mean(
            [math.log(a / b) for a, b in zip(times[(w, i)], times[(w, 0)])])), 4) for i in range(L)}
        print(json.dumps({"workload": w, "ms": r, "min_ms": lo, "ratio_to_first": ratio,
                          "geomean_ratio_to_first": geo,
                          "bitwise_equal": same,
                          "rounds": rounds}), flush=True)


if __name__ == "__main__":
    main()
