"""Batched finite-difference linearisation (hop_linearize_f64) on one GPU.

    python tools/bench_linearize.py [--system quadrotor] [--batch 4096] [--N 100]
                                    [--central] [--cpu-seconds 10]

One JSON line per system / difference scheme: linearised steps per second with
the trajectories resident in HBM, the kernel's average launch time (HIP events
on the launch stream) and its HBM roofline (algorithmic bytes: X, U read once,
A, B, a_res written once per step), next to the reference's loop structure
(oracle/dyn_oracle.linearize_loop: one F call per column, one step at a time)
timed on one host core for a bounded sample of the same trajectories.
Synthetic states around the maker's x0 / u_ref (no dataset exists).
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
    """per launch: X [B, N+1, n] and U [B, N, m] read once; A [B, N, n, n],
    B [B, N, n, m], a_res [B, N, n] written once"""
    return 8 * Bn * ((N + 1) * n + N * m + N * (n * n + n * m + n))


def synth(sid, n, m, Bn, N, seed=5):
    rng = np.random.default_rng(seed)
    x0 = {2: np.r_[2.0, 2.0, 2.0, np.zeros(9)]}.get(sid, np.zeros(n))
    u0 = {2: np.array([9.81, 0.0, 0.0, 0.0])}.get(sid, np.zeros(m))
    X = x0 + 0.3 * rng.standard_normal((Bn, N + 1, n))
    U = u0 + 0.3 * rng.standard_normal((Bn, N, m))
    return X, U


def cpu_baseline(sid, X, U, dt, central, seconds):
    """oracle.linearize_loop (the reference's per-step, per-column F calls) over
    as many of the trajectories as fit in `seconds` on one core"""
    from oracle import dyn_oracle as dyn
    t0 = time.perf_counter()
    steps = 0
    k = 0
    while k < len(X) and (time.perf_counter() - t0) < seconds:
        dyn.linearize_loop(sid, X[k], U[k], dt, central=central)
        steps += U.shape[1]
        k += 1
    dt_s = time.perf_counter() - t0
    return {"value": steps / dt_s, "unit": "linearised steps/s", "cores": 1, "kind": "port",
            "sample": f"{k} trajectories x {U.shape[1]} steps, linearize_loop "
                      f"({'central' if central else 'forward'}), {dt_s:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--system", default="quadrotor", choices=sorted(SYS) + ["all"])
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--N", type=int, default=100)
    ap.add_argument("--central", action="store_true")
    ap.add_argument("--both", action="store_true", help="forward and central")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    args = ap.parse_args()
    import torch
    from time_opt_ilqr_amd import engine, systems
    dev = torch.device("cuda", 0)
    names = sorted(SYS, key=SYS.get) if args.system == "all" else [args.system]
    schemes = [False, True] if args.both else [args.central]
    for name in names:
        sid = SYS[name]
        n, m = engine.system_dims(sid)
        dt = list(systems.MAKERS.values())[sid]()[0].dt  # the maker's default step
        Bn, N = args.batch, args.N
        X, U = synth(sid, n, m, Bn, N)
        Xt = torch.as_tensor(X, device=dev)
        Ut = torch.as_tensor(U, device=dev)
        for central in schemes:
            out = engine.linearize(sid, Xt, Ut, dt, central=central)  # warm-up + buffers
            stream = torch.cuda.current_stream(dev)
            lib = engine._lib.load()
            args_c = (sid, dt, engine._lib.ptr(Xt), engine._lib.ptr(Ut), Bn, N, N, int(central),
                      1e-5, 1e-5, 1e-6, 1e-6, engine._lib.ptr(out.A), engine._lib.ptr(out.B),
                      engine._lib.ptr(out.a_res), None, engine._lib.stream_handle(dev))
            for _ in range(10):
                engine._lib.check(lib.hop_linearize_f64(*args_c))
            torch.cuda.synchronize()
            samples = []
            for _ in range(args.rounds):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.iters):
                    lib.hop_linearize_f64(*args_c)
                e1.record(stream)
                torch.cuda.synchronize()
                samples.append(e0.elapsed_time(e1) / args.iters)
            samples.sort()
            ms = samples[len(samples) // 2]
            byts = algorithmic_bytes(Bn, N, n, m)
            gbs = byts / (ms * 1e-3) / 1e9
            cpu = cpu_baseline(sid, X, U, dt, central, args.cpu_seconds) \
                if args.cpu_seconds > 0 else None
            print(json.dumps({
                "metric": "batched FD linearisation steps/s", "system": name, "n": n, "m": m,
                "scheme": "central" if central else "forward", "batch": Bn, "N": N,
                "value": Bn * N / (ms * 1e-3), "unit": "linearised steps/s",
                "kernel_ms": ms, "kernel_ms_min": samples[0], "dtype": "f64",
                "data": "synthetic",
                "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                             "bytes_per_launch": byts},
                "cpu_baseline": cpu}), flush=True)


if __name__ == "__main__":
    main()
