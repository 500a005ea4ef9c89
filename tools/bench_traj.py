"""Trajectory-form select block on one GPU: in-kernel builders (fused) vs
hop_augment + the augmented-form sweep (unfused) vs the sweep alone on
pre-built blocks.

    python tools/bench_traj.py [--batch 4096] [--n 12] [--m 4] [--N 100]

Synthetic inputs of oracle.synth_traj_problem's distribution drawn with the
device RNG (rho_reg = 1e-12 as the reference).  One JSON line per path.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--n", type=int, default=12)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--N", type=int, default=100)
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=9)
    args = ap.parse_args()
    import torch
    from time_opt_ilqr_amd import _lib, engine
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    Bn, n, m, N = args.batch, args.n, args.m, args.N
    fdt = torch.float64 if args.dtype == "f64" else torch.float32
    kw = dict(device=dev, dtype=fdt, generator=g)
    eye = torch.eye(n, device=dev, dtype=fdt)
    A = eye + 0.05 * torch.randn((Bn, N, n, n), **kw)
    Bm = 0.1 * torch.randn((Bn, N, n, m), **kw)
    X = 0.5 * torch.randn((Bn, N + 1, n), **kw)
    U = 0.3 * torch.randn((Bn, N, m), **kw)
    a_res = 0.02 * torch.randn((Bn, N, n), **kw)
    xg = 0.2 * torch.randn((n,), **kw)
    ur = 0.1 * torch.randn((m,), **kw)
    M = torch.randn((n, n), **kw)
    Q = M @ M.T / n + 0.5 * eye
    Rinv = torch.diag(1.0 / (0.5 + 1.5 * torch.rand((m,), **kw)))
    P = torch.diag(1.0 + 9.0 * torch.rand((n,), **kw))
    w = 0.5
    targs = (A, Bm, a_res, X, U, xg, ur, Q, Rinv, P, w)
    blk = engine.augment(A, Bm, a_res, X, U, xg, ur, Q, P, w)

    def run(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.iters

    def traj_unfused():
        with _lib.options(traj_unfused=True):
            engine.propagate_traj(*targs, t_min=1, t_max=N)

    paths = {
        "traj_fused": lambda: engine.propagate_traj(*targs, t_min=1, t_max=N),
        "traj_fused_wrap": lambda: engine.propagate_traj(*targs, wrap_idx=[n - 1], t_min=1,
                                                         t_max=N),
        "sweep_prebuilt": lambda: engine.propagate(blk.A, blk.B, blk.Q, Rinv, blk.z0, blk.QT,
                                                   t_min=1, t_max=N),
        "augment_only": lambda: engine.augment(A, Bm, a_res, X, U, xg, ur, Q, P, w),
        "traj_unfused": traj_unfused,
    }
    for fn in paths.values():  # warm-up (clocks settle)
        for _ in range(20):
            fn()
    torch.cuda.synchronize()
    samples = {k: [] for k in paths}
    for _ in range(args.rounds):  # interleaved rounds: same clock state for every path
        for k, fn in paths.items():
            samples[k].append(run(fn))
    for name, v in samples.items():
        v = sorted(v)
        ms = v[len(v) // 2]
        print(json.dumps({"path": name, "batch": Bn, "n": n, "m": m, "N": N, "dtype": args.dtype,
                          "ms_median": ms,
                          "ms_min": v[0], "sweeps_per_s": Bn / (ms * 1e-3)}), flush=True)


if __name__ == "__main__":
    main()
