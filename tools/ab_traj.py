"""Same-process interleaved A/B of the trajectory-form select kernel variants on
real quadrotor linearisations (tests/real_lin.py's batch: perturbed rollouts,
central differences, rho_reg = 1e-12).  Variant numbers need the developer
library (HOP_LIB=time_opt_ilqr_amd/libhop_amd_dev.so); 0 = the product default.

    python tools/ab_traj.py --variants 0,97 --rounds 9 --iters 10 [--system quadrotor|synthetic]
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,97")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--system", default="quadrotor")
    ap.add_argument("--finite-only", action="store_true",
                    help="drop problems with a non-finite rollout (the outer loop does)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import real_lin
    from time_opt_ilqr_amd import _lib, engine
    dev = torch.device("cuda", 0)
    if args.system == "synthetic":  # tools/ab_libs.py's select_traj_cf inputs (rho_reg = 1)
        g = torch.Generator(device=dev)
        g.manual_seed(3)
        n, m, N, Bn = 12, 4, 100, args.batch
        kw = dict(device=dev, dtype=torch.float64, generator=g)
        A = torch.eye(n, device=dev, dtype=torch.float64) + 0.05 * torch.randn((Bn, N, n, n), **kw)
        B = 0.1 * torch.randn((Bn, N, n, m), **kw)
        M = torch.randn((n, n), **kw)
        Q = M @ M.T / n + 0.5 * torch.eye(n, device=dev, dtype=torch.float64)
        Ri = torch.linalg.inv(torch.diag(0.5 + 1.5 * torch.rand((m,), **kw)))
        Qf = 10.0 * torch.eye(n, device=dev, dtype=torch.float64)
        X = 0.5 * torch.randn((Bn, N + 1, n), **kw)
        U = 0.3 * torch.randn((Bn, N, m), **kw)
        xg, ur = 0.2 * torch.randn((n,), **kw), 0.1 * torch.randn((m,), **kw)
        ar = 0.02 * torch.randn((Bn, N, n), **kw)
        targs = (A, B, ar, X, U, xg, ur, Q, Ri, Qf, 0.5)
        common = dict(t_min=40, t_max=N, rho_reg=1.0)
    else:
        d = real_lin.build(args.system, args.batch, 1000, dev)
        lin, t = d["lin"], d["t"]
        X, U, A, B, ar = d["X"], d["U"], lin.A, lin.B, lin.a_res
        if args.finite_only:
            keep = torch.isfinite(X[:, :d["T_max"] + 1]).flatten(1).all(1)
            X, U, A, B, ar = (v[keep].contiguous() for v in (X, U, A, B, ar))
        common = dict(wrap_idx=d["wrap"], t_min=d["T_min"], t_max=d["T_max"], n_use=d["T_max"])
        targs = (A, B, ar, X, U, t(d["xg"]), t(d["u_ref"]), t(d["Q"]), t(d["Ri"]), t(d["P"]),
                 t(np.array([d["w"]])))
    variants = args.variants.split(",")
    base = None
    for v in variants:
        with _lib.options(variant=int(v)):
            r = engine.propagate_traj(*targs, **common)
        torch.cuda.synchronize()
        if base is None:
            base = r
        diff = int((r.t_star != base.t_star).sum())
        print(f"variant {v}: T* differs from the first on {diff} of {len(r.t_star)}", flush=True)
    times = {v: [] for v in variants}
    for rnd in range(args.rounds):
        for v in (variants if rnd % 2 == 0 else variants[::-1]):
            with _lib.options(variant=int(v)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    engine.propagate_traj(*targs, **common)
                e1.record()
                torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.iters)
    out = {v: {"median_ms": statistics.median(tt), "min_ms": min(tt)} for v, tt in times.items()}
    print(json.dumps({"system": args.system, "batch": int(X.shape[0]), "ab": out}), flush=True)


if __name__ == "__main__":
    main()
