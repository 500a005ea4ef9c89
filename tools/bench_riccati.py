"""Throughput of the batched Riccati passes on one GPU.

    python tools/bench_riccati.py [--batch 4096] [--n 12] [--m 4] [--N 100]

Synthetic trajectory-form inputs of the oracle's distribution (device RNG),
horizon = N.  Prints one JSON line per mode: ms per launch, problems/s and the
SURVEY.md 8(d) FLOP estimate (4n^3 + 10n^2 m) * T per problem.
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
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch
    from time_opt_ilqr_amd import engine
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    Bn, n, m, N = args.batch, args.n, args.m, args.N
    kw = dict(device=dev, dtype=torch.float64, generator=g)
    A = torch.eye(n, device=dev, dtype=torch.float64) + 0.05 * torch.randn((Bn, N, n, n), **kw)
    Bm = 0.1 * torch.randn((Bn, N, n, m), **kw)
    X = 0.5 * torch.randn((Bn, N + 1, n), **kw)
    U = 0.1 * torch.randn((Bn, N, m), **kw)
    xg = 0.2 * torch.randn((n,), **kw)
    ur = 0.05 * torch.randn((m,), **kw)
    M = torch.randn((n, n), **kw)
    Q = M @ M.T / n + 0.5 * torch.eye(n, device=dev, dtype=torch.float64)
    R = torch.diag(0.5 + 1.5 * torch.rand((m,), **kw))
    Qf = 10.0 * torch.eye(n, device=dev, dtype=torch.float64)
    flop = (4 * n ** 3 + 10 * n * n * m) * N
    for mode in (0, 1):
        run = lambda: engine.riccati(A, Bm, X, U, xg, ur, Q, R, Qf, N, 1e-3, mode=mode)  # noqa: E731
        for _ in range(5):
            r = run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            r = run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        ok = int((r.status != 0).sum())
        print(json.dumps({"mode": mode, "batch": Bn, "n": n, "m": m, "N": N, "ms": ms,
                          "problems_per_s": Bn / (ms * 1e-3),
                          "tflops_est": flop * Bn / (ms * 1e-3) / 1e12,
                          "frac_fp64": flop * Bn / (ms * 1e-3) / 1e12 / 78.6,
                          "nonzero_status": ok}), flush=True)


if __name__ == "__main__":
    main()
