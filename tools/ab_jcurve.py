"""Same-process A/B of brute-force J-curve schedules (developer library: variant
numbers of hop_set_options; 0 = the product default), the bench's bruteforce shape
(B = 4096, N = T_max = 100, n = 12, m = 4).  Order alternates per round; prints the
median ms per launch and checks the curves are bitwise equal.

    HOP_DEV_BUILD=1 HOP_LIB=.../libhop_amd_dev.so python tools/ab_jcurve.py --variants 0,83
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,83")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096)
    args = ap.parse_args()
    import torch
    from time_opt_ilqr_amd import _lib, engine
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(13)
    n, m, N, Bn = 12, 4, 100, args.batch
    kw = dict(device=dev, dtype=torch.float64, generator=g)
    eye = torch.eye(n, device=dev, dtype=torch.float64)
    A = eye + 0.05 * torch.randn((Bn, N, n, n), **kw)
    Bm = 0.1 * torch.randn((Bn, N, n, m), **kw)
    X = 0.5 * torch.randn((Bn, N + 1, n), **kw)
    U = 0.3 * torch.randn((Bn, N, m), **kw)
    xg, ur = 0.2 * torch.randn((n,), **kw), 0.1 * torch.randn((m,), **kw)
    M = torch.randn((n, n), **kw)
    Q = M @ M.T / n + 0.5 * eye
    R = torch.diag(0.5 + 1.5 * torch.rand((m,), **kw))
    Qf = torch.diag(1.0 + 9.0 * torch.rand((n,), **kw))
    vs = [int(v) for v in args.variants.split(",")]
    run = lambda: engine.bruteforce_jcurve(A, Bm, X, U, xg, ur, Q, R, Qf, N,  # noqa: E731
                                           lm_lambda=1e-6, w_stage=0.5)[0]
    outs = {}
    for v in vs:
        with _lib.options(variant=v):
            outs[v] = run().clone()
    times = {v: [] for v in vs}
    for rnd in range(args.rounds):
        for v in (vs if rnd % 2 == 0 else vs[::-1]):
            with _lib.options(variant=v):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / args.iters)
    for v in vs:
        print(json.dumps({"variant": v, "median_ms": round(statistics.median(times[v]), 4),
                          "min_ms": round(min(times[v]), 4),
                          "bitwise_equal_to_first": bool(torch.equal(outs[v].nan_to_num(7.0),
                                                                     outs[vs[0]].nan_to_num(7.0)))}),
              flush=True)


if __name__ == "__main__":
    main()
