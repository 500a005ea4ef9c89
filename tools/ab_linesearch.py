"""Same-process A/B of the quadrotor line search (developer library: 0 = the
product default, two lanes per rollout; 93 = one lane per rollout): interleaved
timing (HIP events, order alternating per round) and a bitwise check of J, the
accepted index, X' and U' between the variants, on bench_forward's problem with
per-problem horizons 1..N (so k >= T steps and the terminal cost run too).

    HOP_DEV_BUILD=1 HOP_LIB=.../libhop_amd_dev.so python tools/ab_linesearch.py --variants 0,93
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,93")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--N", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import numpy as np
    import torch
    from time_opt_ilqr_amd import _lib, engine
    import bench_forward as bf
    dev = torch.device("cuda", 0)
    F, (X, U, K, k), (x0, xg, ur, Q, R, Qf, w, wrap, obs) = bf.problem(2, args.batch, args.N)
    t = lambda a: torch.as_tensor(a, dtype=torch.float64, device=dev)  # noqa: E731
    cost = engine.CostParams(t(xg), t(ur), t(Q), t(R), t(Qf), w, None, wrap)
    Xt, Ut, Kt, kt = t(X), t(U), t(K), t(k)
    rng = np.random.default_rng(1)
    T = torch.as_tensor(rng.integers(0, args.N + 1, args.batch).astype(np.int32), device=dev)
    T[: args.batch // 2] = args.N
    vs = [int(v) for v in args.variants.split(",")]
    run = lambda: engine.forward_linesearch(2, Xt, Ut, T, Kt, kt, cost, F.dt)  # noqa: E731
    outs = {}
    for v in vs:
        with _lib.options(variant=v):
            r = run()
            outs[v] = [x.clone() for x in (r.J, r.accepted, r.X, r.U)]
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
    ref = outs[vs[0]]
    acc = ref[1].cpu().numpy()
    for v in vs:
        same = all(torch.equal(a.nan_to_num(7.0) if a.is_floating_point() else a,
                               b.nan_to_num(7.0) if b.is_floating_point() else b)
                   for a, b in zip(outs[v], ref))
        print(json.dumps({"variant": v, "median_ms": round(statistics.median(times[v]), 4),
                          "min_ms": round(min(times[v]), 4), "bitwise_equal_to_first": bool(same),
                          "accepted_hist": {int(i): int((acc == i).sum()) for i in np.unique(acc)}}),
              flush=True)


if __name__ == "__main__":
    main()
