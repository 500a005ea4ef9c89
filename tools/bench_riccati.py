"""Throughput of the batched Riccati passes on one GPU.

    python tools/bench_riccati.py [--batch 4096] [--n 12] [--m 4] [--N 100] [--variants 0,...]

Synthetic trajectory-form inputs of the oracle's distribution (device RNG),
horizon = N.  The clocks are pre-warmed for --prewarm-s seconds, then every
(variant, mode) is timed in interleaved rounds (same clock state for all; rule 24
of cdna_hip_programming.md 5.4) and the median is reported: one JSON line per
(variant, mode) with ms per launch, problems/s and the SURVEY.md 8(d) FLOP
count (bench.riccati_flops: 4n^3 + 10n^2 m + lower-order terms) * T per problem.  Nonzero variants are developer-build
experiments (HOP_LIB=<libhop_amd_dev.so>).
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--n", type=int, default=12)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--N", type=int, default=100)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--prewarm-s", type=float, default=1.0)
    ap.add_argument("--variants", default="0", help="comma list; nonzero needs HOP_LIB=<dev build>")
    ap.add_argument("--generic", action="store_true", help="also time HOP_OPT_FORCE_GENERIC")
    ap.add_argument("--jcurve", action="store_true",
                    help="also time the brute-force J curve (mode 2 in the output)")
    ap.add_argument("--libs", default="",
                    help="comma list of library paths to A/B in this process (variant 0 of each)")
    args = ap.parse_args()
    import torch
    from time_opt_ilqr_amd import _lib, engine
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
    from bench import riccati_bytes, riccati_flops  # SURVEY.md 8(d) count, term by term
    flop = {md: riccati_flops(n, m, N, md) for md in (0, 1)}
    byts = {md: riccati_bytes(n, m, N, md) for md in (0, 1)}
    # "mode" 2 = the brute-force J curve (hop_bruteforce_jcurve): N value-expansion
    # sweeps of lengths 1..N in one launch; flops summed over the horizons, bytes =
    # the inputs once (A, B, X, U) + J and the per-horizon status written
    flop[2] = sum(riccati_flops(n, m, T, 1) for T in range(1, N + 1))
    byts[2] = 8 * (N * n * n + N * n * m + (N + 1) * n + N * m) + 12 * N
    libs = {"": _lib.load()}
    for p in filter(None, args.libs.split(",")):
        libs[p] = _lib.load(p)
    modes = (0, 1, 2) if args.jcurve else (0, 1)
    cases = [(v, md, False, lp) for lp in libs for v in args.variants.split(",") for md in modes]
    if args.generic:
        cases += [("0", md, True, "") for md in (0, 1)]

    def run(case):
        v, md, gen, lp = case
        _lib._lib = libs[lp]
        with _lib.options(variant=int(v), force_generic=gen):
            if md == 2:
                J, st = engine.bruteforce_jcurve(A, Bm, X, U, xg, ur, Q, R, Qf, N,
                                                 lm_lambda=1e-6, w_stage=0.1)
                return engine.RiccatiResult(None, None, st, None, None, J)
            return engine.riccati(A, Bm, X, U, xg, ur, Q, R, Qf, N, 1e-3, mode=md)

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.prewarm_s:
        for c in cases:
            run(c)
        torch.cuda.synchronize()
    times = {c: [] for c in cases}
    status = {}
    for _ in range(args.rounds):
        for c in cases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                r = run(c)
            e1.record()
            torch.cuda.synchronize()
            times[c].append(e0.elapsed_time(e1) / args.iters)
            status[c] = int((r.status != 0).sum())
    for c in cases:
        ms = statistics.median(times[c])
        print(json.dumps({"lib": os.path.basename(c[3]) or "default", "variant": int(c[0]),
                          "generic": c[2], "mode": c[1], "batch": Bn,
                          "n": n, "m": m, "N": N, "ms": ms, "ms_min": min(times[c]),
                          "problems_per_s": Bn / (ms * 1e-3),
                          "tflops_est": flop[c[1]] * Bn / (ms * 1e-3) / 1e12,
                          "frac_fp64": flop[c[1]] * Bn / (ms * 1e-3) / 1e12 / 78.6,
                          "hbm_tbs": byts[c[1]] * Bn / (ms * 1e-3) / 1e12,
                          "frac_hbm": byts[c[1]] * Bn / (ms * 1e-3) / 1e12 / 8.0,
                          "nonzero_status": status[c]}), flush=True)


if __name__ == "__main__":
    main()
