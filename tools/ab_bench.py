"""Same-process interleaved A/B of LFT kernel variants (hop_set_options: schedule
numbers need a developer build, HOP_DEV_BUILD=1; "g" = HOP_OPT_FORCE_GENERIC,
"r" = HOP_OPT_REFERENCE_ASSOC, "0" = the product default).

    python tools/ab_bench.py --variants 0,1,2,g --rounds 7 --iters 10

Rule: never rank builds by timings from different devices/processes
(cdna_hip_programming.md 5.4 rule 24).  Prints median / min ms per launch.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--N", type=int, default=100)
    ap.add_argument("--s", type=int, default=13)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    args = ap.parse_args()
    import torch
    from time_opt_ilqr_amd import _lib, engine, synth
    dev = torch.device("cuda", 0)
    dt = torch.float64 if args.dtype == "f64" else torch.float32
    A, Bm, Q, Ri, z0, QT = synth.device_batch(args.batch, args.s, args.m, args.N, seed=5,
                                              device=dev, dtype=dt)
    variants = args.variants.split(",")

    def setv(v):
        flags = {"g": _lib.OPT_FORCE_GENERIC, "r": _lib.OPT_REFERENCE_ASSOC}.get(v, 0)
        _lib.check(_lib.load().hop_set_options(flags, 0 if v in "gr" else int(v)))

    ref = None
    for v in variants:  # warm + cross-check
        setv(v)
        r = engine.propagate(A, Bm, Q, Ri, z0, QT)
        torch.cuda.synchronize()
        if ref is None:
            ref = r.J.clone()
        rel = float(((r.J - ref).abs() / ref.abs()).max())
        print(f"variant {v}: max rel vs first = {rel:.3e}", flush=True)
    times = {v: [] for v in variants}
    for rnd in range(args.rounds):
        # alternate the order every round (the first timing of a round can be biased)
        for v in (variants if rnd % 2 == 0 else variants[::-1]):
            setv(v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                engine.propagate(A, Bm, Q, Ri, z0, QT)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.iters)
    out = {v: {"median_ms": statistics.median(t), "min_ms": min(t),
               "sweeps_per_s": args.batch / (statistics.median(t) * 1e-3)} for v, t in times.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
