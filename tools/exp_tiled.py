"""Timing experiment (developer build): the small-s sweep on tile64 blocks (include/hop.h):
the default (fp32: conditioned association + rerun), every problem handed over to the
LFT kernel (HOP_OPT_FORCE_HANDOVER: the LFT association's time plus one conditioned
pass) and the stream alone (variant 78), against batch-major blocks.  J compared.

    HOP_LIB=<libhop_amd_dev.so> python tools/exp_tiled.py [--batch 65536] [--N 200] [--s 5] [--m 1]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--N", type=int, default=200)
    ap.add_argument("--s", type=int, default=5)
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import torch
    from time_opt_ilqr_amd import _lib, engine, synth
    dev = torch.device("cuda", 0)
    dt = torch.float32 if args.dtype == "f32" else torch.float64
    A, Bm, Q, Ri, z0, QT = synth.device_batch(args.batch, args.s, args.m, args.N, seed=5,
                                              device=dev, dtype=dt)
    tiled = [engine.to_tile64(x) for x in (A, Bm, Q, QT)]
    cases = {"batch:0": ((A, Bm, Q, QT), 0, 0), "tile:0": (tiled, 0, 0),
             "tile:handover": (tiled, 0, _lib.OPT_FORCE_HANDOVER), "tile:78": (tiled, 78, 0)}
    lib = _lib.load()

    def run(c):
        (a, b, q, qt), v, flags = cases[c]
        _lib.check(lib.hop_set_options(flags, v))
        return engine.propagate(a, b, q, Ri, z0, qt, t_min=20, t_max=args.N)

    J0 = run("batch:0").J
    for c in ("tile:0", "tile:handover"):
        J = run(c).J
        torch.cuda.synchronize()
        print(c, "max rel vs batch-major:", float(((J - J0).abs() / J0.abs()).max()), flush=True)
    times = {c: [] for c in cases}
    for _ in range(args.rounds):
        for c in cases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                run(c)
            e1.record()
            torch.cuda.synchronize()
            times[c].append(e0.elapsed_time(e1) / args.iters)
    print(json.dumps({c: statistics.median(t) for c, t in times.items()}))


if __name__ == "__main__":
    main()
