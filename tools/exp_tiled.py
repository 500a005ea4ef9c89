"""Timing experiment (developer build): the small-s kernel on a tiled HBM layout
[B/64][N][block elements][64] (variant 79; 78 = its LDS-DMA alone) against the
batch-major layout (variant 0).  Same problems, permuted into tiles; J compared.

    HOP_LIB=<libhop_amd_dev.so> python tools/exp_tiled.py [--batch 65536] [--N 200] [--s 5] [--m 1]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def tile(x):
    B, N = x.shape[:2]
    E = x[0, 0].numel()
    return x.reshape(B // 64, 64, N, E).permute(0, 2, 3, 1).contiguous().reshape(x.shape)


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
    At, Bt, Qt, QTt = tile(A), tile(Bm), tile(Q), tile(QT)
    cases = {"0": (A, Bm, Q, QT), "76": (A, Bm, Q, QT), "79": (At, Bt, Qt, QTt),
             "78": (At, Bt, Qt, QTt), "77": (A, Bm, Q, QT)}
    lib = _lib.load()

    def run(v):
        a, b, q, qt = cases[v]
        _lib.check(lib.hop_set_options(0, int(v)))
        return engine.propagate(a, b, q, Ri, z0, qt)

    J0 = run("0").J
    for v in ("76", "79"):
        J = run(v).J
        torch.cuda.synchronize()
        print(v, "max rel vs 0:", float(((J - J0).abs() / J0.abs()).max()), flush=True)
    times = {v: [] for v in cases}
    for _ in range(args.rounds):
        for v in cases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                run(v)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.iters)
    print(json.dumps({v: statistics.median(t) for v, t in times.items()}))


if __name__ == "__main__":
    main()
