"""Select latency against the batch size (VERDICT r05 missing item 3, the low-occupancy
regime): the LFT sweep + fused argmin at B = 1 .. 4096 for config 2's shape (s = 13,
m = 4, N = 100) and the s = 5 augmented blocks (m = 1, N = 200), fp64, the default
kernels; the time per select and per problem.  One JSON line per (shape, B).

    python tools/bench_small_batch.py [--reps 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from time_opt_ilqr_amd import engine, synth
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for s, m, N in ((13, 4, 100), (5, 1, 200)):
        A, Bm, Q, Ri, z0, QT = synth.device_batch(4096, s, m, N, seed=17, device=dev)
        for B in (1, 4, 16, 64, 256, 1024, 4096):
            args = [x[:B].contiguous() for x in (A, Bm, Q, Ri)] + [z0, QT[:B].contiguous()]
            for _ in range(3):
                r = engine.propagate(*args, t_min=N // 4, t_max=N)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                r = engine.propagate(*args, t_min=N // 4, t_max=N)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            print(json.dumps(dict(s=s, m=m, N=N, batch=B, ms_per_select=round(ms, 4),
                                  us_per_step=round(1e3 * ms / N, 3),
                                  problems_per_s=round(B / ms * 1e3, 1),
                                  status_ok=int(r.status.abs().sum()) == 0)), flush=True)


if __name__ == "__main__":
    main()
