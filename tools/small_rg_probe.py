"""One fp64 s = 5 sweep shape (synthetic blocks, m = 1, N = 200, B = 4,096) launched
--reps times, for rocprofv3 kernel traces / PMC passes of the small-s paths:
--path rowgroup (the default dispatch: lft_sweep_v2.hip SchedCondSmall) or lane
(HOP_OPT_SMALL_LANE: lft_small.hip)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--path", choices=["rowgroup", "lane"], default="rowgroup")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch
    from time_opt_ilqr_amd import _lib, engine, synth
    dev = torch.device("cuda", 0)
    blk = synth.device_batch(a.batch, 5, 1, 200, seed=6, device=dev)
    with _lib.options(small_lane=(a.path == "lane")):
        for _ in range(a.reps):
            r = engine.propagate(*blk, t_min=40, t_max=200)
    torch.cuda.synchronize()
    print(a.path, int(r.t_star.long().sum()), int(r.status.abs().sum()))


if __name__ == "__main__":
    main()
