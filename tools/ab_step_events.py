"""Does the bench's per-step HIP event pair cost wall time?  Config 2 (s = 13, m = 4,
N = 100, B = 4,096, fp64 synthetic blocks), K steps timed by wall clock between two
synchronisations, in alternating rounds: (a) an event pair recorded around every step
(bench.py's timed loop, for kernel_ms), (b) no per-step events, (c) one event pair
around the whole K steps.  The kernel trace of config 2 under rocprofv3 shows a ~10 us
idle gap after each step's rerun launch (tools/launch_gaps.py); this separates the
event records from the launch path itself.

    python tools/ab_step_events.py [--steps 2000] [--rounds 5] [--workload lft|select_gains]
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
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--workload", default="lft")
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    args = argparse.Namespace(s=13, m=4, N=100, dtype="f64", t_min=40, layout="auto",
                              no_alt=True, rho_reg=1e-12)
    launch, _ = bench.WORKLOADS[a.workload](args, 1, 0, 4096, dev)
    for _ in range(200):
        launch()
    torch.cuda.synchronize()
    K = a.steps
    res = {"per_step_events": [], "no_events": [], "outer_events": []}
    for rnd in range(a.rounds):
        order = list(res) if rnd % 2 == 0 else list(reversed(list(res)))
        for mode in order:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(K if mode == "per_step_events" else 1)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if mode == "outer_events":
                ev[0][0].record()
            for i in range(K):
                if mode == "per_step_events":
                    ev[i][0].record()
                launch()
                if mode == "per_step_events":
                    ev[i][1].record()
            if mode == "outer_events":
                ev[0][1].record()
            torch.cuda.synchronize()
            res[mode].append((time.perf_counter() - t0) / K * 1e3)
    out = {m: {"ms_per_step_median": round(statistics.median(v), 5),
               "rounds": [round(x, 5) for x in v]} for m, v in res.items()}
    out["workload"] = a.workload
    out["steps"] = K
    print(json.dumps(out))


if __name__ == "__main__":
    main()
