"""Cost of a genuine hand-over: the config-2 select (s = 13,
m = 4, N = 100, B = 4096, fp64) on a clean batch and on the same batch with one
problem whose stage block needs chol_inv's second jitter (1e-9 -> 1e-8,
utils.py:81-93), on augmented blocks (hop_lft_sweep: the conditioned kernel + the
rerun launch).  Same process, libraries and cases interleaved, HIP events.

    python tools/bench_rerun.py [lib.so ...] [--rounds 9]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import numpy as np
    import torch
    from time_opt_ilqr_amd import _lib, engine, synth
    dev = torch.device("cuda", 0)
    libs = [_lib.load(p) for p in args.libs] if args.libs else [_lib.load()]
    names = [os.path.basename(p) for p in args.libs] if args.libs else ["libhop_amd.so"]
    Bn, s, m, N, b, k = 4096, 13, 4, 100, 1234, 37
    A, Bm, Q, Ri, z0, QT = synth.device_batch(Bn, s, m, N, seed=21, device=dev)
    Qe = Q.clone()
    q = Qe[b, k].cpu().numpy()
    lo = np.linalg.eigvalsh(0.5 * (q + q.T)).min()
    Qe[b, k] = torch.as_tensor(q - np.eye(s) * (lo + 5e-9), device=dev)
    work = {
        "blocks_clean": lambda: engine.propagate(A, Bm, Q, Ri, z0, QT, t_min=40, t_max=N),
        "blocks_escalated": lambda: engine.propagate(A, Bm, Qe, Ri, z0, QT, t_min=40, t_max=N),
    }
    times = {(w, i): [] for w in work for i in range(len(libs))}
    status = {}
    for i, L in enumerate(libs):
        _lib._lib = L
        for w, f in work.items():
            r = f()
            torch.cuda.synchronize()
            status[(w, i)] = int((r.status != 0).sum())
    for rnd in range(args.rounds):
        for w, f in work.items():
            for i in (range(len(libs)) if rnd % 2 == 0 else reversed(range(len(libs)))):
                _lib._lib = libs[i]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    f()
                e1.record()
                torch.cuda.synchronize()
                times[(w, i)].append(e0.elapsed_time(e1) / args.iters)
    for i, nm in enumerate(names):
        med = {w: statistics.median(times[(w, i)]) for w in work}
        print(json.dumps({"lib": nm, "ms": {w: round(v, 4) for w, v in med.items()},
                          "nonzero_status": {w: status[(w, i)] for w in work},
                          "escalated_over_clean": round(med["blocks_escalated"] /
                                                        med["blocks_clean"], 3)}), flush=True)


if __name__ == "__main__":
    main()
