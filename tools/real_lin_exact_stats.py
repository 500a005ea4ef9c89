"""Per-candidate agreement with the exact (50-digit) select on the round-5 fixture
(VERDICT r04 item 1): for every system and every candidate of tools/real_lin_capture.py
(traj = the product select, traj_ref = the reference association on the device, aug =
augmented blocks through the product sweep, aug_ref, aug_gen = round 4's fp64 s = 5
drop-in path, the generic kernel) and the fp64 NumPy reference (the oracle, pinned to
the reference's outputs): T* misses against the exact T* (ties within 1e-9 of the
50-digit curve excepted), J relative error over [T_min, T_max].  CPU only.

    python tools/real_lin_exact_stats.py gpurun_out/<tag>/real_lin_capture.npz [out.jsonl]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TIE = 1e-9
CANDS = ("traj", "traj_ref", "aug", "aug_ref", "aug_gen")


def main():
    cap = np.load(sys.argv[1])
    fx = np.load(os.path.join(REPO, "tests", "golden", "real_lin_batch_hp.npz"))
    out = sys.argv[2] if len(sys.argv) > 2 else None
    lines = []
    for name in ("quadrotor", "segway", "cartpole", "di"):
        p = f"{name}_"
        T_min, T_max = int(fx[p + "meta"][0]), int(fx[p + "meta"][1])
        Jh, th = fx[p + "J_hp"], fx[p + "t_hp"]
        win = slice(T_min - 1, T_max)
        rec = dict(system=name, problems=int(len(th)), T_min=T_min, T_max=T_max,
                   selection_bits={str(b): int(((fx[p + "why"] & b) != 0).sum())
                                   for b in (1, 2, 4, 8, 16, 32, 64)})
        for k in CANDS + ("oracle",):
            J = fx[p + "J_oracle"] if k == "oracle" else cap[p + "J_" + k][:, :T_max]
            ts = fx[p + "t_oracle"] if k == "oracle" else cap[p + "t_" + k]
            rel = np.max(np.abs(J[:, win] - Jh[:, win]) / np.abs(Jh[:, win]), axis=1)
            miss = [b for b in range(len(th)) if ts[b] != th[b] and
                    abs(Jh[b, ts[b] - 1] - Jh[b, th[b] - 1]) > TIE * abs(Jh[b, th[b] - 1])]
            ties = int(sum(1 for b in range(len(th)) if ts[b] != th[b]) - len(miss))
            jstar = np.abs(J[np.arange(len(th)), th - 1] - Jh[np.arange(len(th)), th - 1]) / \
                np.abs(Jh[np.arange(len(th)), th - 1])
            rec[k] = dict(t_star_misses=len(miss), exact_ties=ties,
                          j_rel_max=float(rel.max()), j_rel_p50=float(np.median(rel)),
                          j_rel_gt_1e6=int((rel > 1e-6).sum()),
                          jstar_rel_max=float(jstar.max()),
                          miss_examples=[(int(fx[p + "idx"][b]), int(ts[b]), int(th[b]))
                                         for b in miss[:5]])
        print(json.dumps(rec), flush=True)
        lines.append(rec)
    if out:
        with open(out, "w") as f:
            for r in lines:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
