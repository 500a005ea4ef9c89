"""Randomised bitwise check of the fp64 s <= 5 pipelined rerun against the one-lane rerun
(HOP_OPT_RERUN_LANE): synthetic batches of 1-3 problems per shape whose stage blocks get
random negative shifts at random steps -- magnitudes spread over the jitter ladder's
range (1e-10 .. 10) so that ladders stop at every rung, reach the LU slot, or are not
needed -- and random N (beats cut anywhere).  Prints one JSON line per shape with the
number of cases, ladder / LU counts and mismatches; exits non-zero on a mismatch.

    python tools/stress_small_rerun.py [--cases 40]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from oracle import hop_oracle as orc
    from time_opt_ilqr_amd import _lib, engine
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=40)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    bad_total = 0
    for s, m in ((5, 2), (5, 1), (4, 2), (4, 1), (3, 1), (2, 1)):
        rng = np.random.default_rng(1000 + 10 * s + m)
        n_cases = n_ladder = n_lu = bad = 0
        for c in range(a.cases):
            N = int(rng.integers(1, 180))
            nb = int(rng.integers(1, 4))
            A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(int(rng.integers(1 << 30)), nb, s, m, N)
            Q = Q.copy()
            for b in range(nb):
                ks = rng.choice(N, size=max(1, N // 3), replace=False)
                for k in ks:
                    i = int(rng.integers(s))
                    Q[b, k, i, i] -= 10.0 ** rng.uniform(-10, 1)
            t = lambda x: torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)  # noqa: E731
            args = [t(A), t(Bm), t(Q), t(Ri), t(z0[0]), t(QT)]
            tmin = max(1, N // 4)
            p = engine.propagate(*args, t_min=tmin, t_max=N)
            with _lib.options(rerun_lane=True):
                q = engine.propagate(*args, t_min=tmin, t_max=N)
            torch.cuda.synchronize()
            same = (torch.equal(p.J.nan_to_num(7.0), q.J.nan_to_num(7.0)) and
                    torch.equal(p.status, q.status) and torch.equal(p.t_star, q.t_star) and
                    torch.equal(p.j_star.nan_to_num(7.0), q.j_star.nan_to_num(7.0)))
            st = p.status.cpu().numpy()
            n_cases += 1
            n_ladder += int(((st & _lib.ST_JITTER) != 0).sum())
            n_lu += int(((st & _lib.ST_LU) != 0).sum())
            bad += 0 if same else 1
        bad_total += bad
        print(json.dumps(dict(s=s, m=m, cases=n_cases, problems_with_ladder=n_ladder,
                              problems_with_lu=n_lu, mismatching_cases=bad)), flush=True)
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()
