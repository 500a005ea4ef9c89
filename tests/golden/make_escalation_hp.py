"""50-digit ground truth for the genuine-escalation rerun test
(tests/test_gpu_rerun.py::test_pipelined_rerun_genuine_escalation_in_a_4096_batch).

The problem is config 2's (s = 13, m = 4, N = 100) problem 1234 of
synth.device_batch(seed=21) with Q_37 shifted so that its smallest eigenvalue is
-5e-7: chol_inv (utils.py:81-93) fails at 1e-9, 1e-8, 1e-7 and settles on 1e-6.  The
inputs come from tools/dump_escalation_case.py on the GPU box (the device RNG); this
script evaluates horizon_selection.py:36-86 on them in 50-digit arithmetic (make_hp.
hp_curve, with the reference's jitter 1e-6 at stage 37) and the NumPy oracle, and
writes both curves beside the inputs:

    python tests/golden/make_escalation_hp.py <dump.npz> [out.npz]

On this problem the oracle's fp64 Cholesky inverses are 1.5e-3 from the exact curve
after the escalated stage (E_37 ~ 1e6): an fp64 evaluation of the reference
association is only as good as its conditioning, so the test bounds the device curve
against the exact one, not against the oracle.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import make_hp as mh  # noqa: E402
from oracle import hop_oracle as orc  # noqa: E402


def main():
    d = np.load(sys.argv[1])
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(HERE, "escalation_hp.npz")
    k = int(d["k"])
    N = d["A"].shape[0]
    args = (d["A"], d["B"], d["Q"], d["Ri"], d["z0"], d["QT"])
    o = orc.lft_sweep(*args, N)
    J_hp = np.asarray(mh.hp_curve(*args, N, eps_E={k: "1e-6"}), dtype=np.float64)
    rel = lambda J: np.max(np.abs(J - J_hp) / np.abs(J_hp))  # noqa: E731
    print(f"oracle status {int(o['status'])}; oracle vs 50-digit {rel(o['J']):.3e}; "
          f"device (dump) vs 50-digit {rel(d['J']):.3e}")
    np.savez_compressed(out, A=d["A"], B=d["B"], Q=d["Q"], Ri=d["Ri"], z0=d["z0"], QT=d["QT"],
                        k=k, J_hp=J_hp, J_oracle=o["J"], status_oracle=int(o["status"]))
    print("saved", out)


if __name__ == "__main__":
    main()
