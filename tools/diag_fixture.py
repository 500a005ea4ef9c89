"""Per-horizon J of the select kernels on one real-linearisation fixture problem
against its 50-digit curve (tests/golden/real_lin_hp.npz), without the rerun
launch (developer library: the hand-over reason and horizon in status).

    HOP_LIB=time_opt_ilqr_amd/libhop_amd_dev.so python tools/diag_fixture.py quadrotor 3 [variant...]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
import make_hp as mh  # noqa: E402
from oracle import hop_oracle as orc  # noqa: E402
from time_opt_ilqr_amd import _lib, engine  # noqa: E402

name, idx = sys.argv[1], int(sys.argv[2])
variants = [int(v) for v in sys.argv[3:]] or [0]
d = np.load(os.path.join(REPO, "tests", "golden", "real_lin_hp.npz"))
sid, N, T_min, T_max, _, xg, ur, Q, R, alpha, w, wrap = mh.CASES[name][:12]
t = f"{name}_p{idx}"
dev = torch.device("cuda", 0)
T = lambda x: torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)  # noqa
raw = [T(d[f"{t}_{k}"][None, :N + (k == "X")]) for k in ("A", "B", "a_res", "X", "U")]
n = raw[3].shape[-1]
P = orc.terminal_weight(alpha, n)
Ri = orc.spd_inverse(orc.sym(R))[0]
Jh = d[f"{t}_J_hp"]
for v in variants:
    for rerun in (False, True):
        with _lib.options(variant=v, no_rerun=not rerun):
            r = engine.propagate_traj(*raw, T(xg), T(ur), T(Q), T(Ri), T(P), T(np.array([w])),
                                      wrap_idx=wrap, n_use=N, t_min=T_min, t_max=T_max)
        J = r.J.cpu().numpy()[0]
        st = int(r.status.cpu().numpy()[0])
        rel = np.abs(J - Jh) / np.abs(Jh)
        print(f"variant {v} rerun {rerun}: status {st} (reason {(st >> 5) & 255}, horizon "
              f"{st >> 13}) T* {int(r.t_star[0])} (hp {int(np.argmin(Jh[T_min - 1:T_max]) + T_min)})"
              f" max rel {rel.max():.2e} at {int(rel.argmax()) + 1}")
        worst = np.argsort(-rel)[:6]
        print("   worst horizons:", [(int(i) + 1, float(rel[i])) for i in worst])
