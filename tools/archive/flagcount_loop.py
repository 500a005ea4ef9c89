"""How many problems the conditioned select kernel hands over (ST_RERUN) on the
outer loop's real trajectories (quadrotor, bench_forward.py's batch)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from time_opt_ilqr_amd import _lib, engine, systems  # noqa: E402
from time_opt_ilqr_amd.utils import _sym, chol_inv  # noqa: E402
from oracle import hop_oracle as orc  # noqa: E402

F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap, _ = systems.make_quadrotor(N=100)
N, Bn = 100, 4096
dev = torch.device("cuda", 0)
t = lambda a: torch.as_tensor(np.asarray(a, dtype=float), device=dev)  # noqa: E731
rng = np.random.default_rng(9)
X0 = x0 + 0.2 * rng.standard_normal((Bn, 12))
U = t(np.tile(u_ref, (Bn, N, 1)))
X = engine.rollout(2, t(X0), U, F.dt)
lin = engine.linearize(2, X, U, F.dt)
P = t(_sym(orc.terminal_weight(alpha, 12)))
Ri = t(chol_inv(_sym(R)))
for var, rho in (("54", 1e-12), ("41", 1e-12), ("54", 1.0)):
    # developer build: the conditioned kernel alone, ST_RERUN (16) left set
    _lib.check(_lib.load().hop_set_options(0, int(var)))
    r = engine.propagate_traj(lin.A, lin.B, lin.a_res, X, U, t(xg), t(u_ref), t(Q), Ri, P, w,
                              wrap_idx=wrap, t_min=20, t_max=100, rho_reg=rho)
    st = r.status.cpu().numpy()
    print(f"variant {var} rho_reg={rho}: status histogram", {int(k): int(v) for k, v in
                                                zip(*np.unique(st, return_counts=True))})
