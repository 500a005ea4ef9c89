import os, sys
import numpy as np
import torch
sys.path.insert(0, os.getcwd())
from time_opt_ilqr_amd import _lib, engine, solver, systems
from oracle import ilqr_oracle as io
Bn, N, iters = 4096, 100, 4
F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap, _ = systems.make_quadrotor(N=N)
rng = np.random.default_rng(9)
X0 = x0 + 0.2 * rng.standard_normal((Bn, F.n))
Qf = io.orc.terminal_weight(alpha, F.n)
orig = engine.propagate_traj
def probe(*a, **k):
    with _lib.options(variant=54):
        r = orig(*a, **k)
    st = r.status.cpu().numpy()
    fl = np.nonzero(st & 16)[0]
    r2 = orig(*a, **k)
    if len(fl):
        print("flagged", fl.tolist(), "final status", r2.status.cpu().numpy()[fl].tolist(), "t_star", r2.t_star.cpu().numpy()[fl].tolist(), flush=True)
    return r2
engine.propagate_traj = probe
solver.ilqr_timeopt_batch(2, X0, xg, u_ref, Q, R, Qf, w, N, max(1, N // 5), N, dt=F.dt, max_iter=iters, wrap_idx=wrap, use_central_diff=False)
