"""Per-iteration hand-over count of the select block inside the device outer loop
(quadrotor, tools/bench_forward.py's batch).  Needs the developer library
(HOP_LIB=time_opt_ilqr_amd/libhop_amd_dev.so): each select is run once more as
the closed-form conditioned kernel alone (variant 54, ST_RERUN left set)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from time_opt_ilqr_amd import _lib, engine, solver, systems  # noqa: E402
from oracle import ilqr_oracle as io  # noqa: E402

assert _lib.dev_build(), "run with HOP_LIB=time_opt_ilqr_amd/libhop_amd_dev.so"
Bn, N, iters = int(sys.argv[1]) if len(sys.argv) > 1 else 4096, 100, 4
F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap, _ = systems.make_quadrotor(N=N)
rng = np.random.default_rng(9)
X0 = x0 + 0.2 * rng.standard_normal((Bn, F.n))
Qf = io.orc.terminal_weight(alpha, F.n)
orig = engine.propagate_traj
log = []


def probe(*a, **k):
    with _lib.options(variant=54):
        r = orig(*a, **k)
    st = r.status.cpu().numpy()
    flagged = np.nonzero(st & 16)[0]
    log.append((len(st), flagged.tolist()[:12], len(flagged),
                {int(v): int(c) for v, c in zip(*np.unique(st, return_counts=True))}))
    return orig(*a, **k)


engine.propagate_traj = probe
res = solver.ilqr_timeopt_batch(2, X0, xg, u_ref, Q, R, Qf, w, N, max(1, N // 5), N, dt=F.dt,
                                max_iter=iters, wrap_idx=wrap, use_central_diff=False)
for i, (b, idx, n, hist) in enumerate(log):
    print(f"select {i}: batch {b}, handed over {n}: first {idx}; status histogram {hist}")
print("crashed", int(res["crashed"].sum().item()))
