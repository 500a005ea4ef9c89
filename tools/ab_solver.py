"""Same-process interleaved timing of two versions of the device outer loop:
time_opt_ilqr_amd/solver.py against time_opt_ilqr_amd/_solver_ab.py (e.g. a copy
from git: `git show HEAD~1:time_opt_ilqr_amd/solver.py > time_opt_ilqr_amd/_solver_ab.py`),
quadrotor batch of tools/bench_forward.py, median wall time of --rounds runs each."""
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from time_opt_ilqr_amd import _solver_ab, solver, systems  # noqa: E402
from oracle import ilqr_oracle as io  # noqa: E402

Bn, N, iters, rounds = 4096, 100, 4, int(sys.argv[1]) if len(sys.argv) > 1 else 7
F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap, _ = systems.make_quadrotor(N=N)
rng = np.random.default_rng(9)
X0 = x0 + 0.2 * rng.standard_normal((Bn, F.n))
Qf = io.orc.terminal_weight(alpha, F.n)
kw = dict(dt=F.dt, max_iter=iters, wrap_idx=wrap, use_central_diff=False, stage_timers=False)
mods = {"new": solver, "old": _solver_ab}
for m in mods.values():
    m.ilqr_timeopt_batch(2, X0, xg, u_ref, Q, R, Qf, w, N, N // 5, N, **kw)
torch.cuda.synchronize()
t = {k: [] for k in mods}
res = {}
for _ in range(rounds):
    for k, m in mods.items():
        t0 = time.perf_counter()
        res[k] = m.ilqr_timeopt_batch(2, X0, xg, u_ref, Q, R, Qf, w, N, N // 5, N, **kw)
        torch.cuda.synchronize()
        t[k].append(time.perf_counter() - t0)
same = all(torch.equal(res["new"][f].nan_to_num(7.0) if res["new"][f].is_floating_point()
                       else res["new"][f],
                       res["old"][f].nan_to_num(7.0) if res["old"][f].is_floating_point()
                       else res["old"][f])
           for f in ("X", "U", "J_hist", "T_hist", "n_hist", "T_star", "crashed", "J_curve"))
for k in mods:
    ms = statistics.median(t[k]) * 1e3
    print(f"{k}: {ms:.3f} ms median ({Bn / ms * 1e3:.0f} problems/s), min {min(t[k]) * 1e3:.3f}")
print("outputs bitwise equal:", same)
