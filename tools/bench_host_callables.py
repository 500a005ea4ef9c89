"""Wall time of solver.ilqr_timeopt with the dynamics as a Python callable (host
evaluation, device select / Riccati / accept) against the device dynamics, per system,
and the oracle's scalar loop on one core for scale.  One JSON line per system.

    python tools/bench_host_callables.py [--systems di,quadrotor] [--repeat 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import dyn_oracle as dyn  # noqa: E402
from oracle import ilqr_oracle as io  # noqa: E402
from time_opt_ilqr_amd import host_dynamics, solver, systems  # noqa: E402
from time_opt_ilqr_amd.utils import as_terminal_weight  # noqa: E402


def _solve(F, mk, extra_cost, repeat):
    Fd, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, extra = mk
    best, sol = float("inf"), None
    for _ in range(repeat):
        t0 = time.perf_counter()
        sol = solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max,
                                  max_iter=15, wrap_idx=wrap_idx, extra_stage_cost=extra_cost)
        best = min(best, time.perf_counter() - t0)
    return best, sol


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--systems", default="di,cartpole,quadrotor,pointmass,segway")
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="batch of the row-vectorised run")
    a = ap.parse_args()
    for tag in a.systems.split(","):
        sid = dyn.SYSTEMS[tag]
        mk = list(systems.MAKERS.values())[sid]()
        Fd, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, extra = mk
        ec = extra["extra_stage_cost"] if extra else None
        _solve(Fd, mk, ec, 1)  # warm the device path
        t_dev, s_dev = _solve(Fd, mk, ec, a.repeat)
        obs = None
        host_cost = None
        if extra:
            obs = np.array([[o[0], o[1], r, wt] for o, r, wt in systems.OBSTACLES])
            host_cost = lambda x, u: io.obstacle_cost(x, obs)  # noqa: E731
        t_host, s_host = _solve(dyn._scalar_F(sid, Fd.dt), mk, host_cost, a.repeat)
        Fv = host_dynamics.HostDynamics(dyn._scalar_F(sid, Fd.dt), len(x0), np.atleast_2d(R).shape[0],
                                        vectorized=True)
        t_vec, s_vec = _solve(Fv, mk, host_cost, a.repeat)
        t_dpc = None
        if host_cost is not None:  # the device system with the cost as a Python callable
            t_dpc, s_dpc = _solve(Fd, mk, host_cost, a.repeat)
            assert s_dpc["T_hist"] == s_dev["T_hist"]
        t0 = time.perf_counter()
        o = io.ilqr_timeopt(sid, Fd.dt, x0, xg, u_ref, Q, np.atleast_2d(R),
                            np.asarray(as_terminal_weight(alpha, len(x0))), w, N, T_min, T_max,
                            max_iter=15, wrap_idx=wrap_idx, obstacles=obs)
        t_orc = time.perf_counter() - t0
        print(json.dumps(dict(system=tag, N=N, iters=len(s_host["T_hist"]),
                              same_T_hist=s_host["T_hist"] == s_vec["T_hist"] == s_dev["T_hist"] == o["T_hist"],
                              J_rel=float(abs(s_host["J_hist"][-1] - s_dev["J_hist"][-1]) /
                                          abs(s_dev["J_hist"][-1])),
                              device_dynamics_s=round(t_dev, 4), host_callable_s=round(t_host, 4),
                              host_vectorized_s=round(t_vec, 4),
                              device_dynamics_python_cost_s=None if t_dpc is None else round(t_dpc, 4),
                              oracle_1core_s=round(t_orc, 4))), flush=True)

    # a batch of quadrotor problems (x0 jittered by 1e-3): the device dynamics against the
    # row-vectorised callable through ilqr_timeopt_batch
    import torch
    Fd, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, _ = systems.make_quadrotor()
    X0 = x0 + 1e-3 * np.random.default_rng(0).standard_normal((a.batch, len(x0)))
    Qf = np.asarray(as_terminal_weight(alpha, len(x0)))
    Fv = host_dynamics.HostDynamics(dyn._scalar_F(2, Fd.dt), 12, 4, vectorized=True)
    out = {}
    for name, sysx, kw in (("device_dynamics_s", 2, dict(dt=Fd.dt)), ("host_vectorized_s", Fv, {})):
        best = float("inf")
        for _ in range(2):
            t0 = time.perf_counter()
            r = solver.ilqr_timeopt_batch(sysx, X0, xg, u_ref, Q, np.atleast_2d(R), Qf, w, N, T_min,
                                          T_max, max_iter=15, wrap_idx=wrap_idx, **kw)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        out[name] = round(best, 4)
        out[name.replace("_s", "_T_star")] = np.asarray(r["T_star"].cpu()).tolist()[:4]
    print(json.dumps(dict(system="quadrotor", batch=a.batch, **out)), flush=True)


if __name__ == "__main__":
    main()
