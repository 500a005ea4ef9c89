"""Host-side profile of one solver.ilqr_timeopt solve (device dynamics): where the wall
time of a single solve goes besides the kernels (cProfile, cumulative, top entries).

    python tools/prof_solve_host.py [--system quadrotor] [--top 30]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from time_opt_ilqr_amd import solver, systems
    ap = argparse.ArgumentParser()
    ap.add_argument("--system", default="quadrotor")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    mk = {"di": systems.make_double_integrator, "cartpole": systems.make_cartpole_swingup,
          "quadrotor": systems.make_quadrotor, "pointmass": list(systems.MAKERS.values())[3],
          "segway": systems.make_segway_balance}[a.system]
    F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, extra = mk()
    kw = dict(max_iter=15, wrap_idx=wrap_idx,
              extra_stage_cost=extra["extra_stage_cost"] if extra else None)
    for _ in range(2):
        solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sol = solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, **kw)
    wall = time.perf_counter() - t0
    print(f"{a.system}: wall {wall * 1e3:.2f} ms, {len(sol['T_hist'])} iterations, "
          f"timers {({k: round(v * 1e3, 3) for k, v in sol.get('timers', {}).items()})}")
    pr = cProfile.Profile()
    pr.enable()
    solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, **kw)
    pr.disable()
    out = io.StringIO()
    pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(a.top)
    print(out.getvalue())


if __name__ == "__main__":
    main()
