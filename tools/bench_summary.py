"""The reference's published comparison (plots/summary.csv) on the device.

    python tools/bench_summary.py [--batch 4096] [--runs 5]

For the two summary rows the current solver reproduces (DoubleIntegrator and
Quadrotor_Hover, methods propagator and bruteforce; tests/golden/summary_*.npz,
make_golden.py --summary), with the comparison's settings (max_iter=20,
lm_init=1e-3, central differences, the makers' default N and T range):

  * one solve through the reference-shaped drop-in solver.ilqr_timeopt, stages
    synchronised: per-stage seconds (median of --runs), next to the csv's
    published per-solve stage times (hardware unstated) and the reference run in
    the build container (the capture's own timers, 1 core);
  * the same problem as a batch of --batch solves (x0 jittered by 1e-3 per
    problem, ilqr_timeopt_batch, no stage syncs): solves per second.

One JSON line per (case, method).
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GOLDEN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests",
                      "golden")
STAGES = ("linearize", "select", "backward", "forward")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--runs", type=int, default=5)
    args = ap.parse_args()
    import torch
    from time_opt_ilqr_amd import solver, systems
    from time_opt_ilqr_amd.utils import as_terminal_weight
    for tag, mk in (("di", systems.make_double_integrator), ("quadrotor", systems.make_quadrotor)):
        F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, _ = mk()
        T_max = min(T_max, N)
        for method in ("propagator", "bruteforce"):
            d = np.load(os.path.join(GOLDEN, f"summary_{tag}_{method}.npz"))
            kw = dict(method=method, max_iter=20, lm_init=1e-3, wrap_idx=wrap_idx,
                      use_central_diff=True)
            solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, **kw)
            per, walls, sol = {k: [] for k in STAGES}, [], None
            for _ in range(args.runs):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                sol = solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max,
                                          **kw)
                walls.append(time.perf_counter() - t0)
                for k in STAGES:
                    per[k].append(sol["timers"][k])
            one = {k: statistics.median(v) for k, v in per.items()}
            # the batch: the same problem B times, x0 jittered so the problems differ
            rng = np.random.default_rng(4)
            X0 = np.asarray(x0, float) + 1e-3 * rng.standard_normal((args.batch, F.n))
            Qf = as_terminal_weight(alpha, F.n)
            bkw = dict(dt=F.dt, max_iter=20, lm_init=1e-3, wrap_idx=wrap_idx,
                       use_central_diff=True, method=method, stage_timers=False)
            solver.ilqr_timeopt_batch(F.system_id, X0, xg, u_ref, Q, R, Qf, w, N, T_min, T_max,
                                      **bkw)
            bw = []
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                res = solver.ilqr_timeopt_batch(F.system_id, X0, xg, u_ref, Q, R, Qf, w, N,
                                                T_min, T_max, **bkw)
                torch.cuda.synchronize()
                bw.append(time.perf_counter() - t0)
            bwall = statistics.median(bw)
            print(json.dumps({
                "case": tag, "method": method, "N": N, "T_min": T_min, "T_max": T_max,
                "T_star": sol["T_star"], "J_star": sol["J_hist"][-1],
                "csv_T_star": int(d["csv_T_star"]), "csv_J_star": float(d["csv_J_star"]),
                "iterations": len(sol["J_hist"]),
                "device_one_solve_s": {**{k: round(v, 6) for k, v in one.items()},
                                       "wall": round(statistics.median(walls), 6)},
                "csv_published_s": dict(zip(STAGES, [round(float(v), 6)
                                                     for v in d["csv_timers"]])),
                "reference_here_1core_s": dict(zip(STAGES, [round(float(v), 6)
                                                            for v in d["ref_here_timers"]])),
                "select_speedup_vs_csv": float(d["csv_timers"][1]) / one["select"],
                "batch": args.batch, "batch_wall_s": round(bwall, 6),
                "batch_solves_per_s": args.batch / bwall,
                "batch_crashed": int(res["crashed"].sum().item()),
                "dtype": "f64"}), flush=True)


if __name__ == "__main__":
    main()
