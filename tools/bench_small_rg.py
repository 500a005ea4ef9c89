"""The fp64 s <= 5 sweep by batch size: the row-group kernel (lft_sweep_v2.hip
SchedCondSmall, four problems per wave) against the lane-per-problem kernel
(lft_small.hip), to place the crossover kSmallRowGroupMax.

    python tools/bench_small_rg.py [--out file.jsonl] [--batches 1,64,...]

Each batch size runs in two child processes: the default dispatch (the row-group
kernel up to kSmallRowGroupMax) and HOP_OPT_SMALL_LANE (the lane kernel for every
batch).  Workloads: synthetic SPD blocks of s = 5, m = 1, N = 200
(synth.device_batch) and the bench's cart-pole augmented blocks at rho_reg = 1e-12
(bench._s5_aug_side's construction: the drop-in's path at B = 4,096), and the same
cart-pole linearisation through the trajectory form (propagate_traj: the default
dispatch -- hop_augment + the row-group sweep up to kSmallRowGroupMax, the fused
lane-per-problem kernel above --, HOP_OPT_SMALL_LANE: the fused lane kernel at every
batch, HOP_OPT_TRAJ_UNFUSED: hop_augment + the block sweep at every batch).  HIP events
around 20 launches after 3 warm-ups, on torch's current stream.
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(batches, kind):
    sys.path.insert(0, REPO)
    import numpy as np
    import torch
    from time_opt_ilqr_amd import engine, synth, systems
    from time_opt_ilqr_amd.utils import as_terminal_weight
    dev = torch.device("cuda", 0)
    out = []
    for Bn in batches:
        N, t_min = 200, 40
        if kind == "synthetic":
            A, Bm, Q, Ri, z0, QT = synth.device_batch(Bn, 5, 1, N, seed=5, device=dev)
            lin = X = U = None
        else:
            F, x0, xg, u_ref, Qc, R, alpha, w, _, _, _, wrap, _ = systems.make_cartpole_swingup(N=N)
            g = torch.Generator(device=dev)
            g.manual_seed(29)
            kw = dict(device=dev, dtype=torch.float64, generator=g)
            U = torch.as_tensor(u_ref, device=dev) + 2.0 * torch.randn((Bn, N, F.m), **kw)
            X = engine.rollout(F.system_id, torch.as_tensor(x0, device=dev) +
                               0.3 * torch.randn((Bn, F.n), **kw), U, F.dt)
            t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)  # noqa
            lin = engine.linearize(F.system_id, X, U, F.dt, central=True)
            blk = engine.augment(lin.A, lin.B, lin.a_res, X, U, t(xg), t(u_ref), t(Qc),
                                 t(as_terminal_weight(alpha, F.n)), w, wrap_idx=wrap)
            A, Bm, Q, QT, z0 = blk.A, blk.B, blk.Q, blk.QT, blk.z0
            Ri = torch.linalg.inv(t(R)).contiguous()

        lane = os.environ.get("HOP_BENCH_SMALL_LANE", "0") == "1"

        def run():
            from time_opt_ilqr_amd import _lib
            with _lib.options(small_lane=lane):
                return engine.propagate(A, Bm, Q, Ri, z0, QT, t_min=t_min, t_max=N)

        if kind == "cartpole_traj":  # the trajectory form: fused (lane) or unfused (blocks)
            unf = os.environ.get("HOP_BENCH_TRAJ_UNFUSED", "0") == "1"

            def run():  # noqa: F811
                from time_opt_ilqr_amd import _lib
                with _lib.options(traj_unfused=unf, small_lane=lane):
                    return engine.propagate_traj(lin.A, lin.B, lin.a_res, X, U, t(xg), t(u_ref),
                                                 t(Qc), Ri, t(as_terminal_weight(alpha, F.n)), w,
                                                 wrap_idx=wrap, t_min=t_min, t_max=N)

        r = run()
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        fin = torch.isfinite(r.J).all(dim=1)
        out.append(dict(kind=kind, batch=Bn, ms=ms, sweeps_per_s=Bn / (ms * 1e-3),
                        status_ok=int(((r.status == 0) & fin).sum().item()),
                        t_star_sum=int(r.t_star.long().sum().item())))
        del A, Bm, Q, QT, r, lin, X, U
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--batches", default="1,16,64,256,1024,2048,4096,8192,16384,32768")
    ap.add_argument("--child", default=None)
    ap.add_argument("--kind", default="synthetic")
    a = ap.parse_args()
    batches = [int(b) for b in a.batches.split(",")]
    if a.child:
        child(batches, a.kind)
        return
    rows = []
    for kind in ("synthetic", "cartpole_aug", "cartpole_traj"):
        paths = ((("default", {}), ("lane", {"HOP_BENCH_SMALL_LANE": "1"})) if kind != "cartpole_traj"
                 else (("default", {}), ("traj_fused_lane", {"HOP_BENCH_SMALL_LANE": "1"}),
                       ("traj_unfused", {"HOP_BENCH_TRAJ_UNFUSED": "1"})))
        for label, env in paths:
            e = dict(os.environ, **env)
            p = subprocess.run([sys.executable, __file__, "--child", "1", "--kind", kind,
                                "--batches", a.batches], env=e, capture_output=True, text=True,
                               timeout=600)
            if p.returncode != 0:
                print(p.stdout[-2000:], p.stderr[-2000:], file=sys.stderr)
                sys.exit(p.returncode)
            for r in json.loads(p.stdout.strip().splitlines()[-1]):
                r["path"] = label
                rows.append(r)
                print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
