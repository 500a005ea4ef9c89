"""Agreement with the exact (50-digit) select on every problem of tests/golden/
real_lin_batch_hp.npz, per system and per path, with the library as built (VERDICT r04
item 1: "record the same statistics for the aug path / drop-in and for the oracle"):

  traj      the product select (propagate_traj: hop_lft_sweep_traj_f64)
  traj_ref  the same blocks with the reference association on the device
            (HOP_OPT_REFERENCE_ASSOC: the LFT kernels, horizon_selection.py:36-86)
  aug       hop_augment + propagate (the drop-in propagator_all_Jt_aug's kernels)
  aug_ref   the same with the reference association
  oracle    the fp64 NumPy reference on the same blocks (stored in the fixture)

T* misses against the exact T* (ties within 1e-9 of the 50-digit curve excepted) and
the J relative error over [T_min, T_max].  Inputs regenerated on the device from the
stored x0 / U, fingerprints checked, as tests/test_gpu_real_lin.py does.

    python tools/real_lin_fixture_stats.py [out.jsonl]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def main():
    import torch
    import make_hp_batch as mb
    import test_gpu_real_lin as T
    from oracle import hop_oracle as orc
    from time_opt_ilqr_amd import _lib, engine
    dev = torch.device("cuda", 0)
    golden = os.path.join(REPO, "tests", "golden")
    out = open(sys.argv[1], "w") if len(sys.argv) > 1 else None
    for name in ("quadrotor", "segway", "cartpole", "di"):
        f, F = T._fixture_system(golden, name)
        T_min, T_max = int(f["meta"][0]), int(f["meta"][1])
        t = lambda x: torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)  # noqa
        X = engine.rollout(F.system_id, t(f["X0"]), t(f["U"]), F.dt)
        lin = engine.linearize(F.system_id, X, t(f["U"]), F.dt, central=True)
        fp = mb.fingerprint(lin.A.cpu().numpy()[:, :T_max], lin.B.cpu().numpy()[:, :T_max],
                            lin.a_res.cpu().numpy()[:, :T_max], X.cpu().numpy()[:, :T_max + 1])
        fp_ok = bool(np.allclose(fp, f["fp"], rtol=1e-13, atol=0))
        n = X.shape[-1]
        P = orc.terminal_weight(f["alpha"][()] if f["alpha"].ndim == 0 else f["alpha"], n)
        Ri = orc.spd_inverse(orc.sym(f["R"]))[0]
        wrap = [int(i) for i in f["wrap"]]
        w = float(f["w"][0])
        common = dict(wrap_idx=wrap, t_min=T_min, t_max=T_max)
        U, xg, ur, Q = t(f["U"]), t(f["xg"]), t(f["u_ref"]), t(f["Q"])
        blk = engine.augment(lin.A, lin.B, lin.a_res, X, U, xg, ur, Q, t(P), t(np.array([w])),
                             wrap_idx=wrap, n_build=T_max)
        runs = {}
        for tag, opts in (("traj", {}), ("traj_ref", {"reference_assoc": True})):
            with _lib.options(**opts):
                runs[tag] = engine.propagate_traj(lin.A, lin.B, lin.a_res, X, U, xg, ur, Q, t(Ri),
                                                  t(P), t(np.array([w])), n_use=T_max, **common)
        for tag, opts in (("aug", {}), ("aug_ref", {"reference_assoc": True})):
            with _lib.options(**opts):
                runs[tag] = engine.propagate(blk.A, blk.B, blk.Q, t(Ri), blk.z0, blk.QT,
                                             t_min=T_min, t_max=T_max)
        torch.cuda.synchronize()
        Jh, th = f["J_hp"], f["t_hp"]
        rec = {"system": name, "problems": int(len(th)), "T_min": T_min, "T_max": T_max,
               "inputs_fingerprint_ok": fp_ok}
        cands = {k: (r.J.cpu().numpy(), r.t_star.cpu().numpy(), r.status.cpu().numpy())
                 for k, r in runs.items()}
        cands["oracle"] = (f["J_oracle"], f["t_oracle"], None)
        for k, (J, ts, st) in cands.items():
            miss, rel = T._exact_select_ok(J, ts, Jh, th, T_min, T_max)
            rel = np.where(np.isfinite(rel), rel, np.inf)
            rec[k] = {"t_star_misses": len(miss), "j_rel_max": float(rel.max()),
                      "j_rel_p50": float(np.median(rel)), "j_rel_gt_1e6": int((rel > 1e-6).sum()),
                      "nonzero_status": None if st is None else int((st != 0).sum())}
        line = json.dumps(rec)
        print(line, flush=True)
        if out:
            out.write(line + "\n")


if __name__ == "__main__":
    main()
