"""Capture the real-linearisation problems whose select paths disagree (VERDICT r04
item 1), so that tests/golden/make_hp_batch.py can adjudicate them in 50-digit
arithmetic.

For each system of tests/real_lin.py (4096 device-linearised problems, the
reference's rho_reg = 1e-12) it runs every candidate (traj, traj_ref, aug,
aug_ref, aug_gen, a 32-problem oracle sample) and keeps, per system:

  bit 1   T* of aug_gen (round 4's fp64 s = 5 drop-in path) != traj
  bit 2   T* of traj_ref (the reference association on the device) != traj
  bit 4   T* of aug_ref != traj
  bit 8   T* of aug (augmented blocks, product) != traj
  bit 16  T* of the oracle sample != traj or != aug_gen
  bit 32  the largest J disagreement (aug_gen / traj_ref / aug against traj)
  bit 64  a seeded random sample of the finite problems

(at most `cap` problems of each flip set, seeded), with the exact fp64 inputs the
device produced (x0, U, and the rollout / linearisation they give) and every
candidate's J curve.  Written to <out>/real_lin_capture.npz.

    python tools/real_lin_capture.py <out_dir> [cap] [n_random]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import torch  # noqa: E402

import real_lin  # noqa: E402

out_dir = sys.argv[1]
cap = int(sys.argv[2]) if len(sys.argv) > 2 else 64
n_random = int(sys.argv[3]) if len(sys.argv) > 3 else 32
os.makedirs(out_dir, exist_ok=True)
dev = torch.device("cuda", 0)
CANDS = ("traj", "traj_ref", "aug", "aug_ref", "aug_gen")
save = {}
for seed, name in enumerate(real_lin.SYSTEMS):
    t0 = time.time()
    st, raw = real_lin.stats(name, 4096, 1000 + seed, dev, want_raw=True)
    d, r, ok = raw["d"], raw["r"], raw["ok"]
    T_min, T_max = d["T_min"], d["T_max"]
    rng = np.random.default_rng(5 + seed)
    why = np.zeros(len(ok), dtype=np.int64)

    def pick(mask, bit):
        cand = np.nonzero(mask & ok)[0]
        if len(cand) > cap:
            cand = np.sort(rng.choice(cand, cap, replace=False))
        why[cand] |= bit
        return len(np.nonzero(mask & ok)[0])

    tt = r["traj"][1]
    n_flip = {}
    for bit, k in ((1, "aug_gen"), (2, "traj_ref"), (4, "aug_ref"), (8, "aug")):
        n_flip[k] = pick(r[k][1] != tt, bit)
    oi, ot = raw["oracle_idx"], raw["oracle_t"]
    om = np.zeros(len(ok), dtype=bool)
    om[oi] = (ot != tt[oi]) | (ot != r["aug_gen"][1][oi])
    n_flip["oracle"] = pick(om, 16)
    sl = slice(T_min - 1, T_max)
    Jt = r["traj"][0][:, sl]
    for k in ("aug_gen", "traj_ref", "aug"):
        rel = np.max(np.abs(r[k][0][:, sl] - Jt) / np.maximum(np.abs(Jt), 1e-300), axis=1)
        rel[~ok] = -1
        why[int(np.argmax(rel))] |= 32
    cand = np.nonzero(ok)[0]
    why[np.sort(rng.choice(cand, min(n_random, len(cand)), replace=False))] |= 64
    idx = np.nonzero(why)[0]
    X = d["X"].cpu().numpy()
    lin = d["lin"]
    p = f"{name}_"
    save[p + "idx"] = idx
    save[p + "why"] = why[idx]
    save[p + "X0"] = d["X0"][idx]
    save[p + "U"] = d["U_np"][idx, :T_max]
    save[p + "X"] = X[idx, :T_max + 1]
    save[p + "A"] = lin.A.cpu().numpy()[idx, :T_max]
    save[p + "B"] = lin.B.cpu().numpy()[idx, :T_max]
    save[p + "a_res"] = lin.a_res.cpu().numpy()[idx, :T_max]
    for k in CANDS:
        save[p + "J_" + k] = r[k][0][idx]
        save[p + "t_" + k] = r[k][1][idx]
        save[p + "status_" + k] = r[k][2][idx]
    save[p + "meta"] = np.array([T_min, T_max, d["N"], d["F"].system_id, d["F"].n, d["F"].m])
    for k in ("xg", "u_ref", "Q", "R", "P"):
        save[p + k] = np.asarray(d[k], dtype=np.float64)
    save[p + "alpha"] = np.asarray(d["alpha"], dtype=np.float64)
    save[p + "w"] = np.array([d["w"]])
    save[p + "wrap"] = np.array(list(d["wrap"]), dtype=np.int64)
    print(f"{name}: finite {int(ok.sum())}, flips vs traj {n_flip}, kept {len(idx)} "
          f"({time.time() - t0:.1f} s)", flush=True)
np.savez_compressed(os.path.join(out_dir, "real_lin_capture.npz"), **save)
print("saved", os.path.join(out_dir, "real_lin_capture.npz"))
