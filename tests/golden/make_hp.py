"""High-precision J curves of real linearisations (round 4): the ground truth the
real-input parity tests compare against.

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tests/golden/make_hp.py

On the reference's real select inputs at rho_reg = 1e-12 the fp64 evaluation of
propagator_all_Jt_aug is itself ill-conditioned: on the captured quadrotor problem
of tools/handover_capture.py the NumPy reference (oracle/hop_oracle.py, pinned to
the reference's own outputs) is 1.4e-4 away from the exact value of its own
algorithm.  So every fixture here carries, next to the fp64 oracle's J curve, the
reference's association (horizon_selection.py:36-86: chol_inv = (sym(M) + 1e-9 I)^-1
with no escalation needed on these inputs) evaluated in 50-digit arithmetic
(mpmath) on exactly the fp64 blocks the builders produce (augmented.py:10-87, via
the oracle's builders).

Inputs per system (the makers of systems.py, restated in time_opt_ilqr_amd/systems.py):
perturbed x0 and U = u_ref + noise, X = rollout (oracle/ilqr_oracle.py), (A_k, B_k) by
central differences and a_k = F(x_k, u_k) - x_{k+1} (oracle/dyn_oracle.py, pinned
to linearization.py's outputs by tests/golden/lin_*.npz).  The quadrotor set also
holds the problem the round-3 conditioned kernel handed over inside the device
outer loop (its select inputs were captured on the GPU by tools/handover_capture.py
and are stored as data).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True

import mpmath as mp  # noqa: E402

from oracle import dyn_oracle as dyn  # noqa: E402
from oracle import hop_oracle as orc  # noqa: E402
from oracle import ilqr_oracle as io  # noqa: E402

mp.mp.dps = 50

# name: (system id, N, T_min, T_max, x0, xg, u_ref, Q, R, alpha, w, wrap, x0 jitter, U jitter)
_QUAD_X0 = np.r_[2.0, 2.0, 2.0, np.zeros(9)]
CASES = {
    "quadrotor": (2, 100, 40, 100, _QUAD_X0, np.zeros(12), np.array([9.81, 0.0, 0.0, 0.0]),
                  np.diag([5, 5, 5, 1, 1, 1, 20, 20, 10, 1, 1, 1]).astype(float),
                  np.diag([1e-3, 1e-2, 1e-2, 1e-2]), 300.0, 0.005, [6, 7, 8], 0.1, 0.1),
    "segway": (4, 120, 40, 120, np.array([0.05, 0.0, 0.08, 0.0]), np.zeros(4), np.zeros(1),
               np.diag([1.0, 0.1, 25.0, 1.0]), np.array([[0.25]]),
               np.diag([20.0, 2.0, 250.0, 10.0]), 1e-4, [2], 0.02, 0.2),
    "cartpole": (1, 150, 40, 150, np.zeros(4), np.array([0.0, 0.0, np.pi, 0.0]), np.zeros(1),
                 np.diag([0.01, 0.2, 0.0, 0.2]), np.array([[0.02]]),
                 np.diag([5.0, 5.0, 800.0, 40.0]), 0.03, [2], 0.1, 0.5),
    "di": (0, 120, 10, 80, np.array([1.0, 0.0]), np.array([2.0, 0.0]), np.zeros(1),
           np.diag([1.0, 0.1]), np.array([[1e-2]]), 50.0, 0.02, [], 0.2, 0.2),
}
PER_SYSTEM = 3


def hp_curve(Aa, Ba, Qa, Ri, z0, QT, N, eps_E=None):
    """horizon_selection.py:36-86 (the reference association) in 50-digit arithmetic.
    eps_E: {k: jitter} for stage inverses E_k = chol_inv(Q_k) that the fp64 reference
    escalated (the jitter its ladder settled on, utils.py:81-93); 1e-9 elsewhere."""
    M = lambda a: mp.matrix(np.asarray(a, dtype=float).tolist())  # noqa: E731
    eps = mp.mpf("1e-9")

    def inv(X, e=eps):
        X = (X + X.T) / 2
        return (X + e * mp.eye(X.rows)) ** -1

    Ri_m, z = M(Ri), M(np.asarray(z0).reshape(-1, 1))
    J = []
    for k in range(N):
        Ak, Bk = M(Aa[k]), M(Ba[k])
        Ek = inv(M(Qa[k]), mp.mpf(eps_E[k]) if eps_E and k in eps_E else eps)
        Fk = Ek * Ak.T
        Gk = Ak * Ek * Ak.T + Bk * Ri_m * Bk.T
        Gk = (Gk + Gk.T) / 2
        if k == 0:
            Eb, Fb, Gb = Ek, Fk, Gk
        else:
            W = inv(Ek + Gb)
            FbW = Fb * W
            Eb = Eb - FbW * Fb.T
            Eb = (Eb + Eb.T) / 2
            Fb = FbW * Fk
            Gb = Gk - Fk.T * W * Fk
            Gb = (Gb + Gb.T) / 2
        Wt = inv(inv(M(QT[k])) + Gb)
        X0 = Eb - Fb * Wt * Fb.T
        X0 = (X0 + X0.T) / 2
        J.append(float(0.5 * (z.T * inv(X0) * z)[0, 0]))
    return np.array(J)


def problem(name, seed):
    sid, N, _, _, x0, xg, ur, Q, R, alpha, w, wrap, sx, su = CASES[name]
    n, m = dyn.DIMS[sid]
    dt = dyn.DEFAULT_DT[sid]
    rng = np.random.default_rng(seed)
    for _ in range(20):  # a perturbation whose rollout stays finite
        X0 = x0 + sx * rng.standard_normal(n)
        U = ur + su * rng.standard_normal((N, m))
        X = io.rollout(sid, dt, X0, U)
        if np.isfinite(X).all():
            break
    A, B, a_res = dyn.linearize(sid, X[None], U[None], dt, central=True)
    return dict(A=A[0], B=B[0], a_res=a_res[0], X=X, U=U)


def blocks(name, p):
    sid, N, _, _, _, xg, ur, Q, R, alpha, w, wrap, _, _ = CASES[name]
    Aa, Ba, Qa, _, z0, Ri = orc.augment_stage(list(p["A"][:N]), list(p["B"][:N]), p["a_res"][:N],
                                              p["X"][:N + 1], p["U"][:N], xg, ur, Q, R, w,
                                              wrap_idx=wrap)
    QT = orc.augment_terminal(p["X"][:N + 1], xg, alpha, wrap_idx=wrap)
    return Aa, Ba, Qa, Ri, z0, QT


def main():
    d = {}
    capture = os.path.join(REPO, "gpurun_out", "p2", "handover_capture.npz")
    for name in CASES:
        sid, N, T_min, T_max = CASES[name][:4]
        probs = [problem(name, 7000 + 31 * sid + i) for i in range(PER_SYSTEM)]
        if name == "quadrotor" and os.path.exists(capture):
            c = np.load(capture)
            pre = "s2_p1693_"
            probs.append(dict(A=c[pre + "A"], B=c[pre + "B"], a_res=c[pre + "a_res"],
                              X=c[pre + "X"], U=c[pre + "U"]))
        for i, p in enumerate(probs):
            Aa, Ba, Qa, Ri, z0, QT = blocks(name, p)
            o = orc.lft_sweep(Aa, Ba, Qa, Ri, z0, QT, N)
            Jh = hp_curve(Aa, Ba, Qa, Ri, z0, QT, N)
            tag = f"{name}_p{i}"
            for k, v in p.items():
                d[f"{tag}_{k}"] = v
            d[f"{tag}_J_hp"] = Jh
            d[f"{tag}_J_oracle"] = o["J"]
            d[f"{tag}_status_oracle"] = o["status"]
            rel = np.abs(o["J"] - Jh) / np.abs(Jh)
            t_hp = int(np.argmin(Jh[T_min - 1:T_max]) + T_min)
            t_o = int(np.argmin(o["J"][T_min - 1:T_max]) + T_min)
            print(f"{tag}: oracle fp64 vs 50-digit max {rel.max():.2e} median "
                  f"{np.median(rel):.2e}; T* hp {t_hp} oracle {t_o}", flush=True)
        d[f"{name}_count"] = len(probs)
    np.savez_compressed(os.path.join(HERE, "real_lin_hp.npz"), **d)


def legacy_twin():
    """legacy_twin_hp.npz: the 50-digit curve of the escalated legacy-twin problem
    (tests/golden/legacy_twin_cases.npz, problem 0 of each tag: Q_4 needs the 1e-7
    jitter, ilqr_propagator.py:21-31), whose later horizons the fp64 reference itself
    gets only to ~5e-2 (E_4 ~ 2e7, cancelled by the compose)."""
    d = np.load(os.path.join(HERE, "legacy_twin_cases.npz"))
    out = {}
    for tag, s, m, N in (("s13_m4_N20", 13, 4, 20), ("s5_m1_N20", 5, 1, 20)):
        A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(int(d[f"{tag}_base_seed"]), 3, s, m, N)
        Q = Q.copy()
        Q[0, 4] = d[f"{tag}_Q04"]
        Jh = hp_curve(A[0], Bm[0], Q[0], Ri[0], z0[0], QT[0], N, eps_E={4: "1e-7"})
        out[f"{tag}_J_hp"] = Jh
        rel = np.max(np.abs(d[f"{tag}_J"][0] - Jh) / np.abs(Jh))
        print(f"{tag}: fp64 reference vs 50-digit {rel:.2e}")
    np.savez_compressed(os.path.join(HERE, "legacy_twin_hp.npz"), **out)


if __name__ == "__main__":
    if "--legacy-twin" in sys.argv:
        legacy_twin()
    else:
        main()
