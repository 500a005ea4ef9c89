"""CPU restatement of the forward pass and the outer iLQR loop (SURVEY.md
section 8(f) rank 4).  TEST INFRASTRUCTURE ONLY: imported by tests/ and the
CPU-baseline leg of tools/bench_forward.py, never by the product path
(time_opt_ilqr_amd calls hop_rollout_f64 / hop_forward_linesearch_f64 and
fails loudly without the HIP library).

Restates, in NumPy (scalar per-step loops, as the reference runs them):
  rollout ................................. solver.py:42-62
  cost_timeopt_true ....................... solver.py:65-102
  forward_linesearch_fixedT ............... solver.py:233-286
  ilqr_timeopt(method="propagator") ....... solver.py:449-765 (the propagator
      branch: linearise, augment, propagator J curve, argmin, truncated
      Riccati at T*, forward line search, LM update, stop rule)
with the dynamics of oracle/dyn_oracle.py and the LFT / Riccati restatements
of oracle/hop_oracle.py.

Parity pinning: tests/golden/ilqr_*.npz hold captured forward_linesearch_fixedT
calls (inputs and outputs), rollout, cost_timeopt_true and the J_hist / T_hist
of whole ilqr_timeopt runs of the reference itself on the five benchmark
systems (tests/golden/make_golden.py --ilqr); tests/test_oracle_golden.py
checks this module against them.
"""
from __future__ import annotations

import math

import numpy as np

from oracle import dyn_oracle as dyn
from oracle import hop_oracle as orc

ALPHAS = (1.0, 0.5, 0.25, 0.1, 0.05)  # solver.py:247


def obstacle_cost(x, obstacles):
    """The point-mass extra_stage_cost (systems.py:271-293) for obstacles given
    as rows (cx, cy, radius, weight)."""
    p = np.asarray(x[:2], dtype=float)
    c, cx, cxx = 0.0, np.zeros(len(x)), np.zeros((len(x), len(x)))
    for ox, oy, r, wt in obstacles:
        d = p - np.array([ox, oy])
        s = float(d @ d)
        ci = wt * math.exp(-s / (2.0 * r * r))
        c += ci
        cx[:2] += -(ci / (r * r)) * d
        cxx[:2, :2] += ci * (np.outer(d, d) / (r ** 4) - np.eye(2) / (r * r))
    return c, cx, cxx


def _extra_fn(obstacles):
    if obstacles is None or len(obstacles) == 0:
        return None
    return lambda x, u: obstacle_cost(x, obstacles)


def rollout(sys_id, dt, x0, U, max_state_norm=1e6):
    """solver.py:42-62: X[0] = x0, X[k+1] = F(X[k], U[k]); the first
    non-finite or ||x|| > max_state_norm step sets X[k+1:] = NaN."""
    U = np.asarray(U, dtype=float)
    N, n = U.shape[0], len(x0)
    X = np.zeros((N + 1, n))
    X[0] = x0
    for k in range(N):
        xn = dyn.dynamics(sys_id, X[k], U[k], dt)
        if not np.all(np.isfinite(xn)) or float(np.linalg.norm(xn)) > max_state_norm:
            X[k + 1:] = np.nan
            break
        X[k + 1] = xn
    return X


def cost_true(X, U, xg, u_ref, Q, R, Qf, w, T_star, wrap_idx=None, obstacles=None):
    """solver.py:65-102 with Qf = as_terminal_weight(alpha, n) given."""
    T = int(T_star)
    if T <= 0:
        return float("inf")
    if not np.all(np.isfinite(X[:T + 1])) or not np.all(np.isfinite(U[:T])):
        return float("inf")
    extra = _extra_fn(obstacles)
    c = 0.0
    for k in range(T):
        e = orc.wrap_angles(X[k] - xg, wrap_idx)
        du = np.atleast_1d(U[k] - u_ref)
        if not (np.all(np.isfinite(e)) and np.all(np.isfinite(du))):
            return float("inf")
        c += 0.5 * float(e @ (Q @ e)) + 0.5 * float(du @ (R @ du)) + float(w)
        if extra is not None:
            c += float(extra(X[k], U[k])[0])
    eT = orc.wrap_angles(X[T] - xg, wrap_idx)
    if not np.all(np.isfinite(eT)):
        return float("inf")
    return float(c + 0.5 * float(eT @ (Qf @ eT)))


def forward_linesearch(sys_id, dt, X, U, xg, u_ref, Q, R, Qf, w, T_star, k_list, K_list,
                       alphas=ALPHAS, wrap_idx=None, obstacles=None):
    """solver.py:233-286: first alpha whose rollout under du = K dx + alpha k
    lowers the true cost at T*.  Returns (X', U', J, accepted, alpha index)."""
    T = int(T_star)
    J_old = cost_true(X, U, xg, u_ref, Q, R, Qf, w, T, wrap_idx, obstacles)
    N = len(U)
    for ai, a in enumerate(alphas):
        U_new = U.copy()
        X_new = np.zeros_like(X)
        X_new[0] = X[0]
        ok = True
        for k in range(N):
            if k < T:
                dx = orc.wrap_angles(X_new[k] - X[k], wrap_idx)
                U_new[k] = U[k] + (K_list[k] @ dx + float(a) * np.asarray(k_list[k]).reshape(-1))
            X_new[k + 1] = dyn.dynamics(sys_id, X_new[k], U_new[k], dt)
            if not np.all(np.isfinite(X_new[k + 1])):
                ok = False
                break
        if not ok:
            continue
        J_new = cost_true(X_new, U_new, xg, u_ref, Q, R, Qf, w, T, wrap_idx, obstacles)
        if J_new < J_old:
            return X_new, U_new, J_new, True, ai
    return X, U, J_old, False, -1


def ilqr_timeopt(sys_id, dt, x0, xg, u_ref, Q, R, Qf, w, N, T_min, T_max, max_iter=15,
                 lm_init=1e-3, wrap_idx=None, central=True, obstacles=None,
                 alphas=ALPHAS, U_init=None, method="propagator"):
    """solver.py:449-765, method="propagator" (augmentation with the default
    q_reg 1e-9 / rho_reg 1e-12, the propagator J curve at T_use = T_max) or
    method="bruteforce" (the J curve of solver.py:293-358 at lm_lambda = 1e-6).
    U_init as solver.py:480-490 (1-D = one control per step, padded with its
    last row, truncated to N)."""
    assert method in ("propagator", "bruteforce")
    extra = _extra_fn(obstacles)
    if U_init is None:
        U = np.tile(np.asarray(u_ref, dtype=float).reshape(1, -1), (N, 1))
    else:
        U = np.asarray(U_init, dtype=float)
        if U.ndim == 1:
            U = U.reshape(-1, 1)
        if U.shape[0] < N:
            U = np.vstack([U, np.tile(U[-1:], (N - U.shape[0], 1))])
        U = U[:N]
    X = rollout(sys_id, dt, x0, U)
    J_hist, T_hist = [], []
    lm = float(lm_init)
    n = len(x0)
    m = U.shape[1]
    # alpha as the matrix Qf: the propagator/Riccati restatements take `alpha`
    alpha = Qf

    def select(X, U):
        A, B, a_res = dyn.linearize(sys_id, X, U, dt, central=central)
        if method == "bruteforce":
            J = orc.bruteforce_J(list(A), list(B), X, U, xg, u_ref, Q, R, alpha, w, T_max,
                                 wrap_idx=wrap_idx, extra=extra)
            return A, B, int(np.argmin(J[T_min - 1:T_max]) + T_min)
        Aa, Ba, Qa, _, z0, R_inv = orc.augment_stage(A, B, a_res, X, U, xg, u_ref, Q, R, w,
                                                     wrap_idx=wrap_idx, extra=extra)
        QT = orc.augment_terminal(X, xg, alpha, wrap_idx)
        J = orc.lft_sweep(Aa, Ba, Qa, R_inv, z0, QT, T_max)["J"]
        T_s = int(np.argmin(J[T_min - 1:T_max]) + T_min)
        return A, B, T_s

    def update(A, B, X, U, T_s, lm):
        k_l, K_l, ok = orc.riccati_truncated(list(A), list(B), X, U, xg, u_ref, Q, R, alpha,
                                             T_s, lm_lambda=lm, wrap_idx=wrap_idx, extra=extra)
        if not ok:
            return X, U, float("inf"), False
        Xn, Un, Jn, acc, _ = forward_linesearch(sys_id, dt, X, U, xg, u_ref, Q, R, Qf, w, T_s,
                                                k_l, K_l, alphas, wrap_idx, obstacles)
        return Xn, Un, Jn, acc

    A, B, T_bar = select(X, U)
    k_l, K_l, ok = orc.riccati_truncated(list(A), list(B), X, U, xg, u_ref, Q, R, alpha, T_bar,
                                         lm_lambda=lm, wrap_idx=wrap_idx, extra=extra)
    if ok:
        X, U, J0, _, _ = forward_linesearch(sys_id, dt, X, U, xg, u_ref, Q, R, Qf, w, T_bar,
                                            k_l, K_l, alphas, wrap_idx, obstacles)
        if np.isfinite(J0):
            J_hist.append(float(J0))
            T_hist.append(int(T_bar))
    for _ in range(int(max_iter)):
        A, B, T_star = select(X, U)
        Xn, Un, Jn, acc = update(A, B, X, U, T_star, lm)
        if acc and np.isfinite(Jn):
            X, U = Xn, Un
            T_bar = T_star
            J_hist.append(float(Jn))
            T_hist.append(int(T_star))
            lm = max(lm / 10.0, 1e-12)
        else:
            lm *= 10.0
        if len(J_hist) >= 2:
            rel = abs(J_hist[-1] - J_hist[-2]) / (abs(J_hist[-2]) + 1e-12)
            if rel < 1e-4 and len(T_hist) >= 3 and len(set(T_hist[-3:])) == 1:
                break
    return dict(X=X, U=U, J_hist=J_hist, T_hist=T_hist,
                T_star=int(T_hist[-1] if T_hist else T_bar))
