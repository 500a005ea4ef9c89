"""Caller-side dynamics and stage costs given as Python callables (the reference's own
call form, ``F(x, u) -> x_next`` and ``extra_stage_cost(x, u) -> (c, cx, cxx)``).

The device outer loop (``solver.ilqr_timeopt_batch``) runs the built-in systems'
dynamics, FD linearisation and line search on the GPU.  A user system the device has
no kernel for arrives as a Python callable; these helpers evaluate it on the host,
one problem at a time as the reference does, and hand the arrays to the same device
select (LFT sweep + argmin), truncated Riccati pass and accept / LM / stop step.  The
hot path stays on the GPU; only the callable's own evaluations run here.

Semantics follow the reference functions they stand in for:
  rollout               /root/reference/solver.py:40-59 (divergence check, NaN tail)
  linearize             /root/reference/linearization.py:177-262 (central and forward
                        differences, h = max(eps, rel * max(1, |v|))) and :269-270
                        (affine residuals F(x_k, u_k) - x_{k+1})
  cost_true             /root/reference/solver.py:65-102
  linesearch            /root/reference/solver.py:233-286
"""
from dataclasses import dataclass
from typing import Callable, Optional, Sequence

import numpy as np

from .utils import angle_normalize, wrap_error


@dataclass
class HostDynamics:
    """A user dynamics callable ``F(x, u) -> x_next`` with its state / control sizes.

    ``vectorized=True`` declares that F maps stacked rows ``x [K, n], u [K, m]`` to
    ``[K, n]`` row by row (NumPy broadcasting over the leading axis): the FD
    linearisation then evaluates every perturbed point of every step and problem in one
    call (``linearize_batch``), with the same quotients as the per-call form, and the
    rollouts of a batch (``rollout_batch``) and of every (problem, step size) pair of a
    line search (``linesearch_batch``) advance together, one call per time step."""
    F: Callable
    n: int
    m: int
    name: str = "host"
    vectorized: bool = False

    def __call__(self, x, u):
        return np.asarray(self.F(x, u), dtype=float).reshape(-1)


def rollout(F, x0, U, *, max_state_norm: float = 1e6) -> np.ndarray:
    """One problem: X [N+1, n]; the first non-finite, wrong-sized or too-large state
    and everything after it are NaN."""
    x0 = np.asarray(x0, dtype=float).reshape(-1)
    U = np.asarray(U, dtype=float)
    N, n = U.shape[0], x0.size
    X = np.full((N + 1, n), np.nan)
    X[0] = x0
    with np.errstate(all="ignore"):  # a diverging rollout ends at its first bad state
        for k in range(N):
            xn = np.asarray(F(X[k], U[k]), dtype=float).reshape(-1)
            if xn.size != n or not np.all(np.isfinite(xn)) or \
                    float(np.linalg.norm(xn)) > max_state_norm:
                break
            X[k + 1] = xn
    return X


def rollout_batch(system, X0, U, *, max_state_norm: float = 1e6) -> np.ndarray:
    """A batch (X0 [B, n], U [B, N, m]): X [B, N+1, n], ``rollout`` per problem, or all
    problems a step at a time when the system is declared ``vectorized``."""
    X0 = np.asarray(X0, dtype=float)
    U = np.asarray(U, dtype=float)
    if not getattr(system, "vectorized", False):
        return np.stack([rollout(system, X0[b], U[b], max_state_norm=max_state_norm)
                         for b in range(X0.shape[0])])
    Bn, N = U.shape[:2]
    n = X0.shape[1]
    X = np.full((Bn, N + 1, n), np.nan)
    X[:, 0] = X0
    live = np.arange(Bn)
    with np.errstate(all="ignore"):
        for k in range(N):
            if live.size == 0:
                break
            xn = np.asarray(system.F(X[live, k], U[live, k]), dtype=float).reshape(live.size, n)
            ok = np.isfinite(xn).all(1) & (np.linalg.norm(xn, axis=1) <= max_state_norm)
            X[live[ok], k + 1] = xn[ok]
            live = live[ok]
    return X


def _step(v, eps, rel):
    return max(float(eps), float(rel) * max(1.0, abs(float(v))))


def linearize(F, X, U, *, central: bool = True, epsx: float = 1e-5, epsu: float = 1e-5,
              relx: float = 1e-6, relu: float = 1e-6):
    """One problem: A [N, n, n], B [N, n, m] by finite differences and the affine
    residuals a [N, n] = F(x_k, u_k) - x_{k+1} (non-finite states propagate as NaN,
    quietly)."""
    with np.errstate(all="ignore"):
        return _linearize(F, X, U, central, epsx, epsu, relx, relu)


def _linearize(F, X, U, central, epsx, epsu, relx, relu):
    X = np.asarray(X, dtype=float)
    U = np.asarray(U, dtype=float)
    N, n, m = U.shape[0], X.shape[1], U.shape[1]
    A = np.zeros((N, n, n))
    Bm = np.zeros((N, n, m))
    a = np.zeros((N, n))
    for k in range(N):
        x, u = X[k], U[k]
        f0 = np.asarray(F(x, u), dtype=float).reshape(-1)
        a[k] = f0 - X[k + 1]
        if central:
            for i in range(n):
                h = _step(x[i], epsx, relx)
                xp, xm = x.copy(), x.copy()
                xp[i] += h
                xm[i] -= h
                A[k, :, i] = (np.asarray(F(xp, u), dtype=float).reshape(-1) -
                              np.asarray(F(xm, u), dtype=float).reshape(-1)) / (2.0 * h)
            for j in range(m):
                h = _step(u[j], epsu, relu)
                up, um = u.copy(), u.copy()
                up[j] += h
                um[j] -= h
                Bm[k, :, j] = (np.asarray(F(x, up), dtype=float).reshape(-1) -
                               np.asarray(F(x, um), dtype=float).reshape(-1)) / (2.0 * h)
        else:
            if not np.all(np.isfinite(f0)):  # the forward form marks the whole step
                A[k] = np.nan
                Bm[k] = np.nan
                continue
            for i in range(n):
                h = _step(x[i], epsx, relx)
                e = np.zeros(n)
                e[i] = h
                A[k, :, i] = (np.asarray(F(x + e, u), dtype=float).reshape(-1) - f0) / h
            for j in range(m):
                h = _step(u[j], epsu, relu)
                e = np.zeros(m)
                e[j] = h
                Bm[k, :, j] = (np.asarray(F(x, u + e), dtype=float).reshape(-1) - f0) / h
    return A, Bm, a


def linearize_batch(system, X, U, *, central: bool = True, epsx: float = 1e-5,
                    epsu: float = 1e-5, relx: float = 1e-6, relu: float = 1e-6):
    """A batch of problems (X [B, N+1, n], U [B, N, m]): A [B, N, n, n], B [B, N, n, m],
    a [B, N, n].  One call of F over all perturbed points when the system is declared
    ``vectorized``, else ``linearize`` per problem."""
    X = np.asarray(X, dtype=float)
    U = np.asarray(U, dtype=float)
    if not getattr(system, "vectorized", False):
        parts = [linearize(system, X[b], U[b], central=central, epsx=epsx, epsu=epsu,
                           relx=relx, relu=relu) for b in range(X.shape[0])]
        return tuple(np.stack([q[i] for q in parts]) for i in range(3))
    with np.errstate(all="ignore"):
        return _linearize_vec(system.F, X, U, central, epsx, epsu, relx, relu)


def _linearize_vec(F, X, U, central, epsx, epsu, relx, relu):
    Bn, N, m = U.shape
    n = X.shape[-1]
    x, u = X[:, :N], U
    # h = max(eps, rel * max(1, |v|)) with Python's max: a NaN |v| gives max(1, NaN) = 1
    hx = np.fmax(float(epsx), float(relx) * np.fmax(1.0, np.abs(x)))
    hu = np.fmax(float(epsu), float(relu) * np.fmax(1.0, np.abs(u)))
    P = 1 + (2 if central else 1) * (n + m)   # points per step: f0, then the perturbations
    xs = np.repeat(x[:, :, None, :], P, axis=2)
    us = np.repeat(u[:, :, None, :], P, axis=2)
    i, j = np.arange(n), np.arange(m)
    if central:   # x_i + h, x_i - h, u_j + h, u_j - h: the perturbed component alone
        xs[:, :, 1 + i, i] += hx
        xs[:, :, 1 + n + i, i] -= hx
        us[:, :, 1 + 2 * n + j, j] += hu
        us[:, :, 1 + 2 * n + m + j, j] -= hu
    else:         # x + h e_i, u + h e_j (the per-call form adds the whole vector)
        Ex = np.zeros((Bn, N, n, n))
        Ex[:, :, i, i] = hx
        Eu = np.zeros((Bn, N, m, m))
        Eu[:, :, j, j] = hu
        xs[:, :, 1:1 + n] = x[:, :, None, :] + Ex
        us[:, :, 1 + n:1 + n + m] = u[:, :, None, :] + Eu
    fx = np.asarray(F(xs.reshape(-1, n), us.reshape(-1, m)), dtype=float).reshape(Bn, N, P, n)
    f0 = fx[:, :, 0]
    if central:
        A = (fx[:, :, 1:1 + n] - fx[:, :, 1 + n:1 + 2 * n]) / (2.0 * hx)[..., None]
        Bm = (fx[:, :, 1 + 2 * n:1 + 2 * n + m] - fx[:, :, 1 + 2 * n + m:]) / (2.0 * hu)[..., None]
    else:
        A = (fx[:, :, 1:1 + n] - f0[:, :, None]) / hx[..., None]
        Bm = (fx[:, :, 1 + n:] - f0[:, :, None]) / hu[..., None]
    A, Bm = A.swapaxes(-1, -2).copy(), Bm.swapaxes(-1, -2).copy()
    if not central:  # the forward form marks the whole step when F(x_k, u_k) is not finite
        bad = ~np.isfinite(f0).all(-1)
        A[bad] = np.nan
        Bm[bad] = np.nan
    return A, Bm, f0 - X[:, 1:N + 1]


def stage_cost_terms(extra_stage_cost, X, U):
    """extra_stage_cost at every (x_k, u_k), k < N: c [N], cx [N, n], cxx [N, n, n]
    (the qxx_extra / qx_extra / c_extra arrays of the device select and Riccati)."""
    X = np.asarray(X, dtype=float)
    U = np.asarray(U, dtype=float)
    N, n = U.shape[0], X.shape[1]
    c = np.zeros(N)
    cx = np.zeros((N, n))
    cxx = np.zeros((N, n, n))
    for k in range(N):
        ck, gk, hk = extra_stage_cost(X[k], U[k])
        c[k] = float(ck)
        cx[k] = np.asarray(gk, dtype=float).reshape(n)
        cxx[k] = np.asarray(hk, dtype=float).reshape(n, n)
    return c, cx, cxx


def cost_true(X, U, xg, u_ref, Q, R, Qf, w, T_star: int, wrap_idx: Optional[Sequence[int]] = None,
              extra_stage_cost=None) -> float:
    """Running cost up to T_star plus the terminal cost at T_star (Qf = the terminal
    weight already expanded, as_terminal_weight(alpha))."""
    T = int(T_star)
    if T <= 0:
        return float("inf")
    if not np.all(np.isfinite(X[:T + 1])) or not np.all(np.isfinite(U[:T])):
        return float("inf")
    c = 0.0
    for k in range(T):
        e = np.atleast_1d(wrap_error(X[k] - xg, wrap_idx)).reshape(-1)
        du = np.atleast_1d(U[k] - u_ref).reshape(-1)
        if not np.all(np.isfinite(e)) or not np.all(np.isfinite(du)):
            return float("inf")
        c += 0.5 * float(e @ (Q @ e)) + 0.5 * float(du @ (R @ du)) + float(w)
        if extra_stage_cost is not None:
            c += float(extra_stage_cost(X[k], U[k])[0])
    eT = np.atleast_1d(wrap_error(X[T] - xg, wrap_idx)).reshape(-1)
    if not np.all(np.isfinite(eT)):
        return float("inf")
    return float(c + 0.5 * float(eT @ (Qf @ eT)))


def _wrap_rows(e, wrap_idx):
    """wrap_error on every row of e [R, n] (the same angle_normalize per component)."""
    if not wrap_idx:
        return e
    e = e.copy()
    for i in wrap_idx:
        e[:, i] = angle_normalize(e[:, i])
    return e


def linesearch_batch(system, X, U, T_star, K, kff, active, cost_args, alphas,
                     extra_stage_cost=None):
    """A batch of line searches (X [B, N+1, n], U [B, N, m], T_star [B], K [B, N, m, n],
    kff [B, N, m], active [B]): (X', U', J, J_old, accepted) with accepted = the step-size
    index, -1 when none is accepted, -2 for inactive problems (their X, U kept, J NaN).
    Per problem ``linesearch``; for a ``vectorized`` system (and four or more active
    problems) the step sizes are tried in
    rounds, each round rolling out every problem still without an accepted step size
    together (one F call per time step), so each problem gets the first step size the
    per-call form accepts (the K dx products are stacked matmuls: the same values to
    rounding)."""
    X = np.asarray(X, dtype=float)
    U = np.asarray(U, dtype=float)
    T = np.asarray(T_star).astype(np.int64).reshape(-1)
    act = np.asarray(active).reshape(-1).astype(bool)
    Bn = X.shape[0]
    Xo, Uo = X.copy(), U.copy()
    J = np.full(Bn, np.nan)
    J0 = np.full(Bn, np.nan)
    acc = np.full(Bn, -2, dtype=np.int32)
    # a handful of problems: the per-call loop (stacking rows costs more than it saves)
    if not getattr(system, "vectorized", False) or int(act.sum()) < 4:
        for b in np.nonzero(act)[0]:
            Xo[b], Uo[b], J[b], J0[b], acc[b] = linesearch(system, X[b], U[b], int(T[b]), K[b],
                                                           kff[b], cost_args, alphas,
                                                           extra_stage_cost)
        return Xo, Uo, J, J0, acc
    xg, u_ref, Q, R, Qf, w, wrap_idx = cost_args
    bs = np.nonzero(act)[0]
    N, n = U.shape[1], X.shape[2]
    Kf = np.asarray(K, dtype=float)
    kf = np.asarray(kff, dtype=float).reshape(Bn, N, -1)
    for b in bs:
        J0[b] = cost_true(X[b], U[b], xg, u_ref, Q, R, Qf, w, int(T[b]), wrap_idx, extra_stage_cost)
        J[b], acc[b] = J0[b], -1
    pending = bs
    for ai, al in enumerate(alphas):  # one round per step size, over the problems still open
        if pending.size == 0:
            break
        Xn = np.zeros((pending.size, N + 1, n))
        Xn[:, 0] = X[pending, 0]
        Un = U[pending].copy()
        ok = np.ones(pending.size, dtype=bool)
        with np.errstate(all="ignore"):
            for k in range(N):
                on = k < T[pending]
                if on.any():
                    r = np.nonzero(on)[0]
                    pr = pending[r]
                    dx = _wrap_rows(Xn[r, k] - X[pr, k], wrap_idx)
                    Un[r, k] = U[pr, k] + ((Kf[pr, k] @ dx[:, :, None])[:, :, 0]
                                           + float(al) * kf[pr, k])
                xn = np.asarray(system.F(Xn[:, k], Un[:, k]), dtype=float).reshape(pending.size, n)
                Xn[:, k + 1] = xn
                ok &= np.isfinite(xn).all(1)
        still = []
        for i, b in enumerate(pending):
            if ok[i]:
                Jn = cost_true(Xn[i], Un[i], xg, u_ref, Q, R, Qf, w, int(T[b]), wrap_idx,
                               extra_stage_cost)
                if Jn < J0[b]:
                    Xo[b], Uo[b], J[b], acc[b] = Xn[i], Un[i], Jn, ai
                    continue
            still.append(b)
        pending = np.asarray(still, dtype=np.int64)
    return Xo, Uo, J, J0, acc


def linesearch(F, X, U, T_star: int, K, kff, cost_args, alphas, extra_stage_cost=None):
    """One problem: the first step size whose rollout (controls U + alpha k + K dx up
    to T_star, U beyond) is finite and strictly cheaper than the current trajectory.
    Returns (X', U', J, J_old, index of the accepted step size or -1)."""
    xg, u_ref, Q, R, Qf, w, wrap_idx = cost_args
    T = int(T_star)
    J_old = cost_true(X, U, xg, u_ref, Q, R, Qf, w, T, wrap_idx, extra_stage_cost)
    N = len(U)
    for ai, al in enumerate(alphas):
        Un = U.copy()
        Xn = np.zeros_like(X)
        Xn[0] = X[0]
        ok = True
        with np.errstate(all="ignore"):  # a diverging rollout is rejected, quietly
            for k in range(N):
                if k < T:
                    dx = wrap_error((Xn[k] - X[k]).reshape(-1), wrap_idx)
                    Un[k] = U[k] + ((np.asarray(K[k]) @ dx).reshape(-1)
                                    + float(al) * np.asarray(kff[k]).reshape(-1))
                Xn[k + 1] = np.asarray(F(Xn[k], Un[k]), dtype=float).reshape(-1)
                if not np.all(np.isfinite(Xn[k + 1])):
                    ok = False
                    break
        if not ok:
            continue
        J_new = cost_true(Xn, Un, xg, u_ref, Q, R, Qf, w, T, wrap_idx, extra_stage_cost)
        if J_new < J_old:
            return Xn, Un, J_new, J_old, ai
    return X, U, J_old, J_old, -1
