"""CPU restatement of the horizon-selection hot path (TEST INFRASTRUCTURE ONLY).

This module is the parity oracle for the MI355X engine in ``time_opt_ilqr_amd``.
Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import it, and only as the checker / CPU baseline.  The product
path never calls into this file.

It restates, in batched NumPy, the algorithm of the reference
(dmmsjtu-umich/time-opt-ilqr) for the rows of SURVEY.md section 8(a):

  a1  LFT propagator J(t) for all t ......... horizon_selection.py:36-86
  a2  chol_inv (jitter 1e-9, x10, 8 tries, LU) utils.py:69-93
  a3  chol_solve (jitter, no fallback) ...... utils.py:96-120
  a4  _sym .................................. utils.py:35-37
  a5  augmented stage blocks ................ augmented.py:10-60
  a6  augmented terminal blocks ............. augmented.py:63-87
  a7  terminal weight / angle wrap .......... utils.py:49-62, 127-137
  a8  argmin horizon selection .............. solver.py:522
  a9  truncated Riccati pass (K, k) ......... solver.py:156-230
  a10 value expansions (Vxx, Vx, V0, K, k) .. horizon_selection.py:97-212
  a11 brute-force J(T) curve ................ solver.py:293-358

Parity pinning: tests/golden/*.npz were produced by importing the reference
itself in the build container (tests/golden/make_golden.py).  The tests in
tests/test_oracle_golden.py check this restatement against those vectors.

Status bits (shared with the C ABI, include/hop.h):
  1 = jitter escalated past the first try
  2 = LU fallback used (Cholesky failed for every jitter)
  4 = non-finite input/output encountered
  8 = not positive definite / solve failed (reference: LinAlgError or ok=False)
"""
from __future__ import annotations

import numpy as np

ST_JITTER = 1
ST_LU = 2
ST_NONFINITE = 4
ST_FAIL = 8

JITTER0 = 1e-9


# ---------------------------------------------------------------------------
# a4 / a2 / a3 : small dense helpers
# ---------------------------------------------------------------------------

def sym(M):
    """0.5 (M + M^T) -- utils.py:35-37."""
    return 0.5 * (M + M.T)


def spd_inverse(M, jitter=JITTER0, max_tries=8):
    """Inverse of sym(M) + eps I following utils.py:69-93.

    Returns (inverse, status).  The first attempt already carries eps=jitter;
    every failed Cholesky multiplies eps by 10; after ``max_tries`` failures an
    LU solve of (sym(M) + eps I) is used (status bit 2).
    """
    S = sym(np.asarray(M, dtype=np.float64))
    if not np.isfinite(S).all():
        return np.full_like(S, np.nan), ST_NONFINITE
    eye = np.eye(S.shape[0])
    eps = float(jitter)
    flags = 0
    for attempt in range(int(max_tries)):
        try:
            low = np.linalg.cholesky(S + eps * eye)
        except np.linalg.LinAlgError:
            eps *= 10.0
            flags |= ST_JITTER
            continue
        # two LU-based triangular solves, as the reference does
        half = np.linalg.solve(low, eye)
        return np.linalg.solve(low.T, half), flags
    try:
        return np.linalg.solve(S + eps * eye, eye), flags | ST_LU
    except np.linalg.LinAlgError:
        return np.full_like(S, np.nan), flags | ST_LU | ST_FAIL


def spd_solve(M, rhs, jitter=JITTER0, max_tries=8):
    """(sym(M) + eps I)^{-1} rhs with utils.py:96-120 semantics -> (X, status)."""
    S = sym(np.asarray(M, dtype=np.float64))
    rhs = np.asarray(rhs, dtype=np.float64)
    if not (np.isfinite(S).all() and np.isfinite(rhs).all()):
        return None, ST_NONFINITE
    eye = np.eye(S.shape[0])
    eps = float(jitter)
    flags = 0
    for attempt in range(int(max_tries)):
        try:
            low = np.linalg.cholesky(S + eps * eye)
            X = np.linalg.solve(low.T, np.linalg.solve(low, rhs))
            if not np.isfinite(X).all():
                raise FloatingPointError
            return X, flags
        except (np.linalg.LinAlgError, FloatingPointError):
            eps *= 10.0
            flags |= ST_JITTER
    return None, flags | ST_FAIL


# ---------------------------------------------------------------------------
# a1 : LFT propagator (one problem)
# ---------------------------------------------------------------------------

def lft_sweep(A, Bm, Q, R_inv, z0, QT, N=None, R_list=None, want_efg=False,
              want_prefix=False, max_tries=8):
    """J[t-1] for t = 1..N (horizon_selection.py:36-86), one problem.

    A, Q, QT : (>=N, s, s); Bm : (>=N, s, m); R_inv : (m, m) (cached inverse)
    or None with R_list (N, m, m) (then each stage inverse is spd_inverse(R_k)).
    Returns dict(J, status[, E, F, G][, Ebar, Fbar, Gbar]).
    """
    N = len(A) if N is None else int(N)
    out = {"status": 0}
    if N <= 0:
        out["J"] = np.zeros(0)
        return out
    status = 0
    s = A[0].shape[0]

    def inv(M):
        nonlocal status
        X, st = spd_inverse(M, max_tries=max_tries)
        status |= st
        return X

    if R_inv is None:
        rinv = [inv(R_list[k]) for k in range(N)]
    else:
        rinv = [np.asarray(R_inv, dtype=np.float64)] * N

    # stage blocks (independent per k)
    Es, Fs, Gs = [], [], []
    for k in range(N):
        Ek = inv(Q[k])
        Fk = Ek @ A[k].T
        Gk = sym(A[k] @ Ek @ A[k].T + Bm[k] @ rinv[k] @ Bm[k].T)
        Es.append(Ek)
        Fs.append(Fk)
        Gs.append(Gk)

    # prefix composition; the query for horizon t only needs prefix t-1, so
    # it is evaluated in the same forward pass (fused stage/compose/query).
    J = np.zeros(N)
    z0 = np.asarray(z0, dtype=np.float64).reshape(-1)
    Eb, Fb, Gb = Es[0], Fs[0], Gs[0]
    pre = []
    for k in range(N):
        if k > 0:
            W = inv(Es[k] + Gb)
            FbW = Fb @ W
            Eb = sym(Eb - FbW @ Fb.T)
            Fb = FbW @ Fs[k]
            Gb = sym(Gs[k] - Fs[k].T @ W @ Fs[k])
        if want_prefix:
            pre.append((Eb, Fb, Gb))
        Xt = inv(QT[k])
        Wt = inv(Xt + Gb)
        X0 = sym(Eb - Fb @ Wt @ Fb.T)
        P0 = inv(X0)
        J[k] = 0.5 * float(z0 @ P0 @ z0)
    if not np.isfinite(J).all():
        status |= ST_NONFINITE
    out["J"] = J
    out["status"] = status
    if want_efg:
        out["E"], out["F"], out["G"] = np.array(Es), np.array(Fs), np.array(Gs)
    if want_prefix:
        out["Ebar"] = np.array([p[0] for p in pre])
        out["Fbar"] = np.array([p[1] for p in pre])
        out["Gbar"] = np.array([p[2] for p in pre])
    return out


def lft_sweep_batch(A, Bm, Q, R_inv, z0, QT, N=None, max_tries=8):
    """Loop of lft_sweep over a leading batch axis.  R_inv: (m,m) or (B,m,m)."""
    Bn = A.shape[0]
    N = A.shape[1] if N is None else int(N)
    J = np.zeros((Bn, N))
    st = np.zeros(Bn, dtype=np.int32)
    R_inv = np.asarray(R_inv)
    z0 = np.asarray(z0)
    for b in range(Bn):
        r = R_inv if R_inv.ndim == 2 else R_inv[b]
        z = z0 if z0.ndim == 1 else z0[b]
        o = lft_sweep(A[b], Bm[b], Q[b], r, z, QT[b], N, max_tries=max_tries)
        J[b] = o["J"]
        st[b] = o["status"]
    return J, st


# ---------------------------------------------------------------------------
# a8 : horizon selection
# ---------------------------------------------------------------------------

def select_horizon(J, T_min, T_max):
    """T* = first minimiser of J[T_min-1 : T_max] (+T_min) -- solver.py:522.

    Works on (N,) or (B, N); NaN compares like np.argmin (NaN wins).
    """
    J = np.asarray(J)
    win = J[..., int(T_min) - 1:int(T_max)]
    idx = np.argmin(win, axis=-1)
    Jstar = np.take_along_axis(win, np.expand_dims(idx, -1), -1)[..., 0]
    return idx + int(T_min), Jstar


# ---------------------------------------------------------------------------
# a7 / a5 / a6 : host preparation
# ---------------------------------------------------------------------------

def wrap_angles(e, wrap_idx):
    """utils.py:127-137: (a + pi) mod 2 pi - pi on the listed coordinates."""
    if not wrap_idx:
        return e
    e = np.array(e, dtype=np.float64, copy=True)
    for i in wrap_idx:
        e[..., i] = np.remainder(e[..., i] + np.pi, 2.0 * np.pi) - np.pi
    return e


def terminal_weight(alpha, n):
    """utils.py:49-62."""
    a = np.asarray(alpha, dtype=np.float64)
    if a.ndim == 0:
        return float(a) * np.eye(n)
    if a.ndim == 1:
        if a.shape != (n,):
            raise ValueError("terminal weight vector has wrong shape")
        return np.diag(a)
    if a.shape != (n, n):
        raise ValueError("terminal weight matrix has wrong shape")
    return sym(a)


def augment_stage(A_list, B_list, a_res, X, U, xg, u_ref, Q, R, w, wrap_idx=None,
                  q_reg=1e-9, rho_reg=1e-12, extra=None):
    """augmented.py:10-60 with the affine residuals a_k = F(x_k,u_k) - x_{k+1}
    supplied by the caller (the dynamics F stays on the host)."""
    N = len(A_list)
    n = X.shape[1]
    m = U.shape[1]
    R = sym(np.asarray(R, dtype=np.float64))
    R_inv, _ = spd_inverse(R)
    Qs = sym(np.asarray(Q, dtype=np.float64))
    Aa = np.zeros((N, n + 1, n + 1))
    Ba = np.zeros((N, n + 1, m))
    Qa = np.zeros((N, n + 1, n + 1))
    for k in range(N):
        e = wrap_angles(X[k] - xg, wrap_idx)
        du = np.atleast_1d(U[k] - u_ref)
        Qe = Q @ e
        blk = np.zeros((n + 1, n + 1))
        blk[:n, :n] = Qs + q_reg * np.eye(n)
        blk[:n, n] = Qe
        blk[n, :n] = Qe
        blk[n, n] = float(e @ Q @ e) + 2.0 * float(w) + rho_reg
        if extra is not None:
            c, cx, cxx = extra(X[k], U[k])
            blk[:n, :n] += sym(np.asarray(cxx, dtype=np.float64))
            cx = np.asarray(cx, dtype=np.float64).reshape(-1)
            blk[:n, n] += cx
            blk[n, :n] += cx
            blk[n, n] += 2.0 * float(c)
        Qa[k] = sym(blk)
        Aa[k, :n, :n] = A_list[k]
        Aa[k, :n, n] = np.asarray(a_res[k]).reshape(-1) - B_list[k] @ du
        Aa[k, n, n] = 1.0
        Ba[k, :n, :] = B_list[k]
    z0 = np.zeros(n + 1)
    z0[-1] = 1.0
    return Aa, Ba, Qa, R, z0, R_inv


def augment_terminal(X, xg, alpha, wrap_idx=None, rho_reg=1e-12):
    """augmented.py:63-87: QT[t-1] for t = 1..N (N = len(X) - 1)."""
    n = X.shape[1]
    P = sym(terminal_weight(alpha, n))
    N = X.shape[0] - 1
    out = np.zeros((N, n + 1, n + 1))
    for t in range(1, N + 1):
        e = wrap_angles(X[t] - xg, wrap_idx)
        Pe = P @ e
        blk = np.zeros((n + 1, n + 1))
        blk[:n, :n] = P
        blk[:n, n] = Pe
        blk[n, :n] = Pe
        blk[n, n] = float(e @ Pe) + rho_reg
        out[t - 1] = sym(blk)
    return out


# ---------------------------------------------------------------------------
# a9 / a10 / a11 : Riccati passes
# ---------------------------------------------------------------------------

def riccati_truncated(A_list, B_list, X, U, xg, u_ref, Q, R, alpha, T_star,
                      lm_lambda=1e-3, wrap_idx=None, extra=None, want_v=False):
    """solver.py:156-230.  Returns (k_list, K_list, ok[, Vxx_list, Vx_list]).

    Vxx/Vx are internal in the reference; with want_v they are returned for
    index 0..T_star (index T_star = terminal).
    """
    T = int(T_star)
    if T <= 0:
        return (None, None, False) + ((None, None) if want_v else ())
    n = X.shape[1]
    m = U.shape[1]
    Qf = terminal_weight(alpha, n)
    fail = (None, None, False) + ((None, None) if want_v else ())
    eT = wrap_angles(X[T] - xg, wrap_idx)
    if not np.isfinite(eT).all():
        return fail
    Vx = Qf @ eT
    Vxx = sym(Qf)
    ks, Ks = [None] * T, [None] * T
    Vxxs, Vxs = [None] * (T + 1), [None] * (T + 1)
    Vxxs[T], Vxs[T] = Vxx, Vx
    for k in range(T - 1, -1, -1):
        e = wrap_angles(X[k] - xg, wrap_idx)
        du = np.atleast_1d(U[k] - u_ref)
        if not (np.isfinite(e).all() and np.isfinite(du).all()):
            return fail
        lx = Q @ e
        lu = R @ du
        Qst = Q
        if extra is not None:
            _, cx, cxx = extra(X[k], U[k])
            lx = lx + np.asarray(cx, dtype=np.float64).reshape(-1)
            Qst = sym(Qst + np.asarray(cxx, dtype=np.float64))
        A, B = A_list[k], B_list[k]
        Qx = lx + A.T @ Vx
        Qu = lu + B.T @ Vx
        Qxx = Qst + A.T @ Vxx @ A
        Quu = R + B.T @ Vxx @ B
        Qux = B.T @ Vxx @ A
        Quu_reg = sym(Quu) + float(lm_lambda) * np.eye(m)
        try:
            np.linalg.cholesky(Quu_reg)
        except np.linalg.LinAlgError:
            return fail
        x1, s1 = spd_solve(Quu_reg, Qu)
        x2, s2 = spd_solve(Quu_reg, Qux)
        if x1 is None or x2 is None:
            return fail  # reference raises LinAlgError here; treated as failure
        kap = -x1
        Kk = -x2
        ks[k], Ks[k] = kap, Kk
        Vx = Qx + Kk.T @ Qu + Qux.T @ kap + Kk.T @ Quu @ kap
        Vxx = sym(Qxx + Kk.T @ Qux + Qux.T @ Kk + Kk.T @ Quu @ Kk)
        if not (np.isfinite(Vx).all() and np.isfinite(Vxx).all()):
            return fail
        Vxxs[k], Vxs[k] = Vxx, Vx
    if want_v:
        return ks, Ks, True, Vxxs, Vxs
    return ks, Ks, True


def riccati_expand(A_list, B_list, X, U, xg, u_ref, Q, R, alpha, T_bar, S_right,
                   lm_lambda=1e-6, w_stage=0.0, wrap_idx=None, extra=None,
                   reg_max_tries=12):
    """horizon_selection.py:97-212 -> (Vxx, Vx, V0, K, k), index i = t + S_right.

    Raises FloatingPointError / LinAlgError where the reference does (the
    finiteness checks of horizon_selection.py:138-139, 150-151, 172-173, 179-180,
    188-189, 209-210).
    """
    n = X.shape[1]
    m = U.shape[1]
    Qf = terminal_weight(alpha, n)
    fin = lambda a: bool(np.all(np.isfinite(a)))  # noqa: E731
    L = int(T_bar) + int(S_right)
    Vxx = [np.zeros((n, n)) for _ in range(L + 1)]
    Vx = [np.zeros(n) for _ in range(L + 1)]
    V0 = [0.0] * (L + 1)
    K = [None] * L
    kk = [None] * L
    eT = wrap_angles(X[L] - xg, wrap_idx)
    if not np.isfinite(eT).all():
        raise FloatingPointError("non-finite terminal error")
    Vxx[L] = sym(Qf)
    Vx[L] = Qf @ eT
    V0[L] = 0.5 * float(eT @ (Qf @ eT))
    for i in range(L - 1, -1, -1):
        e = wrap_angles(X[i] - xg, wrap_idx)
        du = np.atleast_1d(U[i] - u_ref)
        if not (np.isfinite(e).all() and np.isfinite(du).all()):
            raise FloatingPointError("non-finite e/du")
        lx = Q @ e
        lu = R @ du
        l0 = 0.5 * float(e @ (Q @ e)) + 0.5 * float(du @ (R @ du)) + float(w_stage)
        Qst = Q
        if extra is not None:
            c, cx, cxx = extra(X[i], U[i])
            l0 += float(c)
            lx = lx + np.asarray(cx, dtype=np.float64).reshape(-1)
            Qst = sym(Qst + np.asarray(cxx, dtype=np.float64))
        A = np.asarray(A_list[i], dtype=np.float64)
        B = np.asarray(B_list[i], dtype=np.float64)
        if not (fin(A) and fin(B) and fin(Vx[i + 1]) and fin(Vxx[i + 1])):
            raise FloatingPointError("non-finite A/B/V")
        Qx = lx + A.T @ Vx[i + 1]
        Qu = lu + B.T @ Vx[i + 1]
        Qxx = Qst + A.T @ Vxx[i + 1] @ A
        Quu = R + B.T @ Vxx[i + 1] @ B
        Qux = B.T @ Vxx[i + 1] @ A
        if not (fin(Qx) and fin(Qu) and fin(Qxx) and fin(Quu) and fin(Qux)):
            raise FloatingPointError("non-finite Q terms")
        lam = float(max(lm_lambda, 1e-12))
        sol = None
        for _ in range(int(reg_max_tries)):
            Quu_reg = sym(Quu) + lam * np.eye(m)
            if not fin(Quu_reg):
                raise FloatingPointError("non-finite Quu_reg")
            a, s1 = spd_solve(Quu_reg, Qu)
            b, s2 = spd_solve(Quu_reg, Qux)
            if a is not None and b is not None:
                sol = (a, b)
                break
            lam *= 10.0
        if sol is None:
            raise np.linalg.LinAlgError("Quu not PD for any regularisation")
        a, b = sol
        kk[i] = -a
        K[i] = -b
        Vxx[i] = sym(Qxx - Qux.T @ b)
        Vx[i] = Qx - Qux.T @ a
        V0[i] = l0 + V0[i + 1] - 0.5 * float(Qu @ a)
        if not (fin(Vxx[i]) and fin(Vx[i]) and np.isfinite(V0[i])):
            raise FloatingPointError("non-finite V")
    return Vxx, Vx, V0, K, kk


def chol_solve_raise(A, B, jitter=JITTER0, max_tries=8):
    """utils.py:96-120 exactly: FloatingPointError on a non-finite A or B, the
    jitter ladder (a non-finite X counts as a failed try), LinAlgError at the end."""
    A = sym(np.asarray(A, dtype=np.float64))
    B = np.asarray(B, dtype=np.float64)
    if not np.all(np.isfinite(A)):
        raise FloatingPointError("Non-finite values in chol_solve(A)")
    if not np.all(np.isfinite(B)):
        raise FloatingPointError("Non-finite values in chol_solve(B)")
    eye = np.eye(A.shape[0])
    eps = float(jitter)
    for _ in range(int(max_tries)):
        try:
            low = np.linalg.cholesky(A + eps * eye)
            X = np.linalg.solve(low.T, np.linalg.solve(low, B))
            if not np.all(np.isfinite(X)):
                raise FloatingPointError
            return X
        except (np.linalg.LinAlgError, FloatingPointError):
            eps *= 10.0
    raise np.linalg.LinAlgError("chol_solve failed: matrix not PD")


def chol_solve_legacy(A, B, jitter=JITTER0, max_tries=4):
    """ilqr_propagator.py:33-43: 4 jitters (no finiteness checks), then the
    least-squares solve of sym(A) (np.linalg.lstsq, rcond=None)."""
    A = sym(np.asarray(A, dtype=np.float64))
    eye = np.eye(A.shape[0])
    eps = float(jitter)
    for _ in range(int(max_tries)):
        try:
            low = np.linalg.cholesky(A + eps * eye)
            return np.linalg.solve(low.T, np.linalg.solve(low, B)), 0
        except np.linalg.LinAlgError:
            eps *= 10.0
    return np.linalg.lstsq(A, B, rcond=None)[0], ST_LU


def riccati_truncated_legacy(A_list, B_list, X, U, xg, u_ref, Q, R, alpha, T_star,
                             lm_lambda=1e-3, wrap_idx=None):
    """ilqr_propagator.py:375-400 (the legacy backward_pass_truncated): Qf = alpha I,
    a Cholesky gate on Quu_reg without jitter ((None, None, False) when it fails),
    then the legacy chol_solve; no finiteness checks."""
    T = int(T_star)
    n, m = X.shape[1], U.shape[1]
    ks, Ks = [None] * T, [None] * T
    eT = wrap_angles(np.asarray(X[T] - xg, dtype=np.float64), wrap_idx).reshape(-1)
    Vx, Vxx = float(alpha) * eT, float(alpha) * np.eye(n)
    for k in range(T - 1, -1, -1):
        e = wrap_angles(np.asarray(X[k] - xg, dtype=np.float64), wrap_idx).reshape(-1)
        du = np.atleast_1d(U[k] - u_ref).reshape(-1)
        A, B = A_list[k], B_list[k]
        Qx, Qu = Q @ e + A.T @ Vx, R @ du + B.T @ Vx
        Qxx, Quu, Qux = Q + A.T @ Vxx @ A, R + B.T @ Vxx @ B, B.T @ Vxx @ A
        Quu_reg = sym(Quu) + float(lm_lambda) * np.eye(m)
        try:
            np.linalg.cholesky(Quu_reg)
        except np.linalg.LinAlgError:
            return None, None, False
        kap = -chol_solve_legacy(Quu_reg, Qu)[0]
        Kk = -chol_solve_legacy(Quu_reg, Qux)[0]
        ks[k], Ks[k] = kap, Kk
        Vx = Qx + Kk.T @ Qu + Qux.T @ kap + Kk.T @ Quu @ kap
        Vxx = sym(Qxx + Kk.T @ Qux + Qux.T @ Kk + Kk.T @ Quu @ Kk)
    return ks, Ks, True


def riccati_expand_legacy(A_list, B_list, X, U, xg, u_ref, Q, R, alpha, T_bar, S_right,
                          lm_lambda=1e-6, w_stage=0.0, wrap_idx=None):
    """ilqr_propagator.py:237-287 (the legacy value_expansions_and_gains_prefix):
    Qf = alpha I, Quu_reg = _sym(Quu) + lm I, the legacy chol_solve (4 jitters,
    then lstsq; never raises for finite data).  Returns (Vxx, Vx, V0, K, k, status)
    with index i = t + S_right; status has ST_LU where lstsq ran."""
    n, m = X.shape[1], U.shape[1]
    L = int(T_bar) + int(S_right)
    Vxx = [np.zeros((n, n)) for _ in range(L + 1)]
    Vx = [np.zeros(n) for _ in range(L + 1)]
    V0 = [0.0] * (L + 1)
    K, kk, st = [None] * L, [None] * L, 0
    eT = wrap_angles(np.asarray(X[L] - xg, dtype=np.float64), wrap_idx).reshape(-1)
    Vxx[L], Vx[L], V0[L] = float(alpha) * np.eye(n), float(alpha) * eT, \
        0.5 * float(alpha) * float(eT @ eT)
    for i in range(L - 1, -1, -1):
        e = wrap_angles(np.asarray(X[i] - xg, dtype=np.float64), wrap_idx).reshape(-1)
        du = np.atleast_1d(U[i] - u_ref).reshape(-1)
        l0 = 0.5 * float(e @ (Q @ e)) + 0.5 * float(du @ (R @ du)) + float(w_stage)
        A, B = A_list[i], B_list[i]
        Qx, Qu = Q @ e + A.T @ Vx[i + 1], R @ du + B.T @ Vx[i + 1]
        Qxx = Q + A.T @ Vxx[i + 1] @ A
        Quu = R + B.T @ Vxx[i + 1] @ B
        Qux = B.T @ Vxx[i + 1] @ A
        Quu_reg = sym(Quu) + float(lm_lambda) * np.eye(m)
        a, s1 = chol_solve_legacy(Quu_reg, Qu)
        b, s2 = chol_solve_legacy(Quu_reg, Qux)
        st |= s1 | s2
        kk[i], K[i] = -a, -b
        Vxx[i] = sym(Qxx - Qux.T @ b)
        Vx[i] = Qx - Qux.T @ a
        V0[i] = l0 + V0[i + 1] - 0.5 * float(Qu.T @ a)
    return Vxx, Vx, V0, K, kk, st


def bruteforce_J(A_list, B_list, X, U, xg, u_ref, Q, R, alpha, w, T_max,
                 lm_lambda=1e-6, wrap_idx=None, extra=None, legacy=False, want_status=False):
    """solver.py:293-358: J[T-1] = V0[0] of a fresh Riccati sweep of length T.

    Unlike value_expansions_and_gains_prefix it checks nothing itself: only its
    chol_solve raises (non-finite Quu_reg / Qu / Qux, or no jitter factors), so a
    non-finite e at t = 0, or a V_0 that overflows, just leaves inf/NaN in J.
    legacy=True restates ilqr_propagator.py:426-454 instead: Vxx_T = alpha I,
    Vx_T = alpha e_T, and the legacy chol_solve (4 jitters, then lstsq; it never
    raises for finite data).  want_status: also return the per-horizon status
    (ST_LU where the legacy lstsq ran)."""
    n, m = X.shape[1], U.shape[1]
    J = np.zeros(int(T_max))
    st = np.zeros(int(T_max), dtype=np.int32)
    Qf = None if legacy else terminal_weight(alpha, n)
    for T in range(1, int(T_max) + 1):
        eT = wrap_angles(np.asarray(X[T] - xg, dtype=np.float64), wrap_idx).reshape(-1)
        if legacy:
            Vxx, Vx, V0 = float(alpha) * np.eye(n), float(alpha) * eT, 0.5 * float(alpha) * float(eT @ eT)
        else:
            Vxx, Vx, V0 = sym(Qf), Qf @ eT, 0.5 * float(eT @ (Qf @ eT))
        for t in range(T - 1, -1, -1):
            e = wrap_angles(np.asarray(X[t] - xg, dtype=np.float64), wrap_idx).reshape(-1)
            du = np.atleast_1d(U[t] - u_ref).reshape(-1)
            lx, lu = Q @ e, R @ du
            l0 = 0.5 * float(e @ (Q @ e)) + 0.5 * float(du @ (R @ du)) + float(w)
            Qst = Q
            if extra is not None and not legacy:
                c, cx, cxx = extra(X[t], U[t])
                l0 += float(c)
                lx = lx + np.asarray(cx, dtype=np.float64).reshape(-1)
                Qst = sym(Qst + np.asarray(cxx, dtype=np.float64))
            A, B = A_list[t], B_list[t]
            Qx = lx + A.T @ Vx
            Qu = lu + B.T @ Vx
            Qxx = Qst + A.T @ Vxx @ A
            Quu = R + B.T @ Vxx @ B
            Qux = B.T @ Vxx @ A
            Quu_reg = sym(Quu) + float(lm_lambda) * np.eye(m)
            if legacy:
                a, s1 = chol_solve_legacy(Quu_reg, Qu)
                b, s2 = chol_solve_legacy(Quu_reg, Qux)
                st[T - 1] |= s1 | s2
            else:
                a = chol_solve_raise(Quu_reg, Qu)
                b = chol_solve_raise(Quu_reg, Qux)
            Vxx = sym(Qxx - Qux.T @ b)
            Vx = Qx - Qux.T @ a
            V0 = l0 + V0 - 0.5 * float(Qu.T @ a)
        J[T - 1] = float(V0)
    return (J, st) if want_status else J


# ---------------------------------------------------------------------------
# Synthetic generators; PCG64 default_rng is platform-stable
# ---------------------------------------------------------------------------

def synth_lft_problem(seed, s, m, N):
    """Well-conditioned augmented LFT inputs for one problem."""
    rng = np.random.default_rng(int(seed))
    n = s - 1
    A = np.zeros((N, s, s))
    Bm = np.zeros((N, s, m))
    Q = np.zeros((N, s, s))
    QT = np.zeros((N, s, s))
    for k in range(N):
        A[k, :n, :n] = np.eye(n) + 0.05 * rng.standard_normal((n, n))
        A[k, :n, n] = 0.1 * rng.standard_normal(n)
        A[k, n, n] = 1.0
        Bm[k, :n, :] = 0.1 * rng.standard_normal((n, m))
        M = rng.standard_normal((s, s))
        Q[k] = M @ M.T / s + np.eye(s)
        M = rng.standard_normal((s, s))
        QT[k] = M @ M.T / s + np.eye(s)
    R = np.diag(rng.uniform(0.5, 2.0, m))
    R_inv, _ = spd_inverse(R)
    z0 = np.zeros(s)
    z0[-1] = 1.0
    return A, Bm, Q, R, R_inv, z0, QT


def synth_lft_batch(base_seed, B, s, m, N):
    """Stack synth_lft_problem(base_seed + i) for i < B."""
    parts = [synth_lft_problem(base_seed + i, s, m, N) for i in range(B)]
    return tuple(np.stack([p[j] for p in parts]) for j in range(7))


def synth_riccati_problem(seed, n, m, N):
    """Trajectory-form Riccati inputs (A_k, B_k, X, U, xg, u_ref, Q, R, alpha)."""
    rng = np.random.default_rng(int(seed))
    A = np.eye(n) + 0.05 * rng.standard_normal((N, n, n))
    B = 0.1 * rng.standard_normal((N, n, m))
    X = 0.5 * rng.standard_normal((N + 1, n))
    U = 0.1 * rng.standard_normal((N, m))
    xg = 0.2 * rng.standard_normal(n)
    u_ref = 0.05 * rng.standard_normal(m)
    M = rng.standard_normal((n, n))
    Q = M @ M.T / n + 0.5 * np.eye(n)
    R = np.diag(rng.uniform(0.5, 2.0, m))
    alpha = float(rng.uniform(5.0, 20.0))
    return A, B, X, U, xg, u_ref, Q, R, alpha


def synth_traj_problem(seed, n, m, N):
    """Trajectory-form select inputs (augmented.py:10-87 + propagator) for one
    problem: A_k, B_k, raw residuals a_k, X, U, xg, u_ref, Q, R, alpha (diagonal
    terminal weight), w and wrap_idx.  Angles of state 0 span several turns so
    the wrap is exercised.  The residual the reference forms,
    F(x_k, u_k) - x_{k+1} with F(x_k, u_k) = x_{k+1} + a_raw_k, is returned as
    a_res (same NumPy expression as compute_affine_residuals)."""
    rng = np.random.default_rng(int(seed))
    A = np.eye(n) + 0.05 * rng.standard_normal((N, n, n))
    B = 0.1 * rng.standard_normal((N, n, m))
    X = 0.5 * rng.standard_normal((N + 1, n))
    X[:, 0] = 6.0 * rng.standard_normal(N + 1)
    U = 0.3 * rng.standard_normal((N, m))
    a_raw = 0.02 * rng.standard_normal((N, n))
    xg = 0.2 * rng.standard_normal(n)
    u_ref = 0.1 * rng.standard_normal(m)
    M = rng.standard_normal((n, n))
    Q = M @ M.T / n + 0.5 * np.eye(n)
    R = np.diag(rng.uniform(0.5, 2.0, m))
    alpha = rng.uniform(1.0, 10.0, n)
    w = float(rng.uniform(0.2, 1.0))
    a_res = np.stack([(X[k + 1] + a_raw[k]) - X[k + 1] for k in range(N)])
    return dict(A=A, B=B, a_res=a_res, X=X, U=U, xg=xg, u_ref=u_ref, Q=Q, R=R, alpha=alpha,
                w=w, wrap_idx=[0], a_raw=a_raw)


# ---------------------------------------------------------------------------
# Config 5: mixed Segway / Cartpole / Quadrotor shapes
# ---------------------------------------------------------------------------

CONFIG5_KINDS = (("segway", 5, 1), ("cartpole", 5, 1), ("quadrotor", 13, 4))


def config5_kind(i):
    """Member i of the config-5 batch: kind i mod 3 -> (name, s, m)."""
    return CONFIG5_KINDS[int(i) % 3]


def synth_config5_problem(base_seed, i, N):
    """Problem i of the mixed batch at its TRUE shape (synth_lft_problem with
    seed base_seed + i and the kind's (s, m))."""
    _, s, m = config5_kind(i)
    return synth_lft_problem(base_seed + int(i), s, m, N)


def embed_block_decoupled(A, Bm, Q, R_inv, z0, QT, s_out, m_out):
    """NumPy statement of the block-decoupled embedding:
    real state dims keep their indices, pad dims sit between them and the
    homogeneous coordinate (last); A_pad = 0, B_pad rows / extra columns 0,
    Q_pad = QT_pad = I, R_inv_pad = I, z0_pad = 0.  One problem, (N, s, s) blocks."""
    N, s = A.shape[0], A.shape[1]
    m = Bm.shape[-1]
    n = s - 1
    idx = list(range(n)) + [s_out - 1]

    def sq(M, fill):
        out = np.zeros((N, s_out, s_out))
        out[:, n:s_out - 1, n:s_out - 1] = fill * np.eye(s_out - 1 - n)
        out[np.ix_(range(N), idx, idx)] = M
        return out

    Bp = np.zeros((N, s_out, m_out))
    Bp[np.ix_(range(N), idx, range(m))] = Bm
    Rp = np.eye(m_out)
    Rp[:m, :m] = R_inv
    zp = np.zeros(s_out)
    zp[idx] = z0
    return sq(A, 0.0), Bp, sq(Q, 1.0), Rp, zp, sq(QT, 1.0)
