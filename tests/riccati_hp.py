"""value_expansions_and_gains_prefix (mode 1) and backward_pass_truncated (mode 0) in
40-digit arithmetic (test infrastructure, mpmath): the referee where the fp64 oracle
and the device disagree by more than 1e-6 per step.

Same recursion as oracle/hop_oracle.py riccati_expand / riccati_truncated
(/root/reference/horizon_selection.py:97-212, solver.py:156-230) on the same fp64
inputs, with the first-attempt regularisation (sym(Quu) + lm I + 1e-9 I for mode 1,
the chol_solve jitter; sym(Quu) + lm I for mode 0's Cholesky gate and solve through
chol_solve's 1e-9): every call here is on inputs whose first attempt succeeds, which
the caller checks (status 0 on both fp64 paths).  Only what the tests compare is
returned: Vxx / Vx / V0 / K (mode 1) or K / k (mode 0), as float64 arrays of the
exact values rounded once.
"""
from __future__ import annotations

import numpy as np

DPS = 40


def _mp():
    import mpmath
    mpmath.mp.dps = DPS
    return mpmath


def _M(mp, a):
    a = np.asarray(a, dtype=np.float64)
    if a.ndim == 1:
        return mp.matrix([[mp.mpf(float(v))] for v in a])
    return mp.matrix([[mp.mpf(float(v)) for v in row] for row in a])


def _np(x):
    return np.array([[float(x[i, j]) for j in range(x.cols)] for i in range(x.rows)])


def _sym(M):
    return (M + M.T) * 0.5


def _wrap(mp, e, wrap_idx):
    if not wrap_idx:
        return e
    e = e.copy()
    pi = mp.mpf(np.pi)  # the fp64 constant the reference's wrap_error uses
    for i in wrap_idx:
        v = e[i]
        e[i] = (v + pi) - 2 * pi * mp.floor((v + pi) / (2 * pi)) - pi
    return e


def riccati_hp(A_list, B_list, X, U, xg, u_ref, Q, R, Qf, T, lm, *, mode, w_stage=0.0,
               wrap_idx=None):
    """mode 1: (Vxx [T+1,n,n], Vx [T+1,n], V0 [T+1], K [T,m,n]); mode 0: (K, k)."""
    mp = _mp()
    n, m = np.shape(X)[1], np.shape(U)[1]
    Qm, Rm, Qfm = _M(mp, Q), _M(mp, R), _M(mp, Qf)
    xgm, urm = _M(mp, xg), _M(mp, u_ref)
    # chol_solve's first attempt adds its 1e-9 jitter to Quu_reg = sym(Quu) + lm I
    # (utils.py:96-120), in both passes
    eps = mp.mpf(float(lm)) + mp.mpf(1e-9)
    I_m = mp.eye(m)
    eT = _wrap(mp, _M(mp, X[T]) - xgm, wrap_idx)
    Vxx = _sym(Qfm)
    Vx = Qfm * eT
    V0 = (eT.T * Qfm * eT)[0] * mp.mpf("0.5")
    out_Vxx, out_Vx, out_V0, out_K, out_k = [None] * (T + 1), [None] * (T + 1), [None] * (T + 1), \
        [None] * T, [None] * T
    out_Vxx[T], out_Vx[T], out_V0[T] = Vxx, Vx, V0
    for i in range(T - 1, -1, -1):
        e = _wrap(mp, _M(mp, X[i]) - xgm, wrap_idx)
        du = _M(mp, U[i]) - urm
        A, B = _M(mp, A_list[i]), _M(mp, B_list[i])
        lx, lu = Qm * e, Rm * du
        Qx = lx + A.T * Vx
        Qu = lu + B.T * Vx
        Qxx = Qm + A.T * Vxx * A
        Quu = Rm + B.T * Vxx * B
        Qux = B.T * Vxx * A
        Qr = _sym(Quu) + I_m * eps
        Qi = mp.inverse(Qr)  # m x m at 40 digits: the solve's error is far below fp64's
        a = Qi * Qu
        b = Qi * Qux
        out_K[i], out_k[i] = -b, -a
        if mode == 1:
            l0 = (e.T * Qm * e)[0] * mp.mpf("0.5") + (du.T * Rm * du)[0] * mp.mpf("0.5") + \
                mp.mpf(w_stage)
            Vxx = _sym(Qxx - Qux.T * b)
            Vx = Qx - Qux.T * a
            V0 = l0 + V0 - (Qu.T * a)[0] * mp.mpf("0.5")
        else:
            K, k = -b, -a
            Vx = Qx + K.T * Qu + Qux.T * k + K.T * Quu * k
            Vxx = _sym(Qxx + K.T * Qux + Qux.T * K + K.T * Quu * K)
        out_Vxx[i], out_Vx[i], out_V0[i] = Vxx, Vx, V0
    K = np.stack([_np(x) for x in out_K])
    if mode == 0:
        return K, np.stack([_np(x)[:, 0] for x in out_k])
    return (np.stack([_np(x) for x in out_Vxx]), np.stack([_np(x)[:, 0] for x in out_Vx]),
            np.array([float(v) for v in out_V0]), K)
