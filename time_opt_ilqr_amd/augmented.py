"""Host assembly of the augmented (n+1) x (n+1) blocks consumed by the sweep.

Mirrors the reference's augmented.py:10-87 call surface.  The affine residual
a_k = F(x_k, u_k) - x_{k+1} needs the Python dynamics F, so this stays on the
host; ``stack_augmented`` packs the result into the batch-major layout of the
device API (engine.propagate).
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

from .utils import _sym, as_terminal_weight, chol_inv, wrap_error


def compute_affine_residuals(F, X: np.ndarray, U: np.ndarray):
    """a_k = F(x_k, u_k) - x_{k+1}  (linearization.py:269-270)."""
    return [(np.asarray(F(X[k], U[k]), dtype=float) - X[k + 1]).reshape(-1, 1)
            for k in range(len(U))]


def build_augmented_sequence_QR(F, A_list, B_list, X, U, xg, u_ref, Q, R, w,
                                wrap_idx: Optional[List[int]] = None, q_reg: float = 1e-9,
                                rho_reg: float = 1e-12, extra_stage_cost=None):
    """Augmented (A, B, Q, R) blocks (augmented.py:10-60)."""
    N = len(A_list)
    n = X.shape[1]
    m = U.shape[1]
    R = _sym(np.asarray(R, dtype=float))
    R_inv = chol_inv(R)
    res = compute_affine_residuals(F, X, U)
    Qs = _sym(np.asarray(Q, dtype=float)) + q_reg * np.eye(n)
    A_aug, B_aug, Q_aug, R_list = [], [], [], []
    for k in range(N):
        e = wrap_error(X[k] - xg, wrap_idx).reshape(-1)
        du = np.atleast_1d(U[k] - u_ref).reshape(-1)
        Qe = (Q @ e).ravel()
        blk = np.zeros((n + 1, n + 1))
        blk[:n, :n] = Qs
        blk[:n, n] = Qe
        blk[n, :n] = Qe
        blk[n, n] = float(e @ Q @ e) + 2.0 * float(w) + rho_reg
        if extra_stage_cost is not None:
            c_x, cx_x, cxx_x = extra_stage_cost(X[k], U[k])
            cx_x = np.asarray(cx_x, dtype=float).reshape(-1)
            blk[:n, :n] += _sym(np.asarray(cxx_x, dtype=float))
            blk[:n, n] += cx_x
            blk[n, :n] += cx_x
            blk[n, n] += 2.0 * float(c_x)
        Ak = np.zeros((n + 1, n + 1))
        Ak[:n, :n] = A_list[k]
        Ak[:n, n] = (res[k] - B_list[k] @ du.reshape(-1, 1)).ravel()
        Ak[n, n] = 1.0
        Bk = np.zeros((n + 1, m))
        Bk[:n, :] = B_list[k]
        A_aug.append(Ak)
        B_aug.append(Bk)
        Q_aug.append(_sym(blk))
        R_list.append(R)
    z0 = np.zeros(n + 1)
    z0[-1] = 1.0
    return A_aug, B_aug, Q_aug, R_list, z0, R_inv


def build_terminal_aug_list(X, xg, alpha, wrap_idx: Optional[List[int]] = None,
                            rho_reg: float = 1e-12):
    """Terminal blocks QT[t-1], t = 1..N (augmented.py:63-87)."""
    n = X.shape[1]
    P = _sym(as_terminal_weight(alpha, n))
    out = []
    for t in range(1, X.shape[0]):
        e = wrap_error(X[t] - xg, wrap_idx).reshape(-1)
        Pe = P @ e
        blk = np.zeros((n + 1, n + 1))
        blk[:-1, :-1] = P
        blk[:-1, -1] = Pe
        blk[-1, :-1] = Pe
        blk[-1, -1] = float(e @ Pe) + rho_reg
        out.append(_sym(blk))
    return out


def stack_augmented(A_aug, B_aug, Q_aug, QT_aug, N: Optional[int] = None):
    """Lists of per-step blocks -> contiguous [N, s, s] / [N, s, m] arrays."""
    N = len(A_aug) if N is None else int(N)
    if len(A_aug) < N or len(B_aug) < N or len(Q_aug) < N or len(QT_aug) < N:
        raise IndexError("list index out of range")  # what the reference loop raises
    return (np.ascontiguousarray(np.stack([np.asarray(a, dtype=float) for a in A_aug[:N]])),
            np.ascontiguousarray(np.stack([np.asarray(b, dtype=float) for b in B_aug[:N]])),
            np.ascontiguousarray(np.stack([np.asarray(q, dtype=float) for q in Q_aug[:N]])),
            np.ascontiguousarray(np.stack([np.asarray(q, dtype=float) for q in QT_aug[:N]])))
