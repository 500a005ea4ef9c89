"""Reference-shaped augmented builders (augmented.py:10-87) on the device.

``build_augmented_sequence_QR`` / ``build_terminal_aug_list`` keep the
reference's names, arguments and list-of-blocks return values, and build the
blocks with the batched device builder (hop_augment_f64, csrc/augment.hip --
the same builders the fused select kernel runs in-kernel).  Only the affine
residual a_k = F(x_k, u_k) - x_{k+1} is evaluated on the host, because F is the
caller's Python dynamics (linearization.py:269-270); batched callers with
device dynamics use engine.linearize's a_res and engine.augment /
engine.propagate_traj directly.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

from . import engine
from .utils import _sym, as_terminal_weight, chol_inv


def compute_affine_residuals(F, X: np.ndarray, U: np.ndarray):
    """a_k = F(x_k, u_k) - x_{k+1}  (linearization.py:269-270)."""
    return [(np.asarray(F(X[k], U[k]), dtype=float) - X[k + 1]).reshape(-1, 1)
            for k in range(len(U))]


def _device_blocks(A_list, B_list, a_res, X, U, xg, u_ref, Q, P, w, wrap_idx, q_reg, rho_reg,
                   extra_stage_cost):
    from .horizon_selection import _to_dev
    N = len(A_list)
    n = X.shape[1]
    m = U.shape[1]
    ex = {}
    if extra_stage_cost is not None:  # per-step cost terms evaluated by the caller's callable
        c, cx, cxx = zip(*(extra_stage_cost(X[k], U[k]) for k in range(N)))
        ex = dict(qxx_extra=_to_dev(np.array(cxx, dtype=float).reshape(1, N, n, n)),
                  qx_extra=_to_dev(np.array(cx, dtype=float).reshape(1, N, n)),
                  c_extra=_to_dev(np.array(c, dtype=float).reshape(1, N)))
    return engine.augment(
        _to_dev(np.asarray(A_list, dtype=float).reshape(1, N, n, n)),
        _to_dev(np.asarray(B_list, dtype=float).reshape(1, N, n, m)),
        _to_dev(np.asarray(a_res, dtype=float).reshape(1, N, n)),
        _to_dev(np.asarray(X[:N + 1], dtype=float)[None]),
        _to_dev(np.asarray(U[:N], dtype=float)[None]),
        _to_dev(np.asarray(xg, dtype=float).reshape(-1)),
        _to_dev(np.atleast_1d(np.asarray(u_ref, dtype=float)).reshape(-1)),
        _to_dev(np.asarray(Q, dtype=float)), _to_dev(P), float(w), wrap_idx=wrap_idx,
        q_reg=q_reg, rho_reg=rho_reg, **ex)


def build_augmented_sequence_QR(F, A_list, B_list, X, U, xg, u_ref, Q, R, w,
                                wrap_idx: Optional[List[int]] = None, q_reg: float = 1e-9,
                                rho_reg: float = 1e-12, extra_stage_cost=None):
    """Augmented (A, B, Q, R) blocks (augmented.py:10-60) ->
    (A_aug, B_aug, Q_aug, R_list, z0, R_inv) as the reference returns them."""
    X = np.asarray(X, dtype=float)
    U = np.asarray(U, dtype=float)
    if U.ndim == 1:
        U = U.reshape(-1, 1)
    N = len(A_list)
    n = X.shape[1]
    R = _sym(np.asarray(R, dtype=float))
    R_inv = chol_inv(R)
    res = compute_affine_residuals(F, X, U[:N])
    blk = _device_blocks(A_list, B_list, res, X, U, xg, u_ref, Q, np.eye(n), w, wrap_idx, q_reg,
                         rho_reg, extra_stage_cost)
    A_aug = list(blk.A[0].cpu().numpy())
    B_aug = list(blk.B[0].cpu().numpy())
    Q_aug = list(blk.Q[0].cpu().numpy())
    return A_aug, B_aug, Q_aug, [R] * N, blk.z0.cpu().numpy(), R_inv


def build_terminal_aug_list(X, xg, alpha, wrap_idx: Optional[List[int]] = None,
                            rho_reg: float = 1e-12):
    """Terminal blocks QT[t-1], t = 1..N (augmented.py:63-87), as a list."""
    X = np.asarray(X, dtype=float)
    n = X.shape[1]
    N = X.shape[0] - 1
    P = _sym(as_terminal_weight(alpha, n))
    zero = [np.zeros((n, n))] * N
    blk = _device_blocks(zero, [np.zeros((n, 1))] * N, np.zeros((N, n)), X, np.zeros((N, 1)), xg,
                         np.zeros(1), np.eye(n), P, 0.0, wrap_idx, 1e-9, rho_reg, None)
    return list(blk.QT[0].cpu().numpy())
