"""Host-side helpers mirroring the reference's utils.py call surface.

Only input preparation lives here (terminal-weight coercion, angle wrapping,
symmetrisation, the m x m SPD inverse used while assembling augmented blocks).
None of it is the horizon-selection hot path, which runs in libhop_amd.so.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np


def _sym(A: np.ndarray) -> np.ndarray:
    """0.5 (A + A^T)  (reference utils.py:35-37)."""
    return 0.5 * (A + A.T)


def as_terminal_weight(alpha, n: int) -> np.ndarray:
    """Scalar / diagonal vector / matrix terminal weight -> (n, n) (utils.py:49-62)."""
    w = np.asarray(alpha, dtype=float)
    if w.ndim == 0:
        return float(w) * np.eye(n)
    if w.ndim == 1:
        if w.shape[0] != n:
            raise ValueError(f"terminal weight vector has shape {w.shape}, expected ({n},)")
        return np.diag(w)
    if w.ndim == 2:
        if w.shape != (n, n):
            raise ValueError(f"terminal weight matrix has shape {w.shape}, expected ({n},{n})")
        return _sym(w)
    raise ValueError(f"unsupported terminal weight ndim={w.ndim}")


def angle_normalize(a):
    """(a + pi) mod 2 pi - pi  (utils.py:127-128)."""
    return (a + np.pi) % (2.0 * np.pi) - np.pi


def wrap_error(e: np.ndarray, wrap_idx: Optional[List[int]] = None) -> np.ndarray:
    """Wrap the listed coordinates of an error vector (utils.py:131-137)."""
    if not wrap_idx:
        return e
    out = np.asarray(e, dtype=float).copy()
    for i in wrap_idx:
        out[i] = angle_normalize(float(out[i]))
    return out


def chol_inv(A: np.ndarray, jitter: float = 1e-9, max_tries: int = 8) -> np.ndarray:
    """SPD inverse with jitter escalation (utils.py:69-93) for small host-side
    blocks (R while assembling the augmented sequence).  The batched sweeps
    invert on the device instead."""
    S = _sym(np.asarray(A, dtype=float))
    if not np.all(np.isfinite(S)):
        raise FloatingPointError("Non-finite values in chol_inv(A)")
    eye = np.eye(S.shape[0])
    eps = float(jitter)
    for _ in range(int(max_tries)):
        try:
            L = np.linalg.cholesky(S + eps * eye)
        except np.linalg.LinAlgError:
            eps *= 10.0
            continue
        return np.linalg.solve(L.T, np.linalg.solve(L, eye))
    try:
        return np.linalg.solve(S + eps * eye, eye)
    except np.linalg.LinAlgError as exc:
        raise np.linalg.LinAlgError(f"chol_inv failed even with jitter={eps:g}: {exc}")
