"""Drop-in, GPU-backed versions of the reference's horizon-selection functions.

Same names, argument meaning and error behaviour as the reference
(horizon_selection.py / solver.py of dmmsjtu-umich/time-opt-ilqr), for callers
that hold one problem as lists of NumPy blocks:

  propagator_all_Jt_aug               horizon_selection.py:36-86
  value_expansions_and_gains_prefix   horizon_selection.py:97-212
  backward_pass_truncated             solver.py:156-230
  bruteforce_all_Jt_backward_expansion solver.py:293-358
  select_horizon                      the argmin at solver.py:522
  select_from_trajectory              the select block of ilqr_timeopt,
                                      solver.py:514-522 (builders + propagator +
                                      argmin, the builders run on the device)

Each call stages the blocks into HBM and runs the batch-of-one kernels of
libhop_amd.so; batched callers should use ``engine.propagate`` directly.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np

from . import _lib, engine
from .augmented import compute_affine_residuals
from .utils import _sym, as_terminal_weight, chol_inv

_DEVICE = None


def _torch():
    import torch
    return torch


def device():
    """The HIP device used by the drop-in functions (fails loudly without one)."""
    global _DEVICE
    torch = _torch()
    if _DEVICE is None:
        if not torch.cuda.is_available():
            raise _lib.HopError("time_opt_ilqr_amd needs a HIP device (MI355X); "
                                "there is no CPU fallback")
        _DEVICE = torch.device("cuda", torch.cuda.current_device())
    return _DEVICE


def _to_dev(a, dtype=None):
    torch = _torch()
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype or torch.float64,
                           device=device())


def _raise_for(status: int, where: str):
    if status & _lib.ST_NONFINITE:
        raise FloatingPointError(f"Non-finite values in {where}")
    if status & _lib.ST_FAIL:
        raise np.linalg.LinAlgError(f"{where}: matrix not positive definite for any jitter")


def propagator_all_Jt_aug(A_aug, B_aug, Q_aug, R_list, z0, QT_aug_list,
                          T_use: Optional[int] = None,
                          R_inv_cached: Optional[np.ndarray] = None) -> np.ndarray:
    """J(T) for all T via the information-form propagator (GPU)."""
    N = len(A_aug) if T_use is None else int(T_use)
    if N <= 0:
        return np.zeros(0, dtype=float)
    if min(len(A_aug), len(B_aug), len(Q_aug), len(QT_aug_list)) < N:
        raise IndexError("list index out of range")
    A = np.stack([np.asarray(x, dtype=float) for x in A_aug[:N]])[None]
    Bm = np.stack([np.asarray(x, dtype=float) for x in B_aug[:N]])[None]
    Q = np.stack([np.asarray(x, dtype=float) for x in Q_aug[:N]])[None]
    QT = np.stack([np.asarray(x, dtype=float) for x in QT_aug_list[:N]])[None]
    if R_inv_cached is None:
        if len(R_list) < N:
            raise IndexError("list index out of range")
        R = np.stack([np.asarray(r, dtype=float) for r in R_list[:N]])[None]
        r_inv = False
    else:
        R = np.asarray(R_inv_cached, dtype=float)
        r_inv = True
    z = np.asarray(z0, dtype=float).reshape(-1)
    res = engine.propagate(_to_dev(A), _to_dev(Bm), _to_dev(Q), _to_dev(R), _to_dev(z),
                           _to_dev(QT), r_is_inverse=r_inv)
    J = res.J[0].cpu().numpy()
    _raise_for(int(res.status[0].item()), "chol_inv(A)")
    return J


def select_horizon(J, T_min: int, T_max: int) -> int:
    """T* = int(np.argmin(J[T_min-1:T_max]) + T_min), computed on the device."""
    torch = _torch()
    Jt = J if isinstance(J, torch.Tensor) else _to_dev(np.asarray(J, dtype=float))
    if Jt.device.type != "cuda":
        Jt = Jt.to(device())
    if not (1 <= int(T_min) <= int(T_max) <= Jt.shape[-1]):
        raise ValueError("attempt to get argmin of an empty sequence")
    ts, _ = engine.select_horizon(Jt, int(T_min), int(T_max))
    return int(ts.item()) if ts.dim() == 0 else ts


def select_from_trajectory(F, A_list, B_list, X, U, xg, u_ref, Q, R, w, alpha,
                           T_min: int, T_max: int, wrap_idx: Optional[List[int]] = None,
                           extra_stage_cost=None) -> Tuple[np.ndarray, int]:
    """The propagator branch of ilqr_timeopt's horizon selection (solver.py:514-522):

        A_aug, B_aug, Q_aug, R_list, z0, R_inv = build_augmented_sequence_QR(...)
        QT_list = build_terminal_aug_list(X, xg, alpha, wrap_idx=wrap_idx)
        J_curve = propagator_all_Jt_aug(..., T_use=T_max, R_inv_cached=R_inv)
        T_bar = int(np.argmin(J_curve[T_min - 1 : T_max]) + T_min)

    Returns (J_curve, T_bar).  The dynamics F (affine residuals), chol_inv(R) and
    the extra stage cost stay on the host as in the reference; the augmented
    blocks are built on the device (inside the sweep for s = 13, m = 4)."""
    X = np.asarray(X, dtype=float)
    U = np.asarray(U, dtype=float).reshape(len(U), -1)
    n, m = X.shape[1], U.shape[1]
    N = len(A_list)
    if int(T_max) > N:
        raise IndexError("list index out of range")
    a_res = np.stack([r.reshape(-1) for r in compute_affine_residuals(F, X, U)])
    R_inv = chol_inv(_sym(np.asarray(R, dtype=float)))
    P = _sym(as_terminal_weight(alpha, n))
    A = np.stack([np.asarray(a, dtype=float) for a in A_list])[None]
    Bm = np.stack([np.asarray(b, dtype=float).reshape(n, m) for b in B_list])[None]
    qxx, qx, c0 = _extra_arrays(extra_stage_cost, X, U, N)
    dv = lambda a: None if a is None else _to_dev(a)  # noqa: E731
    res = engine.propagate_traj(
        dv(A), dv(Bm), dv(a_res[None]), dv(X[None, :N + 1]), dv(U[None, :N]),
        dv(np.asarray(xg, dtype=float).reshape(-1)),
        dv(np.atleast_1d(np.asarray(u_ref, dtype=float)).reshape(-1)),
        dv(np.asarray(Q, dtype=float)), dv(R_inv), dv(P), float(w), wrap_idx=wrap_idx,
        n_use=int(T_max), t_min=int(T_min), t_max=int(T_max), qxx_extra=dv(qxx),
        qx_extra=dv(qx), c_extra=dv(c0))
    J = res.J[0].cpu().numpy()
    _raise_for(int(res.status[0].item()), "chol_inv(A)")
    return J, int(res.t_star[0].item())


def _extra_arrays(extra_stage_cost, X, U, L):
    if extra_stage_cost is None:
        return None, None, None
    n = X.shape[1]
    cxx = np.zeros((L, n, n))
    cx = np.zeros((L, n))
    c0 = np.zeros((L,))
    for i in range(L):
        c, gx, hxx = extra_stage_cost(X[i], U[i])
        c0[i] = float(c)
        cx[i] = np.asarray(gx, dtype=float).reshape(-1)
        cxx[i] = np.asarray(hxx, dtype=float)
    return cxx[None], cx[None], c0[None]


def _riccati_one(A_list, B_list, X, U, xg, u_ref, Q, R, alpha, L, lm, mode, w_stage,
                 wrap_idx, extra_stage_cost, reg_max_tries):
    n, m = X.shape[1], U.shape[1]
    A = np.stack([np.asarray(a, dtype=float) for a in A_list[:L]])[None]
    Bm = np.stack([np.asarray(b, dtype=float) for b in B_list[:L]])[None]
    Xs = np.asarray(X, dtype=float)[None, :L + 1]
    Us = np.asarray(U, dtype=float).reshape(len(U), m)[None, :L]
    Qf = as_terminal_weight(alpha, n)
    qxx, qx, c0 = _extra_arrays(extra_stage_cost, X, U, L)
    dv = lambda a: None if a is None else _to_dev(a)  # noqa: E731
    return engine.riccati(
        dv(A), dv(Bm), dv(Xs), dv(Us), dv(np.asarray(xg, dtype=float).reshape(-1)),
        dv(np.atleast_1d(np.asarray(u_ref, dtype=float)).reshape(-1)), dv(Q), dv(R), dv(Qf),
        [L], [lm], mode=mode, w_stage=w_stage, wrap_idx=wrap_idx, qxx_extra=dv(qxx),
        qx_extra=dv(qx), c_extra=dv(c0), reg_max_tries=reg_max_tries, want_v=True)


def backward_pass_truncated(A_list, B_list, X, U, xg, u_ref, Q, R, alpha, T_star: int, *,
                            lm_lambda: float = 1e-3, wrap_idx=None, extra_stage_cost=None
                            ) -> Tuple[Optional[List[np.ndarray]], Optional[List[np.ndarray]], bool]:
    """Fixed-horizon iLQR backward pass -> (k_list, K_list, ok) (GPU)."""
    T = int(T_star)
    if T <= 0:
        return None, None, False
    X = np.asarray(X, dtype=float)
    U = np.asarray(U, dtype=float)
    if U.ndim == 1:
        U = U.reshape(-1, 1)
    if len(A_list) < T or len(B_list) < T or X.shape[0] < T + 1 or U.shape[0] < T:
        raise IndexError("list index out of range")
    r = _riccati_one(A_list, B_list, X, U, xg, u_ref, np.asarray(Q, float), np.asarray(R, float),
                     alpha, T, float(lm_lambda), 0, 0.0, wrap_idx, extra_stage_cost, 1)
    if int(r.status[0].item()) & _lib.ST_FAIL:
        return None, None, False
    K = r.K[0].cpu().numpy()
    k = r.k[0].cpu().numpy()
    return [k[i].copy() for i in range(T)], [K[i].copy() for i in range(T)], True


def value_expansions_and_gains_prefix(A_list, B_list, X, U, xg, u_ref, Q, R, alpha, T_bar: int,
                                      S_right: int, *, lm_lambda: float = 1e-6,
                                      w_stage: float = 0.0, wrap_idx=None,
                                      extra_stage_cost=None, reg_max_tries: int = 12):
    """One backward sweep over t in [-S_right .. T_bar] -> (Vxx, Vx, V0, K, k) (GPU)."""
    L = int(T_bar) + int(S_right)
    X = np.asarray(X, dtype=float)
    U = np.asarray(U, dtype=float)
    if U.ndim == 1:
        U = U.reshape(-1, 1)
    if len(A_list) < L or len(B_list) < L or X.shape[0] < L + 1 or U.shape[0] < L:
        raise IndexError("list index out of range")
    if L <= 0:
        n = X.shape[1]
        Qf = as_terminal_weight(alpha, n)
        from .utils import wrap_error
        eT = np.atleast_1d(wrap_error(X[0] - xg, wrap_idx)).reshape(-1)
        return [0.5 * (Qf + Qf.T)], [Qf @ eT], [0.5 * float(eT @ (Qf @ eT))], [], []
    r = _riccati_one(A_list, B_list, X, U, xg, u_ref, np.asarray(Q, float), np.asarray(R, float),
                     alpha, L, float(lm_lambda), 1, float(w_stage), wrap_idx, extra_stage_cost,
                     int(reg_max_tries))
    _raise_for(int(r.status[0].item()), "value_expansions_and_gains_prefix")
    Vxx = r.Vxx[0].cpu().numpy()
    Vx = r.Vx[0].cpu().numpy()
    V0 = r.V0[0].cpu().numpy()
    K = r.K[0].cpu().numpy()
    k = r.k[0].cpu().numpy()
    return ([Vxx[i].copy() for i in range(L + 1)], [Vx[i].copy() for i in range(L + 1)],
            [float(V0[i]) for i in range(L + 1)], [K[i].copy() for i in range(L)],
            [k[i].copy() for i in range(L)])


def bruteforce_all_Jt_backward_expansion(A_list, B_list, X, U, xg, u_ref, Q, R, alpha, w,
                                         T_max: int, *, lm_lambda: float = 1e-6, wrap_idx=None,
                                         extra_stage_cost=None) -> np.ndarray:
    """Exact quadratic-model J(T) curve: T_max independent Riccati sweeps of
    lengths 1..T_max, run as ONE launch (hop_bruteforce_jcurve, grid y = horizon)."""
    T_max = int(T_max)
    X = np.asarray(X, dtype=float)
    U = np.asarray(U, dtype=float)
    if U.ndim == 1:
        U = U.reshape(-1, 1)
    if T_max > len(A_list) or T_max > len(B_list) or T_max > len(U) or T_max + 1 > len(X):
        raise IndexError("list index out of range")
    n = X.shape[1]
    A = _to_dev(np.stack([np.asarray(a, dtype=float) for a in A_list[:T_max]])[None])
    Bm = _to_dev(np.stack([np.asarray(b, dtype=float) for b in B_list[:T_max]])[None])
    qxx, qx, c0 = _extra_arrays(extra_stage_cost, X, U, T_max)
    dv = lambda a: None if a is None else _to_dev(a)  # noqa: E731
    J, st = engine.bruteforce_jcurve(
        A, Bm, _to_dev(X[None, :T_max + 1]), _to_dev(U[None, :T_max]),
        _to_dev(np.asarray(xg, float)), _to_dev(np.atleast_1d(np.asarray(u_ref, float))),
        _to_dev(Q), _to_dev(np.atleast_2d(R)), _to_dev(as_terminal_weight(alpha, n)), T_max,
        lm_lambda=float(lm_lambda), w_stage=float(w), wrap_idx=wrap_idx, qxx_extra=dv(qxx),
        qx_extra=dv(qx), c_extra=dv(c0))
    if (st.cpu().numpy() & (_lib.ST_FAIL | _lib.ST_NONFINITE)).any():
        raise np.linalg.LinAlgError("chol_solve failed: matrix not PD after jitter")
    return J[0].cpu().numpy()
