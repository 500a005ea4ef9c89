"""Batched device API of the engine (PyTorch tensors in HBM -> HIP kernels).

``propagate`` / ``select_horizon`` are the north-star names for the batched
LFT sweep and the horizon argmin; ``riccati`` runs the gain / value passes.
All compute happens in libhop_amd.so; torch only owns memory and streams.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence

from . import _lib

_DT = {}


def _torch():
    import torch
    return torch


def _fn(base, dtype):
    torch = _torch()
    lib = _lib.load()
    if dtype == torch.float64:
        return getattr(lib, base + "_f64")
    if dtype == torch.float32:
        return getattr(lib, base + "_f32")
    raise TypeError(f"unsupported dtype {dtype} (float64 / float32)")


def _dev(t, name, dtype=None, device=None):
    torch = _torch()
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise _lib.HopError(f"{name} must live on a HIP device (got {t.device}); "
                            "the engine has no CPU path")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name}: dtype {t.dtype} != {dtype}")
    if device is not None and t.device != device:
        raise ValueError(f"{name} on {t.device}, expected {device}")
    return t.contiguous()


@dataclass
class SweepResult:
    J: "object"            # [B, n_use]
    status: "object"       # [B] int32 (HOP_ST_* bits)
    t_star: "object" = None
    j_star: "object" = None
    efg: "object" = None     # [B, n_use, 3, s, s]  (E_k, F_k, G_k)
    prefix: "object" = None  # [B, n_use, 3, s, s]  (Ebar_k, Fbar_k, Gbar_k)


def propagate(A, B, Q, R, z0, QT, *, n_use: Optional[int] = None, r_is_inverse: bool = True,
              max_tries: int = 8, t_min: Optional[int] = None, t_max: Optional[int] = None,
              return_efg: bool = False, return_prefix: bool = False, out=None) -> SweepResult:
    """Batched LFT sweep (horizon_selection.py:36-86 for every problem of a batch).

    A, Q, QT : [Bn, N, s, s]   B : [Bn, N, s, m]   z0 : [s] or [Bn, s]
    R        : R^-1 if r_is_inverse (R_inv_cached) else raw R_k, shaped
               [m, m] | [Bn or 1, m, m] | [Bn or 1, N, m, m] (per step)
    n_use    : T_use (default N).  t_min/t_max: fuse the argmin (solver.py:522).
    """
    torch = _torch()
    dt = A.dtype
    A = _dev(A, "A", dt)
    dev = A.device
    B = _dev(B, "B", dt, dev)
    Q = _dev(Q, "Q", dt, dev)
    QT = _dev(QT, "QT", dt, dev)
    R = _dev(R, "R", dt, dev)
    z0 = _dev(z0, "z0", dt, dev)
    if A.dim() != 4 or A.shape[-1] != A.shape[-2]:
        raise ValueError(f"A must be [B, N, s, s], got {tuple(A.shape)}")
    Bn, N, s, _ = A.shape
    m = B.shape[-1]
    if tuple(B.shape) != (Bn, N, s, m):
        raise ValueError(f"B must be [B, N, s, m], got {tuple(B.shape)}")
    for name, t in (("Q", Q), ("QT", QT)):
        if tuple(t.shape) != (Bn, N, s, s):
            raise ValueError(f"{name} must be {(Bn, N, s, s)}, got {tuple(t.shape)}")
    n_use = N if n_use is None else int(n_use)
    if n_use > N:
        raise IndexError(f"T_use={n_use} exceeds the {N} stages supplied")
    if R.dim() == 2:
        r_bs, r_ks = 0, 0
    elif R.dim() == 3:
        r_bs, r_ks = (0 if R.shape[0] == 1 else m * m), 0
    elif R.dim() == 4:
        if R.shape[1] < n_use:
            raise IndexError("per-step R has fewer stages than T_use")
        r_bs, r_ks = (0 if R.shape[0] == 1 else R.shape[1] * m * m), m * m
    else:
        raise ValueError("R must be 2-, 3- or 4-D")
    if tuple(R.shape[-2:]) != (m, m):
        raise ValueError(f"R blocks must be {m}x{m}")
    z_bs = 0 if z0.dim() == 1 else s
    if z0.shape[-1] != s or (z0.dim() == 2 and z0.shape[0] not in (1, Bn)):
        raise ValueError("z0 must be [s] or [B, s]")
    if z0.dim() == 2 and z0.shape[0] == 1:
        z_bs = 0
    n_eff = max(n_use, 0)
    J = torch.empty((Bn, n_eff), dtype=dt, device=dev) if out is None else out
    status = torch.zeros((Bn,), dtype=torch.int32, device=dev)
    fuse = t_max is not None
    ts = torch.empty((Bn,), dtype=torch.int32, device=dev) if fuse else None
    js = torch.empty((Bn,), dtype=dt, device=dev) if fuse else None
    efg = torch.empty((Bn, n_eff, 3, s, s), dtype=dt, device=dev) if return_efg else None
    pre = torch.empty((Bn, n_eff, 3, s, s), dtype=dt, device=dev) if return_prefix else None
    rc = _fn("hop_lft_sweep", dt)(
        _lib.ptr(A), _lib.ptr(B), _lib.ptr(Q), _lib.ptr(R), r_bs, r_ks, 1 if r_is_inverse else 0,
        _lib.ptr(QT), _lib.ptr(z0), z_bs, Bn, N, n_use, s, m, int(max_tries),
        int(t_min) if fuse else 0, int(t_max) if fuse else 0,
        _lib.ptr(J), _lib.ptr(status), _lib.ptr(ts), _lib.ptr(js), _lib.ptr(efg), _lib.ptr(pre),
        _lib.stream_handle(dev))
    _lib.check(rc)
    return SweepResult(J, status, ts, js, efg, pre)


def select_horizon(J, t_min: int, t_max: int):
    """First minimiser over J[..., t_min-1 : t_max] (+t_min) -- solver.py:522."""
    torch = _torch()
    J = _dev(J, "J")
    squeeze = J.dim() == 1
    J2 = J.reshape(1, -1) if squeeze else J
    Bn, ld = J2.shape
    ts = torch.empty((Bn,), dtype=torch.int32, device=J.device)
    js = torch.empty((Bn,), dtype=J.dtype, device=J.device)
    rc = _fn("hop_select_horizon", J.dtype)(_lib.ptr(J2), Bn, ld, int(t_min), int(t_max),
                                            _lib.ptr(ts), _lib.ptr(js),
                                            _lib.stream_handle(J.device))
    _lib.check(rc)
    return (ts[0], js[0]) if squeeze else (ts, js)


def wrap_mask(wrap_idx: Optional[Sequence[int]], n: int) -> int:
    mask = 0
    for i in (wrap_idx or []):
        i = int(i)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError(f"wrap index {i} out of range for n={n}")
        mask |= 1 << i
    return mask


@dataclass
class RiccatiResult:
    K: "object"       # [B, N, m, n]
    k: "object"       # [B, N, m]
    status: "object"  # [B] int32
    Vxx: "object" = None  # [B, N+1, n, n]
    Vx: "object" = None   # [B, N+1, n]
    V0: "object" = None   # [B, N+1]


def _bstride(t, per, name, Bn):
    """batch stride (elements) of a block that is either shared ([...]) or per problem."""
    if t.dim() == per:
        return 0
    if t.dim() == per + 1 and t.shape[0] in (1, Bn):
        return 0 if t.shape[0] == 1 else int(t[0].numel())
    raise ValueError(f"{name} has unexpected shape {tuple(t.shape)}")


def riccati(A, Bm, X, U, xg, u_ref, Q, R, Qf, horizon, lm, *, mode: int = 0,
            w_stage: float = 0.0, wrap_idx=None, qxx_extra=None, qx_extra=None, c_extra=None,
            reg_max_tries: int = 12, want_v: bool = False) -> RiccatiResult:
    """Batched Riccati pass.  mode 0: backward_pass_truncated (solver.py:156-230);
    mode 1: value_expansions_and_gains_prefix (horizon_selection.py:97-212).

    A [B,N,n,n], Bm [B,N,n,m], X [B,N+1,n], U [B,N,m]; xg/u_ref/Q/R/Qf shared or
    per problem; horizon [B] int (T* or T_bar+S_right); lm [B] or scalar.
    """
    torch = _torch()
    dt = A.dtype
    A = _dev(A, "A", dt)
    dev = A.device
    Bn, N, n, _ = A.shape
    Bm = _dev(Bm, "Bm", dt, dev)
    m = Bm.shape[-1]
    X = _dev(X, "X", dt, dev)
    U = _dev(U, "U", dt, dev)
    if tuple(X.shape) != (Bn, N + 1, n) or tuple(U.shape) != (Bn, N, m):
        raise ValueError("X must be [B, N+1, n] and U [B, N, m]")
    xg = _dev(xg, "xg", dt, dev)
    u_ref = _dev(u_ref, "u_ref", dt, dev)
    Q = _dev(Q, "Q", dt, dev)
    R = _dev(R, "R", dt, dev)
    Qf = _dev(Qf, "Qf", dt, dev)
    horizon = _dev(torch.as_tensor(horizon, device=dev).to(torch.int32).reshape(-1)
                   .expand(Bn), "horizon")
    lm = _dev(torch.as_tensor(lm, device=dev, dtype=dt).reshape(-1).expand(Bn), "lm")
    ex = [None if t is None else _dev(t, nm, dt, dev)
          for t, nm in ((qxx_extra, "qxx_extra"), (qx_extra, "qx_extra"), (c_extra, "c_extra"))]
    K = torch.zeros((Bn, N, m, n), dtype=dt, device=dev)
    k = torch.zeros((Bn, N, m), dtype=dt, device=dev)
    status = torch.zeros((Bn,), dtype=torch.int32, device=dev)
    want = want_v or mode == 1
    Vxx = torch.zeros((Bn, N + 1, n, n), dtype=dt, device=dev) if want else None
    Vx = torch.zeros((Bn, N + 1, n), dtype=dt, device=dev) if want else None
    V0 = torch.zeros((Bn, N + 1), dtype=dt, device=dev) if want else None
    rc = _fn("hop_riccati", dt)(
        _lib.ptr(A), _lib.ptr(Bm), _lib.ptr(X), _lib.ptr(U),
        _lib.ptr(xg), _bstride(xg, 1, "xg", Bn), _lib.ptr(u_ref), _bstride(u_ref, 1, "u_ref", Bn),
        _lib.ptr(Q), _bstride(Q, 2, "Q", Bn), _lib.ptr(R), _bstride(R, 2, "R", Bn),
        _lib.ptr(Qf), _bstride(Qf, 2, "Qf", Bn),
        _lib.ptr(ex[0]), _lib.ptr(ex[1]), _lib.ptr(ex[2]), _lib.ptr(horizon), _lib.ptr(lm),
        float(w_stage), wrap_mask(wrap_idx, n), int(mode), int(reg_max_tries), Bn, N, n, m,
        _lib.ptr(K), _lib.ptr(k), _lib.ptr(Vxx), _lib.ptr(Vx), _lib.ptr(V0), _lib.ptr(status),
        _lib.stream_handle(dev))
    _lib.check(rc)
    return RiccatiResult(K, k, status, Vxx, Vx, V0)
