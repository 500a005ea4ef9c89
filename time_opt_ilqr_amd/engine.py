"""Batched device API of the engine (PyTorch tensors in HBM -> HIP kernels).

``propagate`` / ``select_horizon`` are the north-star names for the batched
LFT sweep and the horizon argmin; ``riccati`` runs the gain / value passes.
All compute happens in libhop_amd.so; torch only owns memory and streams.
"""
from __future__ import annotations

import numbers
import struct
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


@dataclass
class Tile64:
    """A block tensor in the tile64 layout of include/hop.h: ``data`` is
    [ceil(batch/64), N, rows*cols, 64] (element e of step k of problem b at
    data[b // 64, k, e, b % 64]).  The native layout of the s <= 5 sweep: a wave
    of 64 problems streams each block of a step as one contiguous span."""
    data: "object"
    batch: int
    rows: int
    cols: int

    @property
    def shape(self):
        return (self.batch, int(self.data.shape[1]), self.rows, self.cols)

    def check(self, name="tile64"):
        """The data tensor must be exactly [ceil(batch/64), N, rows*cols, 64]: the
        kernels read whole tiles."""
        d = self.data
        want = ((self.batch + 63) // 64, int(d.shape[1]) if d.dim() == 4 else -1,
                self.rows * self.cols, 64)
        if d.dim() != 4 or tuple(d.shape) != want or not d.is_contiguous():
            raise ValueError(f"{name}: tile64 data must be a contiguous {want} tensor, got "
                             f"{tuple(d.shape)}")
        return self

    @property
    def dtype(self):
        return self.data.dtype

    @property
    def device(self):
        return self.data.device


def to_tile64(x) -> Tile64:
    """[B, N, r, c] batch-major device blocks -> Tile64 (one hop_tile64 copy; padding
    slots of the last tile are 0)."""
    torch = _torch()
    x = _dev(x, "x")
    if x.dim() != 4:
        raise ValueError(f"blocks must be [B, N, r, c], got {tuple(x.shape)}")
    Bn, N, r, c = (int(v) for v in x.shape)
    out = torch.empty(((Bn + 63) // 64, N, r * c, 64), dtype=x.dtype, device=x.device)
    _lib.check(_fn("hop_tile64", x.dtype)(_lib.ptr(x), _lib.ptr(out), Bn, N, r * c, 0,
                                          _lib.stream_handle(x.device)))
    return Tile64(out, Bn, r, c)


def from_tile64(t: Tile64):
    """Tile64 -> [B, N, r, c] batch-major blocks (hop_tile64 inverse)."""
    torch = _torch()
    data = _dev(t.check().data, "tile64 data")
    out = torch.empty(t.shape, dtype=data.dtype, device=data.device)
    _lib.check(_fn("hop_tile64", data.dtype)(_lib.ptr(data), _lib.ptr(out), t.batch,
                                             int(data.shape[1]), t.rows * t.cols, 1,
                                             _lib.stream_handle(data.device)))
    return out


def _propagate_tile64(A, B, Q, R, z0, QT, n_use, r_is_inverse, max_tries, t_min, t_max, out):
    torch = _torch()
    for name, t in (("A", A), ("B", B), ("Q", Q), ("QT", QT)):
        if not isinstance(t, Tile64):
            raise TypeError(f"{name}: tile64 sweep needs every block tensor as Tile64")
    Bn, N, s, _ = A.shape
    m = B.cols
    dt, dev = A.dtype, A.device
    for name, t, cols in (("A", A, s), ("B", B, m), ("Q", Q, s), ("QT", QT, s)):
        t.check(name)
        if t.shape != (Bn, N, s, cols) or t.dtype != dt or t.device != dev:
            raise ValueError(f"{name}: tile64 blocks {t.shape} do not match A {A.shape}")
        _dev(t.data, name, dt, dev)
    R = _dev(R, "R", dt, dev)
    z0 = _dev(z0, "z0", dt, dev)
    n_use = N if n_use is None else int(n_use)
    if n_use > N:
        raise IndexError(f"T_use={n_use} exceeds the {N} stages supplied")
    if R.dim() == 2:
        r_bs = 0
    elif R.dim() == 3:
        r_bs = 0 if R.shape[0] == 1 else m * m
    else:
        raise ValueError("tile64 sweep: R must be [m, m] or [B or 1, m, m] (no per-step R)")
    if tuple(R.shape[-2:]) != (m, m):
        raise ValueError(f"R blocks must be {m}x{m}")
    if z0.shape[-1] != s or (z0.dim() == 2 and z0.shape[0] not in (1, Bn)):
        raise ValueError("z0 must be [s] or [B, s]")
    z_bs = 0 if z0.dim() == 1 or z0.shape[0] == 1 else s
    n_eff = max(n_use, 0)
    J = torch.empty((Bn, n_eff), dtype=dt, device=dev) if out is None else out
    status = (torch.empty if n_eff > 0 else torch.zeros)((Bn,), dtype=torch.int32, device=dev)
    fuse = t_max is not None
    ts = torch.empty((Bn,), dtype=torch.int32, device=dev) if fuse else None
    js = torch.empty((Bn,), dtype=dt, device=dev) if fuse else None
    rc = _fn("hop_lft_sweep_tile64", dt)(
        _lib.ptr(A.data), _lib.ptr(B.data), _lib.ptr(Q.data), _lib.ptr(R), r_bs,
        1 if r_is_inverse else 0, _lib.ptr(QT.data), _lib.ptr(z0), z_bs, Bn, N, n_use, s, m,
        int(max_tries), int(t_min) if fuse else 0, int(t_max) if fuse else 0, _lib.ptr(J),
        _lib.ptr(status), _lib.ptr(ts), _lib.ptr(js), _lib.stream_handle(dev))
    _lib.check(rc)
    return SweepResult(J, status, ts, js)


def propagate(A, B, Q, R, z0, QT, *, n_use: Optional[int] = None, r_is_inverse: bool = True,
              max_tries: int = 8, t_min: Optional[int] = None, t_max: Optional[int] = None,
              return_efg: bool = False, return_prefix: bool = False, out=None) -> SweepResult:
    """Batched LFT sweep (horizon_selection.py:36-86 for every problem of a batch).

    A, Q, QT : [Bn, N, s, s]   B : [Bn, N, s, m]   z0 : [s] or [Bn, s]
    R        : R^-1 if r_is_inverse (R_inv_cached) else raw R_k, shaped
               [m, m] | [Bn or 1, m, m] | [Bn or 1, N, m, m] (per step)
    n_use    : T_use (default N).  t_min/t_max: fuse the argmin (solver.py:522).
    A, B, Q, QT may instead all be ``Tile64`` (s <= 5 shapes; see to_tile64).
    """
    torch = _torch()
    if isinstance(A, Tile64):
        if return_efg or return_prefix:
            raise ValueError("tile64 sweep: no debug outputs")
        return _propagate_tile64(A, B, Q, R, z0, QT, n_use, r_is_inverse, max_tries, t_min,
                                 t_max, out)
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
    # every sweep kernel writes the status of each problem it runs; only the
    # n_use <= 0 call launches nothing (and must report 0)
    status = (torch.empty if n_eff > 0 else torch.zeros)((Bn,), dtype=torch.int32, device=dev)
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


@dataclass
class MixedPlan:
    """Batch slots of each shape group of a mixed batch (see propagate_groups)."""
    slots: list          # per group: int64 device tensor of batch slots
    batch: int


def mixed_plan(order, n_groups: int, device) -> MixedPlan:
    """order[i] = group of batch slot i; slot i takes the next unused member of
    its group (the convention of packing.pack_mixed)."""
    torch = _torch()
    order = torch.as_tensor(order, dtype=torch.int64).cpu().reshape(-1)
    if order.numel() and (int(order.min()) < 0 or int(order.max()) >= n_groups):
        raise ValueError(f"mixed_plan: group ids must lie in [0, {n_groups}) "
                         f"(got {int(order.min())}..{int(order.max())})")
    slots = [torch.nonzero(order == g).reshape(-1).to(device) for g in range(n_groups)]
    if sum(int(sl.numel()) for sl in slots) != order.numel():  # every slot in one group
        raise ValueError("mixed_plan: the groups' slots do not cover the batch")
    return MixedPlan(slots, int(order.numel()))


_SIDE = {}


def _side_stream(device):
    torch = _torch()
    if device not in _SIDE:
        _SIDE[device] = torch.cuda.Stream(device=device)
    return _SIDE[device]


def propagate_groups(groups, plan: MixedPlan, *, t_min: Optional[int] = None,
                     t_max: Optional[int] = None, max_tries: int = 8) -> SweepResult:
    """A mixed batch swept by shape bucket: config 5 without the
    padding to s = 13.  groups[g] = (A, B, Q, R_inv, z0, QT) of group g's members
    at their TRUE shape, in member order (A/B/Q/QT may be Tile64 for s <= 5);
    plan.slots[g] = their batch slots.  Each group runs its own kernel -- the
    s <= 5 groups on a side stream, beside the s = 13 launch -- and J [B, N],
    status, T*, J* come back in batch order.  J equals that of the padded launch
    (packing.pack_mixed: the block-decoupled embedding leaves it unchanged) up to
    rounding; every group needs the same N."""
    torch = _torch()
    if len(groups) != len(plan.slots):
        raise ValueError("one slot list per group")
    first = groups[0][0]
    dev, dt = first.device, first.dtype
    N = int(first.shape[1])
    fuse = t_max is not None
    Bn = plan.batch
    J = torch.empty((Bn, N), dtype=dt, device=dev)
    status = torch.empty((Bn,), dtype=torch.int32, device=dev)
    ts = torch.empty((Bn,), dtype=torch.int32, device=dev) if fuse else None
    js = torch.empty((Bn,), dtype=dt, device=dev) if fuse else None
    main = torch.cuda.current_stream(dev)
    side = _side_stream(dev)
    side.wait_stream(main)
    for grp, slots in zip(groups, plan.slots):
        A = grp[0]
        if int(A.shape[1]) != N or A.dtype != dt:
            raise ValueError("every group needs the same N and dtype")
        if int(A.shape[0]) < int(slots.numel()):
            raise ValueError("a group has fewer members than batch slots")
        s = int(A.shape[2])
        with torch.cuda.stream(side if s <= 5 else main):
            r = propagate(*grp, t_min=t_min, t_max=t_max, max_tries=max_tries)
            cnt = int(slots.numel())
            J.index_copy_(0, slots, r.J[:cnt])
            status.index_copy_(0, slots, r.status[:cnt])
            if fuse:
                ts.index_copy_(0, slots, r.t_star[:cnt])
                js.index_copy_(0, slots, r.j_star[:cnt])
    main.wait_stream(side)
    for t in (J, status, ts, js):
        if t is not None:
            t.record_stream(side)
    return SweepResult(J, status, ts, js)


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


_CONST = {}


def _const_fill(v, n, dtype, dev):
    """A read-only [n] device tensor filled with the scalar v, made once and reused:
    a per-call torch.full is a fill kernel on the stream every step (the select +
    gains step carried two, 9 us of its 459, tools/launch_gaps.py).  Keyed by the
    value's bits (so -0.0 and 0.0, NaN payloads stay distinct).  During a graph
    capture a plain fill is returned (a cached tensor would come from the capture's
    pool); a new entry is synchronised once so another stream can read it at once."""
    torch = _torch()
    val = float(v) if dtype.is_floating_point else int(v)
    if torch.cuda.is_current_stream_capturing():
        return torch.full((n,), val, dtype=dtype, device=dev)
    key = (struct.pack("<d", val) if dtype.is_floating_point else val, n, dtype, str(dev))
    t = _CONST.get(key)
    if t is None:
        if len(_CONST) >= 64:
            _CONST.clear()
        t = torch.full((n,), val, dtype=dtype, device=dev)
        torch.cuda.current_stream(dev).synchronize()
        _CONST[key] = t
    return t


def _per_problem(v, Bn, dtype, dev, name):
    """[Bn] device tensor from a scalar (a cached device fill, _const_fill: no
    host-device copy that would stall the launch queue), a tensor, or an array."""
    torch = _torch()
    if isinstance(v, numbers.Real) and not isinstance(v, bool):
        return _const_fill(v, Bn, dtype, dev)
    t = v if isinstance(v, torch.Tensor) else torch.as_tensor(v)
    return _dev(t.to(device=dev, dtype=dtype).reshape(-1).expand(Bn), name)


def _scalar_or_vec(v, dtype, dev, name):
    """[1] (a device fill) or [n] device tensor."""
    torch = _torch()
    if isinstance(v, numbers.Real) and not isinstance(v, bool):
        return _const_fill(v, 1, dtype, dev)
    t = v if isinstance(v, torch.Tensor) else torch.as_tensor(v)
    return _dev(t.to(device=dev, dtype=dtype).reshape(-1), name)


def riccati(A, Bm, X, U, xg, u_ref, Q, R, Qf, horizon, lm, *, mode: int = 0,
            w_stage: float = 0.0, wrap_idx=None, qxx_extra=None, qx_extra=None, c_extra=None,
            reg_max_tries: int = 12, want_v: bool = False, legacy: bool = False) -> RiccatiResult:
    """Batched Riccati pass.  mode 0: backward_pass_truncated (solver.py:156-230);
    mode 1: value_expansions_and_gains_prefix (horizon_selection.py:97-212).

    A [B,N,n,n], Bm [B,N,n,m], X [B,N+1,n], U [B,N,m]; xg/u_ref/Q/R/Qf shared or
    per problem; horizon [B] int (T* or T_bar+S_right); lm [B] or scalar.
    legacy=True: the legacy twin's passes (ilqr_propagator.py:375-400 / 237-287,
    hop_riccati_legacy_f64): mode 1 solves with its chol_solve (4 jitters, then
    lstsq, ST_LU); mode 0 fails a row at its no-jitter Cholesky gate first, so its
    solves never reach lstsq; no finiteness checks, Qf = alpha I; fp64, no extra
    stage cost.
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
    horizon = _per_problem(horizon, Bn, torch.int32, dev, "horizon")
    lm = _per_problem(lm, Bn, dt, dev, "lm")
    ex = [None if t is None else _dev(t, nm, dt, dev)
          for t, nm in ((qxx_extra, "qxx_extra"), (qx_extra, "qx_extra"), (c_extra, "c_extra"))]
    # outputs are written for steps < horizon[b] (Vxx/Vx/V0 up to horizon[b]) of
    # problems that do not fail; the rest is left unwritten (the reference returns
    # lists of length T*), so no fill kernel runs -- in mode 1 a zero fill of Vxx
    # alone costs about a third of the pass
    K = torch.empty((Bn, N, m, n), dtype=dt, device=dev)
    k = torch.empty((Bn, N, m), dtype=dt, device=dev)
    status = torch.empty((Bn,), dtype=torch.int32, device=dev)
    want = want_v or mode == 1
    Vxx = torch.empty((Bn, N + 1, n, n), dtype=dt, device=dev) if want else None
    Vx = torch.empty((Bn, N + 1, n), dtype=dt, device=dev) if want else None
    V0 = torch.empty((Bn, N + 1), dtype=dt, device=dev) if want else None
    ins = [_lib.ptr(A), _lib.ptr(Bm), _lib.ptr(X), _lib.ptr(U),
           _lib.ptr(xg), _bstride(xg, 1, "xg", Bn), _lib.ptr(u_ref), _bstride(u_ref, 1, "u_ref", Bn),
           _lib.ptr(Q), _bstride(Q, 2, "Q", Bn), _lib.ptr(R), _bstride(R, 2, "R", Bn),
           _lib.ptr(Qf), _bstride(Qf, 2, "Qf", Bn)]
    outs = [_lib.ptr(K), _lib.ptr(k), _lib.ptr(Vxx), _lib.ptr(Vx), _lib.ptr(V0), _lib.ptr(status),
            _lib.stream_handle(dev)]
    if legacy:
        if dt != torch.float64 or any(t is not None for t in ex):
            raise ValueError("legacy passes: fp64 and no extra stage cost (ilqr_propagator.py)")
        rc = _lib.load().hop_riccati_legacy_f64(
            *ins, _lib.ptr(horizon), _lib.ptr(lm), float(w_stage), wrap_mask(wrap_idx, n),
            int(mode), Bn, N, n, m, *outs)
    else:
        rc = _fn("hop_riccati", dt)(
            *ins, _lib.ptr(ex[0]), _lib.ptr(ex[1]), _lib.ptr(ex[2]), _lib.ptr(horizon),
            _lib.ptr(lm), float(w_stage), wrap_mask(wrap_idx, n), int(mode), int(reg_max_tries),
            Bn, N, n, m, *outs)
    _lib.check(rc)
    return RiccatiResult(K, k, status, Vxx, Vx, V0)


def bruteforce_jcurve(A, Bm, X, U, xg, u_ref, Q, R, Qf, t_max: int, *, lm_lambda: float = 1e-6,
                      w_stage: float = 0.0, wrap_idx=None, qxx_extra=None, qx_extra=None,
                      c_extra=None, legacy: bool = False):
    """bruteforce_all_Jt_backward_expansion (solver.py:293-358) for a batch: J [B, t_max]
    with J[:, T-1] = V_0 of the length-T sweep, and the per-horizon status [B, t_max]
    (ST_FAIL / ST_NONFINITE where the reference raises).  All t_max sweeps of every
    problem run in one launch (hop_bruteforce_jcurve_*).  Inputs as riccati().
    legacy=True: the legacy twin's brute force (ilqr_propagator.py:426-454,
    hop_bruteforce_jcurve_legacy_f64): chol_solve with 4 jitters then lstsq (ST_LU
    where it ran), Qf = alpha I; fp64, no extra stage cost."""
    torch = _torch()
    dt = A.dtype
    A = _dev(A, "A", dt)
    dev = A.device
    Bn, N, n, _ = A.shape
    Bm = _dev(Bm, "Bm", dt, dev)
    m = Bm.shape[-1]
    X = _dev(X, "X", dt, dev)
    U = _dev(U, "U", dt, dev)
    if (tuple(Bm.shape) != (Bn, N, n, m) or tuple(X.shape) != (Bn, N + 1, n)
            or tuple(U.shape) != (Bn, N, m)):
        raise ValueError("need A [B, N, n, n], Bm [B, N, n, m], X [B, N+1, n], U [B, N, m]")
    xg = _dev(xg, "xg", dt, dev)
    u_ref = _dev(u_ref, "u_ref", dt, dev)
    Q = _dev(Q, "Q", dt, dev)
    R = _dev(R, "R", dt, dev)
    Qf = _dev(Qf, "Qf", dt, dev)
    ex = [None if t is None else _dev(t, nm, dt, dev)
          for t, nm in ((qxx_extra, "qxx_extra"), (qx_extra, "qx_extra"), (c_extra, "c_extra"))]
    for t, shp in zip(ex, ((Bn, N, n, n), (Bn, N, n), (Bn, N))):
        if t is not None and tuple(t.shape) != shp:
            raise ValueError(f"extra stage-cost term must be {list(shp)}")
    t_max = int(t_max)
    J = torch.empty((Bn, t_max), dtype=dt, device=dev)
    status = torch.empty((Bn, t_max), dtype=torch.int32, device=dev)
    if legacy:
        if dt != torch.float64 or any(t is not None for t in ex):
            raise ValueError("legacy passes: fp64 and no extra stage cost (ilqr_propagator.py)")
        rc = _lib.load().hop_bruteforce_jcurve_legacy_f64(
            _lib.ptr(A), _lib.ptr(Bm), _lib.ptr(X), _lib.ptr(U),
            _lib.ptr(xg), _bstride(xg, 1, "xg", Bn), _lib.ptr(u_ref),
            _bstride(u_ref, 1, "u_ref", Bn), _lib.ptr(Q), _bstride(Q, 2, "Q", Bn), _lib.ptr(R),
            _bstride(R, 2, "R", Bn), _lib.ptr(Qf), _bstride(Qf, 2, "Qf", Bn), float(lm_lambda),
            float(w_stage), wrap_mask(wrap_idx, n), Bn, N, n, m, t_max, _lib.ptr(J),
            _lib.ptr(status), _lib.stream_handle(dev))
        _lib.check(rc)
        return J, status
    rc = _fn("hop_bruteforce_jcurve", dt)(
        _lib.ptr(A), _lib.ptr(Bm), _lib.ptr(X), _lib.ptr(U),
        _lib.ptr(xg), _bstride(xg, 1, "xg", Bn), _lib.ptr(u_ref), _bstride(u_ref, 1, "u_ref", Bn),
        _lib.ptr(Q), _bstride(Q, 2, "Q", Bn), _lib.ptr(R), _bstride(R, 2, "R", Bn),
        _lib.ptr(Qf), _bstride(Qf, 2, "Qf", Bn),
        _lib.ptr(ex[0]), _lib.ptr(ex[1]), _lib.ptr(ex[2]), float(lm_lambda), float(w_stage),
        wrap_mask(wrap_idx, n), Bn, N, n, m, t_max, _lib.ptr(J), _lib.ptr(status),
        _lib.stream_handle(dev))
    _lib.check(rc)
    return J, status


# ---------------------------------------------------------------------------
# trajectory form: augmented.py:10-87 on the device (+ the fused sweep)
# ---------------------------------------------------------------------------
@dataclass
class AugmentedBlocks:
    A: "object"   # [B, N, s, s]
    B: "object"   # [B, N, s, m]
    Q: "object"   # [B, N, s, s]
    QT: "object"  # [B, N, s, s]  (QT[t-1] <-> horizon t)
    z0: "object"  # [s] = e_s


def _traj_args(A, Bm, a_res, X, U, xg, u_ref, Q, P, w, wrap_idx, q_reg, rho_reg,
               qxx_extra, qx_extra, c_extra):
    """Validate the trajectory-form inputs; returns (args, dims, keepalive)."""
    torch = _torch()
    dt = A.dtype
    A = _dev(A, "A", dt)
    dev = A.device
    if A.dim() != 4 or A.shape[-1] != A.shape[-2]:
        raise ValueError(f"A must be [B, N, n, n], got {tuple(A.shape)}")
    Bn, N, n, _ = A.shape
    Bm = _dev(Bm, "Bm", dt, dev)
    m = Bm.shape[-1]
    if tuple(Bm.shape) != (Bn, N, n, m):
        raise ValueError(f"Bm must be [B, N, n, m], got {tuple(Bm.shape)}")
    a_res = _dev(a_res, "a_res", dt, dev)
    X = _dev(X, "X", dt, dev)
    U = _dev(U, "U", dt, dev)
    if tuple(a_res.shape) != (Bn, N, n):
        raise ValueError("a_res must be [B, N, n]")
    if tuple(X.shape) != (Bn, N + 1, n) or tuple(U.shape) != (Bn, N, m):
        raise ValueError("X must be [B, N+1, n] and U [B, N, m]")
    xg = _dev(xg, "xg", dt, dev)
    u_ref = _dev(u_ref, "u_ref", dt, dev)
    Q = _dev(Q, "Q", dt, dev)
    P = _dev(P, "P", dt, dev)
    w = _scalar_or_vec(w, dt, dev, "w")
    if w.numel() not in (1, Bn):
        raise ValueError("w must be a scalar or [B]")
    ex = [None if t is None else _dev(t, nm, dt, dev)
          for t, nm in ((qxx_extra, "qxx_extra"), (qx_extra, "qx_extra"), (c_extra, "c_extra"))]
    if ex[0] is not None and tuple(ex[0].shape) != (Bn, N, n, n):
        raise ValueError("qxx_extra must be [B, N, n, n]")
    if ex[1] is not None and tuple(ex[1].shape) != (Bn, N, n):
        raise ValueError("qx_extra must be [B, N, n]")
    if ex[2] is not None and tuple(ex[2].shape) != (Bn, N):
        raise ValueError("c_extra must be [B, N]")
    args = [_lib.ptr(A), _lib.ptr(Bm), _lib.ptr(a_res), _lib.ptr(X), _lib.ptr(U),
            _lib.ptr(xg), _bstride(xg, 1, "xg", Bn), _lib.ptr(u_ref),
            _bstride(u_ref, 1, "u_ref", Bn), _lib.ptr(Q), _bstride(Q, 2, "Q", Bn),
            _lib.ptr(P), _bstride(P, 2, "P", Bn), _lib.ptr(w), 0 if w.numel() == 1 else 1,
            _lib.ptr(ex[0]), _lib.ptr(ex[1]), _lib.ptr(ex[2]), wrap_mask(wrap_idx, n),
            float(q_reg), float(rho_reg)]
    keep = (A, Bm, a_res, X, U, xg, u_ref, Q, P, w, ex)
    return args, (Bn, N, n, m, dt, dev, any(t is not None for t in ex)), keep


def augment(A, Bm, a_res, X, U, xg, u_ref, Q, P, w, *, wrap_idx=None,
            n_build: Optional[int] = None, q_reg: float = 1e-9, rho_reg: float = 1e-12,
            qxx_extra=None, qx_extra=None, c_extra=None) -> AugmentedBlocks:
    """Batched build_augmented_sequence_QR + build_terminal_aug_list (augmented.py:10-87).

    A [B,N,n,n], Bm [B,N,n,m], a_res [B,N,n] (= F(x_k,u_k) - x_{k+1}), X [B,N+1,n],
    U [B,N,m]; xg/u_ref/Q/P shared or per problem (P = _sym(as_terminal_weight(alpha)));
    w scalar or [B].  Returns the blocks of steps 0..n_build-1 (default N).
    """
    torch = _torch()
    args, (Bn, N, n, m, dt, dev, _), keep = _traj_args(
        A, Bm, a_res, X, U, xg, u_ref, Q, P, w, wrap_idx, q_reg, rho_reg, qxx_extra, qx_extra,
        c_extra)
    nb = N if n_build is None else int(n_build)
    if nb > N:
        raise IndexError(f"n_build={nb} exceeds the {N} stages supplied")
    s = n + 1
    out = AugmentedBlocks(torch.empty((Bn, nb, s, s), dtype=dt, device=dev),
                          torch.empty((Bn, nb, s, m), dtype=dt, device=dev),
                          torch.empty((Bn, nb, s, s), dtype=dt, device=dev),
                          torch.empty((Bn, nb, s, s), dtype=dt, device=dev),
                          torch.empty((s,), dtype=dt, device=dev))
    rc = _fn("hop_augment", dt)(*args, Bn, N, nb, n, m, _lib.ptr(out.A), _lib.ptr(out.B),
                                _lib.ptr(out.Q), _lib.ptr(out.QT), _lib.ptr(out.z0),
                                _lib.stream_handle(dev))
    _lib.check(rc)
    del keep
    return out


def propagate_traj(A, Bm, a_res, X, U, xg, u_ref, Q, R_inv, P, w, *, wrap_idx=None,
                   n_use: Optional[int] = None, t_min: Optional[int] = None,
                   t_max: Optional[int] = None, max_tries: int = 8, q_reg: float = 1e-9,
                   rho_reg: float = 1e-12, qxx_extra=None, qx_extra=None,
                   c_extra=None) -> SweepResult:
    """The select block of solver.py:514-522 for a batch: augmented builders +
    propagator_all_Jt_aug (+ argmin when t_max is given), from trajectory-form
    inputs (see ``augment``).  R_inv = chol_inv(R): [m, m] or [B, m, m].
    For s = 13, m = 4, fp64 (no extras) the blocks are built inside the sweep
    and never written to HBM; otherwise they go through a workspace.
    """
    torch = _torch()
    if isinstance(A, Tile64):
        if any(t is not None for t in (qxx_extra, qx_extra, c_extra)):
            raise ValueError("tile64 trajectory form: no extra_stage_cost")
        return _propagate_traj_tile64(A, Bm, a_res, X, U, xg, u_ref, Q, R_inv, P, w, wrap_idx,
                                      n_use, t_min, t_max, max_tries, q_reg, rho_reg)
    args, (Bn, N, n, m, dt, dev, has_extra), keep = _traj_args(
        A, Bm, a_res, X, U, xg, u_ref, Q, P, w, wrap_idx, q_reg, rho_reg, qxx_extra, qx_extra,
        c_extra)
    R_inv = _dev(R_inv, "R_inv", dt, dev)
    if tuple(R_inv.shape[-2:]) != (m, m):
        raise ValueError(f"R_inv blocks must be {m}x{m}")
    r_bs = _bstride(R_inv, 2, "R_inv", Bn)
    n_use = N if n_use is None else int(n_use)
    if n_use > N:
        raise IndexError(f"T_use={n_use} exceeds the {N} stages supplied")
    n_eff = max(n_use, 0)
    J = torch.empty((Bn, n_eff), dtype=dt, device=dev)
    # every sweep kernel writes the status of each problem it runs
    status = (torch.empty if n_eff > 0 else torch.zeros)((Bn,), dtype=torch.int32, device=dev)
    fuse = t_max is not None
    ts = torch.empty((Bn,), dtype=torch.int32, device=dev) if fuse else None
    js = torch.empty((Bn,), dtype=dt, device=dev) if fuse else None
    lib = _lib.load()
    ws_bytes = int(lib.hop_lft_sweep_traj_workspace_bytes(Bn, n_eff, n, m, A.element_size(),
                                                          1 if has_extra else 0))
    ws = torch.empty((ws_bytes + 256,), dtype=torch.uint8, device=dev) if ws_bytes else None
    ws_ptr = None
    if ws is not None:  # 256-B aligned view
        off = (-ws.data_ptr()) % 256
        ws_ptr = _lib.C.c_void_p(ws.data_ptr() + off)
    rc = _fn("hop_lft_sweep_traj", dt)(
        *args, _lib.ptr(R_inv), r_bs, Bn, N, n_use, n, m, int(max_tries),
        int(t_min) if fuse else 0, int(t_max) if fuse else 0, _lib.ptr(J), _lib.ptr(status),
        _lib.ptr(ts), _lib.ptr(js), ws_ptr, ws_bytes, _lib.stream_handle(dev))
    _lib.check(rc)
    if ws is not None:  # keep the workspace alive until the sweep has consumed it
        ws.record_stream(torch.cuda.current_stream(dev))
    del keep
    return SweepResult(J, status, ts, js)


def _propagate_traj_tile64(A, Bm, a_res, X, U, xg, u_ref, Q, R_inv, P, w, wrap_idx, n_use,
                           t_min, t_max, max_tries, q_reg, rho_reg) -> SweepResult:
    """propagate_traj on the raw linearisation in the tile64 layout (every one of A,
    Bm, a_res, X, U a Tile64, as linearize(..., tile64=True) returns them):
    hop_lft_sweep_traj_tile64_*, small-s shapes."""
    torch = _torch()
    for name, t in (("A", A), ("Bm", Bm), ("a_res", a_res), ("X", X), ("U", U)):
        if not isinstance(t, Tile64):
            raise TypeError(f"{name}: the tile64 trajectory form needs every raw array as Tile64")
    Bn, N, n, _ = A.shape
    m = Bm.cols
    dt, dev = A.dtype, A.device
    for name, t, steps, r, c in (("A", A, N, n, n), ("Bm", Bm, N, n, m), ("a_res", a_res, N, n, 1),
                                 ("X", X, N + 1, n, 1), ("U", U, N, m, 1)):
        t.check(name)
        if t.batch != Bn or t.shape[1] != steps or t.rows * t.cols != r * c or t.dtype != dt \
                or t.device != dev:
            raise ValueError(f"{name}: tile64 {t.shape} does not match A {A.shape}")
    xg, u_ref, Q, P = (_dev(v, nm, dt, dev) for v, nm in ((xg, "xg"), (u_ref, "u_ref"), (Q, "Q"),
                                                           (P, "P")))
    w = _scalar_or_vec(w, dt, dev, "w")
    if w.numel() not in (1, Bn):
        raise ValueError("w must be a scalar or [B]")
    R_inv = _dev(R_inv, "R_inv", dt, dev)
    if tuple(R_inv.shape[-2:]) != (m, m):
        raise ValueError(f"R_inv blocks must be {m}x{m}")
    n_use = N if n_use is None else int(n_use)
    if n_use > N:
        raise IndexError(f"T_use={n_use} exceeds the {N} stages supplied")
    n_eff = max(n_use, 0)
    J = torch.empty((Bn, n_eff), dtype=dt, device=dev)
    status = (torch.empty if n_eff > 0 else torch.zeros)((Bn,), dtype=torch.int32, device=dev)
    fuse = t_max is not None
    ts = torch.empty((Bn,), dtype=torch.int32, device=dev) if fuse else None
    js = torch.empty((Bn,), dtype=dt, device=dev) if fuse else None
    rc = _fn("hop_lft_sweep_traj_tile64", dt)(
        _lib.ptr(A.data), _lib.ptr(Bm.data), _lib.ptr(a_res.data), _lib.ptr(X.data),
        _lib.ptr(U.data), _lib.ptr(xg), _bstride(xg, 1, "xg", Bn), _lib.ptr(u_ref),
        _bstride(u_ref, 1, "u_ref", Bn), _lib.ptr(Q), _bstride(Q, 2, "Q", Bn), _lib.ptr(P),
        _bstride(P, 2, "P", Bn), _lib.ptr(w), 0 if w.numel() == 1 else 1, wrap_mask(wrap_idx, n),
        float(q_reg), float(rho_reg), _lib.ptr(R_inv), _bstride(R_inv, 2, "R_inv", Bn), Bn, N,
        n_use, n, m, int(max_tries), int(t_min) if fuse else 0, int(t_max) if fuse else 0,
        _lib.ptr(J), _lib.ptr(status), _lib.ptr(ts), _lib.ptr(js), _lib.stream_handle(dev))
    _lib.check(rc)
    return SweepResult(J, status, ts, js)


# ---- batched dynamics + finite-difference linearisation

SYSTEM_IDS = {"double_integrator": 0, "di": 0, "cartpole": 1, "quadrotor": 2, "pointmass": 3,
              "segway": 4}


def system_dims(system) -> tuple:
    """(n, m) of a system id or name (hop_system_dims)."""
    sid = system_id(system)
    n, m = _lib.C.c_int32(), _lib.C.c_int32()
    _lib.check(_lib.load().hop_system_dims(sid, _lib.C.byref(n), _lib.C.byref(m)))
    return n.value, m.value


def system_id(system) -> int:
    if isinstance(system, str):
        if system not in SYSTEM_IDS:
            raise ValueError(f"unknown system {system!r} (one of {sorted(SYSTEM_IDS)})")
        return SYSTEM_IDS[system]
    sid = getattr(system, "system_id", system)
    if not isinstance(sid, int) or not 0 <= sid < 5:
        raise ValueError(f"unknown system id {system!r}")
    return sid


@dataclass
class Linearization:
    A: "object"       # [B, N, n, n]
    B: "object"       # [B, N, n, m]
    a_res: "object"   # [B, N, n]  F(x_k, u_k) - x_{k+1}
    Fx: "object" = None  # [B, N, n] F(x_k, u_k) (want_fx=True)
    X: "object" = None   # tile64=True: the trajectory's x_k (k <= n_use) as Tile64
    U: "object" = None   # tile64=True: u_k (k < n_use) as Tile64
    n_use: Optional[int] = None  # steps written (the rest of the tile64 arrays are zero)


def linearize(system, X, U, dt: float, *, central: bool = False, n_use: Optional[int] = None,
              epsx: float = 1e-5, epsu: float = 1e-5, relx: float = 1e-6, relu: float = 1e-6,
              want_fx: bool = False, tile64: bool = False,
              tile64_dtype=None) -> Linearization:
    """Batched linearize_{forward,central}_diff_traj + compute_affine_residuals
    (linearization.py:177-270) for X [B, N+1, n], U [B, N, m] (fp64, on the
    device).  Steps k < n_use (default N) are written; A / B / a_res come out in
    the layout augment / propagate_traj / riccati read.
    tile64=True: A, B, a_res and the trajectory X, U come out as Tile64 (of
    tile64_dtype, default fp64; computed in fp64) -- the layout the small-s
    trajectory-form select streams (propagate_traj on Tile64 inputs)."""
    torch = _torch()
    X = _dev(X, "X", torch.float64)
    U = _dev(U, "U", torch.float64, X.device)
    if X.dim() == 2:  # one problem [N+1, n]: a batch of one (both layouts)
        X, U = X[None], U[None]
    if tile64:
        return _linearize_tile64(system, X, U, dt, central, n_use, epsx, epsu, relx, relu,
                                 tile64_dtype or torch.float64)
    sid = system_id(system)
    n, m = system_dims(sid)
    if X.dim() != 3 or U.dim() != 3 or X.shape[-1] != n or U.shape[-1] != m:
        raise ValueError(f"X must be [B, N+1, {n}] and U [B, N, {m}] for system {sid}")
    Bn, N = U.shape[0], U.shape[1]
    if X.shape[0] != Bn or X.shape[1] != N + 1:
        raise ValueError("X must hold N+1 states per problem (len(U) + 1)")
    n_use = N if n_use is None else int(n_use)
    if n_use > N:
        raise IndexError(f"n_use={n_use} exceeds the {N} steps supplied")
    dev = X.device
    A = torch.empty((Bn, N, n, n), dtype=torch.float64, device=dev)
    Bm = torch.empty((Bn, N, n, m), dtype=torch.float64, device=dev)
    a_res = torch.empty((Bn, N, n), dtype=torch.float64, device=dev)
    Fx = torch.empty((Bn, N, n), dtype=torch.float64, device=dev) if want_fx else None
    rc = _lib.load().hop_linearize_f64(sid, float(dt), _lib.ptr(X), _lib.ptr(U), Bn, N, n_use,
                                       int(bool(central)), float(epsx), float(epsu), float(relx),
                                       float(relu), _lib.ptr(A), _lib.ptr(Bm), _lib.ptr(a_res),
                                       _lib.ptr(Fx), _lib.stream_handle(dev))
    _lib.check(rc)
    return Linearization(A, Bm, a_res, Fx, n_use=n_use)


def _linearize_tile64(system, X, U, dt, central, n_use, epsx, epsu, relx, relu, odt):
    torch = _torch()
    sid = system_id(system)
    n, m = system_dims(sid)
    X = _dev(X, "X", torch.float64)
    U = _dev(U, "U", torch.float64, X.device)
    if X.dim() != 3 or U.dim() != 3 or X.shape[-1] != n or U.shape[-1] != m:
        raise ValueError(f"X must be [B, N+1, {n}] and U [B, N, {m}] for system {sid}")
    Bn, N = U.shape[0], U.shape[1]
    if X.shape[0] != Bn or X.shape[1] != N + 1:
        raise ValueError("X must hold N+1 states per problem (len(U) + 1)")
    n_use = N if n_use is None else int(n_use)
    if n_use > N:
        raise IndexError(f"n_use={n_use} exceeds the {N} steps supplied")
    if odt not in (torch.float64, torch.float32):
        raise TypeError("tile64_dtype must be float64 or float32")
    dev = X.device
    nt = (Bn + 63) // 64
    # steps >= n_use are not written: zero them (a later propagate_traj with its default
    # n_use = N then streams zeros, not uninitialised memory)
    alloc = torch.empty if n_use == N else torch.zeros
    mk = lambda steps, e: alloc((nt, steps, e, 64), dtype=odt, device=dev)  # noqa: E731
    A, Bm, ar, Xt, Ut = mk(N, n * n), mk(N, n * m), mk(N, n), mk(N + 1, n), mk(N, m)
    fn = _lib.load().hop_linearize_tile64_f64 if odt == torch.float64 else \
        _lib.load().hop_linearize_tile64_f32
    rc = fn(sid, float(dt), _lib.ptr(X), _lib.ptr(U), Bn, N, n_use, int(bool(central)),
            float(epsx), float(epsu), float(relx), float(relu), _lib.ptr(A), _lib.ptr(Bm),
            _lib.ptr(ar), _lib.ptr(Xt), _lib.ptr(Ut), _lib.stream_handle(dev))
    _lib.check(rc)
    return Linearization(Tile64(A, Bn, n, n), Tile64(Bm, Bn, n, m), Tile64(ar, Bn, n, 1), None,
                         Tile64(Xt, Bn, n, 1), Tile64(Ut, Bn, m, 1), n_use=n_use)


def dynamics(system, X, U, dt: float):
    """x' = F(x, u) for X [..., n], U [..., m] (fp64, on the device)."""
    torch = _torch()
    sid = system_id(system)
    n, m = system_dims(sid)
    X = _dev(X, "X", torch.float64)
    U = _dev(U, "U", torch.float64, X.device)
    if X.shape[-1] != n or U.shape[-1] != m or X.shape[:-1] != U.shape[:-1]:
        raise ValueError(f"X [..., {n}] and U [..., {m}] with the same leading shape expected")
    cnt = X.numel() // n
    out = torch.empty_like(X)
    rc = _lib.load().hop_dynamics_f64(sid, float(dt), _lib.ptr(X), n, _lib.ptr(U), m, cnt,
                                      _lib.ptr(out), n, _lib.stream_handle(X.device))
    _lib.check(rc)
    return out


# ---- forward pass / outer-loop bookkeeping (forward.hip)

ALPHAS = (1.0, 0.5, 0.25, 0.1, 0.05)  # solver.py:247


@dataclass
class CostParams:
    """Device-resident cost data of cost_timeopt_true (solver.py:65-102): xg [n] or
    [B, n], u_ref [m] or [B, m], Q, R, Qf (= as_terminal_weight(alpha)) shared or per
    problem, w scalar or [B], obstacles [n_obs, 4] = (cx, cy, radius, weight) or None,
    wrap_idx as in the reference."""
    xg: "object"
    u_ref: "object"
    Q: "object"
    R: "object"
    Qf: "object"
    w: "object"
    obstacles: "object" = None
    wrap_idx: Optional[Sequence[int]] = None

    def args(self, Bn, n, m, dev):
        torch = _torch()
        dt = torch.float64
        xg = _dev(self.xg, "xg", dt, dev)
        u_ref = _dev(self.u_ref, "u_ref", dt, dev)
        Q = _dev(self.Q, "Q", dt, dev)
        R = _dev(self.R, "R", dt, dev)
        Qf = _dev(self.Qf, "Qf", dt, dev)
        w = _scalar_or_vec(self.w, dt, dev, "w")
        for t, nm, shp in ((xg, "xg", (n,)), (u_ref, "u_ref", (m,)), (Q, "Q", (n, n)),
                           (R, "R", (m, m)), (Qf, "Qf", (n, n))):
            if tuple(t.shape[-len(shp):]) != shp:
                raise ValueError(f"{nm} must end in {shp}, got {tuple(t.shape)}")
        if w.numel() not in (1, Bn):
            raise ValueError("w must be a scalar or [B]")
        obs = None
        if self.obstacles is not None and len(self.obstacles):
            obs = _dev(torch.as_tensor(self.obstacles, dtype=dt, device=dev), "obstacles", dt, dev)
            if obs.dim() != 2 or obs.shape[1] != 4:
                raise ValueError("obstacles must be [n_obs, 4]")
        n_obs = 0 if obs is None else obs.shape[0]
        args = [_lib.ptr(xg), _bstride(xg, 1, "xg", Bn), _lib.ptr(u_ref),
                _bstride(u_ref, 1, "u_ref", Bn), _lib.ptr(Q), _bstride(Q, 2, "Q", Bn),
                _lib.ptr(R), _bstride(R, 2, "R", Bn), _lib.ptr(Qf), _bstride(Qf, 2, "Qf", Bn),
                _lib.ptr(w), 0 if w.numel() == 1 else 1, _lib.ptr(obs), n_obs,
                wrap_mask(self.wrap_idx, n)]
        return args, (xg, u_ref, Q, R, Qf, w, obs)


def _traj_xu(system, X, U):
    sid = system_id(system)
    n, m = system_dims(sid)
    torch = _torch()
    X = _dev(X, "X", torch.float64)
    dev = X.device
    U = _dev(U, "U", torch.float64, dev)
    if X.dim() != 3 or U.dim() != 3 or X.shape[-1] != n or U.shape[-1] != m \
            or X.shape[0] != U.shape[0] or X.shape[1] != U.shape[1] + 1:
        raise ValueError(f"X must be [B, N+1, {n}] and U [B, N, {m}]")
    return sid, n, m, X, U, dev


def rollout(system, x0, U, dt: float, *, max_state_norm: float = 1e6):
    """Batched rollout (solver.py:42-62): x0 [n] or [B, n], U [B, N, m] -> X [B, N+1, n]."""
    torch = _torch()
    sid = system_id(system)
    n, m = system_dims(sid)
    U = _dev(U, "U", torch.float64)
    dev = U.device
    x0 = _dev(x0, "x0", torch.float64, dev)
    if U.dim() != 3 or U.shape[-1] != m:
        raise ValueError(f"U must be [B, N, {m}]")
    Bn, N = U.shape[0], U.shape[1]
    if x0.shape[-1] != n or (x0.dim() == 2 and x0.shape[0] not in (1, Bn)) or x0.dim() > 2:
        raise ValueError(f"x0 must be [{n}] or [B, {n}]")
    X = torch.empty((Bn, N + 1, n), dtype=torch.float64, device=dev)
    x_bs = n if (x0.dim() == 2 and x0.shape[0] == Bn and Bn > 1) else 0
    rc = _lib.load().hop_rollout_f64(sid, float(dt), _lib.ptr(x0), x_bs, _lib.ptr(U), Bn, N,
                                     float(max_state_norm), _lib.ptr(X), _lib.stream_handle(dev))
    _lib.check(rc)
    return X


def cost_true(system, X, U, T_star, cost: CostParams):
    """Batched cost_timeopt_true (solver.py:65-102) at per-problem horizons T_star [B]."""
    torch = _torch()
    sid, n, m, X, U, dev = _traj_xu(system, X, U)
    Bn, N = U.shape[0], U.shape[1]
    T = _dev(torch.as_tensor(T_star, device=dev).to(torch.int32).reshape(-1).expand(Bn),
             "T_star")
    cargs, keep = cost.args(Bn, n, m, dev)
    J = torch.empty((Bn,), dtype=torch.float64, device=dev)
    rc = _lib.load().hop_cost_true_f64(sid, _lib.ptr(X), _lib.ptr(U), _lib.ptr(T), *cargs, Bn, N,
                                       _lib.ptr(J), _lib.stream_handle(dev))
    _lib.check(rc)
    del keep
    return J


@dataclass
class LineSearchResult:
    X: "object"         # [B, N+1, n]  X' (X where nothing was accepted)
    U: "object"         # [B, N, m]
    J: "object"         # [B]  accepted J' or J_old
    J_old: "object"     # [B]
    accepted: "object"  # [B] int32: alpha index, -1 none, -2 inactive


def forward_linesearch(system, X, U, T_star, K, k, cost: CostParams, dt: float, *,
                       alphas=ALPHAS, active=None) -> LineSearchResult:
    """Batched forward_linesearch_fixedT (solver.py:233-286).  K [B, N, m, n] and
    k [B, N, m] as hop_riccati mode 0 returns them; T_star [B]; active [B] bool/int
    (None = all)."""
    torch = _torch()
    sid, n, m, X, U, dev = _traj_xu(system, X, U)
    Bn, N = U.shape[0], U.shape[1]
    K = _dev(K, "K", torch.float64, dev)
    k = _dev(k, "k", torch.float64, dev)
    if tuple(K.shape) != (Bn, N, m, n) or tuple(k.shape) != (Bn, N, m):
        raise ValueError(f"K must be [B, N, {m}, {n}] and k [B, N, {m}]")
    T = _dev(torch.as_tensor(T_star, device=dev).to(torch.int32).reshape(-1).expand(Bn),
             "T_star")
    act = None if active is None else _dev(torch.as_tensor(active, device=dev).to(torch.int32)
                                           .reshape(-1).expand(Bn), "active")
    al = [float(a) for a in alphas]
    if not 1 <= len(al) <= 8:
        raise ValueError("1..8 step sizes")
    cargs, keep = cost.args(Bn, n, m, dev)
    lib = _lib.load()
    ws_bytes = int(lib.hop_forward_workspace_bytes(sid, Bn, N, len(al)))
    ws = torch.empty((max(ws_bytes, 8),), dtype=torch.uint8, device=dev)
    out = LineSearchResult(torch.empty_like(X), torch.empty_like(U),
                           torch.empty((Bn,), dtype=torch.float64, device=dev),
                           torch.empty((Bn,), dtype=torch.float64, device=dev),
                           torch.empty((Bn,), dtype=torch.int32, device=dev))
    c_al = (_lib.C.c_double * len(al))(*al)
    rc = lib.hop_forward_linesearch_f64(
        sid, float(dt), _lib.ptr(X), _lib.ptr(U), *cargs, _lib.ptr(T), _lib.ptr(act),
        _lib.ptr(K), _lib.ptr(k), c_al, len(al), Bn, N, _lib.C.c_void_p(ws.data_ptr()),
        ws_bytes, _lib.ptr(out.X), _lib.ptr(out.U), _lib.ptr(out.J), _lib.ptr(out.J_old),
        _lib.ptr(out.accepted), _lib.stream_handle(dev))
    _lib.check(rc)
    ws.record_stream(torch.cuda.current_stream(dev))
    del keep
    return out


def obstacle_cost(X, obstacles, *, want=("c", "cx", "cxx")):
    """Point-mass extra_stage_cost (systems.py:271-293) at every state row of X [..., n]:
    returns (c [...], cx [..., n], cxx [..., n, n]) (entries not in `want` are None)."""
    torch = _torch()
    X = _dev(X, "X", torch.float64)
    dev = X.device
    n = X.shape[-1]
    rows = X.reshape(-1, n)
    lead = tuple(X.shape[:-1])
    obs = _dev(torch.as_tensor(obstacles, dtype=torch.float64, device=dev), "obstacles")
    c = torch.empty(lead, dtype=torch.float64, device=dev) if "c" in want else None
    cx = torch.empty(lead + (n,), dtype=torch.float64, device=dev) if "cx" in want else None
    cxx = torch.empty(lead + (n, n), dtype=torch.float64, device=dev) if "cxx" in want else None
    rc = _lib.load().hop_obstacle_cost_f64(_lib.ptr(rows), n, rows.shape[0], n, _lib.ptr(obs),
                                           obs.shape[0], _lib.ptr(c), _lib.ptr(cx),
                                           _lib.ptr(cxx), _lib.stream_handle(dev))
    _lib.check(rc)
    return c, cx, cxx


def ilqr_accept(state, J, accepted, T_star, *, warm: bool = False):
    """Accept / LM / stop-rule update of solver.py:737-752 on the per-problem state
    tensors (lm, T_bar, J_hist, T_hist, n_hist, done) -- see solver.IlqrState."""
    torch = _torch()
    dev = J.device
    Bn = J.shape[0]
    T = _dev(torch.as_tensor(T_star, device=dev).to(torch.int32).reshape(-1).expand(Bn),
             "T_star")
    rc = _lib.load().hop_ilqr_accept_f64(
        Bn, 1 if warm else 0, _lib.ptr(J), _lib.ptr(accepted), _lib.ptr(T), _lib.ptr(state.lm),
        _lib.ptr(state.T_bar), _lib.ptr(state.J_hist), _lib.ptr(state.T_hist),
        _lib.ptr(state.n_hist), state.J_hist.shape[1], _lib.ptr(state.done),
        _lib.stream_handle(dev))
    _lib.check(rc)


def ilqr_select_mask(state, sel_status, ric_status):
    """Crash marking after the select block and the line search's active mask
    (solver.py:514-525, 581-597) in one launch: problems whose select raised
    (ST_FAIL / ST_NONFINITE) and are not done become crashed and done; returns
    active [B] int32 = not done and the Riccati pass succeeded."""
    torch = _torch()
    Bn = state.done.shape[0]
    dev = state.done.device
    sel = _dev(sel_status, "sel_status", torch.int32, dev)
    ric = _dev(ric_status, "ric_status", torch.int32, dev)
    active = torch.empty((Bn,), dtype=torch.int32, device=dev)
    rc = _lib.load().hop_ilqr_select_mask(Bn, _lib.ptr(sel), _lib.ptr(ric), _lib.ptr(state.done),
                                          _lib.ptr(state.crashed), _lib.ptr(active),
                                          _lib.stream_handle(dev))
    _lib.check(rc)
    return active
