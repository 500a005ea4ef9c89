"""Multi-GPU plumbing: one process per GPU, independent problem shards.

The LFT sweeps of different problems never interact, so each
rank owns a contiguous shard of the batch and runs with no communication.  The
only collective is the final all-gather of the per-problem selection
(T*, J*) -- 12 bytes per problem over RCCL/xGMI (or gloo on CPU for tests).
"""
from __future__ import annotations

import os


def env_rank_world():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def shard_bounds(total: int, rank: int, world: int):
    """Contiguous [lo, hi) of problems owned by `rank` (balanced to +-1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(int(total), int(world))
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def _host_collective(group, dev) -> bool:
    """gloo all-gathers host tensors only: a device tensor goes through the host for
    the collective (the real kernels under gloo, several ranks on one GPU: the bench's
    --dist-backend gloo rehearsal and tests/test_gpu_distributed.py).  RCCL keeps them
    on the device."""
    import torch.distributed as dist
    return dev.type != "cpu" and dist.get_backend(group) == "gloo"


def _all_gather_packed(out, packed, group):
    import torch.distributed as dist
    if _host_collective(group, packed.device):
        host = out.cpu()
        dist.all_gather_into_tensor(host, packed.cpu(), group=group)
        out.copy_(host)
    else:
        dist.all_gather_into_tensor(out, packed, group=group)


def all_reduce_max(t, group=None):
    """In-place MAX all-reduce (through the host under gloo, as above)."""
    import torch.distributed as dist
    if _host_collective(group, t.device):
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MAX, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t


def gather_selection(t_star, j_star, total: int, group=None):
    """All-gather every rank's (T*, J*) shard into full [total] tensors.

    Shards may differ by one problem; they are padded to the largest shard for
    all_gather_into_tensor and trimmed afterwards.
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if world == 1:
        return t_star, j_star
    sizes = [shard_bounds(total, r, world) for r in range(world)]
    cap = max(hi - lo for lo, hi in sizes)
    dev = t_star.device
    packed = torch.zeros((cap, 2), dtype=torch.float64, device=dev)
    packed[: t_star.numel(), 0] = t_star.to(torch.float64)
    packed[: j_star.numel(), 1] = j_star.to(torch.float64)
    out = torch.empty((world * cap, 2), dtype=torch.float64, device=dev)
    _all_gather_packed(out, packed, group)
    parts = [out[r * cap: r * cap + (hi - lo)] for r, (lo, hi) in enumerate(sizes)]
    full = torch.cat(parts, 0)
    return full[:, 0].to(torch.int32), full[:, 1].to(j_star.dtype)


def gather_curves(J, total: int, group=None):
    """All-gather every rank's J curves [shard, N] into [total, N] (the optional
    full-curve collection of SURVEY.md 2: the reference's driver plots and writes
    the last J curve, ilqr_propagator.py:825/860).  N * 8 bytes per problem, so
    callers gather curves only when they need them; the bench gathers (T*, J*)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if world == 1:
        return J
    # every rank must pack the same width: an empty shard may hold a [0] tensor, so
    # the curve length is agreed on by one max all-reduce first
    n_loc = torch.tensor([J.shape[1] if J.dim() == 2 else 0], dtype=torch.int64, device=J.device)
    all_reduce_max(n_loc, group)
    N = int(n_loc.item())
    if J.dim() != 2:
        J = J.reshape(0, N)
    sizes = [shard_bounds(total, r, world) for r in range(world)]
    cap = max(hi - lo for lo, hi in sizes)
    packed = torch.full((cap, N), float("nan"), dtype=J.dtype, device=J.device)
    packed[: J.shape[0]] = J
    out = torch.empty((world * cap, N), dtype=J.dtype, device=J.device)
    _all_gather_packed(out, packed, group)
    return torch.cat([out[r * cap: r * cap + (hi - lo)] for r, (lo, hi) in enumerate(sizes)], 0)


def gather_columns(cols, total: int, group=None):
    """All-gather per-problem columns (a list of equal-length 1-D tensors of this
    rank's shard) into full [total] tensors, each returned in its own dtype.  One
    collective: the columns travel packed as float64 (exact for the int32 fields)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return list(cols)
    sizes = [shard_bounds(total, r, world) for r in range(world)]
    cap = max(hi - lo for lo, hi in sizes)
    dev = cols[0].device
    packed = torch.zeros((cap, len(cols)), dtype=torch.float64, device=dev)
    for j, c in enumerate(cols):
        packed[: c.numel(), j] = c.to(torch.float64)
    out = torch.empty((world * cap, len(cols)), dtype=torch.float64, device=dev)
    _all_gather_packed(out, packed, group)
    full = torch.cat([out[r * cap: r * cap + (hi - lo)] for r, (lo, hi) in enumerate(sizes)], 0)
    return [full[:, j].to(c.dtype) for j, c in enumerate(cols)]


def ilqr_timeopt_sharded(system, x0_all, xg, u_ref, Q, R, Qf, w, N: int, T_min: int, T_max: int,
                         *, U_init=None, group=None, device=None, **kw):
    """The device outer loop (solver.ilqr_timeopt_batch, either select method) over a
    batch sharded across the ranks of a node: rank r solves the contiguous problems
    shard_bounds(B, r, world) on its own GPU with no communication inside the loop,
    then one all-gather collects every problem's (T*, final J, accepted iterations,
    crashed).  x0_all [B, n] is the whole batch on every rank (a rank reads only its
    rows); per-problem inputs -- U_init [B, N', m], xg [B, n], u_ref [B, m], Q [B, n, n]
    (the batch shapes ilqr_timeopt_batch accepts) -- are sliced the same way; shared
    ones ([N', m], [n], [m], [n, n]) pass through whole.
    Returns (full: dict of [B] tensors, local: this rank's ilqr_timeopt_batch result
    or None for an empty shard, (lo, hi))."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from . import solver
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    x0_all = np.asarray(x0_all.cpu() if isinstance(x0_all, torch.Tensor) else x0_all,
                        dtype=float)
    if x0_all.ndim != 2:
        raise ValueError("x0_all must be [B, n]")
    total = x0_all.shape[0]
    lo, hi = shard_bounds(total, rank, world)
    dev = device or (torch.device("cuda", torch.cuda.current_device())
                     if torch.cuda.is_available() else torch.device("cpu"))
    def shard(a, batch_ndim, name):
        """rows [lo, hi) of a per-problem input (leading dim == total), else a shared one;
        a leading dimension of 1 is one block in batch form, which ilqr_timeopt_batch
        broadcasts (solver.py: U_init [1, N', m]), so it passes through whole"""
        if a is None or np.ndim(a) < batch_ndim:
            return a
        if np.ndim(a) == batch_ndim and np.shape(a)[0] == 1 and total != 1:
            return a
        if np.ndim(a) > batch_ndim or np.shape(a)[0] != total:
            raise ValueError(f"{name}: per-problem inputs need the leading dimension B={total} "
                             f"(got shape {tuple(np.shape(a))})")
        return a[lo:hi]

    ui = shard(U_init, 3, "U_init")
    xg_r, ur_r, Q_r = shard(xg, 2, "xg"), shard(u_ref, 2, "u_ref"), shard(Q, 3, "Q")
    local = None
    if hi > lo:
        local = solver.ilqr_timeopt_batch(system, x0_all[lo:hi], xg_r, ur_r, Q_r, R, Qf, w, N,
                                          T_min, T_max, U_init=ui, device=dev, **kw)
        nh = local["n_hist"].to(torch.int64)
        last = (nh - 1).clamp(min=0)
        J_last = local["J_hist"].gather(1, last[:, None])[:, 0]
        J_last = torch.where(nh > 0, J_last, torch.full_like(J_last, float("nan")))
        cols = [local["T_star"].to(torch.int32), J_last.to(torch.float64),
                local["n_hist"].to(torch.int32), local["crashed"].to(torch.int32)]
    else:  # an empty shard (more ranks than problems) still joins the collective
        cols = [torch.zeros(0, dtype=torch.int32, device=dev),
                torch.zeros(0, dtype=torch.float64, device=dev),
                torch.zeros(0, dtype=torch.int32, device=dev),
                torch.zeros(0, dtype=torch.int32, device=dev)]
    T, J, nh, cr = gather_columns(cols, total, group)
    return dict(T_star=T, J_star=J, n_hist=nh, crashed=cr), local, (lo, hi)
