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
    dist.all_gather_into_tensor(out, packed, group=group)
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
    N = J.shape[1] if J.dim() == 2 else 0
    sizes = [shard_bounds(total, r, world) for r in range(world)]
    cap = max(hi - lo for lo, hi in sizes)
    packed = torch.full((cap, N), float("nan"), dtype=J.dtype, device=J.device)
    packed[: J.shape[0]] = J
    out = torch.empty((world * cap, N), dtype=J.dtype, device=J.device)
    dist.all_gather_into_tensor(out, packed, group=group)
    return torch.cat([out[r * cap: r * cap + (hi - lo)] for r, (lo, hi) in enumerate(sizes)], 0)
