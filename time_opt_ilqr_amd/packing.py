"""Mixed-shape batches: the block-decoupled embedding.

The reference solves one system at a time, each at its own augmented size
s = n+1 (augmented.py:10-60).  A batch that mixes systems (Segway / Cartpole
s=5, m=1 with Quadrotor s=13, m=4) runs as ONE launch of the s_out x s_out
kernel once every member is embedded so that its J(t) is unchanged:

  * real state dims keep their indices 0..n-1, the homogeneous coordinate moves
    to index s_out-1, pad dims n..s_out-2 sit in between;
  * A_pad = 0 on pad rows/cols, B_pad rows and extra control columns = 0,
    Q_pad = QT_pad = I, R_inv_pad = I on the extra controls, z0_pad = 0.

Every block stays block-diagonal across (real | pad), the pad block never
couples into the z0 quadratic form, so J is the true-s J up to rounding
(oracle: ``embed_block_decoupled``; tests/test_host_cpu.py checks 1e-12).

This is host/device plumbing in torch (gathers into a preallocated batch);
the sweep itself is the same hop_lft_sweep_* launch as any other batch.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Sequence


def _torch():
    import torch
    return torch


def embed_index(s: int, s_out: int):
    """Destination index of each of the s augmented coordinates."""
    if s > s_out:
        raise ValueError(f"cannot embed s={s} into s_out={s_out}")
    return list(range(s - 1)) + [s_out - 1]


def embed_block_decoupled(A, B, Q, R_inv, z0, QT, s_out: int, m_out: int):
    """Embed a batch of true-shape problems into (s_out, m_out) blocks.

    A, Q, QT : [b, N, s, s];  B : [b, N, s, m];  R_inv : [m, m] or [b, m, m];
    z0 : [s] or [b, s].  Returns (A, B, Q, R_inv, z0, QT) at [b, N, s_out, *],
    R_inv [b, m_out, m_out], z0 [b, s_out], same dtype / device.
    """
    torch = _torch()
    b, N, s, _ = A.shape
    m = B.shape[-1]
    if m > m_out:
        raise ValueError(f"cannot embed m={m} into m_out={m_out}")
    idx = torch.as_tensor(embed_index(s, s_out), device=A.device)
    dt, dev = A.dtype, A.device
    n = s - 1
    pad = torch.arange(n, s_out - 1, device=dev)

    def square(M, fill):
        out = torch.zeros((b, N, s_out, s_out), dtype=dt, device=dev)
        out[:, :, pad, pad] = fill
        out[:, :, idx[:, None], idx[None, :]] = M
        return out

    Bp = torch.zeros((b, N, s_out, m_out), dtype=dt, device=dev)
    Bp[:, :, idx, :m] = B
    Rp = torch.eye(m_out, dtype=dt, device=dev).repeat(b, 1, 1)
    Rp[:, :m, :m] = R_inv if R_inv.dim() == 3 else R_inv.expand(b, m, m)
    zp = torch.zeros((b, s_out), dtype=dt, device=dev)
    zp[:, idx] = z0 if z0.dim() == 2 else z0.expand(b, s)
    return square(A, 0.0), Bp, square(Q, 1.0), Rp, zp, square(QT, 1.0)


@dataclass
class MixedBatch:
    """A padded batch plus where each member came from."""
    A: "object"      # [B, N, s_out, s_out]
    B: "object"      # [B, N, s_out, m_out]
    Q: "object"
    R_inv: "object"  # [B, m_out, m_out]
    z0: "object"     # [B, s_out]
    QT: "object"
    kind: "object"   # [B] int64: index into the group list
    true_s: "object"  # [B] int64
    true_m: "object"  # [B] int64


def pack_mixed(groups: Sequence[tuple], order, s_out: int, m_out: int) -> MixedBatch:
    """Interleave groups of true-shape problems into one padded batch.

    groups : list of (A, B, Q, R_inv, z0, QT) tensors, group g holding all the
             members of kind g in their batch order.
    order  : [B] kind of each batch slot (slot i takes the next unused member of
             group order[i]).
    """
    torch = _torch()
    order = torch.as_tensor(order, dtype=torch.int64)
    Bn = int(order.numel())
    ref = groups[0][0]
    N = ref.shape[1]
    dt, dev = ref.dtype, ref.device
    out = MixedBatch(torch.empty((Bn, N, s_out, s_out), dtype=dt, device=dev),
                     torch.empty((Bn, N, s_out, m_out), dtype=dt, device=dev),
                     torch.empty((Bn, N, s_out, s_out), dtype=dt, device=dev),
                     torch.empty((Bn, m_out, m_out), dtype=dt, device=dev),
                     torch.empty((Bn, s_out), dtype=dt, device=dev),
                     torch.empty((Bn, N, s_out, s_out), dtype=dt, device=dev),
                     order.to(dev), torch.empty(Bn, dtype=torch.int64, device=dev),
                     torch.empty(Bn, dtype=torch.int64, device=dev))
    for g, grp in enumerate(groups):
        slots = torch.nonzero(order == g).reshape(-1).to(dev)
        cnt = int(slots.numel())
        if cnt == 0:
            continue
        if grp[0].shape[0] < cnt:
            raise ValueError(f"group {g} has {grp[0].shape[0]} problems, {cnt} slots need it")
        if grp[0].shape[1] != N:
            raise ValueError("every group must have the same number of stages N")
        A, B, Q, Ri, z0, QT = grp
        A, B, Q, QT = A[:cnt], B[:cnt], Q[:cnt], QT[:cnt]
        if Ri.dim() == 3:
            Ri = Ri[:cnt]
        if z0.dim() == 2:
            z0 = z0[:cnt]
        pa, pb, pq, pr, pz, pt = embed_block_decoupled(A, B, Q, Ri, z0, QT, s_out, m_out)
        out.A[slots] = pa
        out.B[slots] = pb
        out.Q[slots] = pq
        out.R_inv[slots] = pr
        out.z0[slots] = pz
        out.QT[slots] = pt
        out.true_s[slots] = A.shape[-1]
        out.true_m[slots] = B.shape[-1]
    return out


def merge_by_shape(groups: Sequence[tuple], order):
    """Regroup a mixed batch by block shape for engine.propagate_groups: kinds
    that share (s, m) -- Segway and Cartpole in config 5 -- become one group (one
    launch), its members in batch-slot order.  groups / order as pack_mixed
    (R_inv and z0 may be shared per kind: [m, m] / [s]).  Returns (shape_groups,
    shape_order) with shape_order[i] = shape group of slot i.  A setup-time
    gather: one copy of the merged members."""
    torch = _torch()
    order = torch.as_tensor(order, dtype=torch.int64).cpu()
    shapes, kind_to_shape = [], []
    for grp in groups:
        key = (int(grp[0].shape[-1]), int(grp[1].shape[-1]))
        if key not in shapes:
            shapes.append(key)
        kind_to_shape.append(shapes.index(key))
    shape_order = torch.as_tensor(kind_to_shape, dtype=torch.int64)[order]
    rank = torch.empty_like(order)  # slot i is the rank[i]-th member of its kind
    for g in range(len(groups)):
        sl = torch.nonzero(order == g).reshape(-1)
        rank[sl] = torch.arange(sl.numel())
    out = []
    for h in range(len(shapes)):
        kinds = [g for g in range(len(groups)) if kind_to_shape[g] == h]
        if len(kinds) == 1:
            out.append(tuple(groups[kinds[0]]))
            continue
        sl = torch.nonzero(shape_order == h).reshape(-1)
        kind_of, rank_of = order[sl], rank[sl]
        parts = []
        for j in range(6):
            ts = [groups[g][j] for g in kinds]
            full_dim = 3 if j == 3 else 2 if j == 4 else None
            if full_dim is not None and all(t.dim() == full_dim - 1 for t in ts) and \
                    all(torch.equal(t, ts[0]) for t in ts):
                parts.append(ts[0])  # one shared block for the merged group
                continue
            if full_dim is not None:  # expand shared per-kind blocks to per member
                ts = [t if t.dim() == full_dim else t.expand((groups[g][0].shape[0],) +
                                                               tuple(t.shape)).contiguous()
                      for g, t in zip(kinds, ts)]
            ref = ts[0]
            rows = torch.empty((sl.numel(),) + tuple(ref.shape[1:]), dtype=ref.dtype,
                               device=ref.device)
            for g, t in zip(kinds, ts):
                m = torch.nonzero(kind_of == g).reshape(-1)
                rows[m.to(ref.device)] = t[rank_of[m].to(ref.device)]
            parts.append(rows)
        out.append(tuple(parts))
    return out, shape_order
