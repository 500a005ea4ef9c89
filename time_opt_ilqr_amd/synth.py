"""Synthetic, well-conditioned LFT inputs generated directly in HBM (bench data).

Same distribution as oracle.hop_oracle.synth_lft_problem:
A = [[I + 0.05 G, 0.1 g], [0, 1]], B = [[0.1 G], [0]], Q = M M^T / s + I,
QT = M' M'^T / s + I, R = diag(U(0.5, 2)), z0 = e_s -- but drawn with torch's
device RNG (not bit-identical to the NumPy stream; parity tests copy subsets
back to the host oracle).
"""
from __future__ import annotations


def device_batch(batch: int, s: int, m: int, N: int, *, seed: int = 0, device=None,
                 dtype=None):
    import torch
    dtype = dtype or torch.float64
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    n = s - 1
    kw = dict(device=device, dtype=torch.float64, generator=g)
    A = torch.zeros((batch, N, s, s), device=device, dtype=torch.float64)
    A[:, :, :n, :n] = torch.eye(n, device=device, dtype=torch.float64) + \
        0.05 * torch.randn((batch, N, n, n), **kw)
    A[:, :, :n, n] = 0.1 * torch.randn((batch, N, n), **kw)
    A[:, :, n, n] = 1.0
    Bm = torch.zeros((batch, N, s, m), device=device, dtype=torch.float64)
    Bm[:, :, :n, :] = 0.1 * torch.randn((batch, N, n, m), **kw)
    eye = torch.eye(s, device=device, dtype=torch.float64)
    M = torch.randn((batch, N, s, s), **kw)
    Q = M @ M.transpose(-1, -2) / s + eye
    M = torch.randn((batch, N, s, s), **kw)
    QT = M @ M.transpose(-1, -2) / s + eye
    r = 0.5 + 1.5 * torch.rand((batch, m), **kw)
    Rinv = torch.diag_embed(1.0 / r)
    z0 = torch.zeros((s,), device=device, dtype=torch.float64)
    z0[-1] = 1.0
    out = (A, Bm, Q, Rinv, z0, QT)
    return tuple(t.to(dtype).contiguous() for t in out)


CONFIG5_KINDS = (("segway", 5, 1), ("cartpole", 5, 1), ("quadrotor", 13, 4))


def config5_batch(batch: int, N: int = 128, *, seed: int = 0, device=None, dtype=None,
                  s_out: int = 13, m_out: int = 4):
    """Config 5: member i is Segway- / Cartpole- / Quadrotor-shaped
    by i mod 3, each drawn at its true (s, m) with ``device_batch`` and embedded
    block-decoupled into (s_out, m_out) (packing.pack_mixed).  Returns
    (MixedBatch, groups) where groups holds the true-shape tensors (for spot
    checks against the oracle)."""
    import torch
    from .packing import pack_mixed
    order = torch.arange(batch) % 3
    groups = []
    for g, (_, s, m) in enumerate(CONFIG5_KINDS):
        cnt = int((order == g).sum())
        groups.append(device_batch(max(cnt, 1), s, m, N, seed=seed * 7 + 101 * g, device=device,
                                   dtype=dtype))
    return pack_mixed(groups, order, s_out, m_out), groups
