"""The pipelined rerun of the s = 13 conditioned kernels' hand-overs (round 5,
VERDICT r04 item 5).

A problem the conditioned kernel hands over with finite inputs (a genuine chol_inv
escalation, /root/reference/utils.py:81-93) is recomputed with the reference
association (horizon_selection.py:36-86).  The rerun launch splits that recompute
over its workgroup's four waves: the stage blocks (:57-64) and the queries (:77-85),
independent per step, on four rows at a time; the compose chain on two waves.  Every
row runs the one-wave LFT kernel's code on the same values, so the outcome must be
bitwise that kernel's (HOP_OPT_REFERENCE_ASSOC: lft_sweep_v2_kernel<SchedLdlDma> on
every problem), and the oracle's status word.
"""
import os

import numpy as np
import pytest

from oracle import hop_oracle as orc

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _t(x, dev):
    import torch
    return torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)


def _same(res, ref, idx=None):
    import torch
    sel = (lambda x: x) if idx is None else (lambda x: x[idx])  # noqa: E731
    assert torch.equal(sel(res.status), sel(ref.status))
    Ja, Jb = sel(res.J).nan_to_num(7.0), sel(ref.J).nan_to_num(7.0)
    rows = torch.nonzero((Ja != Jb).any(dim=-1)).flatten().tolist() if Ja.dim() == 2 else []
    assert torch.equal(Ja, Jb), ("rows differ", rows[:16], float((Ja - Jb).abs().max()))
    if res.t_star is not None:
        assert torch.equal(sel(res.t_star), sel(ref.t_star))
        assert torch.equal(sel(res.j_star).nan_to_num(7.0), sel(ref.j_star).nan_to_num(7.0))


def _escalate(Q, b, k, target=5e-7):
    """Q[b, k] shifted so that its smallest eigenvalue is -target: chol_inv's tries
    at 1e-9 .. 1e-7 fail and 1e-6 succeeds (utils.py:81-93).  (A margin of 5e-9, one
    escalation to 1e-8, leaves E_k ~ 1e8 and W = (E_k + Gbar)^-1 at the edge of
    fp64 Cholesky: the NumPy reference then reaches the LU slot on 4 of 6 seeds, an
    fp64 coin toss no two evaluations share; 5e-7 gives ST_JITTER alone on all.)"""
    Q = Q.copy()
    lo = np.linalg.eigvalsh(orc.sym(Q[b, k])).min()
    Q[b, k] = Q[b, k] - np.eye(Q.shape[-1]) * (lo + target)
    return Q


@pytest.mark.parametrize("Bn,N", [(4, 37), (3, 8), (19, 21)])
def test_pipelined_rerun_forced_is_the_lft_kernel(dev, Bn, N):
    """HOP_OPT_FORCE_HANDOVER hands every problem over.  With at most four problems in
    a workgroup (Bn = 4, 3; the second workgroup of Bn = 19) the rerun runs the
    pipeline on each; with sixteen (the first workgroup of Bn = 19) the LFT body.  N
    not a multiple of the beat, and N = 8 (the pipeline shorter than its depth):
    bitwise the reference-association kernel, J, status, T* and J*."""
    import torch
    from time_opt_ilqr_amd import _lib, engine
    A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(4400 + Bn, Bn, 13, 4, N)
    args = [_t(x, dev) for x in (A, Bm, Q, Ri, z0, QT)]
    kw = dict(t_min=max(1, N // 3), t_max=N)
    with _lib.options(force_handover=True):
        f = engine.propagate(*args, **kw)
    with _lib.options(reference_assoc=True):
        r = engine.propagate(*args, **kw)
    torch.cuda.synchronize()
    _same(f, r)


def test_pipelined_rerun_genuine_escalation_in_a_4096_batch(dev):
    """One finite-input problem of a config-2 batch (s = 13, m = 4, N = 100, B = 4096)
    needs chol_inv's escalated jitter at one stage (Q_37 shifted to a smallest
    eigenvalue of -5e-7: the ladder settles on 1e-6, utils.py:81-93): the conditioned
    kernel hands it over, the rerun's triage finds nothing non-finite and the pipeline
    recomputes it.  Status ST_JITTER (the oracle's word); J / T* / J* bitwise the
    reference-association kernel's; every other problem untouched (status 0).

    J is held against the 50-digit curve of tests/golden/escalation_hp.npz
    (make_escalation_hp.py), not against the oracle: after the escalated stage
    (E_37 ~ 1e6) the oracle's fp64 Cholesky inverses drift 1.5e-3 from the exact
    curve, the device's equilibrated sweeps 2e-4.  Up to the escalated
    stage both agree with it to 1e-10."""
    import torch
    from time_opt_ilqr_amd import _lib, engine, synth
    fx = np.load(os.path.join(GOLDEN, "escalation_hp.npz"))
    Bn, s, m, N, b = 4096, 13, 4, 100, 1234
    k = int(fx["k"])
    A, Bm, Q, Ri, z0, QT = synth.device_batch(Bn, s, m, N, seed=21, device=dev)
    Ri = (Ri if Ri.dim() == 3 else Ri.expand(Bn, m, m)).contiguous()
    z0 = (z0 if z0.dim() == 2 else z0.expand(Bn, s)).contiguous()
    for x, key in ((A, "A"), (Bm, "B"), (Q, "Q"), (QT, "QT"), (Ri, "Ri"), (z0, "z0")):
        x[b] = _t(fx[key], dev)
    kw = dict(t_min=40, t_max=N)
    res = engine.propagate(A, Bm, Q, Ri, z0, QT, **kw)
    with _lib.options(no_rerun=True):
        ho = engine.propagate(A, Bm, Q, Ri, z0, QT, **kw).status.cpu().numpy()
    with _lib.options(reference_assoc=True):
        ref = engine.propagate(A, Bm, Q, Ri, z0, QT, **kw)
    torch.cuda.synchronize()
    handed = np.nonzero(ho & _lib.ST_HANDOVER)[0]
    assert handed.tolist() == [b], handed[:8]
    assert _lib.handover_horizon(int(ho[b])) == k + 1  # the first flagged horizon (hop.h)
    st = res.status.cpu().numpy()
    assert st[b] == int(fx["status_oracle"]) == orc.ST_JITTER and (np.delete(st, b) == 0).all()
    _same(res, ref, slice(b, b + 1))
    Jb, Jh, Jo = res.J[b].cpu().numpy(), fx["J_hp"], fx["J_oracle"]
    rel = lambda J: np.abs(J - Jh) / np.abs(Jh)  # noqa: E731
    assert rel(Jb)[:k].max() <= 1e-10 and rel(Jo)[:k].max() <= 1e-10
    assert rel(Jb).max() <= 5e-4, rel(Jb).max()
    assert rel(Jb).max() <= rel(Jo).max(), (rel(Jb).max(), rel(Jo).max())


def test_pipelined_rerun_several_per_workgroup_and_nonfinite(dev):
    """Workgroups with 1, 2, 4 and 5 escalated problems (the last above kPipeMax:
    the LFT body) and one with a non-finite stage beside an escalated one (the triage
    resolves the first, the pipeline the second), on the trajectory-free blocks path:
    bitwise the reference-association kernel on every recomputed problem."""
    import torch
    from time_opt_ilqr_amd import _lib, engine
    Bn, s, m, N = 96, 13, 4, 30
    A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(4700, Bn, s, m, N)
    Q = Q.copy()
    esc = [0, 16, 17, 32, 33, 34, 35, 48, 49, 50, 51, 52, 64, 65]
    for b in esc:
        Q = _escalate(Q, b, (3 * b) % N)
    Q[66, 9, 2, 3] = np.nan
    args = [_t(x, dev) for x in (A, Bm, Q, Ri, z0, QT)]
    kw = dict(t_min=5, t_max=N)
    res = engine.propagate(*args, **kw)
    with _lib.options(reference_assoc=True):
        ref = engine.propagate(*args, **kw)
    torch.cuda.synchronize()
    # the recomputed problems: bitwise.  Problem 66's hand-over is explained by its
    # non-finite stage: the triage keeps the conditioned kernel's finite prefix (J to
    # ~1e-12 of the reference association) and NaN from the poisoned horizon on, with
    # the reference's status word and argmin (tests/test_gpu_nonfinite.py); the rest
    # keep the conditioned curve and status 0
    _same(res, ref, esc)
    assert torch.equal(res.status, ref.status)
    assert torch.equal(res.J[66].isnan(), ref.J[66].isnan()) and bool(res.J[66].isnan().any())
    assert int(res.t_star[66]) == int(ref.t_star[66])
    rel = ((res.J - ref.J).abs() / ref.J.abs()).nan_to_num(0.0)
    assert float(rel.max()) <= 1e-9


def _traj_batch(dev, Bn, N, seed):
    import torch
    n, m = 12, 4
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    kw = dict(device=dev, dtype=torch.float64, generator=g)
    A = torch.eye(n, device=dev, dtype=torch.float64) + 0.05 * torch.randn((Bn, N, n, n), **kw)
    B = 0.1 * torch.randn((Bn, N, n, m), **kw)
    M = torch.randn((n, n), **kw)
    Q = M @ M.T / n + 0.5 * torch.eye(n, device=dev, dtype=torch.float64)
    Ri = torch.linalg.inv(torch.diag(0.5 + 1.5 * torch.rand((m,), **kw)))
    Qf = 10.0 * torch.eye(n, device=dev, dtype=torch.float64)
    X = 0.5 * torch.randn((Bn, N + 1, n), **kw)
    U = 0.3 * torch.randn((Bn, N, m), **kw)
    xg, ur = 0.2 * torch.randn((n,), **kw), 0.1 * torch.randn((m,), **kw)
    ares = 0.02 * torch.randn((Bn, N, n), **kw)
    return (A, B, ares, X, U, xg, ur, Q, Ri, Qf, 0.5)


@pytest.mark.parametrize("Bn,N,rho", [(4, 37, 1.0), (19, 23, 1e-12), (2, 5, 1e-12)])
def test_pipelined_rerun_trajectory_form_forced_is_the_lft_kernel(dev, Bn, N, rho):
    """The select block's trajectory form (the closed-form conditioned kernel, then
    the rerun launch building Q_aug / QT_aug in-kernel, augmented.py:10-87): every
    problem forced over, the pipeline on workgroups of four or fewer, the LFT body on
    the full one: bitwise the trajectory LFT kernel (HOP_OPT_REFERENCE_ASSOC), with
    wrapped angle states and the reference's rho_reg = 1e-12."""
    import torch
    from time_opt_ilqr_amd import _lib, engine
    args = _traj_batch(dev, Bn, N, 70 + Bn)
    kw = dict(t_min=max(1, N // 3), t_max=N, rho_reg=rho, wrap_idx=[2, 7])
    with _lib.options(force_handover=True):
        f = engine.propagate_traj(*args, **kw)
    with _lib.options(reference_assoc=True):
        r = engine.propagate_traj(*args, **kw)
    torch.cuda.synchronize()
    _same(f, r)
