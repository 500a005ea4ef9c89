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
import numpy as np
import pytest

from oracle import hop_oracle as orc

pytestmark = pytest.mark.gpu


def _t(x, dev):
    import torch
    return torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)


def _same(res, ref, idx=None):
    import torch
    sel = (lambda x: x) if idx is None else (lambda x: x[idx])  # noqa: E731
    assert torch.equal(sel(res.status), sel(ref.status))
    assert torch.equal(sel(res.J).nan_to_num(7.0), sel(ref.J).nan_to_num(7.0))
    if res.t_star is not None:
        assert torch.equal(sel(res.t_star), sel(ref.t_star))
        assert torch.equal(sel(res.j_star).nan_to_num(7.0), sel(ref.j_star).nan_to_num(7.0))


def _escalate(Q, b, k, target=5e-9):
    """Q[b, k] shifted so that its smallest eigenvalue is -target: chol_inv's first
    try (+1e-9) fails and its second (+1e-8) succeeds (utils.py:81-93)."""
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
    needs chol_inv's second jitter (1e-9 -> 1e-8) at one stage: the conditioned kernel
    hands it over, the rerun's triage finds nothing non-finite and the pipeline
    recomputes it.  Status ST_JITTER (the oracle's word), J / T* / J* bitwise the
    reference-association kernel's, J within 1e-9 of the oracle; every other problem
    untouched (the conditioned kernel's own result, status 0)."""
    import torch
    from time_opt_ilqr_amd import _lib, engine, synth
    Bn, s, m, N, b, k = 4096, 13, 4, 100, 1234, 37
    A, Bm, Q, Ri, z0, QT = synth.device_batch(Bn, s, m, N, seed=21, device=dev)
    Qh = _escalate(Q[b:b + 1].cpu().numpy(), 0, k)
    Q[b] = _t(Qh[0], dev)
    kw = dict(t_min=40, t_max=N)
    res = engine.propagate(A, Bm, Q, Ri, z0, QT, **kw)
    with _lib.options(no_rerun=True):
        ho = engine.propagate(A, Bm, Q, Ri, z0, QT, **kw).status.cpu().numpy()
    with _lib.options(reference_assoc=True):
        ref = engine.propagate(A, Bm, Q, Ri, z0, QT, **kw)
    torch.cuda.synchronize()
    handed = np.nonzero(ho & _lib.ST_HANDOVER)[0]
    assert handed.tolist() == [b], handed[:8]
    st = res.status.cpu().numpy()
    assert st[b] == orc.ST_JITTER and (np.delete(st, b) == 0).all()
    _same(res, ref, slice(b, b + 1))
    h = lambda x: x[b].cpu().numpy()  # noqa: E731
    o = orc.lft_sweep(h(A), h(Bm), h(Q), h(Ri) if Ri.dim() == 3 else Ri.cpu().numpy(),
                      h(z0) if z0.dim() == 2 else z0.cpu().numpy(), h(QT))
    assert int(o["status"]) == int(st[b])
    Jb = res.J[b].cpu().numpy()
    assert np.max(np.abs(Jb - o["J"]) / np.abs(o["J"])) <= 1e-9


def test_pipelined_rerun_several_per_workgroup_and_nonfinite(dev):
    """Workgroups with 1, 2, 4 and 5 escalated problems (the last above kPipeMax:
    the LFT body) and one with a non-finite stage beside an escalated one (the triage
    resolves the first, the pipeline the second), on the trajectory-free blocks path:
    bitwise the reference-association kernel on every problem."""
    import torch
    from time_opt_ilqr_amd import _lib, engine
    Bn, s, m, N = 96, 13, 4, 30
    A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(4700, Bn, s, m, N)
    Q = Q.copy()
    for b in [0, 16, 17, 32, 33, 34, 35, 48, 49, 50, 51, 52, 64, 65]:
        Q = _escalate(Q, b, (3 * b) % N)
    Q[66, 9, 2, 3] = np.nan
    args = [_t(x, dev) for x in (A, Bm, Q, Ri, z0, QT)]
    kw = dict(t_min=5, t_max=N)
    res = engine.propagate(*args, **kw)
    with _lib.options(reference_assoc=True):
        ref = engine.propagate(*args, **kw)
    torch.cuda.synchronize()
    _same(res, ref)
