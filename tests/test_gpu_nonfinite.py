"""Non-finite triage of the conditioned kernels' hand-overs.

The reference raises on a non-finite block (chol_inv's _assert_finite,
/root/reference/utils.py:77); the oracle and every kernel report a NaN inverse with
ST_NONFINITE and no ladder.  A problem the s = 13 conditioned kernel hands over
because its inputs turned non-finite is resolved in the rerun launch without the
sequential recompute: J from the conditioned kernel before the first non-finite
horizon, NaN after, status ST_NONFINITE, the fused argmin replayed.  These tests hold
that outcome to the reference association (HOP_OPT_REFERENCE_ASSOC: the
lft_sweep_v2 kernel alone) on the same device inputs: status word, NaN pattern, T*
and J* equal, finite J within 1e-9; and under HOP_OPT_NO_RERUN only the problems the
triage cannot explain stay handed over.
"""
import numpy as np
import pytest

from oracle import hop_oracle as orc

pytestmark = pytest.mark.gpu


def _cmp(res, ref, tag):
    st, st_r = res.status.cpu().numpy(), ref.status.cpu().numpy()
    J, Jr = res.J.cpu().numpy(), ref.J.cpu().numpy()
    assert np.array_equal(st, st_r), (tag, np.nonzero(st != st_r)[0][:8], st[st != st_r][:8],
                                      st_r[st != st_r][:8])
    nan, nan_r = np.isnan(J), np.isnan(Jr)
    bad = np.nonzero((nan != nan_r).any(axis=1))[0]
    assert bad.size == 0, (tag, bad[:8])
    fin = ~nan
    rel = np.abs(J[fin] - Jr[fin]) / np.maximum(np.abs(Jr[fin]), 1e-300)
    assert rel.size == 0 or rel.max() <= 1e-9, (tag, rel.max())
    ts, ts_r = res.t_star.cpu().numpy(), ref.t_star.cpu().numpy()
    assert np.array_equal(ts, ts_r), (tag, np.nonzero(ts != ts_r)[0][:8])
    js, js_r = res.j_star.cpu().numpy(), ref.j_star.cpu().numpy()
    assert np.array_equal(np.isnan(js), np.isnan(js_r)), tag


def test_nonfinite_triage_augmented_blocks_vs_reference_association(dev):
    """Config-2 shape (s = 13, m = 4, N = 100) on pre-built blocks, 192 problems in six
    kinds by b % 6: clean; NaN in Q_k; NaN in QT_k only (later horizons finite: not
    explained, recomputed); inf in A_k; the rollout shape (QT_{k-1}, Q_k, A_k at once);
    NaN in B_k.  Steps k spread over the horizon, the argmin window [40, 100]."""
    import torch
    from time_opt_ilqr_amd import _lib, engine
    Bn, s, m, N = 192, 13, 4, 100
    A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(4242, Bn, s, m, N)
    A, Bm, Q, QT = A.copy(), Bm.copy(), Q.copy(), QT.copy()
    rng = np.random.default_rng(5)
    kinds = np.arange(Bn) % 6
    h_qt = np.zeros(Bn, np.int64)
    for b in range(Bn):
        k = int(rng.integers(1, N))
        i, j = int(rng.integers(0, s)), int(rng.integers(0, s))
        if kinds[b] == 1:
            Q[b, k, i, j] = np.nan
        elif kinds[b] == 2:  # before the last horizon (J(N) alone would be explained)
            QT[b, min(k, N - 2), i, j] = np.nan
            h_qt[b] = min(k, N - 2) + 1
        elif kinds[b] == 3:
            A[b, k, i, j] = np.inf
        elif kinds[b] == 4:
            QT[b, k - 1, i, j] = np.nan
            Q[b, k, j, i] = np.nan
            A[b, k, i, j] = -np.inf
        elif kinds[b] == 5:
            Bm[b, k, i, j % m] = np.nan
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)  # noqa
    args = (t(A), t(Bm), t(Q), t(Ri), t(z0), t(QT))
    kw = dict(t_min=40, t_max=N)
    res = engine.propagate(*args, **kw)
    with _lib.options(reference_assoc=True):
        ref = engine.propagate(*args, **kw)
    torch.cuda.synchronize()
    _cmp(res, ref, "aug")
    with _lib.options(no_rerun=True):
        ho = engine.propagate(*args, **kw).status.cpu().numpy()
    handed = (ho & _lib.ST_HANDOVER) != 0
    # only the terminal-block-only kind is left to the recompute
    assert np.array_equal(handed, kinds == 2), np.nonzero(handed != (kinds == 2))[0][:8]
    # the hand-over word (include/hop.h): the bit, and the first flagged horizon = the
    # poisoned terminal block's (developer builds add the reason field)
    low = (1 << _lib.HANDOVER_SHIFT) - 1
    assert ((ho[handed] & low) == _lib.ST_HANDOVER).all() or _lib.dev_build()
    assert np.array_equal(_lib.handover_horizon(ho[handed]), h_qt[handed])
    assert (ho[kinds == 0] == 0).all()


def test_nonfinite_triage_trajectory_form_vs_reference_association(dev):
    """The select block's trajectory form (closed-form conditioned kernel): raw
    A_k, B_k, a_k, x_k, u_k with a rollout that leaves the finite range at x_k (every
    later x non-finite), a single non-finite x_k, x_N alone, and non-finite A_k, u_k,
    a_k; every kind resolved by the triage (no hand-over left)."""
    import torch
    from time_opt_ilqr_amd import _lib, engine
    Bn, n, m, N = 224, 12, 4, 100
    g = torch.Generator(device=dev)
    g.manual_seed(31)
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
    rng = np.random.default_rng(8)
    kinds = np.arange(Bn) % 7
    for b in range(Bn):
        k = int(rng.integers(1, N))
        i = int(rng.integers(0, n))
        if kinds[b] == 1:  # divergence: x_k .. x_N non-finite
            X[b, k:, i] = float("inf")
            X[b, k + 1:, :] = float("nan")
        elif kinds[b] == 2:
            X[b, k, i] = float("nan")
        elif kinds[b] == 3:
            X[b, N, i] = float("nan")
        elif kinds[b] == 4:
            A[b, k, i, (i + 1) % n] = float("nan")
        elif kinds[b] == 5:
            U[b, k, i % m] = float("-inf")
        elif kinds[b] == 6:
            ares[b, k, i] = float("nan")
    args = (A, B, ares, X, U, xg, ur, Q, Ri, Qf, 0.5)
    kw2 = dict(t_min=40, t_max=N, rho_reg=1.0, wrap_idx=[2])
    res = engine.propagate_traj(*args, **kw2)
    with _lib.options(reference_assoc=True):
        ref = engine.propagate_traj(*args, **kw2)
    torch.cuda.synchronize()
    _cmp(res, ref, "traj")
    with _lib.options(no_rerun=True):
        ho = engine.propagate_traj(*args, **kw2).status.cpu().numpy()
    assert ((ho & _lib.ST_HANDOVER) == 0).all(), np.nonzero(ho & _lib.ST_HANDOVER)[0][:8]
    assert (ho[kinds == 0] == 0).all()


def test_forced_handover_skips_the_triage(dev):
    """HOP_OPT_FORCE_HANDOVER recomputes every problem (the rerun is the LFT kernel,
    bitwise), non-finite inputs included."""
    import torch
    from time_opt_ilqr_amd import _lib, engine
    Bn, s, m, N = 16, 13, 4, 30
    A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(99, Bn, s, m, N)
    Q = Q.copy()
    Q[::3, 7, 2, 2] = np.nan
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)  # noqa
    args = (t(A), t(Bm), t(Q), t(Ri), t(z0), t(QT))
    with _lib.options(force_handover=True):
        f = engine.propagate(*args, t_min=5, t_max=N)
    with _lib.options(reference_assoc=True):
        r = engine.propagate(*args, t_min=5, t_max=N)
    torch.cuda.synchronize()
    assert torch.equal(f.status, r.status)
    assert torch.equal(f.J.nan_to_num(7.0), r.J.nan_to_num(7.0))
