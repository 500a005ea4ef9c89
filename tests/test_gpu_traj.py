"""GPU parity of the trajectory-form path (augmented.py:10-87 on the device):
hop_augment_* (batched builders) and hop_lft_sweep_traj_* (builders + the
propagator, fused into the sweep for s = 13, m = 4 fp64), against the oracle
pinned by the reference's own builders (tests/golden/traj_*.npz).

Tolerances:
  * builder blocks ............. 1e-14 relative (only the order of the Q e / e^T Q e
                                 sums differs from NumPy's)
  * J, well-conditioned terminal blocks (rho_reg = 1) ... 1e-9 relative, same T*
  * J, the reference's rho_reg = 1e-12 (terminal Schur complement 1e-12): the
    same bars as the augmented-form real captures in test_gpu_parity.py
    (the 1e-16 differences of the built blocks are amplified ~1e12)
"""
import os

import numpy as np
import pytest

from oracle import hop_oracle as orc

pytestmark = pytest.mark.gpu


def _t(x, dev, dtype=None):
    import torch
    return torch.as_tensor(np.ascontiguousarray(x), dtype=dtype or torch.float64, device=dev)


def _rel(got, ref):
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return float(np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-300))


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def _batch(seeds, n, m, N):
    ps = [orc.synth_traj_problem(int(s), n, m, N) for s in seeds]
    st = {k: np.stack([p[k] for p in ps]) for k in ("A", "B", "a_res", "X", "U", "xg", "u_ref",
                                                     "Q", "R", "alpha", "w")}
    st["P"] = np.stack([orc.terminal_weight(p["alpha"], n) for p in ps])
    st["R_inv"] = np.stack([orc.spd_inverse(orc.sym(p["R"]))[0] for p in ps])
    st["wrap_idx"] = ps[0]["wrap_idx"]
    return ps, st


def _blocks(p, rho, extra=None):
    Aa, Ba, Qa, _, z0, Ri = orc.augment_stage(list(p["A"]), list(p["B"]), p["a_res"], p["X"],
                                              p["U"], p["xg"], p["u_ref"], p["Q"], p["R"],
                                              p["w"], wrap_idx=p["wrap_idx"], rho_reg=rho,
                                              extra=extra)
    QT = orc.augment_terminal(p["X"], p["xg"], p["alpha"], wrap_idx=p["wrap_idx"], rho_reg=rho)
    return Aa, Ba, Qa, Ri, z0, QT


def _oracle(p, rho, n_use=None, extra=None):
    Aa, Ba, Qa, Ri, z0, QT = _blocks(p, rho, extra)
    return (Aa, Ba, Qa, Ri, z0, QT), orc.lft_sweep(Aa, Ba, Qa, Ri, z0, QT, n_use)


@pytest.fixture(params=[pytest.param("40", marks=pytest.mark.devbuild), "53"])
def traj_variant(request):
    """Fused s=13 trajectory kernels: 53 (default) closed-form stage inverses, 40 stage
    inverses by Gauss-Jordan sweeps on the built images (both + the rerun launch;
    40 is an A/B schedule of developer builds)."""
    from time_opt_ilqr_amd import _lib
    if request.param == "40" and not _lib.dev_build():
        pytest.skip("A/B schedule: developer builds only (HOP_DEV_BUILD=1)")
    with _lib.options(variant=40 if request.param == "40" else 0):
        yield request.param


@pytest.fixture
def unfused():
    """Context: the trajectory form through hop_augment + the augmented-form sweep."""
    from time_opt_ilqr_amd import _lib
    return lambda on=True: _lib.options(traj_unfused=on)


def _dev_args(st, dev, dtype=None):
    return [_t(st[k], dev, dtype) for k in ("A", "B", "a_res", "X", "U", "xg", "u_ref", "Q")]


@pytest.mark.parametrize("n,m,N,dt", [(12, 4, 40, "f64"), (4, 1, 33, "f64"), (2, 1, 20, "f64"),
                                      (5, 2, 17, "f32")])
def test_augment_kernel_matches_oracle_builders(dev, n, m, N, dt):
    import torch
    from time_opt_ilqr_amd import engine
    dtype = torch.float64 if dt == "f64" else torch.float32
    ps, st = _batch(range(900, 907), n, m, N)
    out = engine.augment(*_dev_args(st, dev, dtype), _t(st["P"], dev, dtype),
                         _t(st["w"], dev, dtype), wrap_idx=st["wrap_idx"])
    tol = 1e-14 if dt == "f64" else 2e-6
    for b, p in enumerate(ps):
        Aa, Ba, Qa, Ri, z0, QT = _blocks(p, 1e-12)
        assert _rel(out.A[b].cpu(), Aa) <= tol
        assert _rel(out.B[b].cpu(), Ba) <= tol
        assert _rel(out.Q[b].cpu(), Qa) <= tol
        assert _rel(out.QT[b].cpu(), QT) <= tol
        # structure is exact: A's bottom row [0 .. 0 1], B's zero row, raw blocks copied
        bottom = np.zeros((N, n + 1))
        bottom[:, n] = 1.0
        assert np.array_equal(out.A[b, :, n, :].double().cpu().numpy(), bottom)
        assert np.array_equal(out.B[b, :, n, :].double().cpu().numpy(), np.zeros((N, m)))
        assert np.array_equal(out.A[b, :, :n, :n].cpu().numpy(), st["A"][b].astype(
            out.A.cpu().numpy().dtype))
    assert out.z0.cpu().tolist() == [0.0] * n + [1.0]


@pytest.mark.parametrize("fused", [True, False])
def test_traj_sweep_vs_reference_goldens(dev, golden_dir, fused, traj_variant, unfused):
    """s = 13, m = 4: in-kernel builders (fused) and hop_augment + sweep (unfused)
    against the reference's builders + propagator (traj_synth_n12_m4_N100)."""
    with unfused(not fused):
        _traj_sweep_vs_reference_goldens(dev, golden_dir)


def _traj_sweep_vs_reference_goldens(dev, golden_dir):
    from time_opt_ilqr_amd import engine
    d = _load(golden_dir, "traj_synth_n12_m4_N100.npz")
    n, m, N = int(d["n"]), int(d["m"]), int(d["N"])
    for rho in (1.0, 1e-12):
        idx = [i for i, r in enumerate(d["rho_regs"]) if r == rho]
        ps, st = _batch(d["seeds"][idx], n, m, N)
        res = engine.propagate_traj(*_dev_args(st, dev), _t(st["R_inv"], dev), _t(st["P"], dev),
                                    _t(st["w"], dev), wrap_idx=st["wrap_idx"], rho_reg=rho,
                                    t_min=10, t_max=N)
        J = res.J.cpu().numpy()
        Jref = d["J"][idx]
        T_ref = np.argmin(Jref[:, 9:N], axis=1) + 10
        if rho == 1.0:
            assert _rel(J, Jref) <= 1e-9
            assert (res.status.cpu().numpy() == 0).all()
            assert res.t_star.cpu().tolist() == T_ref.tolist()
        else:
            assert _rel(J, Jref) <= 5e-2
            assert np.isfinite(J).all()


@pytest.mark.parametrize("n,m,N", [(4, 1, 60), (12, 4, 37), (2, 1, 25)])
def test_traj_sweep_batch_vs_oracle(dev, monkeypatch, n, m, N, traj_variant):
    """Batch tails (7 problems), n_use < N, the small-s and generic kernels behind
    the unfused path, and the fused path when the shape has it."""
    from time_opt_ilqr_amd import engine
    ps, st = _batch(range(950, 957), n, m, N)
    n_use = N - 3
    res = engine.propagate_traj(*_dev_args(st, dev), _t(st["R_inv"], dev), _t(st["P"], dev),
                                _t(st["w"], dev), wrap_idx=st["wrap_idx"], rho_reg=1.0,
                                n_use=n_use, t_min=2, t_max=n_use)
    J = res.J.cpu().numpy()
    for b, p in enumerate(ps):
        _, o = _oracle(p, 1.0, n_use)
        assert _rel(J[b], o["J"]) <= 1e-9
        T, _ = orc.select_horizon(o["J"][None], 2, n_use)
        assert int(res.t_star[b]) == int(T[0])
    assert (res.status.cpu().numpy() == 0).all()


def test_traj_fused_equals_unfused(dev, unfused):
    """The fused builder and hop_augment + the augmented-form sweep agree (1e-10:
    the s=13 augmented-form sweep runs the conditioned-prefix association)."""
    from time_opt_ilqr_amd import engine
    ps, st = _batch(range(970, 1003), 12, 4, 50)
    args = (*_dev_args(st, dev), _t(st["R_inv"], dev), _t(st["P"], dev), _t(st["w"], dev))
    a = engine.propagate_traj(*args, wrap_idx=st["wrap_idx"], rho_reg=1.0).J.cpu().numpy()
    with unfused():
        b = engine.propagate_traj(*args, wrap_idx=st["wrap_idx"], rho_reg=1.0).J.cpu().numpy()
    assert _rel(a, b) <= 1e-10


def test_traj_extra_stage_cost(dev):
    """extra_stage_cost (augmented.py:39-46) routes through hop_augment."""
    from time_opt_ilqr_amd import engine
    n, m, N = 12, 4, 24
    ps, st = _batch(range(990, 993), n, m, N)
    rng = np.random.default_rng(5)
    L = rng.standard_normal((3, N, n, n))
    cxx = 0.02 * L @ np.swapaxes(L, -1, -2)  # PSD: the stage blocks stay well-conditioned
    cx = rng.standard_normal((3, N, n)) * 0.1
    c0 = rng.uniform(0, 0.1, (3, N))
    res = engine.propagate_traj(*_dev_args(st, dev), _t(st["R_inv"], dev), _t(st["P"], dev),
                                _t(st["w"], dev), wrap_idx=st["wrap_idx"], rho_reg=1.0,
                                qxx_extra=_t(cxx, dev), qx_extra=_t(cx, dev),
                                c_extra=_t(c0, dev))
    for b, p in enumerate(ps):
        X = p["X"]
        lookup = {X[k].tobytes(): k for k in range(N)}

        def extra(x, u, b=b):
            k = lookup[np.asarray(x).tobytes()]
            return c0[b, k], cx[b, k], cxx[b, k]

        _, o = _oracle(p, 1.0, None, extra=extra)
        assert _rel(res.J[b].cpu(), o["J"]) <= 1e-9
    assert (res.status.cpu().numpy() == 0).all()


@pytest.mark.parametrize("tag,jtol", [("DI_N50", 1e-3), ("Quad_N160", 5e-2)])
def test_traj_real_first_select(dev, golden_dir, tag, jtol, traj_variant):
    """The first select block of ilqr_timeopt on the real systems (raw
    linearisation captured from the reference): T* equal, J at the real-capture
    bars (the Quadrotor shape runs the fused in-kernel builder)."""
    from time_opt_ilqr_amd import engine
    d = _load(golden_dir, f"traj_real_{tag}.npz")
    T_min, T_max = int(d["T_min"]), int(d["T_max"])
    T_use = min(T_max, len(d["U"]))
    x = lambda k: _t(d[k][None], dev)  # noqa: E731
    res = engine.propagate_traj(x("A"), x("B"), x("a_res"), x("X"), x("U"), _t(d["xg"], dev),
                                _t(d["u_ref"], dev), _t(d["Q"], dev), _t(d["R_inv"], dev),
                                _t(d["P"], dev), float(d["w"]),
                                wrap_idx=d["wrap_idx"].tolist(), n_use=T_use, t_min=T_min,
                                t_max=T_max)
    J = res.J[0].cpu().numpy()
    assert np.max(np.abs(J - d["J"]) / np.abs(d["J"])) <= jtol
    T_ref = int(np.argmin(d["J"][T_min - 1:T_max]) + T_min)
    assert int(res.t_star[0]) == T_ref


def test_select_from_trajectory_dropin_DI(dev, golden_dir):
    """The drop-in for solver.py:514-522 on the DoubleIntegrator's first select
    (F reproduces the captured residuals on the trajectory)."""
    from time_opt_ilqr_amd import horizon_selection as hs
    d = _load(golden_dir, "traj_real_DI_N50.npz")
    X, U, a_res = d["X"], d["U"], d["a_res"]
    table = {X[k].tobytes() + U[k].tobytes(): X[k + 1] + a_res[k] for k in range(len(U))}
    F = lambda x, u: table[np.asarray(x).tobytes() + np.asarray(u).tobytes()]  # noqa: E731
    J, T = hs.select_from_trajectory(F, list(d["A"]), list(d["B"]), X, U, d["xg"], d["u_ref"],
                                     d["Q"], d["R"], float(d["w"]), float(d["alpha"]),
                                     int(d["T_min"]), int(d["T_max"]))
    assert np.max(np.abs(J - d["J"]) / np.abs(d["J"])) <= 1e-3
    assert T == int(np.argmin(d["J"][int(d["T_min"]) - 1:int(d["T_max"])]) + int(d["T_min"]))


@pytest.mark.parametrize("fused", [True, False])
def test_traj_nonfinite_and_tiny_horizons(dev, fused, traj_variant, unfused):
    """A NaN in one problem's trajectory flags only that problem (FloatingPointError
    in the reference); n_use = 1 and t_min = t_max work on both paths."""
    with unfused(not fused):
        _traj_nonfinite_and_tiny_horizons(dev)


def _traj_nonfinite_and_tiny_horizons(dev):
    from time_opt_ilqr_amd import engine
    n, m, N = 12, 4, 20
    ps, st = _batch(range(1100, 1105), n, m, N)
    X = st["X"].copy()
    X[2, 7, 3] = np.nan
    st2 = dict(st)
    st2["X"] = X
    args = (*_dev_args(st2, dev), _t(st["R_inv"], dev), _t(st["P"], dev), _t(st["w"], dev))
    res = engine.propagate_traj(*args, wrap_idx=st["wrap_idx"], rho_reg=1.0, t_min=5, t_max=5)
    status = res.status.cpu().numpy()
    p2 = dict(ps[2])
    p2["X"] = X[2]
    _, o2 = _oracle(p2, 1.0)  # the oracle's status word and NaN pattern, exactly
    assert int(status[2]) == int(o2["status"]) == 4
    assert np.array_equal(np.isnan(res.J[2].cpu().numpy()), np.isnan(o2["J"]))
    assert (np.delete(status, 2) == 0).all()
    assert (np.delete(res.t_star.cpu().numpy(), 2) == 5).all()
    J = res.J.cpu().numpy()
    for b in (0, 1, 3, 4):
        _, o = _oracle(ps[b], 1.0)
        assert _rel(J[b], o["J"]) <= 1e-9
    one = engine.propagate_traj(*_dev_args(st, dev), _t(st["R_inv"], dev), _t(st["P"], dev),
                                _t(st["w"], dev), wrap_idx=st["wrap_idx"], rho_reg=1.0, n_use=1)
    for b in range(5):
        _, o = _oracle(ps[b], 1.0, 1)
        assert _rel(one.J[b].cpu(), o["J"]) <= 1e-9


@pytest.mark.parametrize("n,m,dt,tol", [(4, 1, "f32", 2e-3), (4, 2, "f32", 2e-3), (3, 2, "f64", 1e-9),
                                        (2, 1, "f64", 1e-9), (1, 1, "f64", 1e-9)])
def test_traj_small_fused_vs_unfused_and_oracle(dev, unfused, n, m, dt, tol):
    """Small s: the in-register builders of lft_small_traj_kernel against
    hop_augment + the small-s sweep and against the oracle (tails: 67 problems).
    fp64 batches up to kSmallRowGroupMax run unfused by default (augment + the
    row-group kernel); HOP_OPT_SMALL_LANE keeps them on the fused lane kernel."""
    import torch
    from time_opt_ilqr_amd import _lib, engine
    dtype = torch.float64 if dt == "f64" else torch.float32
    N = 45
    ps, st = _batch(range(1200, 1267), n, m, N)
    args = (*_dev_args(st, dev, dtype), _t(st["R_inv"], dev, dtype), _t(st["P"], dev, dtype),
            _t(st["w"], dev, dtype))
    kw = dict(wrap_idx=st["wrap_idx"], rho_reg=1.0, t_min=3, t_max=N)
    with _lib.options(small_lane=True):
        a = engine.propagate_traj(*args, **kw)  # fused, one problem per lane
    with unfused():
        b = engine.propagate_traj(*args, **kw)
    d = engine.propagate_traj(*args, **kw)
    Ja, Jb = a.J.double().cpu().numpy(), b.J.double().cpu().numpy()
    assert _rel(Ja, Jb) <= (1e-11 if dt == "f64" else 2e-3)  # fp32: the 2e-3 bar
    if dt == "f64" and (n + 1, m) in ((2, 1), (3, 1), (4, 1), (4, 2), (5, 1), (5, 2)):
        assert torch.equal(d.J, b.J)  # the default is the unfused row-group path
    else:
        assert torch.equal(d.J, a.J)
    for i in (0, 33, 66):
        _, o = _oracle(ps[i], 1.0)
        assert _rel(Ja[i], o["J"]) <= tol
    if dt == "f64":
        assert (a.status.cpu().numpy() == 0).all()
        for i in range(0, 67, 11):
            _, o = _oracle(ps[i], 1.0)
            T, _ = orc.select_horizon(o["J"][None], 3, N)
            assert int(a.t_star[i]) == int(T[0])


def test_traj_closed_form_kernel_alone(dev):
    """The closed-form trajectory kernel: nothing handed over at rho_reg = 1 (the
    result is not bitwise the reference-association kernel's), J within 1e-10 of
    the reference association (HOP_OPT_REFERENCE_ASSOC) and of the Gauss-Jordan
    conditioned kernel (variant 41, developer builds), same T*."""
    import torch
    from time_opt_ilqr_amd import _lib, engine
    ps, st = _batch(range(1200, 1237), 12, 4, 60)
    args = (*_dev_args(st, dev), _t(st["R_inv"], dev), _t(st["P"], dev), _t(st["w"], dev))
    kw = dict(wrap_idx=st["wrap_idx"], rho_reg=1.0, t_min=3, t_max=60)
    cf = engine.propagate_traj(*args, **kw)
    with _lib.options(reference_assoc=True):
        ref = engine.propagate_traj(*args, **kw)
    assert (cf.status.cpu().numpy() == 0).all()
    assert not torch.equal(cf.J, ref.J)
    assert _rel(cf.J.cpu().numpy(), ref.J.cpu().numpy()) <= 1e-10
    assert cf.t_star.cpu().tolist() == ref.t_star.cpu().tolist()
    if _lib.dev_build():
        with _lib.options(variant=54):
            cf2 = engine.propagate_traj(*args, **kw)
        with _lib.options(variant=41):
            gj = engine.propagate_traj(*args, **kw)
        assert (cf2.status.cpu().numpy() == 0).all()
        assert _rel(cf2.J.cpu().numpy(), gj.J.cpu().numpy()) <= 1e-10
    for b in (0, 36):
        _, o = _oracle(ps[b], 1.0)
        assert _rel(cf.J[b].cpu().numpy(), o["J"]) <= 1e-9


def test_reference_shaped_augmented_builders(dev):
    """augmented.build_augmented_sequence_QR / build_terminal_aug_list (the
    reference's names and return values, augmented.py:10-87) built on the device:
    against the oracle's builders, with a wrapped state, per-step residuals from
    the caller's F and an extra stage cost."""
    from time_opt_ilqr_amd import augmented
    rng = np.random.default_rng(0)
    n, m, N = 4, 2, 6
    A = [np.eye(n) + 0.1 * rng.standard_normal((n, n)) for _ in range(N)]
    B = [0.1 * rng.standard_normal((n, m)) for _ in range(N)]
    X = rng.standard_normal((N + 1, n))
    X[:, 2] *= 5.0
    U = rng.standard_normal((N, m))
    xg = rng.standard_normal(n)
    ur = rng.standard_normal(m)
    Q = np.diag(rng.uniform(1, 2, n))
    R = np.diag(rng.uniform(1, 2, m))

    def F(x, u):
        return 0.9 * x + 0.05 * np.concatenate([u, u])[:n]

    def extra(x, u):
        return 0.3 * float(x @ x), 0.6 * x, 0.6 * np.eye(n)

    for esc in (None, extra):
        Aa, Ba, Qa, Rl, z0, Ri = augmented.build_augmented_sequence_QR(
            F, A, B, X, U, xg, ur, Q, R, 0.03, wrap_idx=[2], extra_stage_cost=esc)
        res = [F(X[k], U[k]) - X[k + 1] for k in range(N)]
        oA, oB, oQ, oR, oz, oRi = orc.augment_stage(A, B, res, X, U, xg, ur, Q, R, 0.03,
                                                     wrap_idx=[2], extra=esc)
        assert _rel(np.array(Aa), oA) <= 1e-14 and _rel(np.array(Qa), oQ) <= 1e-14
        assert np.array_equal(np.array(Ba), oB) and np.allclose(Ri, oRi)
        assert np.array_equal(z0, oz) and len(Rl) == N
    alpha = np.array([1.0, 2.0, 3.0, 4.0])
    QT = augmented.build_terminal_aug_list(X, xg, alpha, wrap_idx=[2])
    oQT = orc.augment_terminal(X, xg, alpha, wrap_idx=[2])
    assert len(QT) == N and _rel(np.array(QT), oQT) <= 1e-14


# ---- tile64 raw linearisation (hop_linearize_tile64_* -> hop_lft_sweep_traj_tile64_*)

@pytest.mark.parametrize("sid,central", [(1, True), (1, False), (0, True), (4, False)])
def test_linearize_tile64_equals_batch_major(dev, sid, central):
    """hop_linearize_tile64_*: the same values as hop_linearize_f64 (fp64 output:
    bitwise; fp32 output: the fp64 result rounded once), laid out as tile64, with
    the trajectory copies X (rows 0 .. n_use) / U (rows < n_use) and zero padding
    slots; a ragged batch (70 = one full tile + 6) and n_use < N."""
    import torch
    from time_opt_ilqr_amd import engine
    from oracle import dyn_oracle as dyn
    n, m = dyn.DIMS[sid]
    Bn, N, n_use = 70, 23, 19
    rng = np.random.default_rng(40 + sid)
    X = 0.7 * rng.standard_normal((Bn, N + 1, n))
    U = 0.5 * rng.standard_normal((Bn, N, m))
    Xt, Ut = _t(X, dev), _t(U, dev)
    dt = dyn.DEFAULT_DT[sid]
    ref = engine.linearize(sid, Xt, Ut, dt, central=central, n_use=n_use)
    for odt in (torch.float64, torch.float32):
        t = engine.linearize(sid, Xt, Ut, dt, central=central, n_use=n_use, tile64=True,
                             tile64_dtype=odt)
        for got, want, steps in ((t.A, ref.A, n_use), (t.B, ref.B, n_use),
                                 (t.a_res, ref.a_res[..., None], n_use)):
            bm = engine.from_tile64(got)[:, :steps].reshape(Bn, steps, -1)
            w = want[:, :steps].reshape(Bn, steps, -1).to(odt)
            assert torch.equal(bm, w)
            assert (got.data[-1, :steps, :, Bn % 64:] == 0).all()  # padding slots
        assert torch.equal(engine.from_tile64(t.X)[:, :n_use + 1, :, 0], Xt[:, :n_use + 1].to(odt))
        assert torch.equal(engine.from_tile64(t.U)[:, :n_use, :, 0], Ut[:, :n_use].to(odt))


@pytest.mark.parametrize("n,m,dt", [(4, 1, "f32"), (4, 2, "f32"), (2, 1, "f64"), (3, 1, "f64"),
                                    (4, 1, "f64"), (4, 2, "f64")])
def test_traj_tile64_equals_batch_major_and_oracle(dev, n, m, dt):
    """hop_lft_sweep_traj_tile64_* on tile64 raw arrays (a ragged 67-problem batch):
    fp64 (the conditioned association + the LFT rerun on both layouts, s up to 5)
    bitwise the batch-major trajectory kernel's J / T* / status; fp32 (the same
    association) within the fp32 bar of it, T* equal except at near-ties; the oracle
    on a sample at the fp64 / fp32 bars."""
    import torch
    from time_opt_ilqr_amd import engine
    from time_opt_ilqr_amd import _lib
    dtype = torch.float64 if dt == "f64" else torch.float32
    N = 45
    ps, st = _batch(range(1300, 1367), n, m, N)
    raw = _dev_args(st, dev, dtype)
    shared = (raw[5], raw[6], raw[7], _t(st["R_inv"], dev, dtype), _t(st["P"], dev, dtype),
              _t(st["w"], dev, dtype))
    kw = dict(wrap_idx=st["wrap_idx"], rho_reg=1.0, t_min=3, t_max=N)
    with _lib.options(small_lane=True):  # fp64: the fused lane kernel, like tile64's
        bm = engine.propagate_traj(*raw[:5], *shared, **kw)
    t64 = [engine.to_tile64(x if x.dim() == 4 else x[..., None]) for x in raw[:5]]
    tl = engine.propagate_traj(*t64, *shared, **kw)
    if dt == "f64":
        assert torch.equal(tl.J, bm.J) and torch.equal(tl.t_star, bm.t_star)
        assert torch.equal(tl.status, bm.status) and (tl.status == 0).all()
        # the batch-major default (hop_augment + the row-group kernel): within 1e-11
        d = engine.propagate_traj(*raw[:5], *shared, **kw)
        assert _rel(d.J.cpu().numpy(), tl.J.cpu().numpy()) <= 1e-11
        assert torch.equal(d.t_star, tl.t_star)
    else:
        from test_gpu_configs import _same_sweep
        _same_sweep(tl, bm, False, tol=2e-3)
    J = tl.J.double().cpu().numpy()
    tol = 1e-9 if dt == "f64" else 2e-3
    for i in (0, 33, 63, 64, 66):
        _, o = _oracle(ps[i], 1.0)
        assert _rel(J[i], o["J"]) <= tol


def test_traj_tile64_config3_size_from_linearisation(dev):
    """Config 3's shape end to end (s = 5, m = 1, N = 200, B = 65,536, fp32): cart-pole
    rollouts linearised straight into fp32 tile64 (hop_linearize_tile64_f32), then
    the tile64 select; problems spread over the batch against the oracle's builders
    and propagator on the same (fp32-rounded) raw arrays, at the fp32 bar.  The cost
    is a well-conditioned one (the maker's zero angle weight puts 1e9 entries in
    E_k = (Q_aug + eps I)^-1, and rho_reg = 1e-12 Schur complements, neither of which
    an fp32 sweep resolves)."""
    import torch
    from time_opt_ilqr_amd import engine, systems
    F, x0, xg, u_ref, _, _, _, _, _, _, _, wrap, _ = systems.make_cartpole_swingup(N=200)
    Q, R, alpha, w = np.diag([1.0, 0.5, 2.0, 0.5]), np.array([[0.1]]), np.array([5.0, 5.0, 20.0,
                                                                                   5.0]), 0.03
    Bn, N, T_min = 65536, 200, 40
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    U = 2.0 * torch.randn((Bn, N, 1), device=dev, dtype=torch.float64, generator=g)
    X0 = torch.as_tensor(x0, device=dev) + 0.3 * torch.randn((Bn, 4), device=dev,
                                                               dtype=torch.float64, generator=g)
    X = engine.rollout(F.system_id, X0, U, F.dt)
    lin = engine.linearize(F.system_id, X, U, F.dt, central=True, tile64=True,
                           tile64_dtype=torch.float32)
    P = orc.terminal_weight(alpha, 4)
    Ri = orc.spd_inverse(orc.sym(R))[0]
    f = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float32), device=dev)  # noqa: E731
    res = engine.propagate_traj(lin.A, lin.B, lin.a_res, lin.X, lin.U, f(xg), f(u_ref), f(Q),
                                f(Ri), f(P), f([w]), wrap_idx=wrap, rho_reg=1.0, t_min=T_min,
                                t_max=N)
    torch.cuda.synchronize()
    assert torch.isfinite(res.J).all()
    Ab, Bb, ab = (engine.from_tile64(t).double().cpu().numpy() for t in (lin.A, lin.B, lin.a_res))
    Xb = engine.from_tile64(lin.X).double().cpu().numpy()[..., 0]
    Ub = engine.from_tile64(lin.U).double().cpu().numpy()[..., 0]
    for b in (0, 1, 63, 64, 40000, Bn - 1):
        p = dict(A=Ab[b], B=Bb[b], a_res=ab[b, :, :, 0], X=Xb[b], U=Ub[b], xg=xg, u_ref=u_ref,
                 Q=Q, R=R, alpha=alpha, w=w, wrap_idx=wrap)
        _, o = _oracle(p, 1.0)
        assert _rel(res.J[b].double().cpu().numpy(), o["J"]) <= 2e-3, b
