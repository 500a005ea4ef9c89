"""GPU parity of the batched dynamics + finite-difference linearisation
(hop_linearize_f64 / hop_dynamics_f64, csrc/linearize.hip) against the
reference's own outputs (tests/golden/lin_*.npz) and the oracle
(oracle/dyn_oracle.py, pinned bit for bit by those fixtures).

Tolerances (written where they are used):
  * double integrator, point mass, segway: bit-exact (no libm call; the kernel
    is compiled without FMA contraction and angle_normalize is exact)
  * cart-pole, quadrotor: the device's sin / cos / tan (ROCm ocml) may differ
    from glibc / NumPy in the last bit, so F is compared to 2e-15 max(1, |F|)
    and A, B (1 ulp of F over h = 1e-5 ~ 1e-10) to 1e-8 absolute; the NaN
    pattern (quadrotor guards, forward-difference NaN blocks) must be identical.
"""
import os

import numpy as np
import pytest

from oracle import dyn_oracle as dyn

pytestmark = pytest.mark.gpu

NAMES = ["di", "cartpole", "quadrotor", "pointmass", "segway"]
EXACT = {0, 3, 4}


def _t(x, dev):
    import torch
    return torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)


def _np(t):
    return t.detach().cpu().numpy()


def _same(a, b):
    return np.asarray(a).shape == np.asarray(b).shape and np.array_equal(a, b, equal_nan=True)


def _close(got, ref, f_tol=2e-15, ab_tol=1e-8, kind="ab"):
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape
    assert np.array_equal(np.isnan(got), np.isnan(ref)), "NaN pattern differs"
    # +-inf (e.g. a_res = F(x_k) - x_{k+1} with x_{k+1} = inf) must match exactly
    assert np.array_equal(got[np.isinf(ref)], ref[np.isinf(ref)]), "inf entries differ"
    ok = np.isfinite(ref)
    tol = ab_tol if kind == "ab" else f_tol * np.maximum(1.0, np.abs(ref[ok]))
    err = np.abs(got[ok] - ref[ok])
    assert (err <= tol).all(), float(err.max())
    return float(err.max()) if err.size else 0.0


def _check(sid, got, ref):
    """got/ref = (A, B, a_res[, Fx]); exact for the libm-free systems"""
    for i, (g, r) in enumerate(zip(got, ref)):
        if sid in EXACT:
            assert _same(g, r), (sid, i)
        else:
            _close(g, r, kind="ab" if i < 2 else "f")


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("central", [False, True])
def test_linearize_vs_reference_fixture(dev, golden_dir, name, central):
    from time_opt_ilqr_amd import engine
    d = np.load(os.path.join(golden_dir, f"lin_{name}.npz"))
    sid, dt = dyn.SYSTEMS[name], float(d["dt"])
    r = engine.linearize(sid, _t(d["X"], dev)[None], _t(d["U"], dev)[None], dt, central=central,
                         want_fx=True)
    tag = "cen" if central else "fwd"
    _check(sid, (_np(r.A)[0], _np(r.B)[0], _np(r.a_res)[0], _np(r.Fx)[0]),
           (d["A_" + tag], d["B_" + tag], d["a_res"], d["Fx"]))


@pytest.mark.parametrize("name", NAMES)
def test_reference_shaped_dropins(dev, golden_dir, name):
    """linearization.linearize_{forward,central}_diff_traj / compute_affine_residuals
    with a systems.make_* F: same lists as the reference's"""
    from time_opt_ilqr_amd import linearization as lin, systems
    d = np.load(os.path.join(golden_dir, f"lin_{name}.npz"))
    sid = dyn.SYSTEMS[name]
    mk = list(systems.MAKERS.values())[sid]
    F = mk(dt=float(d["dt"]))[0]
    X, U = d["X"], d["U"]
    Af, Bf = lin.linearize_forward_diff_traj(F, X, U)
    Ac, Bc = lin.linearize_central_diff_traj(F, X, U)
    res = lin.compute_affine_residuals(F, X, U)
    assert len(Af) == len(Bf) == len(Ac) == len(res) == len(U)
    assert res[0].shape == (F.n, 1)
    _check(sid, (np.array(Af), np.array(Bf), np.array(res)[..., 0]),
           (d["A_fwd"], d["B_fwd"], d["a_res"]))
    _check(sid, (np.array(Ac), np.array(Bc)), (d["A_cen"], d["B_cen"]))
    fx = F(X[1], U[1])
    _check(sid, (fx,), (d["Fx"][1],)) if sid in EXACT else _close(fx, d["Fx"][1], kind="f")
    assert lin.linearize_forward_diff_traj(F, X[:1], U[:0]) == ([], [])


def _random_batch(sid, Bn, N, seed, scale):
    n, m = dyn.DIMS[sid]
    rng = np.random.default_rng(seed)
    X = scale * rng.standard_normal((Bn, N + 1, n))
    U = scale * rng.standard_normal((Bn, N, m))
    if sid == 2:
        U[..., 0] += 9.81
        X[0, 2, 7] = np.pi / 2      # |cos(pitch)| guard
        X[1, 4, 9] = 5e3            # |omega| guard
        X[2, 6, 0] = np.inf         # non-finite state
        X[3, 1, 7] = np.pi / 2 - 1e-3 - 5e-6  # only the +h pitch column trips the guard
    return X, U


@pytest.mark.parametrize("sid", range(5))
@pytest.mark.parametrize("central", [False, True])
def test_linearize_random_batch_vs_oracle(dev, sid, central):
    """ragged batch (not a multiple of the 64-step tile), guard states included"""
    from time_opt_ilqr_amd import engine
    X, U = _random_batch(sid, 37, 29, 500 + sid, 1.5)
    dt = dyn.DEFAULT_DT[sid]
    r = engine.linearize(sid, _t(X, dev), _t(U, dev), dt, central=central)
    ref = dyn.linearize(sid, X, U, dt, central=central)
    if sid == 2:  # the vectorised oracle's 3x3 products carry no FMA: 1 ulp in F
        for i, (g, rr) in enumerate(zip((_np(r.A), _np(r.B), _np(r.a_res)), ref)):
            _close(g, rr, kind="ab" if i < 2 else "f")
    else:
        _check(sid, (_np(r.A), _np(r.B), _np(r.a_res)), ref)


def test_linearize_n_use_and_nullable_outputs(dev):
    """steps k >= n_use and the nullable a_res / Fx are left untouched"""
    import torch
    from time_opt_ilqr_amd import _lib
    lib = _lib.load()
    X, U = _random_batch(4, 5, 40, 9, 1.0)
    Xt, Ut = _t(X, dev), _t(U, dev)
    A = torch.full((5, 40, 4, 4), -7.0, dtype=torch.float64, device=dev)
    B = torch.full((5, 40, 4, 1), -7.0, dtype=torch.float64, device=dev)
    rc = lib.hop_linearize_f64(4, 0.02, _lib.ptr(Xt), _lib.ptr(Ut), 5, 40, 17, 0, 1e-5, 1e-5,
                               1e-6, 1e-6, _lib.ptr(A), _lib.ptr(B), None, None,
                               _lib.stream_handle(dev))
    _lib.check(rc)
    torch.cuda.synchronize()
    An, Bn = _np(A), _np(B)
    assert (An[:, 17:] == -7.0).all() and (Bn[:, 17:] == -7.0).all()
    Ao, Bo, _ = dyn.linearize(4, X[:, :18], U[:, :17], 0.02)
    assert _same(An[:, :17], Ao) and _same(Bn[:, :17], Bo)


@pytest.mark.parametrize("sid", range(5))
def test_dynamics_kernel_vs_oracle(dev, sid):
    from time_opt_ilqr_amd import engine
    X, U = _random_batch(sid, 9, 33, 40 + sid, 2.0)
    X = X[:, :-1]
    dt = dyn.DEFAULT_DT[sid]
    out = _np(engine.dynamics(sid, _t(X, dev), _t(U, dev), dt))
    ref = dyn.dynamics(sid, X, U, dt)
    if sid in EXACT:
        assert _same(out, ref)
    else:
        _close(out, ref, kind="f")


def test_quadrotor_bench_size_properties(dev):
    """at the bench size (4096 problems x 100 steps): a sample of problems against
    the oracle, forward vs central differences close, the residual equal to F - x'"""
    import torch
    from time_opt_ilqr_amd import engine
    Bn, N = 4096, 100
    X, U = _random_batch(2, Bn, N, 77, 0.3)
    X[..., :3] += 2.0
    Xt, Ut = _t(X, dev), _t(U, dev)
    fw = engine.linearize(2, Xt, Ut, 0.05, want_fx=True)
    ce = engine.linearize(2, Xt, Ut, 0.05, central=True)
    torch.cuda.synchronize()
    pick = np.array([0, 1, 2, 3, 511, 2048, 4095])
    ref = dyn.linearize(2, X[pick], U[pick], 0.05)
    for i, (g, rr) in enumerate(zip((fw.A, fw.B, fw.a_res), ref)):
        _close(_np(g[pick]), rr, kind="ab" if i < 2 else "f")
    ok = torch.isfinite(fw.A).flatten(2).all(-1) & torch.isfinite(ce.A).flatten(2).all(-1)
    assert ok.float().mean().item() > 0.99
    assert (fw.A - ce.A).abs()[ok].max().item() < 1e-3
    res = fw.Fx - Xt[:, 1:]
    assert torch.equal(torch.nan_to_num(res, 1.0), torch.nan_to_num(fw.a_res, 1.0))


def test_linearize_feeds_the_select_block(dev):
    """device linearisation -> propagate_traj (fused builders + sweep + argmin)
    gives the same T* / J as the oracle's linearisation fed to the same sweep"""
    import torch
    from time_opt_ilqr_amd import engine, systems
    from oracle import hop_oracle as orc
    F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, _ = systems.make_quadrotor(N=60)
    T_min, T_max = 10, 60
    rng = np.random.default_rng(3)
    Bn = 8
    X = x0 + 0.1 * rng.standard_normal((Bn, N + 1, 12))
    U = u_ref + 0.1 * rng.standard_normal((Bn, N, 4))
    lin = engine.linearize(F.system_id, _t(X, dev), _t(U, dev), F.dt)
    Ao, Bo, aro = dyn.linearize(2, X, U, F.dt)
    P = orc.terminal_weight(alpha, 12)
    Ri = orc.spd_inverse(orc.sym(R))[0]
    # rho_reg = 1: a well-conditioned terminal block, so 1e-10 differences in A
    # are not amplified (test_gpu_traj.py documents the 1e-12 case)
    common = dict(wrap_idx=wrap_idx, t_min=T_min, t_max=T_max, rho_reg=1.0)
    args = (_t(X, dev), _t(U, dev), _t(xg, dev), _t(u_ref, dev), _t(Q, dev), _t(Ri, dev),
            _t(P, dev), _t(np.array([w]), dev))
    g = engine.propagate_traj(lin.A, lin.B, lin.a_res, *args, **common)
    o = engine.propagate_traj(_t(Ao, dev), _t(Bo, dev), _t(aro, dev), *args, **common)
    torch.cuda.synchronize()
    assert torch.equal(g.t_star, o.t_star)
    Jg, Jo = _np(g.J), _np(o.J)
    assert np.max(np.abs(Jg - Jo) / np.maximum(np.abs(Jo), 1.0)) < 1e-6
