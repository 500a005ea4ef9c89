"""CPU: the dynamics / finite-difference linearisation row.

* the NumPy oracle (oracle/dyn_oracle.py) reproduces the reference's own outputs
  (tests/golden/lin_*.npz, made by importing the reference: make_golden.py --lin)
  bit for bit, for F, both linearisations and the affine residuals;
* the kernel's per-step arithmetic (csrc/dynamics.hpp, built for the host as
  dyn_host.cpp) reproduces them bit for bit too, and the oracle on random batches;
* hop_linearize_f64 / hop_dynamics_f64 reject bad calls before any launch, and
  the Python drop-ins refuse CPU tensors and arbitrary Python dynamics.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from oracle import dyn_oracle as dyn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["di", "cartpole", "quadrotor", "pointmass", "segway"]
_P = C.c_void_p


def _p(a):
    return a.ctypes.data_as(_P)


def _same(a, b):
    """bit-for-bit equal, NaN where the reference has NaN"""
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and np.array_equal(a, b, equal_nan=True)


@pytest.fixture(scope="module")
def dyn_host(tmp_path_factory):
    """g++ build of csrc/dynamics.hpp (the linearisation kernel's per-step math)."""
    d = tmp_path_factory.mktemp("dyn")
    so = str(d / "libdyn_host.so")
    src = os.path.join(REPO, "time_opt_ilqr_amd", "csrc", "dyn_host.cpp")
    # plain libm sin / cos / tan calls: GCC would otherwise fuse sin + cos of one
    # argument into sincos(), which differs from sin() in the last bit on some inputs
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-builtin-sin",
                           "-fno-builtin-cos", "-fno-builtin-tan", "-shared", "-fPIC",
                           "-DHOP_HD=", src, "-o", so])
    lib = C.CDLL(so)
    lib.dyn_host_linearize.argtypes = [C.c_int, C.c_double, _P, _P, C.c_int64, C.c_int, C.c_int,
                                       C.c_int] + [C.c_double] * 4 + [_P] * 4
    return lib


def _host_lin(lib, sid, X, U, dt, central, n_use=None):
    X, U = np.ascontiguousarray(X, float), np.ascontiguousarray(U, float)
    if X.ndim == 2:
        X, U = X[None], U[None]
    Bn, N, m = U.shape
    n = X.shape[-1]
    n_use = N if n_use is None else n_use
    A = np.full((Bn, N, n, n), -7.0)
    B = np.full((Bn, N, n, m), -7.0)
    ar = np.full((Bn, N, n), -7.0)
    Fx = np.full((Bn, N, n), -7.0)
    assert lib.dyn_host_linearize(sid, dt, _p(X), _p(U), Bn, N, n_use, int(central), 1e-5, 1e-5,
                                  1e-6, 1e-6, _p(A), _p(B), _p(ar), _p(Fx)) == 0
    return A, B, ar, Fx


@pytest.mark.parametrize("name", NAMES)
def test_oracle_dynamics_and_linearisations_vs_reference(golden_dir, name):
    d = np.load(os.path.join(golden_dir, f"lin_{name}.npz"))
    sid, dt = dyn.SYSTEMS[name], float(d["dt"])
    X, U = d["X"], d["U"]
    assert _same(dyn.dynamics(sid, X[:-1], U, dt), d["Fx"])
    for central, tag in ((False, "fwd"), (True, "cen")):
        A, B, ar = dyn.linearize(sid, X, U, dt, central=central)
        assert _same(A, d["A_" + tag]) and _same(B, d["B_" + tag]) and _same(ar, d["a_res"])
        A, B, ar = dyn.linearize_loop(sid, X, U, dt, central=central)
        assert _same(A, d["A_" + tag]) and _same(B, d["B_" + tag]) and _same(ar, d["a_res"])


def test_quadrotor_fixture_covers_every_guard(golden_dir):
    """the capture holds one state per NaN guard of systems.py:175-191; forward
    differences give all-NaN blocks there, central ones NaN columns"""
    d = np.load(os.path.join(golden_dir, "lin_quadrotor.npz"))
    bad = np.isnan(d["Fx"]).all(-1)
    assert sorted(np.flatnonzero(bad).tolist()) == [3, 5, 7, 9, 11]
    assert np.isnan(d["A_fwd"][bad]).all() and np.isnan(d["B_fwd"][bad]).all()
    assert np.isfinite(d["A_fwd"][~bad]).all()


@pytest.mark.parametrize("name", NAMES)
def test_kernel_math_vs_reference(dyn_host, golden_dir, name):
    """csrc/dynamics.hpp on the host == the reference, bit for bit (including the
    quadrotor, whose BLAS products are formed in OpenBLAS's FMA order)."""
    d = np.load(os.path.join(golden_dir, f"lin_{name}.npz"))
    sid, dt = dyn.SYSTEMS[name], float(d["dt"])
    for central, tag in ((False, "fwd"), (True, "cen")):
        A, B, ar, Fx = _host_lin(dyn_host, sid, d["X"], d["U"], dt, central)
        assert _same(Fx[0], d["Fx"]) and _same(ar[0], d["a_res"])
        assert _same(A[0], d["A_" + tag]) and _same(B[0], d["B_" + tag])


def _random_batch(sid, Bn, N, seed, scale):
    n, m = dyn.DIMS[sid]
    rng = np.random.default_rng(seed)
    X = scale * rng.standard_normal((Bn, N + 1, n))
    U = scale * rng.standard_normal((Bn, N, m))
    if sid == 2:
        U[..., 0] += 9.81
        X[0, 2, 7] = np.pi / 2  # singular pitch
        X[1, 4, 9] = 5e3        # |omega| guard
    return X, U


def close_lin(got, ref, f_tol=2e-15, ab_tol=1e-8):
    """(A, B, a_res) parity where the arithmetic may differ in the last bit of F:
    same NaN pattern; |dF| <= f_tol max(1, |F|); |dA|, |dB| <= ab_tol (1 ulp of F
    over h = 1e-5 is ~1e-10)"""
    for i, (g, r) in enumerate(zip(got, ref)):
        g, r = np.asarray(g), np.asarray(r)
        assert g.shape == r.shape
        assert np.array_equal(np.isnan(g), np.isnan(r))
        ok = ~np.isnan(r)
        tol = ab_tol if i < 2 else f_tol * np.maximum(1.0, np.abs(r[ok]))
        assert (np.abs(g[ok] - r[ok]) <= tol).all(), float(np.max(np.abs(g[ok] - r[ok])))


@pytest.mark.parametrize("sid", range(5))
def test_kernel_math_vs_oracle_random_batch(dyn_host, sid):
    """random batches incl. quadrotor guard states; bit-exact except the quadrotor:
    its vectorised oracle forms the 3x3 products without FMA (the reference's BLAS
    and the kernel use FMA chains) and NumPy's SIMD tan differs from libm's in the
    last bit on ~0.5% of arguments, so F agrees to 1 ulp there (the per-call loop
    oracle, which is the reference's arithmetic, is compared the same way)"""
    X, U = _random_batch(sid, 6, 30, 100 + sid, 2.0)
    dt = dyn.DEFAULT_DT[sid]
    for central in (False, True):
        A, B, ar, _ = _host_lin(dyn_host, sid, X, U, dt, central)
        ref = dyn.linearize(sid, X, U, dt, central=central)
        if sid == 2:
            close_lin((A, B, ar), ref)
        else:
            assert _same(A, ref[0]) and _same(B, ref[1]) and _same(ar, ref[2])
        Al, Bl, arl = dyn.linearize_loop(sid, X[0], U[0], dt, central=central)
        if sid == 2:
            close_lin((A[0], B[0], ar[0]), (Al, Bl, arl))
        else:
            assert _same(A[0], Al) and _same(B[0], Bl) and _same(ar[0], arl)


def test_kernel_math_n_use_leaves_the_tail(dyn_host):
    X, U = _random_batch(1, 3, 12, 7, 1.0)
    A, B, ar, Fx = _host_lin(dyn_host, 1, X, U, 0.02, False, n_use=5)
    assert (A[:, 5:] == -7.0).all() and (B[:, 5:] == -7.0).all() and (ar[:, 5:] == -7.0).all()
    Ao, Bo, aro = dyn.linearize(1, X[:, :6], U[:, :5], 0.02)
    assert _same(A[:, :5], Ao) and _same(B[:, :5], Bo) and _same(ar[:, :5], aro)


@pytest.fixture(scope="module")
def lib():
    from time_opt_ilqr_amd import _lib, build
    build.build(verbose=False)
    return _lib.load()


def test_linearize_entry_validation_without_gpu(lib):
    nul = None
    args = lambda sys_id, batch, na, nu, cen: (sys_id, 0.05, nul, nul, batch, na, nu, cen,  # noqa
                                               1e-5, 1e-5, 1e-6, 1e-6, nul, nul, nul, nul, nul)
    assert lib.hop_linearize_f64(*args(5, 1, 10, 10, 0)) == -1
    assert b"system" in lib.hop_last_error()
    assert lib.hop_linearize_f64(*args(2, -1, 10, 10, 0)) == -1
    assert lib.hop_linearize_f64(*args(2, 1, 10, 11, 0)) == -1
    assert lib.hop_linearize_f64(*args(2, 1, 10, 10, 2)) == -1
    assert lib.hop_linearize_f64(*args(2, 1, 10, 10, 0)) == -1  # null pointers
    assert lib.hop_linearize_f64(*args(2, 0, 10, 10, 0)) == 0   # empty batch: nothing to do
    assert lib.hop_linearize_f64(*args(2, 4, 10, 0, 0)) == 0    # len(U) == 0: [] in the reference
    assert lib.hop_dynamics_f64(7, 0.05, nul, 12, nul, 4, 3, nul, 12, nul) == -1
    assert lib.hop_dynamics_f64(2, 0.05, nul, 11, nul, 4, 3, nul, 12, nul) == -1
    assert lib.hop_dynamics_f64(2, 0.05, nul, 12, nul, 4, 0, nul, 12, nul) == 0
    n, m = C.c_int32(), C.c_int32()
    for sid, dims in dyn.DIMS.items():
        assert lib.hop_system_dims(sid, C.byref(n), C.byref(m)) == 0
        assert (n.value, m.value) == dims
    assert lib.hop_system_dims(-1, nul, nul) == -1


def test_linearize_has_no_cpu_fallback():
    import torch
    from time_opt_ilqr_amd import HopError, engine, linearization, systems
    X = torch.zeros((1, 4, 4), dtype=torch.float64)
    U = torch.zeros((1, 3, 1), dtype=torch.float64)
    with pytest.raises(HopError):
        engine.linearize("cartpole", X, U, 0.02)
    with pytest.raises(TypeError):
        linearization.linearize_forward_diff_traj(lambda x, u: x, np.zeros((4, 4)), np.zeros((3, 1)))
    F = systems.make_cartpole_swingup()[0]
    assert (F.system_id, F.n, F.m, F.dt) == (1, 4, 1, 0.02)


def test_makers_match_reference_problem_data():
    """the makers' problem data equal the reference's (systems.py), recorded as
    JSON-free constants in the oracle fixtures' generator: spot-check the shapes
    and the values the engine consumes"""
    from time_opt_ilqr_amd import systems
    for name, mk in systems.MAKERS.items():
        F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, extra = mk()
        assert x0.shape == (F.n,) and xg.shape == (F.n,) and u_ref.shape == (F.m,)
        assert Q.shape == (F.n, F.n) and R.shape == (F.m, F.m)
        assert 1 <= T_min <= T_max
    c, cx, cxx = systems.obstacle_stage_cost(np.array([0.0, 0.2, 0.0, 0.0]))
    assert c > 6.0 and cx.shape == (4,) and cxx.shape == (4, 4)
