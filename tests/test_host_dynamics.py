"""Host side of the Python-callable path (time_opt_ilqr_amd/host_dynamics.py): a user
dynamics F(x, u) or stage cost the device has no kernel for is evaluated on the host
per problem, the reference's own call form.  CPU tests:

  * linearize equals the oracle's loop form (oracle/dyn_oracle.py _linearize_loop)
    bit for bit on random trajectories with the quadrotor's NaN guards tripped, and the
    reference's fixtures (tests/golden/lin_*.npz) bit for bit -- the oracle dynamics
    are pinned to those fixtures bit for bit, so the same F gives the same quotients;
  * rollout / cost_true / linesearch against the reference's captured calls
    (tests/golden/ilqr_*.npz: X0 / X_big, cost_J, every forward_linesearch_fixedT
    call of the reference's run) and the oracle's line search on a mixed batch.

Tolerances are written where they are used.  The device side of this path (select,
Riccati, accept on the GPU around these host evaluations) is
tests/test_gpu_forward.py::test_ilqr_outer_loop_host_callables_vs_reference.
"""
import os

import numpy as np
import pytest

from oracle import dyn_oracle as dyn
from oracle import ilqr_oracle as io
from time_opt_ilqr_amd import host_dynamics as hd

TAGS = ["di", "cartpole", "quadrotor", "pointmass", "segway"]


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and np.array_equal(a, b, equal_nan=True)


def _rel(got, ref):
    got, ref = np.asarray(got, float), np.asarray(ref, float)
    return float(np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-300))


def _obs(tag):
    if tag != "pointmass":
        return None, None
    from time_opt_ilqr_amd.systems import OBSTACLES
    rows = np.array([[o[0], o[1], r, wt] for o, r, wt in OBSTACLES])
    return rows, (lambda x, u: io.obstacle_cost(x, rows))


def _random_traj(sid, N, seed):
    n, m = dyn.DIMS[sid]
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((N + 1, n))
    U = rng.standard_normal((N, m))
    if sid == 2:
        U[:, 0] += 9.81
        X[2, 7] = np.pi / 2                  # |cos(pitch)| guard: F is NaN
        X[4, 9] = 5e3                        # |omega| guard
        X[6, 0] = np.inf                     # non-finite state
        X[1, 7] = np.pi / 2 - 1e-3 - 5e-6    # only the +h pitch column trips the guard
    return X, U


@pytest.mark.parametrize("sid", range(5))
@pytest.mark.parametrize("central", [False, True])
def test_linearize_equals_oracle_loop_bitwise(sid, central):
    X, U = _random_traj(sid, 12, 40 + sid)
    F = dyn._scalar_F(sid, 0.05)
    with np.errstate(all="ignore"):
        got = hd.linearize(F, X, U, central=central)
        ref = dyn._linearize_loop(F, X, U, central, 1e-5, 1e-5, 1e-6, 1e-6)
    for g, r in zip(got, ref):
        assert _same(g, r)
    if sid == 2:
        assert np.isnan(got[0]).any()  # the guards were tripped


@pytest.mark.parametrize("tag", TAGS)
def test_linearize_vs_reference_fixture_bitwise(golden_dir, tag):
    d = np.load(os.path.join(golden_dir, f"lin_{tag}.npz"))
    F = dyn._scalar_F(dyn.SYSTEMS[tag], float(d["dt"]))
    for central, k in ((False, "fwd"), (True, "cen")):
        A, B, a = hd.linearize(F, d["X"], d["U"], central=central)
        assert _same(A, d["A_" + k]) and _same(B, d["B_" + k]) and _same(a, d["a_res"])


@pytest.mark.parametrize("tag", TAGS)
def test_rollout_and_cost_vs_reference_captures(golden_dir, tag):
    d = np.load(os.path.join(golden_dir, f"ilqr_{tag}.npz"))
    sid, dt, N = dyn.SYSTEMS[tag], float(d["dt"]), int(d["N"])
    wrap = [int(i) for i in d["wrap_idx"]]
    F = dyn._scalar_F(sid, dt)
    X0 = hd.rollout(F, d["x0"], np.tile(d["u_ref"].reshape(1, -1), (N, 1)))
    assert _same(X0, d["X0"])  # the oracle dynamics are the reference's bit for bit
    Xb = hd.rollout(F, d["x0"], d["U_big"], max_state_norm=1e3)
    assert _same(np.isnan(Xb), np.isnan(d["X_big"]))
    _, extra = _obs(tag)
    for T, Jr in zip(d["cost_T"], d["cost_J"]):
        J = hd.cost_true(d["X"], d["U"], d["xg"], d["u_ref"], d["Q"], d["R"], d["Qf"],
                         float(d["w"]), int(T), wrap, extra)
        assert abs(J - float(Jr)) <= 1e-13 * max(1.0, abs(float(Jr)))
    assert hd.cost_true(d["X"], d["U"], d["xg"], d["u_ref"], d["Q"], d["R"], d["Qf"],
                        float(d["w"]), 0, wrap, extra) == float("inf")


@pytest.mark.parametrize("tag", TAGS)
def test_linesearch_vs_reference_captures(golden_dir, tag):
    """every captured forward_linesearch_fixedT call of the reference's run"""
    d = np.load(os.path.join(golden_dir, f"ilqr_{tag}.npz"))
    sid, dt = dyn.SYSTEMS[tag], float(d["dt"])
    wrap = [int(i) for i in d["wrap_idx"]]
    F = dyn._scalar_F(sid, dt)
    _, extra = _obs(tag)
    args = (d["xg"], d["u_ref"], d["Q"], d["R"], d["Qf"], float(d["w"]), wrap)
    for i in range(int(d["n_fwd"])):
        g = lambda k: d[f"f{i}_{k}"]  # noqa: E731
        Xn, Un, J, J0, ai = hd.linesearch(F, g("X"), g("U"), int(g("T_star")), g("K"), g("k"),
                                          args, io.ALPHAS, extra)
        assert (ai >= 0) == bool(g("acc")), (i, ai)
        Jr = float(g("J"))
        # the reference sums the same terms in the same order: 1e-13 covers NumPy's
        # pairwise e @ Q @ e against the reference's expression
        assert abs(J - Jr) <= 1e-13 * max(1.0, abs(Jr))
        assert _rel(Xn, g("X_new")) <= 1e-13 and _rel(Un, g("U_new")) <= 1e-13


def test_linesearch_mixed_batch_vs_oracle(golden_dir):
    """quadrotor with the feed-forward scaled per problem (x1 .. x300, negated):
    every outcome -- accepted at several step sizes, NaN-guard rejections, nothing
    accepted, T* = 0 and short horizons -- equals the oracle's forward_linesearch"""
    d = np.load(os.path.join(golden_dir, "ilqr_quadrotor.npz"))
    g = lambda k: d[f"f1_{k}"]  # noqa: E731
    dt, N, T0 = float(d["dt"]), int(d["N"]), int(g("T_star"))
    wrap = [int(i) for i in d["wrap_idx"]]
    F = dyn._scalar_F(2, dt)
    K = np.zeros((N, 4, 12))
    k0 = np.zeros((N, 4))
    K[:T0], k0[:T0] = g("K"), g("k")
    args = (d["xg"], d["u_ref"], d["Q"], d["R"], d["Qf"], float(d["w"]), wrap)
    seen = set()
    for sc, T in [(1, T0), (3, T0), (10, T0), (30, T0), (100, T0), (300, T0), (-1, T0),
                  (-10, T0), (0.3, T0), (1, 0), (1, 1), (1, 5), (1, T0 // 2), (1, N)]:
        k = k0 * sc
        with np.errstate(all="ignore"):
            Xn, Un, J, _, ai = hd.linesearch(F, g("X"), g("U"), T, K, k, args, io.ALPHAS)
            Xo, Uo, Jo, ok, ao = io.forward_linesearch(2, dt, g("X"), g("U"), d["xg"], d["u_ref"],
                                                       d["Q"], d["R"], d["Qf"], float(d["w"]), T,
                                                       k, K, wrap_idx=wrap)
        seen.add(ai)
        assert ai == ao and (ai >= 0) == ok
        assert J == Jo or (np.isinf(J) and np.isinf(Jo))
        assert _same(Xn, Xo) and _same(Un, Uo)
    assert -1 in seen and 0 in seen and len(seen) >= 3, seen


def test_stage_cost_terms_and_host_dynamics_wrapper():
    rows, extra = _obs("pointmass")
    rng = np.random.default_rng(3)
    X = rng.uniform(-2.5, 2.5, (9, 4))
    U = rng.standard_normal((8, 2))
    c, cx, cxx = hd.stage_cost_terms(extra, X, U)
    assert c.shape == (8,) and cx.shape == (8, 4) and cxx.shape == (8, 4, 4)
    for k in range(8):
        rc, rcx, rcxx = io.obstacle_cost(X[k], rows)
        assert c[k] == rc and _same(cx[k], rcx) and _same(cxx[k], rcxx)
    Fh = hd.HostDynamics(dyn._scalar_F(3, 0.1), 4, 2)
    assert Fh(X[0], U[0]).shape == (4,)
    # a callable returning the wrong size ends the rollout like a non-finite state
    X1 = hd.rollout(lambda x, u: np.zeros(3), X[0], U)
    assert np.isnan(X1[1:]).all() and _same(X1[0], X[0])


@pytest.mark.parametrize("sid", range(5))
@pytest.mark.parametrize("central", [False, True])
def test_linearize_batch_vectorized_equals_per_call(sid, central):
    """HostDynamics(vectorized=True): one F call over every perturbed point of every
    step and problem gives the per-call quotients -- bit for bit where F's row results
    do not depend on the stacking (every system but the quadrotor, whose stacked 3x3
    matmuls may round differently from single ones: 1e-8 absolute on A, B as the
    device linearisation's bar, the NaN pattern equal)"""
    n, m = dyn.DIMS[sid]
    F = dyn._scalar_F(sid, 0.05)
    X = np.stack([_random_traj(sid, 9, 70 + b)[0] for b in range(3)])
    U = np.stack([_random_traj(sid, 9, 70 + b)[1] for b in range(3)])
    X[1, 3, 0] = np.nan
    per = hd.linearize_batch(hd.HostDynamics(F, n, m), X, U, central=central)
    vec = hd.linearize_batch(hd.HostDynamics(F, n, m, vectorized=True), X, U, central=central)
    for g, r in zip(vec, per):
        assert g.shape == r.shape
        if sid == 2:
            assert np.array_equal(np.isnan(g), np.isnan(r))
            ok = np.isfinite(r)
            assert np.all(np.abs(g[ok] - r[ok]) <= 1e-8)
        else:
            assert _same(g, r)


@pytest.mark.parametrize("tag", TAGS)
def test_rollout_batch_vectorized_vs_per_call(golden_dir, tag):
    """rollout_batch: every problem a time step at a time (one F call per step) against
    rollout per problem: the divergence cut at the same step, the states equal (bit for
    bit but for the quadrotor's stacked 3 x 3 matmuls: 1e-13 relative)"""
    d = np.load(os.path.join(golden_dir, f"ilqr_{tag}.npz"))
    sid, dt, N = dyn.SYSTEMS[tag], float(d["dt"]), int(d["N"])
    n, m = dyn.DIMS[sid]
    F = dyn._scalar_F(sid, dt)
    X0 = np.stack([d["x0"], d["x0"], d["x0"] + 0.1])
    U = np.stack([d["U_big"], np.tile(d["u_ref"].reshape(1, -1), (N, 1)), d["U"]])
    per = hd.rollout_batch(hd.HostDynamics(F, n, m), X0, U, max_state_norm=1e3)
    vec = hd.rollout_batch(hd.HostDynamics(F, n, m, vectorized=True), X0, U, max_state_norm=1e3)
    assert np.array_equal(np.isnan(per), np.isnan(vec))
    assert np.array_equal(np.isnan(per[0]), np.isnan(d["X_big"]))
    if sid == 2:
        assert _rel(np.nan_to_num(vec), np.nan_to_num(per)) <= 1e-13
    else:
        assert _same(vec, per)


@pytest.mark.parametrize("tag", ["quadrotor", "pointmass", "cartpole"])
def test_linesearch_batch_vectorized_vs_per_call(golden_dir, tag):
    """linesearch_batch: all (problem, step size) rollouts together against the per-call
    line search per problem, on a batch built from a captured call with the feed-forward
    scaled per problem (several accepted step sizes, rejections, NaN guards on the
    quadrotor), one inactive problem, T* = 0 and short horizons: the same accepted index
    everywhere, J / X' / U' equal to rounding (1e-12)"""
    d = np.load(os.path.join(golden_dir, f"ilqr_{tag}.npz"))
    sid, dt, N = dyn.SYSTEMS[tag], float(d["dt"]), int(d["N"])
    n, m = dyn.DIMS[sid]
    g = lambda k: d[f"f1_{k}"]  # noqa: E731
    T0 = int(g("T_star"))
    F = dyn._scalar_F(sid, dt)
    _, extra = _obs(tag)
    wrap = [int(i) for i in d["wrap_idx"]]
    args = (d["xg"], d["u_ref"], d["Q"], d["R"], d["Qf"], float(d["w"]), wrap)
    sc = np.array([1, 3, 10, 30, 100, 300, -1, -10, 0.3])
    Bn = 14
    X = np.stack([g("X")] * Bn)
    U = np.stack([g("U")] * Bn)
    K = np.zeros((Bn, N, m, n))
    k = np.zeros((Bn, N, m))
    K[:, :T0] = g("K")
    k[:, :T0] = g("k").reshape(T0, m)[None] * sc[np.arange(Bn) % len(sc), None, None]
    T = np.full(Bn, T0)
    T[9:13] = [0, 1, 5, T0 // 2]
    active = np.ones(Bn, dtype=bool)
    active[4] = False
    per = hd.linesearch_batch(hd.HostDynamics(F, n, m), X, U, T, K, k, active, args, io.ALPHAS,
                              extra)
    vec = hd.linesearch_batch(hd.HostDynamics(F, n, m, vectorized=True), X, U, T, K, k, active,
                              args, io.ALPHAS, extra)
    assert np.array_equal(per[4], vec[4]) and per[4][4] == -2
    for b in range(Bn):
        if not active[b]:
            assert _same(vec[0][b], X[b]) and np.isnan(vec[2][b])
            continue
        Jp, Jv = per[2][b], vec[2][b]
        assert Jp == Jv or abs(Jp - Jv) <= 1e-12 * abs(Jp) or (np.isinf(Jp) and np.isinf(Jv))
        assert _rel(vec[0][b], per[0][b]) <= 1e-12 and _rel(vec[1][b], per[1][b]) <= 1e-12
    assert len(set(per[4].tolist())) >= 3


def test_ilqr_timeopt_routes_callables(monkeypatch):
    """solver.ilqr_timeopt's routing (no GPU: the batched loop is stubbed): a built-in
    system with its own cost stays on the device; a Python stage cost with a built-in
    system keeps F on the device kernel as row-vectorised host dynamics; any other
    callable F is host dynamics (per call); a HostDynamics passes through"""
    import torch
    from time_opt_ilqr_amd import solver, systems
    seen = {}

    def fake_batch(system, x0, *a, **kw):
        seen["system"], seen["kw"] = system, kw
        N = a[6]
        n = x0.shape[1]
        return {"crashed": torch.zeros(1, dtype=torch.int32), "n_hist": torch.ones(1, dtype=torch.int32),
                "X": torch.zeros(1, N + 1, n), "U": torch.zeros(1, N, 1), "J_hist": torch.zeros(1, 1),
                "T_hist": torch.ones(1, 1, dtype=torch.int32), "timers": {},
                "J_curve": torch.zeros(1, N), "T_star": torch.ones(1, dtype=torch.int32)}

    monkeypatch.setattr(solver, "ilqr_timeopt_batch", fake_batch)
    monkeypatch.setattr(solver, "_dev", lambda: torch.device("cpu"))
    F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, extra = \
        systems.make_double_integrator(N=20)
    args = (x0, xg, u_ref, Q, R, alpha, w, 20, 5, 20)
    solver.ilqr_timeopt(F, *args)
    assert seen["system"] == F.system_id and "dt" in seen["kw"]
    cost = lambda x, u: (0.0, np.zeros(2), np.zeros((2, 2)))  # noqa: E731
    solver.ilqr_timeopt(F, *args, extra_stage_cost=cost)
    s = seen["system"]
    assert isinstance(s, hd.HostDynamics) and s.vectorized and (s.n, s.m) == (2, 1)
    assert seen["kw"]["extra_stage_cost"] is cost
    Fp = dyn._scalar_F(0, F.dt)
    solver.ilqr_timeopt(Fp, *args)
    s = seen["system"]
    assert isinstance(s, hd.HostDynamics) and not s.vectorized and s.F is Fp
    Fh = hd.HostDynamics(Fp, 2, 1, vectorized=True)
    solver.ilqr_timeopt(Fh, *args)
    assert seen["system"] is Fh
    with pytest.raises(TypeError):
        solver.ilqr_timeopt(42, *args)
