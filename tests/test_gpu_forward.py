"""GPU parity of the forward pass and the device outer loop (forward.hip,
solver.py) against the reference's own captures (tests/golden/ilqr_*.npz,
make_golden.py --ilqr) and the oracle (oracle/ilqr_oracle.py, pinned by them).

Tolerances (written where they are used):
  * J (true cost): 1e-12 relative -- the kernel's dot products run as fma
    chains where NumPy hands them to BLAS, so the last bits differ;
  * X', U' of an accepted step: 1e-12 relative to the trajectory's scale
    (bit-exact dynamics for DI / point mass / segway, ocml trig for the others);
  * whole outer loop: the same T_hist and accepted iterations, J_hist to 1e-9
    relative (each iteration re-linearises, so 1e-16 differences compound).
"""
import os

import numpy as np
import pytest

from oracle import dyn_oracle as dyn
from oracle import ilqr_oracle as io

pytestmark = pytest.mark.gpu

TAGS = ["di", "cartpole", "quadrotor", "pointmass", "segway"]


def _t(x, dev):
    import torch
    return torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)


def _np(t):
    return t.detach().cpu().numpy()


def _rel(got, ref):
    got, ref = np.asarray(got, float), np.asarray(ref, float)
    return float(np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-300))


def _case(golden_dir, tag):
    d = np.load(os.path.join(golden_dir, f"ilqr_{tag}.npz"))
    obs = None
    if tag == "pointmass":
        from time_opt_ilqr_amd.systems import OBSTACLES
        obs = np.array([[o[0], o[1], r, wt] for o, r, wt in OBSTACLES])
    return d, dyn.SYSTEMS[tag], [int(i) for i in d["wrap_idx"]], obs


def _cost(d, wrap, obs, dev):
    from time_opt_ilqr_amd import engine
    return engine.CostParams(_t(d["xg"], dev), _t(d["u_ref"], dev), _t(d["Q"], dev),
                             _t(d["R"], dev), _t(d["Qf"], dev), float(d["w"]),
                             None if obs is None else _t(obs, dev), wrap)


@pytest.mark.parametrize("tag", TAGS)
def test_forward_linesearch_vs_reference_captures(dev, golden_dir, tag):
    """every captured forward_linesearch_fixedT call, batched into one launch"""
    from time_opt_ilqr_amd import engine
    d, sid, wrap, obs = _case(golden_dir, tag)
    nf = int(d["n_fwd"])
    N = int(d["N"])
    n, m = dyn.DIMS[sid]
    g = lambda i, k: d[f"f{i}_{k}"]  # noqa: E731
    X = np.stack([g(i, "X") for i in range(nf)])
    U = np.stack([g(i, "U") for i in range(nf)])
    T = [int(g(i, "T_star")) for i in range(nf)]
    K = np.zeros((nf, N, m, n))
    k = np.zeros((nf, N, m))
    for i in range(nf):
        K[i, :T[i]] = g(i, "K")
        k[i, :T[i]] = g(i, "k")
    r = engine.forward_linesearch(sid, _t(X, dev), _t(U, dev), T, _t(K, dev), _t(k, dev),
                                  _cost(d, wrap, obs, dev), float(d["dt"]))
    acc = _np(r.accepted)
    for i in range(nf):
        assert (acc[i] >= 0) == bool(g(i, "acc")), (i, acc[i])
        Jr = float(g(i, "J"))
        assert abs(float(r.J[i]) - Jr) <= 1e-12 * max(1.0, abs(Jr))
        assert _rel(_np(r.X[i]), g(i, "X_new")) <= 1e-12
        assert _rel(_np(r.U[i]), g(i, "U_new")) <= 1e-12


@pytest.mark.parametrize("tag", TAGS)
def test_rollout_and_cost_vs_reference(dev, golden_dir, tag):
    from time_opt_ilqr_amd import engine
    d, sid, wrap, obs = _case(golden_dir, tag)
    N, dt = int(d["N"]), float(d["dt"])
    U0 = np.tile(d["u_ref"].reshape(1, -1), (N, 1))
    X0 = _np(engine.rollout(sid, _t(d["x0"], dev), _t(U0, dev)[None], dt))[0]
    assert np.array_equal(np.isnan(X0), np.isnan(d["X0"]))
    assert _rel(np.nan_to_num(X0), np.nan_to_num(d["X0"])) <= 1e-13
    Xb = _np(engine.rollout(sid, _t(d["x0"], dev), _t(d["U_big"], dev)[None], dt,
                            max_state_norm=1e3))[0]
    assert np.array_equal(np.isnan(Xb), np.isnan(d["X_big"]))
    Ts = [int(t) for t in d["cost_T"]]
    B = len(Ts)
    J = _np(engine.cost_true(sid, _t(np.stack([d["X"]] * B), dev),
                             _t(np.stack([d["U"]] * B), dev), Ts, _cost(d, wrap, obs, dev)))
    assert np.all(np.abs(J - d["cost_J"]) <= 1e-12 * np.maximum(1.0, np.abs(d["cost_J"])))


def test_cost_edge_cases(dev, golden_dir):
    """T* <= 0 -> inf, non-finite data -> inf, T* > N -> NaN (reference: IndexError)"""
    from time_opt_ilqr_amd import engine
    d, sid, wrap, obs = _case(golden_dir, "di")
    N = int(d["N"])
    X = np.stack([d["X"]] * 4)
    U = np.stack([d["U"]] * 4)
    X[2, 3, 0] = np.nan
    J = _np(engine.cost_true(sid, _t(X, dev), _t(U, dev), [0, -3, 10, N + 1],
                             _cost(d, wrap, obs, dev)))
    assert np.isposinf(J[0]) and np.isposinf(J[1]) and np.isposinf(J[2]) and np.isnan(J[3])
    J = _np(engine.cost_true(sid, _t(X, dev), _t(U, dev), [2, 3, 2, N], _cost(d, wrap, obs, dev)))
    assert np.isfinite(J[2])  # the NaN in X[3] is not read at T* = 2
    ref = io.cost_true(d["X"], d["U"], d["xg"], d["u_ref"], d["Q"], d["R"], d["Qf"],
                       float(d["w"]), N, wrap)
    assert abs(J[3] - ref) <= 1e-12 * abs(ref)


def test_linesearch_mixed_batch_vs_oracle(dev, golden_dir):
    """quadrotor, 37 problems (ragged) built from a captured line search with the
    feed-forward k scaled per problem (x1 .. x300, negated): every step-size index
    is accepted somewhere, large steps trip the dynamics' NaN guards, negated
    steps accept nothing; one problem is inactive, one has T* = 0, several have
    shorter horizons"""
    import torch
    from time_opt_ilqr_amd import engine
    d, sid, wrap, obs = _case(golden_dir, "quadrotor")
    g = lambda k: d[f"f1_{k}"]  # noqa: E731
    N, T0 = int(d["N"]), int(g("T_star"))
    Bn = 37
    scales = np.array([1, 3, 10, 30, 100, 300, -1, -10, 0.3])
    sc = scales[np.arange(Bn) % len(scales)]
    X = np.stack([g("X")] * Bn)
    U = np.stack([g("U")] * Bn)
    K = np.zeros((Bn, N, 4, 12))
    k = np.zeros((Bn, N, 4))
    K[:, :T0] = g("K")
    k[:, :T0] = g("k")[None] * sc[:, None, None]
    T = np.full(Bn, T0)
    T[3] = 0
    T[10:14] = [1, 5, T0 // 2, N]
    active = np.ones(Bn, dtype=np.int32)
    active[7] = 0
    r = engine.forward_linesearch(2, _t(X, dev), _t(U, dev), torch.as_tensor(T), _t(K, dev),
                                  _t(k, dev), _cost(d, wrap, obs, dev), float(d["dt"]),
                                  active=torch.as_tensor(active))
    acc = _np(r.accepted)
    seen = set()
    for b in range(Bn):
        if not active[b]:
            assert acc[b] == -2 and np.array_equal(_np(r.X[b]), X[b], equal_nan=True)
            continue
        Xo, Uo, Jo, ok, ai = io.forward_linesearch(2, float(d["dt"]), X[b], U[b], d["xg"],
                                                   d["u_ref"], d["Q"], d["R"], d["Qf"],
                                                   float(d["w"]), int(T[b]), k[b], K[b],
                                                   wrap_idx=wrap)
        seen.add(ai)
        assert acc[b] == ai, (b, acc[b], ai)
        Jg = float(r.J[b])
        assert abs(Jg - Jo) <= 1e-12 * max(1.0, abs(Jo)) or (np.isinf(Jo) and np.isinf(Jg))
        assert _rel(_np(r.X[b]), Xo) <= 1e-11
        assert _rel(_np(r.U[b]), Uo) <= 1e-11
    assert -1 in seen and 0 in seen and len(seen) >= 4, seen


def test_linesearch_two_lane_and_one_lane_layouts_bitwise(dev, golden_dir):
    """The quadrotor line search runs two lanes per (problem, alpha) rollout while the
    launch fits one wave per SIMD (37 problems here) and one lane per rollout beyond
    that (6,000 problems: 66,000 two-lane lanes would exceed the 65,536 of one wave per
    SIMD).  The same problems at both sizes: J, the accepted index, X' and U' bitwise
    equal; per-problem horizons, scaled feed-forwards (rejections, non-finite steps)."""
    import torch
    from time_opt_ilqr_amd import engine
    d, sid, wrap, obs = _case(golden_dir, "quadrotor")
    g = lambda k: d[f"f1_{k}"]  # noqa: E731
    N, T0 = int(d["N"]), int(g("T_star"))
    nb = 37
    scales = np.array([1, 3, 10, 30, 100, 300, -1, -10, 0.3])
    sc = scales[np.arange(nb) % len(scales)]
    X = np.stack([g("X")] * nb)
    U = np.stack([g("U")] * nb)
    K = np.zeros((nb, N, 4, 12))
    k = np.zeros((nb, N, 4))
    K[:, :T0] = g("K")
    k[:, :T0] = g("k")[None] * sc[:, None, None]
    T = np.full(nb, T0)
    T[3], T[10:14] = 0, [1, 5, T0 // 2, N]
    cost = _cost(d, wrap, obs, dev)
    small = engine.forward_linesearch(2, _t(X, dev), _t(U, dev), torch.as_tensor(T), _t(K, dev),
                                      _t(k, dev), cost, float(d["dt"]))
    rep = (6000 + nb - 1) // nb
    big = engine.forward_linesearch(2, _t(np.tile(X, (rep, 1, 1)), dev),
                                    _t(np.tile(U, (rep, 1, 1)), dev),
                                    torch.as_tensor(np.tile(T, rep)), _t(np.tile(K, (rep, 1, 1, 1)), dev),
                                    _t(np.tile(k, (rep, 1, 1)), dev), cost, float(d["dt"]))
    for j in (0, rep // 2, rep - 1):
        sl = slice(j * nb, (j + 1) * nb)
        assert torch.equal(big.accepted[sl], small.accepted)
        assert torch.equal(big.J[sl].nan_to_num(7.0), small.J.nan_to_num(7.0))
        assert torch.equal(big.X[sl].nan_to_num(7.0), small.X.nan_to_num(7.0))
        assert torch.equal(big.U[sl].nan_to_num(7.0), small.U.nan_to_num(7.0))
    assert len(set(small.accepted.tolist())) >= 3


def test_obstacle_cost_kernel(dev):
    from time_opt_ilqr_amd import engine, systems
    rng = np.random.default_rng(5)
    X = rng.uniform(-2.5, 2.5, (3, 17, 4))
    obs = np.array([[o[0], o[1], r, wt] for o, r, wt in systems.OBSTACLES])
    c, cx, cxx = engine.obstacle_cost(_t(X, dev), _t(obs, dev))
    for idx in np.ndindex(3, 17):
        rc, rcx, rcxx = systems.obstacle_stage_cost(X[idx])
        assert abs(float(c[idx]) - rc) <= 1e-14 * max(1.0, abs(rc))
        assert np.allclose(_np(cx[idx]), rcx, rtol=1e-13, atol=1e-15)
        assert np.allclose(_np(cxx[idx]), rcxx, rtol=1e-13, atol=1e-15)


@pytest.mark.parametrize("tag", TAGS)
def test_ilqr_outer_loop_vs_reference(dev, golden_dir, tag):
    """solver.ilqr_timeopt (device end to end) against the reference's run"""
    from time_opt_ilqr_amd import solver, systems
    d, sid, wrap, obs = _case(golden_dir, tag)
    mk = list(systems.MAKERS.values())[sid]
    F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap_idx, extra = mk(N=int(d["N"]))
    sol = solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, int(d["N"]), int(d["T_min"]),
                              int(d["T_max"]), max_iter=int(d["max_iter"]), wrap_idx=wrap_idx,
                              use_central_diff=bool(d["central"]),
                              extra_stage_cost=extra["extra_stage_cost"] if extra else None)
    # cart-pole: the zero angle weight makes E_k = (Q_k + 1e-9 I)^-1 reach 5e8, so the
    # compose inverse W has cond ~1e9 and the J curve / gains carry ~1e-9 relative
    # rounding differences from the reference's LAPACK path (same T* everywhere)
    tol = 1e-8 if tag == "cartpole" else 1e-9
    assert sol["T_hist"] == [int(t) for t in d["T_hist"]]
    assert _rel(np.array(sol["J_hist"]), d["J_hist"]) <= tol
    assert sol["T_star"] == int(d["T_star"])
    assert _rel(np.nan_to_num(sol["X"]), np.nan_to_num(d["X"])) <= 100 * tol
    # the last select's J curve (solver.py:751-762), as the reference driver plots it;
    # these real terminal blocks are ill-conditioned: real-capture bar
    # over the selection window [T_min, T_max] (cart-pole's horizons far below T_min
    # differ by O(1) relative between any two LAPACK-free rounding orders: its zero
    # angle weight puts 5e8 entries into E_k)
    assert sol["J_curve"].shape == d["J_curve"].shape
    jc_tol = 1e-3 if tag in ("di", "pointmass") else 5e-2
    win = slice(int(d["T_min"]) - 1, int(d["T_max"]))
    got, ref = sol["J_curve"][win], d["J_curve"][win]
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(got), fin)
    assert np.max(np.abs(got[fin] - ref[fin]) / np.abs(ref[fin])) <= jc_tol


def test_ilqr_batch_mixed_problems_vs_oracle(dev):
    """a batch of DI problems with different x0: per-problem T_hist / J_hist /
    stop iteration equal the oracle's scalar runs"""
    import torch
    from time_opt_ilqr_amd import solver, systems
    F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, _ = \
        systems.make_double_integrator(N=50)
    rng = np.random.default_rng(2)
    Bn = 6
    X0 = x0 + rng.uniform(-1.5, 1.5, (Bn, 2))
    Qf = np.asarray(io.orc.terminal_weight(alpha, 2))
    res = solver.ilqr_timeopt_batch(0, X0, xg, u_ref, Q, R, Qf, w, 50, 10, 50, dt=F.dt,
                                    max_iter=12, use_central_diff=False)
    nh = _np(res["n_hist"])
    for b in range(Bn):
        o = io.ilqr_timeopt(0, F.dt, X0[b], xg, u_ref, Q, R, Qf, w, 50, 10, 50, max_iter=12,
                            central=False)
        assert _np(res["T_hist"][b, :nh[b]]).tolist() == o["T_hist"]
        assert _rel(_np(res["J_hist"][b, :nh[b]]), o["J_hist"]) <= 1e-9
        assert int(res["T_star"][b]) == o["T_star"]
    assert not bool(torch.as_tensor(res["crashed"]).any())


def test_reference_shaped_forward_dropins(dev, golden_dir):
    from time_opt_ilqr_amd import solver, systems
    d, sid, wrap, obs = _case(golden_dir, "segway")
    F = systems.make_segway_balance(N=int(d["N"]))[0]
    g = lambda k: d[f"f0_{k}"]  # noqa: E731
    T = int(g("T_star"))
    Xn, Un, J, acc = solver.forward_linesearch_fixedT(
        F, g("X"), g("U"), d["xg"], d["u_ref"], d["Q"], d["R"], d["Qf"], float(d["w"]), T,
        list(g("k")), list(g("K")), wrap_idx=wrap)
    assert acc == bool(g("acc")) and abs(J - float(g("J"))) <= 1e-12 * abs(float(g("J")))
    assert _rel(Xn, g("X_new")) <= 1e-12
    X0 = solver.rollout(F, d["x0"], np.tile(d["u_ref"], (int(d["N"]), 1)))
    assert _rel(X0, d["X0"]) <= 1e-13
    Jc = solver.cost_timeopt_true(d["X"], d["U"], d["xg"], d["u_ref"], d["Q"], d["R"], d["Qf"],
                                  float(d["w"]), int(d["cost_T"][2]), wrap)
    assert abs(Jc - float(d["cost_J"][2])) <= 1e-12 * abs(float(d["cost_J"][2]))
    assert solver.cost_timeopt_true(d["X"], d["U"], d["xg"], d["u_ref"], d["Q"], d["R"],
                                    d["Qf"], float(d["w"]), 0) == float("inf")


@pytest.mark.parametrize("wrap", [[6, 7], [], [0, 6, 7, 8]])
def test_linesearch_nondefault_wrap_vs_oracle(dev, golden_dir, wrap):
    """a wrap_idx other than the system's default takes the runtime-mask kernel"""
    from time_opt_ilqr_amd import engine
    d, sid, _, obs = _case(golden_dir, "quadrotor")
    g = lambda k: d[f"f0_{k}"]  # noqa: E731
    N, T0 = int(d["N"]), int(g("T_star"))
    K = np.zeros((1, N, 4, 12))
    k = np.zeros((1, N, 4))
    K[0, :T0] = g("K")
    k[0, :T0] = g("k")
    X = g("X").copy()
    X[:, 7] += 2 * np.pi  # wrapped components differ by a full turn
    r = engine.forward_linesearch(2, _t(X[None], dev), _t(g("U")[None], dev), [T0],
                                  _t(K, dev), _t(k, dev), _cost(d, wrap, obs, dev),
                                  float(d["dt"]))
    Xo, Uo, Jo, ok, ai = io.forward_linesearch(2, float(d["dt"]), X, g("U"), d["xg"],
                                               d["u_ref"], d["Q"], d["R"], d["Qf"],
                                               float(d["w"]), T0, k[0], K[0], wrap_idx=wrap)
    assert int(r.accepted[0]) == ai
    Jg = float(r.J[0])
    assert abs(Jg - Jo) <= 1e-12 * max(1.0, abs(Jo)) or (np.isinf(Jo) and np.isinf(Jg))
    assert _rel(_np(r.U[0]), Uo) <= 1e-11


def test_dropin_input_shapes_like_the_reference(dev):
    """Reference input conventions the drop-ins keep:
    a 1-D U_init on an m=1 system is one control per step (solver.py:484-485);
    a [1, N, m] U_init is shared by a batch; cost_timeopt_true reads only
    X[:T+1] and U[:T] (solver.py:80-102); a per-problem Qf is rejected, never
    symmetrised across problems; timers are the reference's four keys and NaN
    when the stages are not synchronised."""
    import torch
    from time_opt_ilqr_amd import solver, systems
    F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, _ = \
        systems.make_double_integrator(N=50)
    U1 = 0.05 * np.sin(np.arange(40))
    sol = solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, 50, 10, 50, U_init=U1,
                              max_iter=3, use_central_diff=False)
    o = io.ilqr_timeopt(0, F.dt, x0, xg, u_ref, Q, R, np.asarray(io.orc.terminal_weight(alpha, 2)),
                        w, 50, 10, 50, max_iter=3, central=False,
                        U_init=U1)
    assert sol["T_hist"] == o["T_hist"]
    assert sorted(sol["timers"]) == ["backward", "forward", "linearize", "select"]
    Qf = np.asarray(io.orc.terminal_weight(alpha, 2))
    X0 = np.stack([x0, x0 + 0.3])
    res = solver.ilqr_timeopt_batch(0, X0, xg, u_ref, Q, R, Qf, w, 50, 10, 50, dt=F.dt,
                                    U_init=U1.reshape(1, -1, 1), max_iter=2,
                                    use_central_diff=False, stage_timers=False)
    assert all(np.isnan(v) for v in res["timers"].values())
    assert res["J_curve"].shape == (2, 50)
    with pytest.raises(ValueError):
        solver.ilqr_timeopt_batch(0, X0, xg, u_ref, Q, R, np.stack([Qf, Qf]), w, 50, 10, 50,
                                  dt=F.dt, max_iter=1)
    X, U = sol["X"], sol["U"]
    T = sol["T_star"]
    full = solver.cost_timeopt_true(X, U, xg, u_ref, Q, R, alpha, w, T)
    short = solver.cost_timeopt_true(X[:T + 1], U[:T], xg, u_ref, Q, R, alpha, w, T)
    assert full == short
    del torch


def test_ilqr_batch_nonfinite_initial_trajectories_crash_up_front(dev):
    """Problems whose initial rollout is not finite on the rows the select reads raise
    in the reference's first select (chol_inv's _assert_finite, utils.py:77): they
    are reported crashed with nothing recorded, their J curve NaN and their select
    status non-finite, and the other problems' runs are bitwise those of the batch
    without them."""
    import torch
    from time_opt_ilqr_amd import solver, systems
    F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap_idx, _ = systems.make_quadrotor(N=40)
    rng = np.random.default_rng(5)
    Bn = 7
    X0 = x0 + 0.2 * rng.standard_normal((Bn, 12))
    X0[2, 9] = 2e3    # |omega| > 1e3: the quadrotor's guard makes X[1:] NaN
    X0[5, 7] = np.nan
    Qf = np.asarray(io.orc.terminal_weight(alpha, 12))
    kw = dict(dt=F.dt, max_iter=4, wrap_idx=wrap_idx, use_central_diff=False)
    res = solver.ilqr_timeopt_batch(2, X0, xg, u_ref, Q, R, Qf, w, 40, 8, 40, **kw)
    keep = [0, 1, 3, 4, 6]
    ref = solver.ilqr_timeopt_batch(2, X0[keep], xg, u_ref, Q, R, Qf, w, 40, 8, 40, **kw)
    assert _np(res["crashed"]).tolist() == [0, 0, 1, 0, 0, 1, 0]
    assert _np(res["n_hist"])[[2, 5]].tolist() == [0, 0]
    assert bool(torch.isnan(res["J_curve"][[2, 5]]).all())
    st0 = _np(res["select_status"][:, 0])
    assert (st0[[2, 5]] & 4).all() and (st0[keep] == _np(ref["select_status"][:, 0])).all()
    for f in ("n_hist", "T_hist", "J_hist", "T_star", "X", "U", "J_curve"):
        a, b = res[f][keep], ref[f]
        assert torch.equal(a.nan_to_num(7.0) if a.is_floating_point() else a,
                           b.nan_to_num(7.0) if b.is_floating_point() else b), f


# ---------------------------------------------------------------------------
# method="bruteforce" (solver.py:525-532 / 607-614 with solver.py:293-358)
# ---------------------------------------------------------------------------
BF_TAGS = ["di", "cartpole", "segway", "quadrotor", "pointmass"]


def _bf_case(golden_dir, tag):
    d = np.load(os.path.join(golden_dir, f"ilqr_bf_{tag}.npz"))
    obs = None
    if tag == "pointmass":
        from time_opt_ilqr_amd.systems import OBSTACLES
        obs = np.array([[o[0], o[1], r, wt] for o, r, wt in OBSTACLES])
    return d, dyn.SYSTEMS[tag], [int(i) for i in d["wrap_idx"]], obs


@pytest.mark.parametrize("tag", BF_TAGS)
def test_ilqr_bruteforce_outer_loop_vs_reference(dev, golden_dir, tag):
    """solver.ilqr_timeopt(method="bruteforce") against the reference's run: same
    T_hist, J_hist to 1e-9 relative (cart-pole 1e-8), the last J curve to 1e-8 (a
    Riccati sweep per horizon: no ill-conditioned augmented blocks)"""
    from time_opt_ilqr_amd import solver, systems
    d, sid, wrap, obs = _bf_case(golden_dir, tag)
    mk = list(systems.MAKERS.values())[sid]
    F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap_idx, extra = mk(N=int(d["N"]))
    sol = solver.ilqr_timeopt_baseline1(
        F, x0, xg, u_ref, Q, R, alpha, w, int(d["N"]), int(d["T_min"]), int(d["T_max"]),
        max_iter=int(d["max_iter"]), wrap_idx=wrap_idx, use_central_diff=bool(d["central"]),
        extra_stage_cost=extra["extra_stage_cost"] if extra else None)
    # cart-pole: the zero angle weight leaves near-singular Quu blocks early on, so
    # the 1e-16 rounding differences of fma chains vs BLAS compound over its four
    # re-linearised iterations to ~3e-9 (same T_hist); the others stay below 1e-9
    tol = 1e-8 if tag == "cartpole" else 1e-9
    assert sol["T_hist"] == [int(t) for t in d["T_hist"]]
    assert _rel(np.array(sol["J_hist"]), d["J_hist"]) <= tol
    assert sol["T_star"] == int(d["T_star"])
    assert _rel(sol["X"], d["X"]) <= 100 * tol
    # the last J curve is evaluated on the final (iterated) trajectory: 1e-8 relative
    assert sol["J_curve"].shape == d["J_curve"].shape
    assert np.max(np.abs(sol["J_curve"] - d["J_curve"]) / np.abs(d["J_curve"])) <= 1e-8


@pytest.mark.parametrize("sid,N,T_max", [(2, 40, 33), (0, 30, 30), (4, 25, 20)])
def test_bruteforce_jcurve_equals_per_horizon_riccati(dev, sid, N, T_max):
    """the one-launch J curve (grid y = horizon) against T_max separate mode-1 passes
    at horizon T: bit-identical V_0 and status (same kernel arithmetic).  sid 2 =
    quadrotor (the exact-size fp64 kernel), 0 / 4 the generic kernel; a ragged batch
    (B = 9) and one problem with a NaN state at step 7 (fails for every T >= 7)"""
    import torch
    from time_opt_ilqr_amd import _lib, engine
    n, m = dyn.DIMS[sid]
    rng = np.random.default_rng(11 + sid)
    Bn = 9
    X = rng.standard_normal((Bn, N + 1, n)) * 0.3
    U = rng.standard_normal((Bn, N, m)) * 0.1
    lin = engine.linearize(sid, _t(X, dev), _t(U, dev), 0.05, central=False)
    X[4, 7, 0] = np.nan
    Xd, Ud = _t(X, dev), _t(U, dev)
    xg, ur = _t(rng.standard_normal(n), dev), _t(np.zeros(m), dev)
    Q = _t(np.diag(rng.uniform(0.5, 2, n)), dev)
    R = _t(np.diag(rng.uniform(0.5, 2, m)), dev)
    Qf = _t(10 * np.eye(n), dev)
    wrap = [n - 1] if sid == 4 else None
    J, st = engine.bruteforce_jcurve(lin.A, lin.B, Xd, Ud, xg, ur, Q, R, Qf, T_max,
                                     lm_lambda=1e-6, w_stage=0.7, wrap_idx=wrap)
    J, st = _np(J), _np(st)
    for T in range(1, T_max + 1):
        r = engine.riccati(lin.A, lin.B, Xd, Ud, xg, ur, Q, R, Qf,
                           torch.full((Bn,), T, dtype=torch.int32), 1e-6, mode=1, w_stage=0.7,
                           wrap_idx=wrap, reg_max_tries=1)
        rs = _np(r.status)
        assert np.array_equal(st[:, T - 1], rs), T
        ok = (rs & _lib.ST_FAIL) == 0
        assert np.array_equal(J[ok, T - 1], _np(r.V0[:, 0])[ok]), T
        assert np.isnan(J[~ok, T - 1]).all()
    # horizon T reads X[0..T]: T >= 7 sees the NaN (column T-1 >= 6)
    assert (st[4, 6:] & _lib.ST_NONFINITE).all() and not (st[4, :6] & _lib.ST_FAIL).any()


def test_bruteforce_jcurve_shared_q_two_wave_kernel_bitwise(dev):
    """a batch-shared Q runs the J curve at two waves per SIMD (one step image, one Q
    image per wave, Q's rows re-read from LDS); a per-problem Q (the same matrix
    repeated) the one-wave layout: bit-identical curves and status.  Quadrotor sizes
    (the exact-size kernel), ragged B = 37, odd T_max, a NaN state, and a
    non-symmetric Q so lx = Q e and the Qxx start (Q's rows vs columns) are told apart"""
    import torch
    from time_opt_ilqr_amd import engine
    n, m = dyn.DIMS[2]
    rng = np.random.default_rng(29)
    Bn, N, T_max = 37, 40, 31
    X = rng.standard_normal((Bn, N + 1, n)) * 0.3
    U = rng.standard_normal((Bn, N, m)) * 0.1
    lin = engine.linearize(2, _t(X, dev), _t(U, dev), 0.05, central=False)
    X[5, 9, 3] = np.nan
    Xd, Ud = _t(X, dev), _t(U, dev)
    xg, ur = _t(rng.standard_normal(n) * 0.2, dev), _t(rng.standard_normal(m) * 0.1, dev)
    Qn = np.diag(rng.uniform(0.5, 2, n)) + 0.05 * rng.standard_normal((n, n))
    Q = _t(Qn, dev)
    R = _t(np.diag(rng.uniform(0.5, 2, m)), dev)
    Qf = _t(np.diag(rng.uniform(2, 10, n)), dev)
    kw = dict(lm_lambda=1e-6, w_stage=0.4)
    J1, s1 = engine.bruteforce_jcurve(lin.A, lin.B, Xd, Ud, xg, ur, Q, R, Qf, T_max, **kw)
    Qb = Q.unsqueeze(0).repeat(Bn, 1, 1).contiguous()
    J2, s2 = engine.bruteforce_jcurve(lin.A, lin.B, Xd, Ud, xg, ur, Qb, R, Qf, T_max, **kw)
    assert torch.equal(s1, s2)
    assert torch.equal(J1.nan_to_num(7.0), J2.nan_to_num(7.0))
    # horizon T reads X[0..T]: T >= 9 (column 8 on) sees the NaN
    assert torch.isnan(J1[5, 8:]).all() and torch.isfinite(J1[5, :8]).all()


def test_bruteforce_jcurve_oracle_and_limits(dev):
    """against the oracle's bruteforce_J on a DI problem, and the entry's checks"""
    from time_opt_ilqr_amd import _lib, engine
    from oracle import hop_oracle as orc
    rng = np.random.default_rng(3)
    N, T_max = 24, 24
    X = rng.standard_normal((N + 1, 2))
    U = rng.standard_normal((N, 1))
    A, B, _ = dyn.linearize(0, X, U, 0.1, central=True)
    xg, ur, Q, R = np.array([1.0, 0.0]), np.zeros(1), np.diag([1.0, 0.1]), np.eye(1) * 0.1
    Qf = np.diag([50.0, 5.0])
    J, st = engine.bruteforce_jcurve(_t(A[None], dev), _t(B[None], dev), _t(X[None], dev),
                                     _t(U[None], dev), _t(xg, dev), _t(ur, dev), _t(Q, dev),
                                     _t(R, dev), _t(Qf, dev), T_max, w_stage=0.25)
    ref = orc.bruteforce_J(list(A), list(B), X, U, xg, ur, Q, R, Qf, 0.25, T_max)
    assert (_np(st) == 0).all()
    assert _rel(_np(J)[0], ref) <= 1e-12
    with pytest.raises(_lib.HopError):  # t_max > N: the reference's IndexError
        engine.bruteforce_jcurve(_t(A[None], dev), _t(B[None], dev), _t(X[None], dev),
                                 _t(U[None], dev), _t(xg, dev), _t(ur, dev), _t(Q, dev),
                                 _t(R, dev), _t(Qf, dev), N + 1)
    Je, se = engine.bruteforce_jcurve(_t(A[None], dev)[:0], _t(B[None], dev)[:0],
                                      _t(X[None], dev)[:0], _t(U[None], dev)[:0], _t(xg, dev),
                                      _t(ur, dev), _t(Q, dev), _t(R, dev), _t(Qf, dev), T_max)
    assert Je.shape == (0, T_max) and se.shape == (0, T_max)


def test_ilqr_batch_bruteforce_mixed_problems_vs_oracle(dev):
    """a batch of quadrotor problems with different x0 through
    ilqr_timeopt_batch(method="bruteforce"), each against the oracle's outer loop"""
    from time_opt_ilqr_amd import solver
    d, sid, wrap, obs = _bf_case(os.path.join(os.path.dirname(__file__), "golden"), "quadrotor")
    N, T_min, T_max = int(d["N"]), int(d["T_min"]), int(d["T_max"])
    rng = np.random.default_rng(8)
    Bn = 5
    x0 = np.stack([d["x0"]] * Bn)
    x0[1:, :3] += rng.uniform(-0.5, 0.5, (Bn - 1, 3))
    res = solver.ilqr_timeopt_batch(sid, x0, d["xg"], d["u_ref"], d["Q"], d["R"], d["Qf"],
                                    float(d["w"]), N, T_min, T_max, dt=float(d["dt"]),
                                    max_iter=3, wrap_idx=wrap, use_central_diff=False,
                                    device=dev, method="bruteforce")
    for b in range(Bn):
        o = io.ilqr_timeopt(sid, float(d["dt"]), x0[b], d["xg"], d["u_ref"], d["Q"], d["R"],
                            d["Qf"], float(d["w"]), N, T_min, T_max, max_iter=3, wrap_idx=wrap,
                            central=False, method="bruteforce")
        nh = int(res["n_hist"][b])
        assert [int(t) for t in _np(res["T_hist"][b, :nh])] == o["T_hist"], b
        assert _rel(_np(res["J_hist"][b, :nh]), o["J_hist"]) <= 1e-9, b
    assert not _np(res["crashed"]).any()


def test_ilqr_batch_bruteforce_per_problem_goals_vs_oracle(dev):
    """per-problem goals xg [B, n] (the non-compact batch path: stopped rows are
    masked, not gathered out) with method="bruteforce": each problem against the
    oracle's scalar bruteforce loop"""
    from time_opt_ilqr_amd import solver, systems
    F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, _ = \
        systems.make_double_integrator(N=40)
    rng = np.random.default_rng(21)
    Bn = 5
    XG = np.asarray(xg, float) + rng.uniform(-1.0, 1.0, (Bn, 2))
    Qf = np.asarray(io.orc.terminal_weight(alpha, 2))
    res = solver.ilqr_timeopt_batch(0, np.stack([x0] * Bn), XG, u_ref, Q, R, Qf, w, 40, 8, 40,
                                    dt=F.dt, max_iter=6, use_central_diff=False,
                                    method="bruteforce")
    nh = _np(res["n_hist"])
    for b in range(Bn):
        o = io.ilqr_timeopt(0, F.dt, x0, XG[b], u_ref, Q, R, Qf, w, 40, 8, 40, max_iter=6,
                            central=False, method="bruteforce")
        assert _np(res["T_hist"][b, :nh[b]]).tolist() == o["T_hist"], b
        assert _rel(_np(res["J_hist"][b, :nh[b]]), o["J_hist"]) <= 1e-9, b
        assert int(res["T_star"][b]) == o["T_star"]
    assert len(set(_np(res["T_star"]).tolist())) > 1  # the goals give different horizons


@pytest.mark.parametrize("tag,method", [("di", "propagator"), ("di", "bruteforce"),
                                        ("quadrotor", "propagator"),
                                        ("quadrotor", "bruteforce")])
def test_summary_csv_rows_on_the_device(dev, golden_dir, tag, method):
    """The reference's published comparison (plots/summary.csv, written by the legacy
    driver with max_iter=20, central differences, the makers' default N / T range):
    the device drop-in reproduces the reference's current-solver run of it (T_hist,
    J_hist 1e-9) and the committed csv row's T* and J* (to 1e-9), for both methods."""
    from time_opt_ilqr_amd import solver, systems
    d = np.load(os.path.join(golden_dir, f"summary_{tag}_{method}.npz"))
    mk = systems.make_double_integrator if tag == "di" else systems.make_quadrotor
    F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, _ = mk()
    assert (N, T_min, min(T_max, N)) == (int(d["N"]), int(d["T_min"]), int(d["T_max"]))
    sol = solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, int(d["T_max"]),
                              method=method, max_iter=20, lm_init=1e-3, wrap_idx=wrap_idx,
                              use_central_diff=True)
    assert sol["T_hist"] == [int(t) for t in d["T_hist"]]
    assert _rel(np.array(sol["J_hist"]), d["J_hist"]) <= 1e-9
    assert sol["T_star"] == int(d["csv_T_star"])
    assert abs(sol["J_hist"][-1] - float(d["csv_J_star"])) <= 1e-9 * abs(float(d["csv_J_star"]))
    assert len(sol["J_hist"]) == int(d["csv_n_iterations"])


def test_bruteforce_jcurve_fp32_entry(dev):
    """hop_bruteforce_jcurve_f32 (the generic kernel's fp32 instantiation) against the
    fp64 curve on the same well-conditioned quadrotor linearisation: 1e-4 relative
    (fp32 accumulation over up to 40 steps)"""
    import torch
    from time_opt_ilqr_amd import engine
    n, m, N, Bn = 12, 4, 40, 6
    rng = np.random.default_rng(17)
    X = rng.standard_normal((Bn, N + 1, n)) * 0.3
    U = rng.standard_normal((Bn, N, m)) * 0.1
    lin = engine.linearize(2, _t(X, dev), _t(U, dev), 0.05, central=False)
    args64 = [lin.A, lin.B, _t(X, dev), _t(U, dev), _t(np.zeros(n), dev),
              _t(np.array([9.81, 0, 0, 0]), dev), _t(np.diag(rng.uniform(0.5, 2, n)), dev),
              _t(np.diag(rng.uniform(0.5, 2, m)), dev), _t(20 * np.eye(n), dev)]
    J64, s64 = engine.bruteforce_jcurve(*args64, N, lm_lambda=1e-6, w_stage=0.05)
    J32, s32 = engine.bruteforce_jcurve(*[a.to(torch.float32) for a in args64], N,
                                        lm_lambda=1e-6, w_stage=0.05)
    assert J32.dtype == torch.float32 and J32.shape == (Bn, N)
    assert (_np(s64) == 0).all() and (_np(s32) == 0).all()
    assert _rel(_np(J32).astype(np.float64), _np(J64)) <= 1e-4


def test_bruteforce_jcurve_full_size_spot_checks(dev):
    """the bench size (B = 4096, N = T_max = 100, quadrotor shape; 409,600 sweeps in
    one launch): the first, a middle and the last problem against the oracle's
    bruteforce_J at 1e-9 relative, every status 0"""
    import torch
    from time_opt_ilqr_amd import engine
    from oracle import hop_oracle as orc
    Bn, N, n, m = 4096, 100, 12, 4
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    kw = dict(device=dev, dtype=torch.float64, generator=g)
    A = torch.eye(n, device=dev, dtype=torch.float64) + 0.05 * torch.randn((Bn, N, n, n), **kw)
    Bm = 0.1 * torch.randn((Bn, N, n, m), **kw)
    X = 0.5 * torch.randn((Bn, N + 1, n), **kw)
    U = 0.1 * torch.randn((Bn, N, m), **kw)
    xg = 0.2 * torch.randn((n,), **kw)
    ur = 0.05 * torch.randn((m,), **kw)
    M = torch.randn((n, n), **kw)
    Q = M @ M.T / n + 0.5 * torch.eye(n, device=dev, dtype=torch.float64)
    R = torch.diag(0.5 + 1.5 * torch.rand((m,), **kw))
    Qf = 10.0 * torch.eye(n, device=dev, dtype=torch.float64)
    J, st = engine.bruteforce_jcurve(A, Bm, X, U, xg, ur, Q, R, Qf, N, lm_lambda=1e-6,
                                     w_stage=0.1)
    assert int((st != 0).sum()) == 0
    Jn = _np(J)
    for b in (0, Bn // 2 + 3, Bn - 1):
        ref = orc.bruteforce_J(list(_np(A[b])), list(_np(Bm[b])), _np(X[b]), _np(U[b]), _np(xg),
                               _np(ur), _np(Q), _np(R), _np(Qf), 0.1, N)
        assert _rel(Jn[b], ref) <= 1e-9, b


def test_integration_md_ctypes_stubs_run(dev):
    """INTEGRATION.md's ctypes stubs (the binding a maintainer would add to the
    reference) run as written against the in-tree library and agree with engine"""
    import re
    import torch
    from time_opt_ilqr_amd import _lib, engine
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    text = open(os.path.join(repo, "INTEGRATION.md")).read()
    blocks = [b for b in re.findall(r"```python\n(.*?)```", text, re.S)
              if "hop_lft_sweep_f64" in b or "hop_bruteforce_jcurve_f64" in b
              or "hop_bruteforce_jcurve_legacy_f64" in b]
    assert len(blocks) == 3
    ns = {}
    code = "\n".join(blocks).replace("/path/to/time_opt_ilqr_amd/libhop_amd.so", _lib.LIB_PATH)
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    rng = np.random.default_rng(9)
    n, m, N, Bn = 4, 2, 12, 3
    A = np.eye(n) + 0.05 * rng.standard_normal((Bn, N, n, n))
    Bm = 0.1 * rng.standard_normal((Bn, N, n, m))
    X = 0.5 * rng.standard_normal((Bn, N + 1, n))
    U = 0.1 * rng.standard_normal((Bn, N, m))
    xg, ur = np.zeros(n), np.zeros(m)
    Q, R, Qf = np.eye(n), 0.5 * np.eye(m), 10 * np.eye(n)
    J, st = ns["bruteforce_all_Jt_batched"](A, Bm, X, U, xg, ur, Q, R, Qf, N, 0.1)
    Je, se = engine.bruteforce_jcurve(_t(A, dev), _t(Bm, dev), _t(X, dev), _t(U, dev), _t(xg, dev),
                                      _t(ur, dev), _t(Q, dev), _t(R, dev), _t(Qf, dev), N,
                                      w_stage=0.1)
    assert np.array_equal(J, _np(Je)) and np.array_equal(st, _np(se)) and (st == 0).all()
    # the legacy twin's brute force (ilqr_propagator.py:426-454), Qf = alpha I
    Jg, sg = ns["legacy_bruteforce_all_Jt_batched"](A, Bm, X, U, xg, ur, Q, R, 10.0, N, 0.1)
    Jge, sge = engine.bruteforce_jcurve(_t(A, dev), _t(Bm, dev), _t(X, dev), _t(U, dev),
                                        _t(xg, dev), _t(ur, dev), _t(Q, dev), _t(R, dev),
                                        _t(10.0 * np.eye(n), dev), N, w_stage=0.1, legacy=True)
    assert np.array_equal(Jg, _np(Jge)) and np.array_equal(sg, _np(sge))
    assert np.allclose(Jg, J, rtol=1e-9)  # well-conditioned: the legacy solve is the same
    from oracle import hop_oracle as orc
    Aa, Ba, Qa, Ra, Ri, z0, QT = orc.synth_lft_batch(40, 2, 5, 1, 16)
    Jl, stl, tsl = ns["propagator_all_Jt_aug_batched"](Aa, Ba, Qa, Ri[0], z0[0], QT, 16, 3, 16)
    r = engine.propagate(_t(Aa, dev), _t(Ba, dev), _t(Qa, dev), _t(Ri[0], dev), _t(z0[0], dev),
                         _t(QT, dev), t_min=3, t_max=16)
    assert _rel(Jl, _np(r.J)) <= 1e-12 and np.array_equal(tsl, _np(r.t_star))
    assert (stl == 0).all()
    del torch


def test_ilqr_batch_large_batch_spot_checks(dev):
    """the device outer loop at B = 65,536 quadrotor problems (16x the bench batch:
    A_k alone is 7.5 GB, the line search's candidate rows 4.2 GB): the first, a
    middle and the last problem against the oracle's scalar loop"""
    from time_opt_ilqr_amd import solver, systems
    F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap, _ = systems.make_quadrotor(N=100)
    Bn, N, T_min, T_max = 65536, 100, 20, 100
    rng = np.random.default_rng(31)
    X0 = x0 + 0.2 * rng.standard_normal((Bn, 12))
    Qf = np.asarray(io.orc.terminal_weight(alpha, 12))
    res = solver.ilqr_timeopt_batch(2, X0, xg, u_ref, Q, R, Qf, w, N, T_min, T_max, dt=F.dt,
                                    max_iter=2, wrap_idx=wrap, use_central_diff=False,
                                    device=dev, stage_timers=False)
    nh = _np(res["n_hist"])
    for b in (0, Bn // 2 + 1, Bn - 1):
        o = io.ilqr_timeopt(2, F.dt, X0[b], xg, u_ref, Q, R, Qf, w, N, T_min, T_max, max_iter=2,
                            wrap_idx=wrap, central=False)
        assert _np(res["T_hist"][b, :nh[b]]).tolist() == o["T_hist"], b
        assert _rel(_np(res["J_hist"][b, :nh[b]]), o["J_hist"]) <= 1e-9, b


@pytest.mark.gpu
@pytest.mark.parametrize("n,m", [(4, 2), (12, 4)])
def test_bruteforce_jcurve_edge_cases_vs_reference(dev, golden_dir, n, m):
    """Where solver.py:293-358 raises and where it does not (reference goldens,
    bruteforce_edge_cases.npz): only its chol_solve raises, so a non-finite e at
    t = 0 or an overflowing terminal V_0 leaves inf/NaN in J with a clean status,
    while a non-finite A_0, du_0 or later state fails a horizon (the reference
    raises out of the whole call).  n=4/m=2 runs the generic kernel, n=12/m=4 the
    exact-size one."""
    from time_opt_ilqr_amd import _lib, engine
    from oracle import hop_oracle as orc
    d = np.load(os.path.join(golden_dir, "bruteforce_edge_cases.npz"))
    tag, N = f"n{n}_m{m}", 12
    names = ("clean", "e0_nan", "xT_huge", "A0_inf", "du0_nan", "x3_nan")
    _, B, _, _, xg, ur, Q, R, alpha = orc.synth_riccati_problem(int(d[f"{tag}_seed"]), n, m, N)
    A = np.stack([d[f"{tag}_{k}_A"] for k in names])
    X = np.stack([d[f"{tag}_{k}_X"] for k in names])
    U = np.stack([d[f"{tag}_{k}_U"] for k in names])
    Bb = np.stack([B] * len(names))
    Qf = alpha * np.eye(n)
    J, st = engine.bruteforce_jcurve(_t(A, dev), _t(Bb, dev), _t(X, dev), _t(U, dev), _t(xg, dev),
                                     _t(ur, dev), _t(Q, dev), _t(R, dev), _t(Qf, dev), N,
                                     lm_lambda=1e-6, w_stage=0.5)
    J, st = _np(J), _np(st)
    for b, k in enumerate(names):
        raised = str(d[f"{tag}_{k}_raised"])
        if raised:
            assert (st[b] & _lib.ST_FAIL).any(), k
        else:
            ref = d[f"{tag}_{k}_J"]
            assert (st[b] == 0).all(), (k, st[b])
            assert np.array_equal(np.isfinite(J[b]), np.isfinite(ref)), (k, J[b], ref)
            f = np.isfinite(ref)
            if f.any():
                assert np.max(np.abs(J[b][f] - ref[f]) / np.abs(ref[f])) <= 1e-9, k


@pytest.mark.gpu
@pytest.mark.parametrize("n,m", [(4, 2), (12, 4)])
def test_legacy_bruteforce_lstsq_vs_reference(dev, golden_dir, n, m):
    """The legacy twin's brute force (ilqr_propagator.py:426-454) with its chol_solve
    (ilqr_propagator.py:33-43: 4 jitters, then np.linalg.lstsq): problem 0's R[0,0] =
    -1 makes Quu_reg indefinite, every such solve takes the least-squares fallback
    (ST_LU) instead of failing; problem 1 is clean.  Reference goldens
    legacy_bruteforce_cases.npz; the generic kernel runs both shapes."""
    from time_opt_ilqr_amd import _lib, engine
    from oracle import hop_oracle as orc
    d = np.load(os.path.join(golden_dir, "legacy_bruteforce_cases.npz"))
    tag, N = f"n{n}_m{m}", 10
    for i in range(2):
        A, B, X, U, xg, ur, Q, R, alpha = orc.synth_riccati_problem(int(d[f"{tag}_seed"]) + i, n,
                                                                   m, N)
        R = d[f"{tag}_p{i}_R"]
        J, st = engine.bruteforce_jcurve(_t(A[None], dev), _t(B[None], dev), _t(X[None], dev),
                                         _t(U[None], dev), _t(xg, dev), _t(ur, dev), _t(Q, dev),
                                         _t(R, dev), _t(alpha * np.eye(n), dev), N,
                                         lm_lambda=1e-6, w_stage=0.5, legacy=True)
        J, st = _np(J)[0], _np(st)[0]
        assert _rel(J, d[f"{tag}_p{i}_J"]) <= 1e-10, (i, J, d[f"{tag}_p{i}_J"])
        assert not (st & _lib.ST_FAIL).any()
        assert bool((st & _lib.ST_LU).any()) == (int(d[f"{tag}_p{i}_lstsq_calls"]) > 0)
        if i == 0:  # the modern brute force raises there (chol_solve has no fallback)
            Jm, sm = engine.bruteforce_jcurve(_t(A[None], dev), _t(B[None], dev),
                                              _t(X[None], dev), _t(U[None], dev), _t(xg, dev),
                                              _t(ur, dev), _t(Q, dev), _t(R, dev),
                                              _t(alpha * np.eye(n), dev), N, lm_lambda=1e-6,
                                              w_stage=0.5)
            assert (_np(sm)[0] & _lib.ST_FAIL).any()


@pytest.mark.gpu
@pytest.mark.parametrize("n,m", [(4, 2), (12, 4)])
def test_legacy_riccati_passes_vs_reference(dev, golden_dir, n, m):
    """The legacy twin's Riccati passes (hop_riccati_legacy_f64) against the
    reference's own (legacy_riccati_cases.npz): mode 0 = backward_pass_truncated
    (ilqr_propagator.py:375-400: no-jitter Cholesky gate, then chol_solve), mode 1 =
    value_expansions_and_gains_prefix (ilqr_propagator.py:237-287: chol_solve's 4
    jitters, then lstsq).  Problem 1's R[0, 0] = -1 makes Quu_reg indefinite:
    mode 0 fails the row (ok=False), mode 1 takes the least-squares fallback
    (ST_LU) at the steps where the reference calls lstsq.  n=4/m=2 and n=12/m=4
    both run the generic kernel (the legacy passes have no exact-size form)."""
    from time_opt_ilqr_amd import _lib, engine
    from oracle import hop_oracle as orc
    d = np.load(os.path.join(golden_dir, "legacy_riccati_cases.npz"))
    tag, N = f"n{n}_m{m}", 10
    T_star, T_bar, S_right, lm = d[f"{tag}_params"]
    T_star, T_bar, S_right = int(T_star), int(T_bar), int(S_right)
    L = T_bar + S_right
    for i in range(2):
        A, B, X, U, xg, ur, Q, R, alpha = orc.synth_riccati_problem(int(d[f"{tag}_seed"]) + i, n,
                                                                   m, N)
        R = d[f"{tag}_p{i}_R"]
        args = (_t(A[None], dev), _t(B[None], dev), _t(X[None], dev), _t(U[None], dev),
                _t(xg, dev), _t(ur, dev), _t(Q, dev), _t(R, dev), _t(alpha * np.eye(n), dev))
        r0 = engine.riccati(*args, T_star, float(lm), mode=0, legacy=True)
        st0 = int(_np(r0.status)[0])
        if bool(d[f"{tag}_p{i}_m0_ok"]):
            assert st0 & _lib.ST_FAIL == 0 and st0 & _lib.ST_LU == 0, st0
            assert _rel(_np(r0.K)[0, :T_star], d[f"{tag}_p{i}_m0_K"]) <= 1e-10
            assert _rel(_np(r0.k)[0, :T_star], d[f"{tag}_p{i}_m0_k"]) <= 1e-10
        else:  # (None, None, False): the gate fails the row, no lstsq
            assert st0 & _lib.ST_FAIL and not st0 & _lib.ST_LU, st0
        r1 = engine.riccati(*args, L, float(lm), mode=1, w_stage=0.5, legacy=True)
        st1 = int(_np(r1.status)[0])
        assert st1 & _lib.ST_FAIL == 0, st1
        assert bool(st1 & _lib.ST_LU) == (int(d[f"{tag}_p{i}_m1_lstsq_calls"]) > 0), st1
        tol = 1e-10 if i == 0 else 1e-8  # the pinv solve: Jacobi vs LAPACK's SVD
        assert _rel(_np(r1.K)[0, :L], d[f"{tag}_p{i}_m1_K"]) <= tol
        assert _rel(_np(r1.k)[0, :L], d[f"{tag}_p{i}_m1_k"]) <= tol
        assert _rel(_np(r1.Vxx)[0, :L + 1], d[f"{tag}_p{i}_m1_Vxx"]) <= tol
        assert _rel(_np(r1.Vx)[0, :L + 1], d[f"{tag}_p{i}_m1_Vx"]) <= tol
        assert _rel(_np(r1.V0)[0, :L + 1], d[f"{tag}_p{i}_m1_V0"]) <= tol


@pytest.mark.parametrize("tag", TAGS)
def test_zero_step_is_rejected_like_the_reference(dev, golden_dir, tag):
    """the reference rolls out every candidate with the same F as the
    current trajectory, so a zero step (K = 0, k = 0) reproduces X bit for bit and
    J_new < J_old (strict, solver.py:233-286) rejects it.  On the device the first
    iteration's X comes from hop_rollout_f64 and the candidates from the line search's
    rollouts: they must be the same arithmetic, or an ulp of J accepts the step."""
    import torch
    from time_opt_ilqr_amd import engine
    d, sid, wrap, obs = _case(golden_dir, tag)
    N, dt = int(d["N"]), float(d["dt"])
    n, m = d["Q"].shape[0], d["R"].shape[0]
    Bn = 64
    rng = np.random.default_rng(61)
    x0 = d["x0"] + 0.05 * rng.standard_normal((Bn, n))
    U = d["u_ref"].reshape(1, 1, -1) + 0.1 * rng.standard_normal((Bn, N, m))
    X = engine.rollout(sid, _t(x0, dev), _t(U, dev), dt)
    T = np.full(Bn, N, dtype=np.int32)
    T[::3] = N // 2
    K = torch.zeros((Bn, N, m, n), dtype=torch.float64, device=dev)
    k = torch.zeros((Bn, N, m), dtype=torch.float64, device=dev)
    r = engine.forward_linesearch(sid, X, _t(U, dev), T, K, k, _cost(d, wrap, obs, dev), dt)
    torch.cuda.synchronize()
    fin = np.isfinite(_np(r.J_old))
    assert fin.any()
    acc = _np(r.accepted)  # alpha index, -1 none accepted
    assert (acc == -1).all(), np.nonzero(acc != -1)[0][:8]
    assert torch.equal(r.X[torch.as_tensor(fin)], X[torch.as_tensor(fin)])
    assert torch.equal(r.J, r.J_old)


@pytest.mark.parametrize("vectorized", [False, True])
@pytest.mark.parametrize("tag", TAGS)
def test_ilqr_outer_loop_host_callables_vs_reference(dev, golden_dir, tag, vectorized):
    """solver.ilqr_timeopt with the dynamics as a plain Python callable F(x, u) (the
    oracle's NumPy dynamics, the reference's bit for bit) and, for the point mass, the
    obstacle cost as a plain callable too: the host evaluates F and the stage cost per
    problem (host_dynamics.py) while the select, Riccati and accept steps run on the
    device; ``vectorized``: F declared row-vectorised, so the linearisation is one call.
    Same bars as the device-dynamics run above."""
    from time_opt_ilqr_amd import solver, systems
    d, sid, wrap, obs = _case(golden_dir, tag)
    mk = list(systems.MAKERS.values())[sid]
    Fd, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap_idx, extra = mk(N=int(d["N"]))
    F = dyn._scalar_F(sid, Fd.dt)
    if vectorized:  # one F call per iteration for the whole FD linearisation
        from time_opt_ilqr_amd.host_dynamics import HostDynamics
        F = HostDynamics(F, len(x0), np.atleast_2d(R).shape[0], vectorized=True)
    cost = None
    if extra:
        cost = lambda x, u: io.obstacle_cost(x, obs)  # noqa: E731
    sol = solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, int(d["N"]), int(d["T_min"]),
                              int(d["T_max"]), max_iter=int(d["max_iter"]), wrap_idx=wrap_idx,
                              use_central_diff=bool(d["central"]), extra_stage_cost=cost)
    tol = 1e-8 if tag == "cartpole" else 1e-9
    assert sol["T_hist"] == [int(t) for t in d["T_hist"]]
    assert _rel(np.array(sol["J_hist"]), d["J_hist"]) <= tol
    assert sol["T_star"] == int(d["T_star"])
    assert _rel(np.nan_to_num(sol["X"]), np.nan_to_num(d["X"])) <= 100 * tol


@pytest.mark.parametrize("vectorized", [False, True])
@pytest.mark.parametrize("tag", ["di", "pointmass"])
def test_ilqr_batch_host_callables_vs_oracle(dev, tag, vectorized):
    """ilqr_timeopt_batch with a Python-callable system (host_dynamics.HostDynamics: the
    host rolls out, linearises and line-searches every problem, the device selects,
    runs the Riccati pass and accepts): a batch with different x0 -- double integrator,
    and the point mass with its obstacle cost as a plain callable (every select hands
    over: the pipelined s <= 5 rerun on two problems) -- per-problem T_hist / J_hist /
    T* equal to the oracle's scalar runs"""
    from time_opt_ilqr_amd import host_dynamics, solver, systems
    sid = dyn.SYSTEMS[tag]
    mk = list(systems.MAKERS.values())[sid]
    F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, extra = \
        mk(N=50) if tag == "di" else mk()
    T_max = min(T_max, N)
    n, m = dyn.DIMS[sid]
    rng = np.random.default_rng(2)
    Bn = 5 if tag == "di" else 2
    X0 = x0 + rng.uniform(-1.5 if tag == "di" else -0.05, 1.5 if tag == "di" else 0.05, (Bn, n))
    Qf = np.asarray(io.orc.terminal_weight(alpha, n))
    obs, cost = None, None
    if extra:
        obs = np.array([[o[0], o[1], r, wt] for o, r, wt in systems.OBSTACLES])
        cost = lambda x, u: io.obstacle_cost(x, obs)  # noqa: E731
    iters = 12 if tag == "di" else 6
    sysh = host_dynamics.HostDynamics(dyn._scalar_F(sid, F.dt), n, m, vectorized=vectorized)
    res = solver.ilqr_timeopt_batch(sysh, X0, xg, u_ref, Q, np.atleast_2d(R), Qf, w, N, T_min,
                                    T_max, max_iter=iters, wrap_idx=wrap_idx,
                                    use_central_diff=tag != "di", extra_stage_cost=cost)
    nh = _np(res["n_hist"])
    for b in range(Bn):
        o = io.ilqr_timeopt(sid, F.dt, X0[b], xg, u_ref, Q, np.atleast_2d(R), Qf, w, N, T_min,
                            T_max, max_iter=iters, wrap_idx=wrap_idx, central=tag != "di",
                            obstacles=obs)
        assert _np(res["T_hist"][b, :nh[b]]).tolist() == o["T_hist"]
        assert _rel(_np(res["J_hist"][b, :nh[b]]), o["J_hist"]) <= 1e-9
        assert int(res["T_star"][b]) == o["T_star"]


@pytest.mark.parametrize("tag", ["di", "segway", "pointmass"])
def test_ilqr_bruteforce_outer_loop_host_callables_vs_reference(dev, golden_dir, tag):
    """method="bruteforce" (baseline1) with the dynamics as a plain Python callable and,
    for the point mass, the obstacle cost as a plain callable: the host evaluates them
    (host_dynamics.py), the device runs the brute-force J curve, the Riccati pass and the
    accept step; the reference's run reproduced to the device-dynamics test's bars"""
    from time_opt_ilqr_amd import solver, systems
    d, sid, wrap, obs = _bf_case(golden_dir, tag)
    mk = list(systems.MAKERS.values())[sid]
    Fd, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap_idx, extra = mk(N=int(d["N"]))
    cost = (lambda x, u: io.obstacle_cost(x, obs)) if extra else None  # noqa: E731
    sol = solver.ilqr_timeopt_baseline1(
        dyn._scalar_F(sid, Fd.dt), x0, xg, u_ref, Q, R, alpha, w, int(d["N"]), int(d["T_min"]),
        int(d["T_max"]), max_iter=int(d["max_iter"]), wrap_idx=wrap_idx,
        use_central_diff=bool(d["central"]), extra_stage_cost=cost)
    assert sol["T_hist"] == [int(t) for t in d["T_hist"]]
    assert _rel(np.array(sol["J_hist"]), d["J_hist"]) <= 1e-9
    assert sol["T_star"] == int(d["T_star"])
    assert np.max(np.abs(sol["J_curve"] - d["J_curve"]) / np.abs(d["J_curve"])) <= 1e-8


@pytest.mark.parametrize("tag", ["pointmass", "quadrotor"])
def test_ilqr_device_dynamics_python_cost_vs_reference(dev, golden_dir, tag):
    """a built-in system's DeviceDynamics with a Python stage cost (the obstacle cost as
    a plain callable for the point mass; a zero callable cost for the quadrotor): the
    host takes the cost and F's rows run on the device kernel in one launch per
    evaluation round (solver._device_rows); the reference's run reproduced"""
    from time_opt_ilqr_amd import solver, systems
    d, sid, wrap, obs = _case(golden_dir, tag)
    mk = list(systems.MAKERS.values())[sid]
    F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap_idx, extra = mk(N=int(d["N"]))
    n = len(x0)
    if extra:
        cost = lambda x, u: io.obstacle_cost(x, obs)  # noqa: E731
    else:
        cost = lambda x, u: (0.0, np.zeros(n), np.zeros((n, n)))  # noqa: E731
    sol = solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, int(d["N"]), int(d["T_min"]),
                              int(d["T_max"]), max_iter=int(d["max_iter"]), wrap_idx=wrap_idx,
                              use_central_diff=bool(d["central"]), extra_stage_cost=cost)
    assert sol["T_hist"] == [int(t) for t in d["T_hist"]]
    assert _rel(np.array(sol["J_hist"]), d["J_hist"]) <= 1e-9
    assert sol["T_star"] == int(d["T_star"])
