"""GPU: feedback gains and cost-to-go, per step, on real linearisations.

The north star's parity claim is "K_k / V_k matching NumPy to 1e-6 rel on identical
linearisations".  These tests check it step by step (tests/gain_check.py:
||got_k - ref_k|| / ||ref_k|| for every k, not one max-norm over the whole array):

  * the reference's own backward_pass_truncated output on the captured quadrotor and
    double-integrator linearisations (tests/golden/real_*.npz bwd_K / bwd_k, made by
    tests/golden/make_golden.py from /root/reference/solver.py:156-230 inside
    ilqr_timeopt): the device Riccati kernel (mode 0) and the drop-in
    horizon_selection.backward_pass_truncated;
  * value_expansions_and_gains_prefix (mode 1, horizon_selection.py:97-212) on the same
    inputs against the oracle (pinned to the reference by tests/test_oracle_golden.py);
  * the select + gains block of one outer iteration (solver.py:581-597: the
    trajectory-form select at rho_reg = 1e-12, then the truncated Riccati pass at each
    problem's T*) on all 347 problems of the 50-digit real-linearisation fixture
    (tests/golden/real_lin_batch_hp.npz): device K / k at the device T* against the
    oracle's backward_pass_truncated on the same device linearisation.
"""
import os

import numpy as np
import pytest

from gain_check import assert_per_step
from oracle import hop_oracle as orc

pytestmark = pytest.mark.gpu

TOL = 1e-6  # BASELINE.json north_star: K_k / V_k to 1e-6 relative, fp64


def _t(x, dev, dtype=None):
    import torch
    return torch.as_tensor(np.ascontiguousarray(x), dtype=dtype or torch.float64, device=dev)


@pytest.mark.parametrize("tag", ["Quad_N160", "DI_N50"])
def test_riccati_real_capture_per_step_vs_reference(dev, golden_dir, tag):
    """Device mode 0 against the reference's own K_k / k_k, every step; the drop-in
    likewise; mode 1 against the oracle's value expansions, every step."""
    import torch
    from time_opt_ilqr_amd import engine
    from time_opt_ilqr_amd import horizon_selection as hs
    d = np.load(os.path.join(golden_dir, f"real_{tag}.npz"))
    A, B, X, U = d["bwd_A"], d["bwd_B"], d["bwd_X"], d["bwd_U"]
    n, m = X.shape[1], U.shape[1]
    T, lm = int(d["bwd_T_star"]), float(d["bwd_lm"])
    wrap = [int(i) for i in d["wrap_idx"]] or None
    alpha, w = float(d["alpha"]), float(d["w"])
    Qf = orc.terminal_weight(alpha, n)
    args = [_t(x[None], dev) for x in (A, B, X, U)] + [_t(x, dev) for x in
                                                        (d["xg"], d["u_ref"], d["Q"], d["R"], Qf)]
    assert d["bwd_K"].shape == (T, m, n)
    r0 = engine.riccati(*args, torch.tensor([T], dtype=torch.int32, device=dev), lm, mode=0,
                        wrap_idx=wrap)
    assert int(r0.status[0]) == 0
    assert_per_step(r0.K[0, :T].cpu().numpy(), d["bwd_K"], TOL, f"{tag} K")
    assert_per_step(r0.k[0, :T].cpu().numpy(), d["bwd_k"], TOL, f"{tag} k")
    k, K, ok = hs.backward_pass_truncated(list(A), list(B), X, U, d["xg"], d["u_ref"], d["Q"],
                                          d["R"], alpha, T, lm_lambda=lm, wrap_idx=wrap)
    assert ok and len(K) == T
    assert_per_step(np.array(K), d["bwd_K"], TOL, f"{tag} drop-in K")
    assert_per_step(np.array(k), d["bwd_k"], TOL, f"{tag} drop-in k")
    # mode 1 (the brute-force / value-expansion pass) at the same horizon
    r1 = engine.riccati(*args, torch.tensor([T], dtype=torch.int32, device=dev), 1e-6, mode=1,
                        w_stage=w, wrap_idx=wrap)
    assert int(r1.status[0]) == 0
    Vxx, Vx, V0, K2, k2 = orc.riccati_expand(list(A), list(B), X, U, d["xg"], d["u_ref"],
                                             d["Q"], d["R"], alpha, T, 0, lm_lambda=1e-6,
                                             w_stage=w, wrap_idx=wrap)
    for f, ref in (("Vxx", Vxx), ("Vx", Vx), ("V0", V0)):
        assert_per_step(getattr(r1, f)[0, :T + 1].cpu().numpy(), np.array(ref), TOL, f"{tag} {f}")
    assert_per_step(r1.K[0, :T].cpu().numpy(), np.array(K2), TOL, f"{tag} mode-1 K")
    assert_per_step(r1.k[0, :T].cpu().numpy(), np.array(k2), TOL, f"{tag} mode-1 k")


@pytest.mark.parametrize("name", ["quadrotor", "segway", "cartpole", "di"])
def test_select_gains_real_fixture_per_step(dev, golden_dir, name):
    """solver.py:581-597 on every problem of the 50-digit fixture: the product select
    (propagate_traj, rho_reg = 1e-12) picks T*, then the device's truncated Riccati pass
    at that T* (lm = lm_init = 1e-3, solver.py:465) gives K_k / k_k within 1e-6 of the
    oracle's backward_pass_truncated on the same linearisation, every step of every
    problem; value_expansions_and_gains_prefix (mode 1) likewise on the first 16."""
    import torch
    from test_gpu_real_lin import _fixture_system
    from time_opt_ilqr_amd import engine
    f, F = _fixture_system(golden_dir, name)
    T_min, T_max = int(f["meta"][0]), int(f["meta"][1])
    t = lambda x: _t(x, dev)  # noqa: E731
    U = t(f["U"])
    X = engine.rollout(F.system_id, t(f["X0"]), U, F.dt)
    lin = engine.linearize(F.system_id, X, U, F.dt, central=True)
    n = X.shape[-1]
    alpha = f["alpha"][()] if f["alpha"].ndim == 0 else f["alpha"]
    P = orc.terminal_weight(alpha, n)
    Ri = orc.spd_inverse(orc.sym(f["R"]))[0]
    wrap = [int(i) for i in f["wrap"]] or None
    w = float(f["w"][0])
    sel = engine.propagate_traj(lin.A, lin.B, lin.a_res, X, U, t(f["xg"]), t(f["u_ref"]),
                                t(f["Q"]), t(Ri), t(P), t(np.array([w])), n_use=T_max,
                                wrap_idx=wrap, t_min=T_min, t_max=T_max)
    assert (sel.status.cpu().numpy() == 0).all()
    shared = [t(x) for x in (f["xg"], f["u_ref"], f["Q"], f["R"], P)]
    r0 = engine.riccati(lin.A, lin.B, X, U, *shared, sel.t_star, 1e-3, mode=0, wrap_idx=wrap)
    r1 = engine.riccati(lin.A, lin.B, X, U, *shared, sel.t_star, 1e-6, mode=1, w_stage=w,
                        wrap_idx=wrap)
    torch.cuda.synchronize()
    ts = sel.t_star.cpu().numpy()
    assert (ts >= T_min).all() and (ts <= T_max).all()
    st0, st1 = r0.status.cpu().numpy(), r1.status.cpu().numpy()
    Ah, Bh, Xh, Uh = (x.cpu().numpy() for x in (lin.A, lin.B, X, U))
    K0, k0 = r0.K.cpu().numpy(), r0.k.cpu().numpy()
    worst = 0.0
    for b in range(len(ts)):
        T = int(ts[b])
        k, K, ok = orc.riccati_truncated(list(Ah[b, :T]), list(Bh[b, :T]), Xh[b, :T + 1], Uh[b, :T],
                                         f["xg"], f["u_ref"], f["Q"], f["R"], alpha, T,
                                         lm_lambda=1e-3, wrap_idx=wrap)
        assert ok and st0[b] == 0, (b, int(st0[b]))
        worst = max(worst, assert_per_step(K0[b, :T], np.array(K), TOL, f"{name} {b} K"),
                    assert_per_step(k0[b, :T], np.array(k), TOL, f"{name} {b} k"))
        if b < 16:
            Vxx, Vx, V0, K2, k2 = orc.riccati_expand(list(Ah[b, :T]), list(Bh[b, :T]),
                                                     Xh[b, :T + 1], Uh[b, :T], f["xg"],
                                                     f["u_ref"], f["Q"], f["R"], alpha, T, 0,
                                                     lm_lambda=1e-6, w_stage=w, wrap_idx=wrap)
            assert st1[b] == 0
            for fld, ref in (("Vxx", Vxx), ("Vx", Vx), ("V0", V0)):
                got = getattr(r1, fld)[b, :T + 1].cpu().numpy()
                worst = max(worst, assert_per_step(got, np.array(ref), TOL, f"{name} {b} {fld}"))
            worst = max(worst, assert_per_step(r1.K[b, :T].cpu().numpy(), np.array(K2), TOL,
                                               f"{name} {b} mode-1 K"))
    print(f"{name}: {len(ts)} problems, worst per-step relative error {worst:.2e}")


def test_riccati_ill_conditioned_quadrotor_vs_40_digit(dev, golden_dir):
    """The fixture's quadrotor problem 9 near the pitch singularity: |A_k| up to 3e4,
    Vxx up to 3e10 and cond(Quu_reg) 3.5e7 at lm = 1e-6.  Round 5's offset-form Quu
    sweep left mode 1's Vxx 5e-6 off the oracle at step 34 (an entry of M^-1 ~ 1/d kept
    as 1 - that loses u d); the equilibrated sweep (riccati_fast.hip) is within 1e-6 per
    step of the same recursion evaluated in 40-digit arithmetic (tests/riccati_hp.py)
    on the device's own linearisation, mode 1 and mode 0 alike, as the fp64 oracle is."""
    import torch
    import riccati_hp as rh
    from gain_check import per_step_rel
    from test_gpu_real_lin import _fixture_system
    from time_opt_ilqr_amd import engine
    f, F = _fixture_system(golden_dir, "quadrotor")
    b = 9
    U = _t(f["U"][b:b + 1], dev)
    X = engine.rollout(F.system_id, _t(f["X0"][b:b + 1], dev), U, F.dt)
    lin = engine.linearize(F.system_id, X, U, F.dt, central=True)
    T = int(f["t_hp"][b])
    alpha = f["alpha"][()] if f["alpha"].ndim == 0 else f["alpha"]
    P = orc.terminal_weight(alpha, 12)
    wrap = [int(i) for i in f["wrap"]]
    w = float(f["w"][0])
    shared = [_t(x, dev) for x in (f["xg"], f["u_ref"], f["Q"], f["R"], P)]
    Tt = torch.tensor([T], dtype=torch.int32, device=dev)
    r1 = engine.riccati(lin.A, lin.B, X, U, *shared, Tt, 1e-6, mode=1, w_stage=w, wrap_idx=wrap)
    r0 = engine.riccati(lin.A, lin.B, X, U, *shared, Tt, 1e-3, mode=0, wrap_idx=wrap)
    torch.cuda.synchronize()
    assert int(r1.status[0]) == 0 and int(r0.status[0]) == 0
    A, B, Xh, Uh = (x[0].cpu().numpy() for x in (lin.A, lin.B, X, U))
    args = (A[:T], B[:T], Xh[:T + 1], Uh[:T], f["xg"], f["u_ref"], f["Q"], f["R"], P, T)
    Vh, Vxh, V0h, K1h = rh.riccati_hp(*args, 1e-6, mode=1, w_stage=w, wrap_idx=wrap)
    K0h, k0h = rh.riccati_hp(*args, 1e-3, mode=0, wrap_idx=wrap)
    for got, ref, what in ((r1.Vxx[0, :T + 1], Vh, "Vxx"), (r1.Vx[0, :T + 1], Vxh, "Vx"),
                           (r1.V0[0, :T + 1], V0h, "V0"), (r1.K[0, :T], K1h, "mode-1 K"),
                           (r0.K[0, :T], K0h, "mode-0 K"), (r0.k[0, :T], k0h, "mode-0 k")):
        assert_per_step(got.cpu().numpy(), ref, TOL, what)
    Vxx_o = orc.riccati_expand(list(A[:T]), list(B[:T]), Xh[:T + 1], Uh[:T], f["xg"], f["u_ref"],
                               f["Q"], f["R"], alpha, T, 0, lm_lambda=1e-6, w_stage=w,
                               wrap_idx=wrap)[0]
    dev_err = per_step_rel(r1.Vxx[0, :T + 1].cpu().numpy(), Vh)[0]
    orc_err = per_step_rel(np.array(Vxx_o), Vh)[0]
    print(f"quadrotor 9, T* {T}: Vxx per-step error vs 40 digits: device {dev_err:.1e}, "
          f"fp64 oracle {orc_err:.1e}")
