"""GPU: the small-s row-group path.

fp64 augmented blocks at s <= 5 (the drop-in propagator_all_Jt_aug on the reference's
own Segway / Cart-pole / DI / point-mass shapes, horizon_selection.py:36-86) at
batches up to lft_sweep_v2.hip's kSmallRowGroupMax run on the conditioned kernel's
row-group layout (SchedCondSmall: four problems per wave, one per 16-lane DPP row)
instead of lft_small.hip's one problem per lane, which at B = 4,096 filled 64 of the
1,024 SIMDs.  Checked here:

  * against the lane kernel (the previous default, which larger batches keep) on the
    same problems: J within 1e-12, T* and status equal, every small shape;
  * a forced hand-over: the rerun launch (lft_small.hip's LFT instantiation, the
    reference association) recomputes every problem, bitwise HOP_OPT_REFERENCE_ASSOC;
  * a genuine chol_inv escalation in a real cart-pole batch (the zero angle weight
    Q[2,2] = 0, /root/reference/systems.py:103, pushed just below zero at one stage:
    utils.py:69-93's jitter ladder): that problem's status and J are bitwise the
    reference association's, the rest of the batch bitwise what it is without it.
The 50-digit fixture tests (tests/test_gpu_real_lin.py, the `aug` path and the
drop-in) run on this path too.
"""
import numpy as np
import pytest

from oracle import hop_oracle as orc

pytestmark = pytest.mark.gpu

RG_MAX = 16384  # lft_sweep_v2.hip kSmallRowGroupMax


def _t(x, dev):
    import torch
    return torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)


@pytest.mark.parametrize("s,m,N", [(5, 1, 200), (5, 2, 60), (4, 2, 60), (4, 1, 60), (3, 1, 50),
                                   (2, 1, 50)])
def test_rowgroup_matches_lane_kernel(dev, s, m, N):
    """The same RG_MAX problems through the row-group kernel (a batch of RG_MAX) and
    through the lane-per-problem kernel (the same problems as the head of a batch one
    larger, which the dispatch gives to lft_small.hip)."""
    import torch
    from time_opt_ilqr_amd import engine, synth
    A, Bm, Q, Ri, z0, QT = synth.device_batch(RG_MAX + 1, s, m, N, seed=600 + 10 * s + m,
                                              device=dev)
    t_min = max(1, N // 4)
    lane = engine.propagate(A, Bm, Q, Ri, z0, QT, t_min=t_min, t_max=N)
    h = slice(0, RG_MAX)
    rg = engine.propagate(A[h].contiguous(), Bm[h].contiguous(), Q[h].contiguous(),
                          Ri[h].contiguous(), z0, QT[h].contiguous(), t_min=t_min, t_max=N)
    torch.cuda.synchronize()
    assert int(rg.status.abs().sum()) == 0 and int(lane.status.abs().sum()) == 0
    Jr, Jl = rg.J.cpu().numpy(), lane.J[h].cpu().numpy()
    rel = float(np.max(np.abs(Jr - Jl) / np.abs(Jl)))
    assert rel <= 1e-12, rel
    assert not np.array_equal(Jr, Jl)  # two kernels, not one
    assert np.array_equal(rg.t_star.cpu().numpy(), lane.t_star[h].cpu().numpy())
    # HOP_OPT_SMALL_LANE puts a batch under the crossover on the lane kernel: bitwise
    # the same problems in the batch above it (one problem per lane, batch-independent)
    from time_opt_ilqr_amd import _lib
    q = slice(0, 256)
    with _lib.options(small_lane=True):
        ln = engine.propagate(A[q].contiguous(), Bm[q].contiguous(), Q[q].contiguous(),
                              Ri[q].contiguous(), z0, QT[q].contiguous(), t_min=t_min, t_max=N)
    assert torch.equal(ln.J, lane.J[q]) and torch.equal(ln.t_star, lane.t_star[q])


@pytest.mark.parametrize("s,m", [(5, 1), (3, 1), (4, 2)])
def test_rowgroup_forced_handover_is_the_lft_kernel(dev, s, m):
    import torch
    from time_opt_ilqr_amd import _lib, engine
    Bn, N = 131, 40
    A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(7300 + s, Bn, s, m, N)
    Q = Q.copy()
    Q[70, 5] = -np.eye(s)  # chol_inv's LU slot
    args = [_t(x, dev) for x in (A, Bm, Q, Ri, z0[0], QT)]
    with _lib.options(force_handover=True):
        f = engine.propagate(*args, t_min=3, t_max=N)
    with _lib.options(reference_assoc=True):
        r = engine.propagate(*args, t_min=3, t_max=N)
    d = engine.propagate(*args, t_min=3, t_max=N)
    with _lib.options(no_rerun=True):
        ho = engine.propagate(*args, t_min=3, t_max=N).status.cpu().numpy()
    assert torch.equal(f.J, r.J) and torch.equal(f.status, r.status)
    assert torch.equal(f.t_star, r.t_star) and torch.equal(f.j_star, r.j_star)
    assert int(r.status[70]) & orc.ST_LU
    # default: only the bad problem is handed over, and it is the LFT kernel's
    assert (ho & _lib.ST_HANDOVER).nonzero()[0].tolist() == [70]
    assert torch.equal(d.status, r.status) and torch.equal(d.J[70], r.J[70])
    ok = torch.ones(Bn, dtype=torch.bool)
    ok[70] = False
    assert float(((d.J[ok] - r.J[ok]).abs() / r.J[ok].abs()).max()) <= 1e-9


def test_rowgroup_genuine_escalation_real_cartpole(dev, golden_dir):
    import torch
    from test_gpu_real_lin import _fixture_system
    from time_opt_ilqr_amd import _lib, engine
    f, F = _fixture_system(golden_dir, "cartpole")
    T_min, T_max = int(f["meta"][0]), int(f["meta"][1])
    nb = 64
    U = _t(f["U"][:nb], dev)
    X = engine.rollout(F.system_id, _t(f["X0"][:nb], dev), U, F.dt)
    lin = engine.linearize(F.system_id, X, U, F.dt, central=True)
    P = orc.terminal_weight(f["alpha"], X.shape[-1])
    Ri = orc.spd_inverse(orc.sym(f["R"]))[0]
    wrap = [int(i) for i in f["wrap"]]
    assert float(f["Q"][2, 2]) == 0.0  # systems.py:103: the zero angle weight
    blk = engine.augment(lin.A, lin.B, lin.a_res, X, U, _t(f["xg"], dev), _t(f["u_ref"], dev),
                         _t(f["Q"], dev), _t(P, dev), _t(np.array([float(f["w"][0])]), dev),
                         wrap_idx=wrap, n_build=T_max)
    Qa = blk.Q.clone()
    b, k = 37, 11
    Qa[b, k, 2, 2] -= 1e-7  # q_reg (1e-9) on a zero weight, now just indefinite
    args = (blk.A, blk.B, Qa, _t(Ri, dev), blk.z0, blk.QT)
    d0 = engine.propagate(blk.A, blk.B, blk.Q, _t(Ri, dev), blk.z0, blk.QT, t_min=T_min,
                          t_max=T_max)
    d = engine.propagate(*args, t_min=T_min, t_max=T_max)
    with _lib.options(reference_assoc=True):
        r = engine.propagate(*args, t_min=T_min, t_max=T_max)
    with _lib.options(no_rerun=True):
        ho = engine.propagate(*args, t_min=T_min, t_max=T_max).status.cpu().numpy()
    torch.cuda.synchronize()
    assert b in (ho & _lib.ST_HANDOVER).nonzero()[0].tolist()
    assert int(r.status[b]) & orc.ST_JITTER  # the ladder ran (utils.py:69-93)
    assert int(d.status[b]) == int(r.status[b])
    assert torch.equal(d.J[b], r.J[b]) and int(d.t_star[b]) == int(r.t_star[b])
    # every other problem: untouched by its neighbour's hand-over (bitwise the run
    # without the perturbation)
    oth = torch.ones(nb, dtype=torch.bool, device=d.J.device)
    oth[b] = False
    assert torch.equal(d.J[oth], d0.J[oth]) and torch.equal(d.status[oth], d0.status[oth])
    assert torch.equal(d.t_star[oth], d0.t_star[oth])


@pytest.mark.parametrize("s,m", [(5, 2), (5, 1), (4, 2), (3, 1), (2, 1)])
@pytest.mark.parametrize("N", [1, 63, 64, 65, 150])
def test_pipelined_small_rerun_bitwise(dev, s, m, N):
    """The fp64 s <= 5 rerun launch's pipeline (lft_small.hip lft_small_rerun_kernel:
    stage blocks, compose chain and queries on three waves in beats of 64 steps)
    against the one-lane LFT kernel (HOP_OPT_RERUN_LANE) and the reference association
    alone: J, status, T*, J* bitwise.  Hand-overs are chol_inv LU slots (Q_k = -I) at
    one and two problems of a workgroup (the pipeline) and at four and five (more than
    kSmallPipeMax = 3: the one-lane body); beats are cut at N = 1, 63, 64, 65, 150."""
    import torch
    from time_opt_ilqr_amd import _lib, engine
    Bn = 600
    A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(8100 + 7 * s + m, Bn, s, m, N)
    Q = Q.copy()
    # problems per workgroup: 192 (s = 5, three waves) or 256 (four)
    ppb = 192 if s == 5 else 256
    bad = [3] + [ppb + 10, ppb + 70] + [2 * ppb + i for i in (0, 1, 63, 64)]
    if 3 * ppb + 5 < Bn:
        bad += [3 * ppb + i for i in (5, 6, 7, 8, 9)]
    for j, b in enumerate(bad):
        Q[b, (7 * j) % N] = -np.eye(s)  # chol_inv's ladder ends in the LU slot
    args = [_t(x, dev) for x in (A, Bm, Q, Ri, z0[0], QT)]
    t_min = max(1, N // 3)
    d = engine.propagate(*args, t_min=t_min, t_max=N)
    with _lib.options(rerun_lane=True):
        ln = engine.propagate(*args, t_min=t_min, t_max=N)
    with _lib.options(reference_assoc=True):
        r = engine.propagate(*args, t_min=t_min, t_max=N)
    torch.cuda.synchronize()
    st = d.status.cpu().numpy()
    assert all(int(st[b]) & orc.ST_LU for b in bad), st[bad]
    for o in (ln, r):
        for b in bad:
            assert torch.equal(d.J[b].nan_to_num(7.0), o.J[b].nan_to_num(7.0)), b
        assert torch.equal(d.status[bad], o.status[bad])
        assert torch.equal(d.t_star[bad], o.t_star[bad])
        assert torch.equal(d.j_star[bad].nan_to_num(7.0), o.j_star[bad].nan_to_num(7.0))
    # the problems nobody handed over keep the conditioned kernel's values
    ok = np.ones(Bn, dtype=bool)
    ok[bad] = False
    okt = torch.as_tensor(ok, device=d.J.device)
    assert torch.equal(d.J[okt], ln.J[okt]) and int(d.status[okt].abs().sum()) == 0


def test_pipelined_small_rerun_point_mass_outer_loop(dev):
    """The point-mass obstacle run (every select hands its problem over: the obstacle
    Hessian makes Q_k indefinite) through the pipelined rerun and through the
    one-lane rerun: identical T_hist and J_hist, bit for bit"""
    from time_opt_ilqr_amd import _lib, solver, systems
    F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, wrap_idx, extra = \
        systems.make_point_mass_obstacles() if hasattr(systems, "make_point_mass_obstacles") \
        else list(systems.MAKERS.values())[3]()
    kw = dict(max_iter=15, wrap_idx=wrap_idx, extra_stage_cost=extra["extra_stage_cost"])
    a = solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, **kw)
    with _lib.options(rerun_lane=True):
        b = solver.ilqr_timeopt(F, x0, xg, u_ref, Q, R, alpha, w, N, T_min, T_max, **kw)
    assert a["T_hist"] == b["T_hist"] and a["J_hist"] == b["J_hist"]
    assert np.array_equal(a["J_curve"], b["J_curve"], equal_nan=True)


@pytest.mark.parametrize("nb", [1, 2, 3, 4])
def test_pipelined_small_rerun_many_lu_steps_bitwise(dev, nb):
    """Real cart-pole augmented blocks (fp64, s = 5, N = 200) with the stage block made
    indefinite at every other step, so chol_inv's ladder ends in the LU slot there and
    the chain's W_k often does too: the pipelined rerun (one to three hand-overs per
    workgroup; four run the one-lane body) against the one-lane rerun and the reference
    association alone, J / status / T* bitwise (a side-by-side ladder once differed
    here in the last bits from step 125 on: tools/dbg_handover.py)"""
    import torch
    from time_opt_ilqr_amd import _lib, engine, systems
    from time_opt_ilqr_amd.utils import as_terminal_weight
    N, Bn = 200, 8
    F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, wrap, _ = systems.make_cartpole_swingup(N=N)
    g = torch.Generator(device=dev)
    g.manual_seed(29)
    kw = dict(device=dev, dtype=torch.float64, generator=g)
    U = torch.as_tensor(u_ref, device=dev) + 2.0 * torch.randn((Bn, N, F.m), **kw)
    X = engine.rollout(F.system_id, torch.as_tensor(x0, device=dev) +
                       0.3 * torch.randn((Bn, F.n), **kw), U, F.dt)
    P = _t(as_terminal_weight(alpha, F.n), dev)
    Ri = torch.linalg.inv(_t(R, dev)).contiguous()
    lin = engine.linearize(F.system_id, X, U, F.dt, central=True)
    blk = engine.augment(lin.A, lin.B, lin.a_res, X, U, _t(xg, dev), _t(u_ref, dev), _t(Q, dev),
                         P, w, wrap_idx=wrap)
    h = slice(0, nb)
    Qh = blk.Q[h].clone()
    Qh[:, 1::2, 0, 0] -= 1.0
    args = (blk.A[h].contiguous(), blk.B[h].contiguous(), Qh, Ri, blk.z0, blk.QT[h].contiguous())
    a = engine.propagate(*args, t_min=50, t_max=N)
    with _lib.options(rerun_lane=True):
        b = engine.propagate(*args, t_min=50, t_max=N)
    with _lib.options(reference_assoc=True):
        c = engine.propagate(*args, t_min=50, t_max=N)
    torch.cuda.synchronize()
    assert all(int(v) & orc.ST_LU for v in a.status.tolist())
    for o in (b, c):
        assert torch.equal(a.J.nan_to_num(7.0), o.J.nan_to_num(7.0))
        assert torch.equal(a.status, o.status) and torch.equal(a.t_star, o.t_star)
