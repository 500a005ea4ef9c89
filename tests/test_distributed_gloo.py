"""CPU, world_size 2 over gloo: the multi-GPU plumbing of bench.py / the engine
(contiguous problem shards, no data-path collective, one all-gather of
(T*, J*)) reassembles exactly the single-process selection.  The per-shard
compute is stood in by the CPU oracle (no GPU here)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, total, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import hop_oracle as orc
        from time_opt_ilqr_amd import distributed as hd
        lo, hi = hd.shard_bounds(total, rank, world)
        A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(100 + lo, hi - lo, 4, 1, 12) \
            if hi > lo else [np.zeros((0,))] * 7
        ts = torch.zeros(hi - lo, dtype=torch.int32)
        js = torch.zeros(hi - lo, dtype=torch.float64)
        Jc = torch.zeros((hi - lo, 12), dtype=torch.float64)
        for i in range(hi - lo):
            # problem index lo+i uses seed 100+lo+i in both paths
            A1, B1, Q1, R1, Ri1, z1, QT1 = orc.synth_lft_problem(100 + lo + i, 4, 1, 12)
            o = orc.lft_sweep(A1, B1, Q1, Ri1, z1, QT1)
            t, j = orc.select_horizon(o["J"], 3, 12)
            ts[i], js[i] = int(t), float(j)
            Jc[i] = torch.as_tensor(o["J"])
        T, J = hd.gather_selection(ts, js, total)
        curves = hd.gather_curves(Jc, total)
        if rank == 0:
            np.savez(os.path.join(out_dir, "gathered.npz"), T=T.numpy(), J=J.numpy(),
                     curves=curves.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 9), (2, 16), (4, 9), (4, 3)])
def test_gloo_shards_and_gather(tmp_path, world, total):
    """world 2 and a 4-rank rehearsal (uneven shards, and more ranks than
    problems for some: 3 problems over 4 ranks leaves one rank empty)."""
    mp.spawn(_worker, args=(world, _free_port(), total, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "gathered.npz")
    from oracle import hop_oracle as orc
    T_ref, J_ref, C_ref = [], [], []
    for b in range(total):
        A1, B1, Q1, R1, Ri1, z1, QT1 = orc.synth_lft_problem(100 + b, 4, 1, 12)
        o = orc.lft_sweep(A1, B1, Q1, Ri1, z1, QT1)
        t, j = orc.select_horizon(o["J"], 3, 12)
        T_ref.append(int(t))
        J_ref.append(float(j))
        C_ref.append(o["J"])
    assert got["T"].tolist() == T_ref
    assert np.array_equal(got["J"], np.array(J_ref))
    assert np.array_equal(got["curves"], np.array(C_ref).reshape(total, 12))


def _oracle_batch(system, x0, xg, u_ref, Q, R, Qf, w, N, T_min, T_max, *, U_init=None,
                  device=None, dt=0.05, max_iter=4, use_central_diff=False,
                  method="propagator", **kw):
    """CPU stand-in for solver.ilqr_timeopt_batch (no GPU here): the oracle's scalar
    outer loop per problem, returned in the batch function's layout"""
    from oracle import ilqr_oracle as io
    Bn, H = len(x0), max_iter + 1
    J_hist = torch.zeros((Bn, H), dtype=torch.float64)
    T_hist = torch.zeros((Bn, H), dtype=torch.int32)
    n_hist = torch.zeros(Bn, dtype=torch.int32)
    T_star = torch.zeros(Bn, dtype=torch.int32)
    for b in range(Bn):
        o = io.ilqr_timeopt(0, dt, x0[b], xg, u_ref, Q, R, Qf, w, N, T_min, T_max,
                            max_iter=max_iter, central=use_central_diff, method=method)
        k = len(o["J_hist"])
        J_hist[b, :k] = torch.as_tensor(o["J_hist"])
        T_hist[b, :k] = torch.as_tensor(o["T_hist"], dtype=torch.int32)
        n_hist[b], T_star[b] = k, o["T_star"]
    return dict(J_hist=J_hist, T_hist=T_hist, n_hist=n_hist, T_star=T_star,
                crashed=torch.zeros(Bn, dtype=torch.int32))


def _case_di():
    from time_opt_ilqr_amd import systems
    from oracle import ilqr_oracle as io
    F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, _, _ = systems.make_double_integrator(N=30)
    Qf = np.asarray(io.orc.terminal_weight(alpha, 2))
    return F, x0, xg, u_ref, Q, R, Qf, w


def _worker_loop(rank, world, port, total, method, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from time_opt_ilqr_amd import distributed as hd
        from time_opt_ilqr_amd import solver
        solver.ilqr_timeopt_batch = _oracle_batch  # the GPU outer loop's stand-in
        F, x0, xg, u_ref, Q, R, Qf, w = _case_di()
        X0 = x0 + np.linspace(-1.0, 1.0, total)[:, None] * np.array([1.0, 0.3])
        full, local, (lo, hi) = hd.ilqr_timeopt_sharded(
            0, X0, xg, u_ref, Q, R, Qf, w, 30, 8, 30, dt=F.dt, max_iter=4,
            use_central_diff=False, method=method, device=torch.device("cpu"))
        assert (local is None) == (hi == lo)
        if rank == 0:
            np.savez(os.path.join(out_dir, "loop.npz"), **{k: v.numpy() for k, v in full.items()})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total,method", [(2, 5, "propagator"), (3, 2, "bruteforce")])
def test_gloo_sharded_outer_loop(tmp_path, world, total, method):
    """ilqr_timeopt_sharded: contiguous shards (one empty when there are more ranks
    than problems), one all-gather of (T*, final J, iterations, crashed) that
    reassembles exactly the single-process per-problem results"""
    mp.spawn(_worker_loop, args=(world, _free_port(), total, method, str(tmp_path)), nprocs=world,
             join=True)
    got = np.load(tmp_path / "loop.npz")
    F, x0, xg, u_ref, Q, R, Qf, w = _case_di()
    X0 = x0 + np.linspace(-1.0, 1.0, total)[:, None] * np.array([1.0, 0.3])
    ref = _oracle_batch(0, X0, xg, u_ref, Q, R, Qf, w, 30, 8, 30, dt=F.dt, max_iter=4,
                        method=method)
    nh = ref["n_hist"].numpy()
    assert got["T_star"].tolist() == ref["T_star"].tolist()
    assert got["n_hist"].tolist() == nh.tolist()
    J_last = np.array([ref["J_hist"][b, nh[b] - 1].item() for b in range(total)])
    assert np.array_equal(got["J_star"], J_last)
    assert not got["crashed"].any()


def test_sharded_inputs_broadcast_leading_one(monkeypatch):
    """ilqr_timeopt_sharded's per-problem slicing: a batch-form input with a leading
    dimension of 1 (one shared U_init [1, N', m], which ilqr_timeopt_batch
    broadcasts) passes through whole; [B, ...] is sliced; any other leading size
    is refused"""
    from time_opt_ilqr_amd import distributed as hd
    from time_opt_ilqr_amd import solver
    seen = {}

    def standin(system, x0, xg, u_ref, Q, R, Qf, w, N, T_min, T_max, *, U_init=None, **kw):
        seen["U_init"], seen["xg"] = U_init, xg
        return _oracle_batch(0, x0, np.zeros(2) + 2.0, u_ref, Q, R, Qf, w, N, T_min, T_max,
                             max_iter=1)

    monkeypatch.setattr(solver, "ilqr_timeopt_batch", standin)
    F, x0, xg, u_ref, Q, R, Qf, w = _case_di()
    X0 = np.stack([x0] * 3)
    U1 = np.zeros((1, 30, 1))
    hd.ilqr_timeopt_sharded(0, X0, xg, u_ref, Q, R, Qf, w, 30, 8, 30, U_init=U1,
                            device=torch.device("cpu"))
    assert seen["U_init"].shape == (1, 30, 1)
    hd.ilqr_timeopt_sharded(0, X0, np.stack([xg] * 3), u_ref, Q, R, Qf, w, 30, 8, 30,
                            U_init=np.zeros((3, 30, 1)), device=torch.device("cpu"))
    assert seen["U_init"].shape == (3, 30, 1) and seen["xg"].shape == (3, 2)
    with pytest.raises(ValueError):
        hd.ilqr_timeopt_sharded(0, X0, xg, u_ref, Q, R, Qf, w, 30, 8, 30,
                                U_init=np.zeros((2, 30, 1)), device=torch.device("cpu"))
