"""The sharded path with the real kernels (the CPU gloo tests
stand the oracle in for the GPU compute): two ranks on the one GPU of the box, gloo
for the collective (RCCL refuses two ranks on one device), each rank sweeping its
contiguous shard of a config-2-shaped batch with hop_lft_sweep_f64 + the fused
argmin, then distributed.gather_selection: the gathered (T*, J*) must be bitwise the
single-process sweep of the whole batch (problems are independent),
for even and uneven shards and for a rank with an empty shard.  The device outer
loop's sharded form (ilqr_timeopt_sharded) runs the same way on a small DI batch."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, total, out_dir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from time_opt_ilqr_amd import distributed as hd
        from time_opt_ilqr_amd import engine, synth
        dev = torch.device("cuda", 0)
        N = 40
        # every rank draws the same global batch (seeded device RNG) and sweeps its shard
        A, Bm, Q, Ri, z0, QT = synth.device_batch(total, 13, 4, N, seed=77, device=dev)
        lo, hi = hd.shard_bounds(total, rank, world)
        sl = slice(lo, hi)
        ri = Ri[sl] if Ri.dim() == 3 else Ri
        if hi > lo:
            res = engine.propagate(A[sl].contiguous(), Bm[sl].contiguous(), Q[sl].contiguous(),
                                   ri.contiguous(), z0, QT[sl].contiguous(), t_min=10, t_max=N)
            ts, js = res.t_star.cpu(), res.j_star.cpu()
        else:
            ts = torch.zeros(0, dtype=torch.int32)
            js = torch.zeros(0, dtype=torch.float64)
        T, J = hd.gather_selection(ts, js, total)
        if rank == 0:
            full = engine.propagate(A, Bm, Q, Ri, z0, QT, t_min=10, t_max=N)
            torch.cuda.synchronize()
            np.savez(os.path.join(out_dir, "gathered.npz"), T=T.numpy(), J=J.numpy(),
                     T_full=full.t_star.cpu().numpy(), J_full=full.j_star.cpu().numpy(),
                     st=full.status.cpu().numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 4096), (2, 4097), (3, 2)])
def test_sharded_sweep_on_the_gpu_equals_one_process(tmp_path, world, total):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), total, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "gathered.npz")
    assert (got["st"] == 0).all()
    assert np.array_equal(got["T"], got["T_full"])
    assert np.array_equal(got["J"], got["J_full"])


def _case_di():
    from time_opt_ilqr_amd import systems
    from oracle import ilqr_oracle as io
    F, x0, xg, u_ref, Q, R, alpha, w, _, _, _, _, _ = systems.make_double_integrator(N=30)
    Qf = np.asarray(io.orc.terminal_weight(alpha, 2))
    return F, x0, xg, u_ref, Q, R, Qf, w


def _worker_loop(rank, world, port, total, method, out_dir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from time_opt_ilqr_amd import distributed as hd
        from time_opt_ilqr_amd import solver
        dev = torch.device("cuda", 0)
        F, x0, xg, u_ref, Q, R, Qf, w = _case_di()
        X0 = x0 + np.linspace(-1.0, 1.0, total)[:, None] * np.array([1.0, 0.3])
        kw = dict(dt=F.dt, max_iter=4, use_central_diff=False, method=method)
        full, local, (lo, hi) = hd.ilqr_timeopt_sharded(0, X0, xg, u_ref, Q, R, Qf, w, 30, 8, 30,
                                                         device=dev, **kw)
        assert (local is None) == (hi == lo)
        if rank == 0:
            ref = solver.ilqr_timeopt_batch(0, X0, xg, u_ref, Q, R, Qf, w, 30, 8, 30, device=dev,
                                            **kw)
            nh = ref["n_hist"].to(torch.int64)
            J_last = ref["J_hist"].gather(1, (nh - 1).clamp(min=0)[:, None])[:, 0]
            np.savez(os.path.join(out_dir, "loop.npz"),
                     **{k: v.cpu().numpy() for k, v in full.items()},
                     ref_T=ref["T_star"].cpu().numpy(), ref_n=nh.cpu().numpy(),
                     ref_J=J_last.cpu().numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total,method", [(2, 5, "propagator"), (3, 2, "bruteforce")])
def test_sharded_outer_loop_on_the_gpu_equals_one_process(tmp_path, world, total, method):
    """ilqr_timeopt_sharded with the device outer loop on every rank (one shard empty
    when there are more ranks than problems): the all-gathered T*, final J and
    iteration counts are the single-process batch's, bitwise."""
    import torch.multiprocessing as mp
    mp.spawn(_worker_loop, args=(world, _free_port(), total, method, str(tmp_path)),
             nprocs=world, join=True)
    got = np.load(tmp_path / "loop.npz")
    assert got["T_star"].tolist() == got["ref_T"].tolist()
    assert got["n_hist"].tolist() == got["ref_n"].tolist()
    assert np.array_equal(got["J_star"], got["ref_J"])
    assert not got["crashed"].any()
