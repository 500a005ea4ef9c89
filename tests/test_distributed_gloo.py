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
