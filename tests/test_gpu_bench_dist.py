"""GPU: bench.py's N > 1 path with the real kernels.

The driver's only multi-GPU run is its SCALE pass on an 8-GPU node.  This rehearses
the same code on the one-GPU box: `bench.py --gpus 2 --dist-backend gloo` starts two
ranks itself (torch.distributed.run as a child process), rank 0 builds, both pass the
barrier, each sweeps its contiguous shard with the product kernels on the shared GPU,
(T*, J*) is all-gathered every timed step, and the timings are MAX-all-reduced.  RCCL
(the default backend) refuses two ranks on one device, so the collectives go through
the host (distributed._host_collective); everything else is the nccl path's code.

The gathered selection must be bitwise what one process computes on the same shards
(problems are independent), and the line must carry n_gpus = 2 and
config 4's global batch: 2 x 32,768 (weak) or 262,144 (strong).
"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _env():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
              "LOCAL_WORLD_SIZE", "GROUP_RANK"):
        env.pop(k, None)
    env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


@pytest.mark.parametrize("scaling,global_batch", [("weak", 65536), ("strong", 262144)])
def test_bench_two_ranks_real_kernels_gloo(dev, tmp_path, scaling, global_batch):
    import torch
    sys.path.insert(0, REPO)
    import bench
    from time_opt_ilqr_amd import distributed as hd
    out = tmp_path / "gathered.npz"
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", "2",
           "--dist-backend", "gloo", "--scaling", scaling, "--steps", "3", "--warmup", "1",
           "--prewarm-s", "0", "--no-cpu-baseline", "--no-alt", "--no-h2d",
           "--gather-out", str(out)]
    p = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == scaling
    assert line["config"]["global_batch"] == global_batch
    assert line["config"]["parallelism"] == "dp2" and line["config"]["dist_backend"] == "gloo"
    assert line["status_ok"] is True
    assert line["value"] > 0 and line["ms_per_step"] > 0
    got = np.load(out)
    assert got["t_star"].shape == (global_batch,)
    # one process, the same shards (the workload seeds each shard by its first index)
    args = argparse.Namespace(s=13, m=4, N=100, dtype="f64", t_min=40, layout="auto",
                              no_alt=True)
    for r in range(2):
        lo, hi = hd.shard_bounds(global_batch, r, 2)
        launch, _ = bench._lft_workload(args, 2, lo, hi, dev)
        res = launch()
        torch.cuda.synchronize()
        assert int(res.status.abs().sum()) == 0
        assert np.array_equal(got["t_star"][lo:hi], res.t_star.cpu().numpy()), r
        assert np.array_equal(got["j_star"][lo:hi], res.j_star.cpu().numpy()), r
        del launch, res
        torch.cuda.empty_cache()
