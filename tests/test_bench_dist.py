"""CPU: bench.py's own multi-rank path.

`python bench.py --gpus 2 --dry-run` with no torchrun environment must start two
ranks itself (torch.distributed.run as a child process), shard the batch
contiguously, all-gather (T*, J*) over gloo and print n_gpus == 2 with the global
batch; a rank count that disagrees with --gpus, or more --gpus than visible HIP
devices, must fail loudly instead of timing one rank."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tests"))


def _env():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
              "LOCAL_WORLD_SIZE", "GROUP_RANK"):
        env.pop(k, None)
    env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "1"
    return env


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus,batch", [(2, 5), (3, 2)])
def test_bench_self_launch_dry_run_gathers_every_shard(tmp_path, gpus, batch):
    out = tmp_path / "g.npz"
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--dry-run",
           "--batch", str(batch), "--steps", "2", "--warmup", "1", "--prewarm-s", "0",
           "--no-cpu-baseline", "--dry-out", str(out)]
    p = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    line = _json_line(p.stdout)
    assert line["dry_run"] is True
    assert line["n_gpus"] == gpus
    assert line["config"]["global_batch"] == gpus * batch
    assert line["config"]["parallelism"] == f"dp{gpus}"
    assert line["status_ok"] is True
    got = np.load(out)
    import bench_dry_standin as sd
    ref = [sd.select_for(i) for i in range(gpus * batch)]
    assert got["t_star"].tolist() == [r[0] for r in ref]
    assert np.array_equal(got["j_star"], np.array([r[1] for r in ref]))


def test_bench_world_mismatch_fails():
    env = _env()
    env.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--dry-run", "--no-cpu-baseline"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode != 0
    assert "WORLD_SIZE=1" in p.stderr
    assert '"n_gpus"' not in p.stdout


def test_bench_more_gpus_than_devices_fails():
    """No HIP device here: --gpus 2 (a GPU run, not --dry-run) must refuse before
    launching anything rather than print a one-rank line."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two devices visible")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--no-cpu-baseline"], env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 2, p.stdout + p.stderr
    assert "HIP device" in p.stderr
    assert '"n_gpus"' not in p.stdout


@pytest.mark.parametrize("gpus,total", [(2, 7), (3, 5)])
def test_bench_strong_scaling_dry_run_shards_the_global_batch(tmp_path, gpus, total):
    """--scaling strong: the global batch stays fixed and is split into contiguous
    shards (sizes differ by at most one); the line names the mode and every
    problem's (T*, J*) comes back in order"""
    out = tmp_path / "s.npz"
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--dry-run",
           "--scaling", "strong", "--global-batch", str(total), "--steps", "2", "--warmup", "1",
           "--prewarm-s", "0", "--no-cpu-baseline", "--dry-out", str(out)]
    p = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    line = _json_line(p.stdout)
    assert line["n_gpus"] == gpus and line["scaling"] == "strong"
    assert line["config"]["global_batch"] == total and line["config"]["scaling"] == "strong"
    assert line["config"]["batch_per_gpu"] == -(-total // gpus)  # rank 0's shard
    got = np.load(out)
    import bench_dry_standin as sd
    ref = [sd.select_for(i) for i in range(total)]
    assert got["t_star"].tolist() == [r[0] for r in ref]
    assert np.array_equal(got["j_star"], np.array([r[1] for r in ref]))
