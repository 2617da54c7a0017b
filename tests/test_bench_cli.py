"""bench.py's rank handling on the CPU (nothing here touches a GPU).

Config 5 (``main.py:294-299``, ``device: [0,1,2,3]`` in
``config/nturgbd-cross-subject/train_joint.yaml:35``) is measured by ``bench.py --gpus N``:
without a launcher it starts the N ranks itself (``launch_command``, a child
``torch.distributed.run``); under a launcher the launcher's WORLD_SIZE must equal ``--gpus``.
The end-to-end two-rank line (``world_size`` / ``backend`` in ``config``) is
``tests/test_gpu_dist.py::test_bench_two_ranks_same_device``.
"""
import os
import subprocess
import sys

import pytest

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_check_world_rules():
    assert bench.check_world(1, {}) == 1
    assert bench.check_world(8, {}) is None                 # start the 8 ranks first
    assert bench.check_world(4, {"WORLD_SIZE": "4"}) == 4
    with pytest.raises(SystemExit) as e:
        bench.check_world(8, {"WORLD_SIZE": "1"})
    assert e.value.code == 2
    with pytest.raises(SystemExit):
        bench.check_world(1, {"WORLD_SIZE": "2"})


def test_launch_command_runs_this_bench_under_torchrun():
    cmd = bench.launch_command(["--gpus", "8", "--steps", "5"], 8, 29999)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29999" in cmd
    i = cmd.index(os.path.join(REPO, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "5"]


@pytest.mark.parametrize("env_ws, gpus", [("2", "1"), ("1", "8"), ("4", "2")])
def test_world_size_mismatch_exits_nonzero(env_ws, gpus):
    env = dict(os.environ, WORLD_SIZE=env_ws, RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", gpus,
                        "--steps", "1", "--warmup", "0"], env=env, capture_output=True,
                       text=True, timeout=300, cwd=REPO)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "WORLD_SIZE" in r.stderr and not r.stdout.strip()


def test_more_ranks_than_visible_gpus_exits_nonzero():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""   # (no GPU in this container anyway)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8",
                        "--steps", "1"], env=env, capture_output=True, text=True,
                       timeout=300, cwd=REPO)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "GPUs are visible" in r.stderr
