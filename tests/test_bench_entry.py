"""bench.py's process entry on CPU (no GPU call is made before these checks):
`--gpus N` against the launcher's WORLD_SIZE, and the command that starts
N ranks when no launcher is around (the driver's plain `bench.py --gpus N`).
The GPU half (the ranks actually rendering, one JSON line with n_gpus N and
the N = 1 image hash) is tests/test_boundary_gpu.py::
test_bench_entry_two_ranks_gloo_matches_one."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_world_check():
    assert bench.world_check(1, {}) == 1
    assert bench.world_check(8, {}) is None                  # spawn the 8 ranks
    assert bench.world_check(8, {"WORLD_SIZE": "8"}) == 8
    assert bench.world_check(1, {"WORLD_SIZE": "1"}) == 1
    with pytest.raises(SystemExit) as e:
        bench.world_check(3, {"WORLD_SIZE": "2"})
    assert e.value.code == 2
    with pytest.raises(SystemExit):
        bench.world_check(1, {"WORLD_SIZE": "8"})


def test_launcher_cmd_is_the_drivers_form():
    cmd = bench.launcher_cmd(4, ["--gpus", "4", "--steps", "2"], 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node" in cmd and cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-5:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "2"]


def test_mismatched_world_size_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2
    assert "WORLD_SIZE=2" in p.stderr
    assert '"metric"' not in p.stdout
