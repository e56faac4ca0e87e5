"""Host check of the OccX / lane-walk decision (csrc/zrt_internal.h
occx_usable, tests/cpp/occx_plan_check.cpp): a grid of more than 2^24 4^3
bricks (> 2^30 cells, still a valid reference grid) must fall back to the lane
walk rather than fail context creation."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_occx_decision(tmp_path):
    exe = tmp_path / "occxchk"
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "zig_raytracing_contest_amd", "csrc"),
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "cpp", "occx_plan_check.cpp"),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
