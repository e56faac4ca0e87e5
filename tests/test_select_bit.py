"""Host check of the park kernel's pair-refill select (csrc/dda.h select_bit,
the byte-table select that picks the r-th candidate pair of a cell range)
against a bit loop (tests/cpp/select_check.cpp).  The kernel compiles the same
header; its images are checked against the oracle in test_gpu_parity.py."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_select_bit_matches_bit_loop(tmp_path):
    exe = tmp_path / "selchk"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off",
                    "-I", os.path.join(ROOT, "zig_raytracing_contest_amd", "csrc"),
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "select_check.cpp"), "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    res = json.loads(r.stdout)
    assert res["fails"] == 0 and res["checked"] > 10000000, res


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_item_division_matches_hardware_division(tmp_path):
    """dda.h div_magic / div_by: the kernels' pixel-major item -> (pixel,
    sample) split, every samples-per-pass divisor S < 2^16."""
    exe = tmp_path / "divchk"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off",
                    "-I", os.path.join(ROOT, "zig_raytracing_contest_amd", "csrc"),
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "div_check.cpp"), "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe), "64"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    res = json.loads(r.stdout)
    assert res["fails"] == 0 and res["checked"] > 8000000, res
