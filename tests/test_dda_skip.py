"""Host check of the exact empty-brick skip (csrc/dda.h BRICK_SKIP4) against
the cell-by-cell Iterator.next walk (DDA_STEP): same cells of occupied
bricks, bit-identical DDA state, same grid exit (tests/cpp/dda_skip_check.cpp);
and the park kernel's DDAW_STEP against DDA_STEP, step by step.
The GPU kernels compile the same header; their images are checked against
the oracle in test_gpu_parity.py."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
@pytest.mark.parametrize("bm", [0, 1])
def test_brick_skip_matches_cell_walk(tmp_path, bm):
    """bm = 1: the same checks on brick-major packed words (power-of-two grids;
    the kernels' layout for them since r05ag)."""
    exe = tmp_path / "ddachk"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", f"-DPK_BM_TEST={bm}",
                    "-I", os.path.join(ROOT, "zig_raytracing_contest_amd", "csrc"),
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "dda_skip_check.cpp"), "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe), "60", "6000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    import json
    res = json.loads(r.stdout)
    assert res["fails"] == 0 and res["walk_fails"] == 0 and res["walk_steps"] > 100000, res
    # the packed-word checks ran on grids of this layout (for bm = 1
    # the checker skips grids that do not pack brick-major, so zero counts
    # would pass silently): brick skips, fast-forwards and their steps
    assert res["layout_grids"] >= 10 and res["skipv"] > 1000 and res["ff"] > 1000 and res["ff_steps"] > 10000, res
