"""Host check of the park walk's escape table and of the primary walk's
frustum bound (csrc/escape.h): on random
grids and rays, no cell the cell-by-cell walk (Iterator.next, linalg.zig:478)
visits after a brick whose escape bit is set for the ray's direction bin
holds a triangle, so stopping the walk there leaves traceRay's result
(stage3.zig:152-185) unchanged (tests/cpp/escape_check.cpp).  The GPU images
with the table on are checked against the oracle in test_gpu_parity.py."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_escape_table_is_sound(tmp_path):
    exe = tmp_path / "escchk"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off",
                    "-I", os.path.join(ROOT, "zig_raytracing_contest_amd", "csrc"),
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "escape_check.cpp"), "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe), "24", "20000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    res = {}
    for line in r.stdout.splitlines():
        res.update(json.loads(line))
    # the table must actually fire (not vacuously sound) and never be wrong
    assert res["unsound"] == 0 and res["box_fails"] == 0, res
    assert res["escapes"] > 10000 and res["steps_after_escape"] > 100000, res
    # the primary frustum bound (escape.h frustum_bound lo): no ray of a block
    # enters an occupied cell below the block's bound, and the bound covers
    # most of the cells the rays pass
    assert res["frustum_unsound"] == 0, res
    assert res["frustum_cells_below_bound"] > 0.3 * res["frustum_steps"], res
    # the far bound: no occupied cell entered at or past it, and it cuts walks
    assert res["frustum_far_unsound"] == 0, res
    assert res["frustum_cells_past_far"] > 0.02 * res["frustum_steps"], res
    # the gap: no occupied cell entered inside it, and it holds cells
    assert res["frustum_gap_unsound"] == 0, res
    assert res["frustum_gap_blocks"] > 20 and res["frustum_cells_in_gap"] > 5000, res
    # zero / non-finite cell_size axes: no proof at all
    assert res["flat_grid_bits"] == 0 and res["flat_grid_bounds"] == 0, res
