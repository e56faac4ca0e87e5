"""Parity of the benchmarked frames at their own size.

Every BASELINE config the bench and the config log quote (cfg2, cfg3, cfg5,
and cfg4 on one GPU) is rendered at FULL size with the product kernels and
the product schedule -- the pass split of the 144 GiB budget, two pass sets on
two HIP streams with the lead, kParkChunk-entry park chunks (render.hip) over
hundreds of millions of queue entries, pixel-major items -- and a pixel subset of the frame is compared against the
oracle's render_pixels (oracle/zrt_oracle.c, the reference's renderWorker
restated, stage3.zig:222-245) with the same counter RNG: RGB8 AND linear
radiance bit-equal.  The subset is every 499th pixel plus every pixel of two
64x64 tiles (the top-left corner tile and one at the frame centre), so the
oracle side costs seconds.

A frame's pixels are independent (the RNG is keyed by pixel and sample), so
a pixel's value does not depend on which other pixels the oracle renders.
"""
import os

import numpy as np
import pytest

from zig_raytracing_contest_amd import RenderScene, camera_for, native, scenes

pytestmark = pytest.mark.gpu


def _threads():
    avail = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(avail, omp if omp > 0 else 16))


def _subset(w, h, stride=499, tile=64):
    pix = set(range(0, w * h, stride))
    for ty, tx in ((0, 0), (h // 2 // tile * tile, w // 2 // tile * tile)):
        for y in range(ty, min(h, ty + tile)):
            pix.update(range(y * w + tx, y * w + min(w, tx + tile)))
    return np.array(sorted(pix), np.uint32)


# (config, passes the default split must produce at that size: the schedule
# under test is the product's, not a thumbnail's)
FRAMES = [("cfg2", 2), ("cfg3", 2), ("cfg5", 2), ("cfg4", 2)]


@pytest.mark.parametrize("cfg,min_passes", FRAMES)
def test_benchmark_frame_subset_bitexact(oracle_mod, cfg, min_passes):
    d = scenes.CONFIGS[cfg]
    soup = scenes.get_scene(d["scene"])
    c = soup.camera(d["camera"])
    cam = camera_for(soup, d["camera"], d["width"], d["height"])
    rs = RenderScene(soup, device=0)
    try:
        img, res = rs.render(cam, num_samples=d["spp"], max_bounce=d["max_bounce"], linear=True)
        prof = rs.context.profile()
    finally:
        rs.close()
    assert prof["passes"] >= min_passes and prof["sets"] == 2, prof
    assert res["stats"]["samples"] == cam.w * cam.h * d["spp"]
    pixels = _subset(cam.w, cam.h)
    ocam = oracle_mod.camera_from_matrix(c.matrix, c.yfov, c.aspect, None if c.aspect else d["width"], d["height"])
    assert (ocam.w, ocam.h) == (cam.w, cam.h)
    rgb, lin, _ = oracle_mod.OracleScene(soup).render_pixels(ocam, d["spp"], d["max_bounce"], pixels,
                                                               oracle_mod.RNG_PATH, 0, _threads())
    packed = native.tile_pixels(cam.w, cam.h)
    where = np.empty(cam.w * cam.h, np.int64)
    where[packed] = np.arange(packed.size)
    gpu_lin = res["linear"][where[pixels]]
    gpu_rgb = img.reshape(-1, 3)[pixels]
    bad = np.flatnonzero(np.any(gpu_rgb != rgb, axis=1))
    assert bad.size == 0, f"{bad.size} of {pixels.size} pixels differ, first {pixels[bad[:5]]}"
    assert np.array_equal(gpu_lin.view(np.uint32), lin.view(np.uint32))
