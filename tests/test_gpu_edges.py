"""GPU edge cases against the CPU oracle, bit for bit (image, linear radiance
and the traversal counters), on both ways of making a context (host build +
upload, and the device build straight into the context):

- image sizes that are not multiples of the 8x8 wave block or the 64x64 tile
  (1x1, 7x13, 65x3, 129x67): the ragged edges of stage3.zig:228-229's split;
- a camera inside the grid's bbox (Grid.traceRay's origin-inside branch,
  linalg.zig:443-469) and one that sees only sky (getEnvColor, stage3.zig:144-150);
- degenerate triangles (zero area, collinear, repeated vertices) mixed into a
  mesh: Moller-Trumbore's det == 0 path (linalg.zig:683-722) and the SAT
  build (linalg.zig:516-563);
- a one-triangle scene, grid resolutions 1x1x1 and non-cubic, and grids
  large enough for coarser occupancy bricks (300x260x280, 640x256x512);
- max_bounce 0 (primary rays only);
- grids with an axis above 1024 cells (the unpacked walk);
- the capacity guard's premise: counting, timed and counting renders on one
  context at growing sizes (every buffer regrown before its launch).
"""
import dataclasses
import math

import numpy as np
import pytest

from zig_raytracing_contest_amd import RenderScene, camera_for, native, scenes

pytestmark = pytest.mark.gpu


def _with_camera(soup, eye, target, yfov_deg=50.0):
    cam = scenes.CameraDef("Edge", scenes.look_at(eye, target), math.radians(yfov_deg), None)
    return dataclasses.replace(soup, cameras=[cam])


def _degenerate_sphere():
    s = scenes.get_scene("sphere")
    v = np.array([[0.2, 0.1, 0.9], [0.2, 0.1, 0.9], [0.2, 0.1, 0.9],      # one point
                  [-0.5, 0.0, 1.1], [0.0, 0.0, 1.1], [0.5, 0.0, 1.1],    # collinear
                  [0.3, -0.4, 1.05], [0.3, -0.4, 1.05], [0.6, 0.2, 1.05],  # two equal vertices
                  [-0.2, 0.3, 1.2], [0.1, 0.3, 1.2], [-0.2, 0.6, 1.2]],  # a proper one on top
                 np.float32).reshape(4, 9)
    n = np.tile(np.array([0, 0, 1], np.float32), (4, 3))
    uv = np.zeros((4, 6), np.float32)
    return dataclasses.replace(s, name="sphere_degenerate", pos=np.concatenate([s.pos, v]),
                               nrm=np.concatenate([s.nrm, n]), uv=np.concatenate([s.uv, uv]),
                               mat=np.concatenate([s.mat, np.zeros(4, s.mat.dtype)]))


def _one_triangle():
    s = scenes.get_scene("sphere")
    pos = np.array([[-1, -1, 0, 1, -1, 0, 0, 1, 0]], np.float32)
    nrm = np.tile(np.array([0, 0, 1], np.float32), (1, 3))
    return dataclasses.replace(s, name="one_triangle", pos=pos, nrm=nrm,
                               uv=np.zeros((1, 6), np.float32), mat=np.zeros(1, s.mat.dtype))


def _cornell_inside():
    s = scenes.get_scene("cornell")
    lo = s.pos.reshape(-1, 3).min(0)
    hi = s.pos.reshape(-1, 3).max(0)
    mid = (lo + hi) / 2
    eye = mid + (hi - lo) * np.array([0.1, 0.15, 0.2])
    return _with_camera(s, tuple(float(x) for x in eye), tuple(float(x) for x in lo), 70.0)


def _sky_only():
    return _with_camera(scenes.get_scene("sphere"), (0, 0, 3), (0, 0, 6))


SCENES = {"sphere": lambda: scenes.get_scene("sphere"), "degenerate": _degenerate_sphere,
          "one_triangle": _one_triangle, "cornell_inside": _cornell_inside, "sky_only": _sky_only}

# (scene, w, h, spp, max_bounce, grid resolution)
CASES = [("sphere", 1, 1, 3, 4, (128, 128, 128)),
         ("sphere", 7, 13, 2, 4, (128, 128, 128)),
         ("sphere", 65, 3, 2, 4, (128, 128, 128)),
         ("sphere", 129, 67, 1, 4, (128, 128, 128)),
         ("degenerate", 48, 40, 2, 4, (128, 128, 128)),
         ("degenerate", 48, 40, 2, 4, (3, 5, 2)),
         ("one_triangle", 40, 40, 2, 4, (128, 128, 128)),
         ("one_triangle", 40, 40, 2, 4, (1, 1, 1)),
         ("cornell_inside", 64, 48, 2, 4, (128, 128, 128)),
         ("cornell_inside", 64, 48, 2, 4, (31, 64, 17)),
         ("cornell_inside", 64, 48, 4, 0, (128, 128, 128)),
         ("sky_only", 32, 24, 2, 4, (128, 128, 128)),
         # grids whose 4^3-brick bits exceed wf_kernel's LDS share: coarser
         # occupancy bricks (8^3, 16^3), and no OccX (the lane-walk fallback)
         ("cornell_inside", 48, 40, 2, 4, (300, 260, 280)),
         ("sphere", 32, 24, 1, 3, (640, 256, 512)),
         # an axis above 1024 cells: the unpacked ("wide") wf_kernel
         # instantiations for the primary and the bounce launches
         ("sphere", 40, 32, 2, 4, (1100, 8, 8)),
         ("cornell_inside", 40, 32, 2, 4, (12, 1030, 9))]


@pytest.fixture(scope="module")
def soups():
    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = SCENES[name]()
        return cache[name]
    return get


_ORACLE = {}

# the timed kernels' variants: defaults, the escape table
# forced on / off (wf_park_kernel<true> / <false>) and the primary frustum
# bounds forced on (small frames skip them by default): every one of them on
# every degenerate grid (flat, 1x1x1, 3x5x2, coarse bricks, wide axes, sky)
# ... and (round 6) the IEEE-division lane walk that scenes with edges of
# 2^62 or more take (ZRT_FLAG_MT_EXACT forces it on any scene), and the park
# release forced on / off
MODES = {"default": 0, "escape": native.FLAG_ESCAPE, "no_escape": native.FLAG_NO_ESCAPE,
         "frustum": native.FLAG_FRUSTUM, "mt_exact": native.FLAG_MT_EXACT,
         "release": native.FLAG_RELEASE, "no_release": native.FLAG_NO_RELEASE}


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("device_build", [False, True], ids=["host-build", "device-build"])
@pytest.mark.parametrize("name,w,h,spp,mb,res", CASES)
def test_edge_render_bitexact_vs_oracle(oracle_mod, soups, name, w, h, spp, mb, res, device_build, mode):
    soup = soups(name)
    cam = camera_for(soup, None, w, h)
    key = (name, w, h, spp, mb, res)
    if key not in _ORACLE:
        c = soup.camera(None)
        ocam = oracle_mod.camera_from_matrix(c.matrix, c.yfov, None, w, h)
        _ORACLE[key] = oracle_mod.OracleScene(soup, res).render(ocam, spp, mb, oracle_mod.RNG_PATH, 0, 16)
    rgb, lin, ctr = _ORACLE[key]
    pix = native.tile_pixels(cam.w, cam.h)
    rs = RenderScene(soup, res, device_build=device_build)
    try:
        if mode == "default":   # the counting build (trace_kernel): the counters
            img, out = rs.render(cam, num_samples=spp, max_bounce=mb, stats=True, linear=True)
            assert np.array_equal(out["linear"].view(np.uint32), lin[pix].view(np.uint32))
            assert np.array_equal(img.reshape(-1, 3), rgb)
            st = out["stats"]
            assert (st["segments"], st["cells_visited"], st["triangle_tests"], st["hits"]) == \
                tuple(int(x) for x in ctr[:4])
            if name == "sky_only":   # the walk still runs: the box behind the camera is entered
                assert st["hits"] == 0
        fast, fo = rs.render(cam, num_samples=spp, max_bounce=mb, linear=True, flags=MODES[mode])
    finally:
        rs.close()
    assert np.array_equal(fast.reshape(-1, 3), rgb)
    assert np.array_equal(fo["linear"].view(np.uint32), lin[pix].view(np.uint32))


def test_growing_frames_counting_timed_counting(oracle_mod):
    """Round 2 once rendered a counting frame through a d_out that the timed
    path had never allocated.  One fresh context, frames of growing size,
    alternating counting (trace_kernel) and timed (wavefront) renders: every
    one equals the oracle, so every buffer was regrown before its launch
    (zrt_context_render checks each one's capacity before launching)."""
    soup = scenes.get_scene("cornell")
    c = soup.camera(None)
    rs = RenderScene(soup)
    osc = oracle_mod.OracleScene(soup)
    try:
        for w, h, spp in ((16, 16, 1), (48, 40, 3), (96, 64, 5), (160, 120, 2)):
            cam = camera_for(soup, None, w, h)
            ocam = oracle_mod.camera_from_matrix(c.matrix, c.yfov, None, w, h)
            rgb, _, _ = osc.render(ocam, spp, 4, oracle_mod.RNG_PATH, 0, 16, want_linear=False)
            for counting in (True, False, True):
                img, _ = rs.render(cam, num_samples=spp, max_bounce=4, stats=counting)
                assert np.array_equal(img.reshape(-1, 3), rgb), (w, h, spp, counting)
    finally:
        rs.close()


def _far_vertex(scale):
    """The sphere with one vertex moved to (scale, scale, scale): the
    triangles around it get edge components near `scale` (Moller-Trumbore
    dets up to ~scale^2, past the short reciprocal's 2^126 from 2^62 on)."""
    s = scenes.get_scene("sphere")
    pos = s.pos.astype(np.float32).copy()
    pos[0, 0:3] = np.float32(scale)
    return dataclasses.replace(s, name=f"far_vertex_{scale}", pos=pos)


def _far_floor(scale):
    """The sphere over a floor triangle with edges of 2 * scale, facing up
    (y = -1.5): Moller-Trumbore's det for a ray down onto it is
    4 scale^2 |d.y|, so from scale 2^62 on the bounce rays that hit it have
    dets of 2^124 .. 2^128 and past (the short reciprocal's 2^126 limit, the
    subnormal reciprocals, the overflow to inf)."""
    s = scenes.get_scene("sphere")
    S = np.float32(scale)
    tri = np.array([[-S, -1.5, -S, 0, -1.5, S, S, -1.5, -S]], np.float32)
    n = np.tile(np.array([0, 1, 0], np.float32), (1, 3))
    return dataclasses.replace(s, name=f"far_floor_{scale}", pos=np.concatenate([s.pos, tri]),
                               nrm=np.concatenate([s.nrm, n]), uv=np.concatenate([s.uv, np.zeros((1, 6), np.float32)]),
                               mat=np.concatenate([s.mat, np.zeros(1, s.mat.dtype)]))


# (scene, scale, needs the IEEE-division kernels)
FAR = [("vertex", 2.0 ** 40, False), ("vertex", 2.0 ** 62, True), ("vertex", 2.0 ** 64, True),
       ("vertex", 2.0 ** 100, True), ("vertex", float("inf"), True), ("vertex", float("nan"), False),
       ("floor", 2.0 ** 40, False), ("floor", 2.0 ** 62, True), ("floor", 2.0 ** 63, True),
       ("floor", 2.0 ** 64, True)]


@pytest.mark.parametrize("device_build", [False, True], ids=["host-build", "device-build"])
@pytest.mark.parametrize("kind,scale,exact", FAR, ids=[f"{k}-2^{int(np.log2(s))}" if np.isfinite(s) else f"{k}-{s}"
                                                        for k, s, _ in FAR])
def test_far_vertex_scene_renders_bitexact_vs_oracle(oracle_mod, kind, scale, exact, device_build):
    """the contexts no longer refuse scenes the reference
    renders (linalg.zig:696-722 takes any f32).  A scene with an edge
    component of 2^62 or more, or infinite, renders through the lane walk
    with the IEEE division (the bounce launches are the wf_kernel class, no
    park launch); image, linear radiance and counters equal the oracle's."""
    soup = _far_vertex(scale) if kind == "vertex" else _far_floor(scale)
    w, h, spp, mb, res = 40, 32, 2, 4, (16, 16, 16)
    cam = camera_for(soup, None, w, h)
    c = soup.camera(None)
    ocam = oracle_mod.camera_from_matrix(c.matrix, c.yfov, None, w, h)
    rgb, lin, ctr = oracle_mod.OracleScene(soup, res).render(ocam, spp, mb, oracle_mod.RNG_PATH, 0, 16)
    pix = native.tile_pixels(cam.w, cam.h)
    rs = RenderScene(soup, res, device_build=device_build)
    try:
        img, out = rs.render(cam, num_samples=spp, max_bounce=mb, stats=True, linear=True)
        assert np.array_equal(img.reshape(-1, 3), rgb)
        assert np.array_equal(out["linear"].view(np.uint32), lin[pix].view(np.uint32))
        st = out["stats"]
        assert (st["segments"], st["cells_visited"], st["triangle_tests"], st["hits"]) == \
            tuple(int(x) for x in ctr[:4])
        fast, fo = rs.render(cam, num_samples=spp, max_bounce=mb, linear=True)
        kinds = rs.context.profile()["kernels"]
        assert np.array_equal(fast.reshape(-1, 3), rgb)
        assert np.array_equal(fo["linear"].view(np.uint32), lin[pix].view(np.uint32))
        if exact:
            assert "park" not in kinds and "bounce" in kinds, kinds
        elif scale == 2.0 ** 40:
            assert "park" in kinds, kinds
        if kind == "floor":       # the floor is seen: hits beyond the sphere's
            assert st["hits"] > 0
    finally:
        rs.close()
