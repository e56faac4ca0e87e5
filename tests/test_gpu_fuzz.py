"""Seeded random scenes against the CPU oracle, bit for bit, in every kernel
mode (round 6).  The fixed edge cases (test_gpu_edges.py) and the benchmark
stand-ins pin the paths one at a time; this file draws scenes that mix them:

- triangle families: small random triangles, axis-aligned quads (shared
  coordinates: the DDA's ties, linalg.zig:478-496), slivers and degenerate
  ones (Moller-Trumbore's det near 0, linalg.zig:683-722), huge triangles
  spanning the box (refs in many cells: the SAT build, linalg.zig:516-563),
  exact duplicates (equal t: the first ref in cell order wins);
- materials: random RGBA textures of 1-17 texels a side, repeat or clamp
  wrap, uvs outside [0, 1], OPAQUE / MASK / BLEND alpha, emissive factors and
  textures (stage1.zig:381-496, stage3.zig:82-123);
- cameras outside and inside the grid's box, wide and narrow fields of view;
- grid resolutions from 1 to 64 cells per axis (and one above 1024: the wide
  walk), image sizes 1-40 pixels, 1-3 spp, max_bounce 0-5, and the seed.

Each scene renders through the counting build (image, linear radiance and
the traversal counters) and then through the timed kernels in every mode
(escape table forced on / off, frustum bounds, IEEE division, park release
forced on / off).  The images are the oracle's whatever is drawn.
"""
import math
import os

import numpy as np
import pytest

from zig_raytracing_contest_amd import RenderScene, camera_for, native, scenes

MODES = {"default": 0, "escape": native.FLAG_ESCAPE, "no_escape": native.FLAG_NO_ESCAPE,
         "frustum": native.FLAG_FRUSTUM, "mt_exact": native.FLAG_MT_EXACT,
         "release": native.FLAG_RELEASE, "no_release": native.FLAG_NO_RELEASE}
F32 = np.float32


def _texture(rng):
    h, w = (int(x) for x in rng.integers(1, 18, 2))
    rgba = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    if rng.random() < 0.5:           # a mask with hard holes
        rgba[..., 3] = np.where(rng.random((h, w)) < 0.4, 0, 255).astype(np.uint8)
    return scenes.Texture(rgba, wrap_s_clamp=bool(rng.random() < 0.3), wrap_t_clamp=bool(rng.random() < 0.3),
                          has_alpha=bool(rng.random() < 0.8))


def _material(rng, ntex):
    base_tex = int(rng.integers(0, ntex)) if ntex and rng.random() < 0.6 else None
    emis_tex = int(rng.integers(0, ntex)) if ntex and rng.random() < 0.15 else None
    emis = tuple(float(x) for x in (rng.random(3) * 4.0 if rng.random() < 0.3 else np.zeros(3)))
    if emis_tex is not None and not any(emis):
        emis = (1.0, 1.0, 1.0)
    return scenes.Material(base_color=tuple(float(x) for x in rng.random(4)), base_texture=base_tex,
                           emissive=emis, emissive_texture=emis_tex,
                           alpha_mode=str(rng.choice(["OPAQUE", "MASK", "BLEND"])),
                           alpha_cutoff=float(rng.random()))


def _triangles(rng, n):
    """(n, 9) f32 triangles in roughly [-1, 1]^3, from the families above."""
    out = []
    while sum(len(t) for t in out) < n:
        kind = rng.integers(0, 5)
        if kind == 0:                                   # small random triangles
            c = rng.uniform(-1, 1, (8, 1, 3))
            out.append((c + rng.normal(0, 0.15, (8, 3, 3))).reshape(-1, 9))
        elif kind == 1:                                 # an axis-aligned quad (two triangles)
            ax = int(rng.integers(0, 3))
            lo, hi = np.sort(rng.uniform(-1, 1, (2, 2)), axis=0)
            k = F32(rng.choice([-0.5, 0.0, 0.25, 0.5, float(rng.uniform(-1, 1))]))
            q = np.array([[lo[0], lo[1]], [hi[0], lo[1]], [hi[0], hi[1]], [lo[0], hi[1]]], F32)
            v = np.insert(q, ax, k, axis=1)
            out.append(np.stack([np.concatenate([v[0], v[1], v[2]]), np.concatenate([v[0], v[2], v[3]])]))
        elif kind == 2:                                 # slivers and degenerate triangles
            a = rng.uniform(-1, 1, 3)
            b = rng.uniform(-1, 1, 3)
            t = rng.uniform(0, 1)
            eps = float(rng.choice([0.0, 1e-7, 1e-5, 1e-3]))
            c = a + t * (b - a) + eps * rng.normal(size=3)
            out.append(np.concatenate([a, b, c])[None, :])
            out.append(np.concatenate([a, a, b])[None, :])
        elif kind == 3:                                 # a huge triangle across the box
            out.append(rng.uniform(-3, 3, (1, 9)))
        else:                                           # duplicates of what is there
            if out:
                prev = np.concatenate(out)
                out.append(prev[rng.integers(0, len(prev), 3)])
    return np.ascontiguousarray(np.concatenate(out)[:n], F32)


def _scene(seed):
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.choice([1, 2, 17, 90, 400, 2000]))
    pos = _triangles(rng, n)
    v = pos.reshape(n, 3, 3)
    fn = np.cross(v[:, 1] - v[:, 0], v[:, 2] - v[:, 0])
    fn = fn / np.maximum(np.linalg.norm(fn, axis=1, keepdims=True), 1e-20)
    nrm = np.repeat(fn, 3, axis=0).reshape(n, 9) + rng.normal(0, 0.05, (n, 9))
    nrm = np.ascontiguousarray(nrm, F32)
    uv = np.ascontiguousarray(rng.uniform(-2, 3, (n, 6)), F32)
    textures = [_texture(rng) for _ in range(int(rng.integers(0, 4)))]
    materials = [_material(rng, len(textures)) for _ in range(int(rng.integers(1, 5)))]
    mat = rng.integers(0, len(materials), n).astype(np.uint32)
    lo, hi = v.reshape(-1, 3).min(0), v.reshape(-1, 3).max(0)
    mid = (lo + hi) / 2
    if rng.random() < 0.3:           # inside the box
        eye = mid + (hi - lo) * rng.uniform(-0.3, 0.3, 3)
    else:
        eye = mid + rng.normal(0, 1, 3) * 2.5 * max(float(np.max(hi - lo)), 1e-3)
    target = mid + rng.normal(0, 0.3, 3)
    yfov = math.radians(float(rng.choice([20.0, 50.0, 90.0, 120.0])))
    cam = scenes.CameraDef("Fuzz", scenes.look_at(tuple(float(x) for x in eye), tuple(float(x) for x in target)),
                           yfov, None)
    soup = scenes.SceneSoup(f"fuzz{seed}", pos, nrm, uv, mat, materials, textures, [cam]).bake_materials()
    if rng.random() < 0.1:
        res = (1100, int(rng.integers(1, 9)), int(rng.integers(1, 9)))
    else:
        res = tuple(int(x) for x in rng.integers(1, 65, 3))
    w, h = (int(x) for x in rng.integers(1, 41, 2)) if rng.random() < 0.8 else (int(x) for x in rng.integers(41, 97, 2))
    spp = int(rng.integers(1, 4))
    mb = int(rng.integers(0, 6))
    rseed = int(rng.integers(0, 2 ** 31))
    return soup, res, w, h, spp, mb, rseed


# ZRT_FUZZ_SEEDS=n widens the draw (round 6 ran 2,000 once: profiles/r06)
SEEDS = list(range(int(os.environ.get("ZRT_FUZZ_SEEDS", "160"))))
_KINDS = {}


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_fuzz_scene_bitexact_vs_oracle(oracle_mod, seed):
    soup, res, w, h, spp, mb, rseed = _scene(seed)
    c = soup.camera(None)
    ocam = oracle_mod.camera_from_matrix(c.matrix, c.yfov, None, w, h)
    rgb, lin, ctr = oracle_mod.OracleScene(soup, res).render(ocam, spp, mb, oracle_mod.RNG_PATH, rseed, 16)
    cam = camera_for(soup, None, w, h)
    pix = native.tile_pixels(cam.w, cam.h)
    rs = RenderScene(soup, res, device_build=bool(seed % 2))
    try:
        img, out = rs.render(cam, num_samples=spp, max_bounce=mb, seed=rseed, stats=True, linear=True)
        info = (seed, soup.num_triangles, res, w, h, spp, mb)
        assert np.array_equal(img.reshape(-1, 3), rgb), info
        assert np.array_equal(out["linear"].view(np.uint32), lin[pix].view(np.uint32)), info
        st = out["stats"]
        assert (st["segments"], st["cells_visited"], st["triangle_tests"], st["hits"]) == \
            tuple(int(x) for x in ctr[:4]), info
        for mode, flags in MODES.items():
            fast, fo = rs.render(cam, num_samples=spp, max_bounce=mb, seed=rseed, linear=True, flags=flags)
            _KINDS.setdefault(seed, set()).update(rs.context.profile()["kernels"])
            assert np.array_equal(fast.reshape(-1, 3), rgb), (mode,) + info
            assert np.array_equal(fo["linear"].view(np.uint32), lin[pix].view(np.uint32)), (mode,) + info
    finally:
        rs.close()


def test_fuzz_scenes_cover_the_families():
    """The draws reach what the file promises (checked on the host: no GPU
    call): cameras inside the box, wide grids, max_bounce 0, 1-pixel sides,
    masked materials and clamp-wrapped textures."""
    draws = [_scene(s) for s in SEEDS]
    assert any(r[0] > 1024 for _, r, *_ in draws)
    assert any(mb == 0 for *_, mb, _ in draws)
    assert any(min(w, h) == 1 for _, _, w, h, *_ in draws) or any(w * h < 40 for _, _, w, h, *_ in draws)
    assert any(m.alpha_mode == "MASK" and m.base_texture is not None for s, *_ in draws for m in s.materials)
    assert any(t.wrap_s_clamp or t.wrap_t_clamp for s, *_ in draws for t in s.textures)
    assert any(s.num_triangles >= 400 for s, *_ in draws)


MEDIUM = list(range(12))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", MEDIUM)
def test_fuzz_medium_scene_bitexact_vs_oracle(oracle_mod, seed):
    """Larger draws (128-320 pixels a side, 4-16 spp, 2,000-20,000
    triangles, 16-128 cells per axis): queues long enough for several park
    chunks per wave, the two pass sets and multi-pass splits
    (samples_per_pass); default, release forced on and the escape table forced
    on, each equal to the oracle's whole frame."""
    rng = np.random.default_rng(5000 + seed)
    soup, _, _, _, _, _, rseed = _scene(seed + 10000)
    n = int(rng.integers(2000, 20001))
    pos = _triangles(rng, n)
    v = pos.reshape(n, 3, 3)
    fn = np.cross(v[:, 1] - v[:, 0], v[:, 2] - v[:, 0])
    fn = fn / np.maximum(np.linalg.norm(fn, axis=1, keepdims=True), 1e-20)
    soup.pos = pos
    soup.nrm = np.ascontiguousarray(np.repeat(fn, 3, axis=0).reshape(n, 9), F32)
    soup.uv = np.ascontiguousarray(rng.uniform(-2, 3, (n, 6)), F32)
    soup.mat = rng.integers(0, soup.num_materials, n).astype(np.uint32)
    res = tuple(int(x) for x in rng.integers(16, 129, 3))
    w, h = (int(x) for x in rng.integers(128, 321, 2))
    spp = int(rng.integers(4, 17))
    mb = int(rng.integers(1, 6))
    c = soup.camera(None)
    ocam = oracle_mod.camera_from_matrix(c.matrix, c.yfov, None, w, h)
    rgb, lin, ctr = oracle_mod.OracleScene(soup, res).render(ocam, spp, mb, oracle_mod.RNG_PATH, rseed, 16)
    cam = camera_for(soup, None, w, h)
    pix = native.tile_pixels(cam.w, cam.h)
    rs = RenderScene(soup, res, device_build=bool(seed % 2))
    info = (seed, n, res, w, h, spp, mb)
    try:
        for flags, spp_pass in ((0, 0), (native.FLAG_RELEASE, 0), (native.FLAG_ESCAPE, 0), (0, max(1, spp // 3))):
            fast, fo = rs.render(cam, num_samples=spp, max_bounce=mb, seed=rseed, linear=True, flags=flags,
                                 samples_per_pass=spp_pass)
            assert np.array_equal(fast.reshape(-1, 3), rgb), (flags, spp_pass) + info
            assert np.array_equal(fo["linear"].view(np.uint32), lin[pix].view(np.uint32)), (flags, spp_pass) + info
            assert fo["stats"]["segments"] == int(ctr[0]), (flags, spp_pass) + info
    finally:
        rs.close()


@pytest.mark.gpu
def test_fuzz_reached_every_bounce_kernel():
    """(runs after the scenes above) the draws rendered bounces through both
    the park kernel and the lane walk (wide grids, the IEEE-division mode)."""
    if len(_KINDS) < len(SEEDS):
        pytest.skip("the fuzz scenes did not all run in this session")
    seen = set().union(*_KINDS.values())
    assert {"park", "bounce", "primary"} <= seen, seen
