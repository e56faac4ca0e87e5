"""Host-side logic that runs without a GPU: camera rules, tile sharding,
config.json, C-ABI exports."""
import json
import math
import re

import numpy as np
import pytest

from zig_raytracing_contest_amd import Config, camera_for, native, scenes

ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))


def test_abi_exports_every_declared_symbol():
    hdr = open(f"{ROOT}/include/zrt.h").read()
    declared = set(re.findall(r"\b(zrt_[a-z0-9_]+)\s*\(", hdr))
    L = native.lib()
    missing = [s for s in sorted(declared) if not hasattr(L, s)]
    assert not missing, missing
    assert L.zrt_abi_version() == 2
    assert L.zrt_error_string(-5) == b"unsupported configuration"
    assert set(native.EXPORTS) <= declared


def test_render_flags_match_the_header():
    """Every ZRT_FLAG_* of zrt.h has its native.FLAG_* twin with the same bit."""
    hdr = open(f"{ROOT}/include/zrt.h").read()
    flags = dict(re.findall(r"#define ZRT_FLAG_([A-Z_]+)\s+(0x[0-9a-fA-F]+)u", hdr))
    assert "NO_FRUSTUM" in flags and len(flags) >= 8, flags
    for name, val in flags.items():
        assert getattr(native, "FLAG_" + name) == int(val, 16), name


def test_render_config_layout_is_abi_stable():
    """ABI 2 took the device list out of the reserved words: same size and
    offsets of every ABI-1 field."""
    import ctypes as C
    rc = native.RenderConfig
    assert C.sizeof(rc) == 56
    assert rc.samples_per_pass.offset == 36 and rc.num_devices.offset == 40 and rc.devices.offset == 48


@pytest.mark.parametrize("name,cam,w,h", [("sphere", None, 256, 256), ("cornell", None, 512, 512),
                                          ("contest", "Camera 1", None, 1080),
                                          ("contest", "Camera 2", 3840, None),
                                          ("sponza", None, None, 1080)])
def test_camera_matches_oracle(oracle_mod, name, cam, w, h):
    soup = scenes.get_scene(name)
    c = soup.camera(cam)
    a = camera_for(soup, cam, w, h)
    b = oracle_mod.camera_from_matrix(c.matrix, c.yfov, c.aspect, w, h)
    assert (a.w, a.h) == (b.w, b.h)
    for k1, k2 in (("origin", "origin"), ("lower_left_corner", "llc"), ("right", "right"),
                   ("up", "up")):
        assert list(getattr(a, k1)) == list(getattr(b, k2)), k1


def test_camera_size_rules():
    m = scenes.look_at((0, 0, 3), (0, 0, 0))
    # stage1.zig:322-342
    with pytest.raises(native.ZrtError):
        native.camera_from_matrix(m, 0.8, None, None, None)       # OutputImgSizeIsNotSpecified
    with pytest.raises(native.ZrtError):
        native.camera_from_matrix(m, 0.8, 1.5, 100, 100)          # CameraHasAspectRatio
    with pytest.raises(native.ZrtError):
        native.camera_from_matrix(m, 0.8, None, 100, None)        # CameraHasntAspectRatio
    c = native.camera_from_matrix(m, 0.8, 16 / 9, None, 1080)
    assert (c.w, c.h) == (1920, 1080)
    c = native.camera_from_matrix(m, 0.8, 16 / 9, 1920, None)
    assert (c.w, c.h) == (1920, 1080)
    # up points world-down so row 0 is the top image row
    assert c.up[1] < 0


@pytest.mark.parametrize("w,h,tile,n", [(256, 256, 64, 1), (1920, 1080, 64, 8), (100, 37, 16, 3),
                                        (1, 1, 8, 2), (130, 70, 64, 5)])
def test_tile_partition_is_exact(w, h, tile, n):
    seen = np.zeros(w * h, np.int32)
    for r in range(n):
        px = native.tile_pixels(w, h, tile, r, n)
        seen[px] += 1
    assert (seen == 1).all()


def test_tile_order_blocks_of_64():
    px = native.tile_pixels(128, 128, 64, 0, 1)
    # first wave = first 8x8 block of the first tile
    blk = px[:64]
    assert sorted(blk.tolist()) == sorted(y * 128 + x for y in range(8) for x in range(8))


def test_config_json(tmp_path):
    p = tmp_path / "config.json"
    p.write_text(json.dumps({"grid_resolution": [128, 128, 128], "num_threads": None,
                             "num_samples": 3, "max_bounce": 4}))
    c = Config.load(str(p))
    assert c.grid_resolution == (128, 128, 128) and c.num_threads is None
    assert (c.num_samples, c.max_bounce) == (3, 4)
    p.write_text(json.dumps({"grid_resolution": [1, 2, 3], "num_samples": 1, "max_bounce": 1,
                             "bogus": 1}))
    with pytest.raises(ValueError):
        Config.load(str(p))


def test_reference_config_json_parses():
    ref = f"{ROOT}/config.json"
    c = Config.load(ref)
    assert c.grid_resolution == (128, 128, 128) and c.num_samples == 3 and c.max_bounce == 4


def test_render_needs_gpu_and_fails_loudly():
    if native.device_count() > 0:
        pytest.skip("GPU present")
    soup = scenes.get_scene("sphere")
    g = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat, (32, 32, 32))
    keep = []
    native.attach_materials(g.scene, soup.tex_desc, soup.texels, keep)
    with pytest.raises(native.ZrtError) as e:
        native.Context(g.scene)
    assert e.value.status == -2


def test_contexts_take_triangles_beyond_the_short_reciprocal_range():
    """Both context creators take every coordinate the reference takes
    (linalg.zig:696-722): an edge component of 2^62 or more, or infinite, is
    no longer refused (ZRT_ERR_UNSUPPORTED until round 5) but selects the
    IEEE-division kernels (zrt_context::mt_exact; rendered against the oracle
    by tests/test_gpu_edges.py::test_far_vertex_scene_renders_bitexact_vs_oracle).
    Without a GPU both creators get past validation and stop at the device
    probe (ZRT_ERR_NO_DEVICE)."""
    if native.device_count() > 0:
        pytest.skip("GPU present (the renders are the -m gpu test)")
    soup = scenes.get_scene("sphere")
    keep = []
    for scale in (2.0 ** 40, 2.0 ** 62, 2.0 ** 100, float("inf"), float("nan")):
        pos = soup.pos.astype(np.float32).copy()
        pos[0, 0:3] = scale
        g = native.Geometry(pos, soup.nrm, soup.uv, soup.mat, (8, 8, 8))
        native.attach_materials(g.scene, soup.tex_desc, soup.texels, keep)
        with pytest.raises(native.ZrtError) as e:
            native.Context(g.scene)
        assert e.value.status == -2, scale
        with pytest.raises(native.ZrtError) as e:
            native.Context.built(pos, soup.nrm, soup.uv, soup.mat, g.scene, (8, 8, 8))
        assert e.value.status == -2, scale


@pytest.mark.parametrize("w,h", [(1920, 1080), (7, 3), (1, 1), (640, 2000)])
def test_png_write_parallel_deflate_roundtrip(tmp_path, w, h):
    """zrt_png_write (main.zig:129-140 stbi_write_png stand-in): the zlib
    stream is deflated in row pieces on host threads and must still decode,
    pixel for pixel, with an independent reader."""
    import ctypes as C
    from zig_raytracing_contest_amd import pngio
    rng = np.random.default_rng(w * 7 + h)
    y, x = np.mgrid[0:h, 0:w]
    img = np.stack([(x * 255 // max(w - 1, 1)), (y * 255 // max(h - 1, 1)),
                    rng.integers(0, 256, (h, w))], -1).astype(np.uint8)
    p = str(tmp_path / "o.png")
    L = native.lib()
    L.zrt_png_write.argtypes = [C.c_char_p, C.c_void_p, C.c_uint32, C.c_uint32]
    assert L.zrt_png_write(p.encode(), img.ctypes.data, w, h) == 0
    got = pngio.read(p)
    assert got.shape[:2] == (h, w)
    assert np.array_equal(got[..., :3], img)
