"""stage1 (glTF load, textures, cameras) through the C ABI vs the generator.

The scenes are written by scenes.write_gltf with identity node transforms, so
the loaded soup must equal the generated one bit for bit (normals after the
reference loader's normalize, stage1.zig:246), the material table must equal
scenes.SceneSoup.bake_materials (stb's LDR->linear texels x factor, 1x1
dummies, clamp/repeat ranges, MASK alpha), and cameras must follow
stage1.zig:282-371 including its error cases.
"""
import json
import os

import numpy as np
import pytest

from zig_raytracing_contest_amd import camera_for, native, pngio, scenes


@pytest.fixture(scope="module")
def gltf_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("gltf")
    for n in ("sphere", "cornell", "contest"):
        scenes.write_gltf(scenes.get_scene(n), str(d / f"{n}.gltf"))
    return d


@pytest.mark.parametrize("name", ["sphere", "cornell", "contest"])
def test_soup_roundtrip(gltf_dir, name):
    soup = scenes.get_scene(name)
    g = native.Gltf(str(gltf_dir / f"{name}.gltf"), num_threads=4)
    pos, nrm, uv, mat = g.soup()
    assert pos.shape == soup.pos.shape
    assert np.array_equal(pos, soup.pos)
    assert np.array_equal(uv, soup.uv)
    assert np.array_equal(mat, soup.mat)
    exp_n = scenes.f32_normalize(soup.nrm.reshape(-1, 3)).reshape(-1, 9)
    assert np.array_equal(nrm, exp_n)


@pytest.mark.parametrize("name", ["sphere", "cornell", "contest"])
def test_materials_match_stage1(gltf_dir, name):
    soup = scenes.get_scene(name)
    g = native.Gltf(str(gltf_dir / f"{name}.gltf"))
    desc, tex = g.materials()
    assert desc.shape == soup.tex_desc.shape
    assert np.array_equal(desc[..., 1:], soup.tex_desc[..., 1:])
    for m in range(desc.shape[0]):
        for k, ch in ((0, 3), (1, 3), (2, 1)):
            n = int(desc[m, k, 1] * desc[m, k, 2] * ch)
            a = tex[desc[m, k, 0]:desc[m, k, 0] + n]
            b = soup.texels[soup.tex_desc[m, k, 0]:soup.tex_desc[m, k, 0] + n]
            assert np.array_equal(a, b), (m, k)


def test_cameras(gltf_dir):
    soup = scenes.get_scene("contest")
    g = native.Gltf(str(gltf_dir / "contest.gltf"))
    for name, w, h in (("Camera 1", None, 1080), ("Camera 2", 640, None)):
        a = g.camera(name, w, h)
        b = camera_for(soup, name, w, h)
        assert (a.w, a.h) == (b.w, b.h)
        for k in ("origin", "lower_left_corner", "right", "up"):
            assert list(getattr(a, k)) == list(getattr(b, k))
    with pytest.raises(native.ZrtError) as e:
        g.camera("nope", None, 1080)
    assert e.value.status == -8                     # CameraNotFound
    with pytest.raises(native.ZrtError) as e:
        g.camera("Camera 1", 100, 100)
    assert e.value.status == -9                     # CameraHasAspectRatio
    with pytest.raises(native.ZrtError):
        g.camera("Camera 1")                        # OutputImgSizeIsNotSpecified


def test_png_decode_variants(tmp_path):
    """PNG decode as stb (req_comp 4): RGB, RGBA, gray, gray+alpha, palette+tRNS."""
    rng = np.random.default_rng(3)
    rgba = rng.integers(0, 256, (7, 5, 4), dtype=np.uint8)
    for c in (3, 4):
        p = tmp_path / f"t{c}.png"
        pngio.write(str(p), rgba[..., :c])
        doc = {"asset": {"version": "2.0"}, "images": [{"uri": p.name}],
               "textures": [{"source": 0}], "materials": [
                   {"pbrMetallicRoughness": {"baseColorTexture": {"index": 0}},
                    "alphaMode": "BLEND"}]}
        gp = tmp_path / f"t{c}.gltf"
        gp.write_text(json.dumps(doc))
        desc, tex = native.Gltf(str(gp)).materials()
        base = tex[desc[0, 0, 0]:desc[0, 0, 0] + 35 * 3].reshape(7, 5, 3)
        assert np.array_equal(base, scenes.srgb8_to_linear(rgba[..., :3]))
        alpha_w = desc[0, 2, 1]
        if c == 4:   # BLEND with an alpha channel -> alpha texture
            a = tex[desc[0, 2, 0]:desc[0, 2, 0] + 35].reshape(7, 5)
            assert alpha_w == 5 and np.array_equal(a, scenes.alpha8_to_float(rgba[..., 3]))
        else:        # no alpha channel -> 1x1 dummy 1.0
            assert alpha_w == 1 and tex[desc[0, 2, 0]] == 1.0


def test_load_errors(tmp_path):
    with pytest.raises(native.ZrtError) as e:
        native.Gltf(str(tmp_path / "missing.gltf"))
    assert e.value.status == -6
    bad = tmp_path / "bad.gltf"
    bad.write_text("{not json")
    with pytest.raises(native.ZrtError) as e:
        native.Gltf(str(bad))
    assert e.value.status == -7


def _texels_to_u8(lin):
    """Invert the loader's per-byte sRGB->linear map (scenes.srgb8_to_linear)."""
    lut = scenes.srgb8_to_linear(np.arange(256, dtype=np.uint8))
    idx = np.searchsorted(lut, lin)
    idx = np.clip(idx, 0, 255)
    assert np.array_equal(lut[idx], lin)
    return idx.astype(np.int32)


@pytest.mark.parametrize("w,h,mode,kw", [
    (37, 23, "RGB", dict(quality=90, subsampling=0)),                    # baseline 4:4:4
    (64, 48, "RGB", dict(quality=75, subsampling=2)),                    # 4:2:0
    (33, 17, "RGB", dict(quality=85, subsampling=1)),                    # 4:2:2, odd size
    (50, 41, "RGB", dict(quality=80, subsampling=2, progressive=True)),  # progressive
    (40, 40, "RGB", dict(quality=95, subsampling=0, progressive=True)),
    (29, 31, "L", dict(quality=90)),                                     # grayscale
    (48, 32, "RGB", dict(quality=70, subsampling=2, restart_marker_blocks=2)),   # DRI
])
def test_jpeg_texture_decode(tmp_path, w, h, mode, kw):
    """JPEG textures (stage1.zig:58 stbi_loadf_from_memory on a JPEG; SURVEY.md
    §8 f1): the loader's decode against an independent decoder (PIL/libjpeg)
    on PIL-encoded images.  stb_image itself is not in the reference tree,
    so these texels are parity unpinned; the bar is a small per-channel
    tolerance (different IDCT rounding / upsampling filters)."""
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(w * h)
    y, x = np.mgrid[0:h, 0:w]
    base = np.stack([x * 255 // w, y * 255 // h, (x + y) * 127 // (w + h) + 60], -1)
    img = np.clip(base + rng.integers(-20, 21, base.shape), 0, 255).astype(np.uint8)
    pil = Image.fromarray(img if mode == "RGB" else img[..., 0], mode)
    p = tmp_path / "t.jpg"
    pil.save(str(p), "JPEG", **kw)
    ref = np.asarray(Image.open(str(p)).convert("RGB")).astype(np.int32)
    doc = {"asset": {"version": "2.0"}, "images": [{"uri": p.name}],
           "textures": [{"source": 0}], "materials": [
               {"pbrMetallicRoughness": {"baseColorTexture": {"index": 0}}}]}
    gp = tmp_path / "t.gltf"
    gp.write_text(json.dumps(doc))
    desc, tex = native.Gltf(str(gp)).materials()
    assert (desc[0, 0, 1], desc[0, 0, 2]) == (w, h)
    got = _texels_to_u8(tex[desc[0, 0, 0]:desc[0, 0, 0] + w * h * 3].reshape(h, w, 3))
    d = np.abs(got - ref)
    assert d.max() <= 3, (d.max(), d.mean())
    assert d.mean() < 0.5, d.mean()
