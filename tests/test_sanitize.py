"""The byte parsers under AddressSanitizer + UndefinedBehaviorSanitizer (CPU).

gltf.cpp (+ json.h, GLB container, data URIs), png.cpp and jpeg.cpp read
untrusted files (stage1.zig:30-110 loadGltfFile / stbi_loadf_from_memory on
the reference side).  tests/cpp/parser_fuzz.cpp links exactly those sources
with -fsanitize=address,undefined, loads valid seeds -- a small textured,
alpha-masked glTF with .bin and PNG images, the same with a JPEG texture, as
GLB, with a base64 data-URI buffer, and PNG / JPEG images in the encodings
the loader supports -- then deterministic truncations and byte flips of each
file.  Any out-of-bounds access, signed overflow, bad shift or leak aborts
the run; a mutant may only load or return an error.
"""
import base64
import dataclasses
import json
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

from zig_raytracing_contest_amd import pngio, scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zig_raytracing_contest_amd", "csrc")


def _small_textured(tmp):
    soup = scenes.get_scene("contest")
    keep = np.concatenate([np.arange(0, 120), np.flatnonzero(soup.mat == 5)[:40]])   # ground + leaf cards
    small = dataclasses.replace(soup, pos=soup.pos[keep], nrm=soup.nrm[keep], uv=soup.uv[keep],
                                mat=soup.mat[keep])
    out = [scenes.write_gltf(small, os.path.join(tmp, "g", "small.gltf"))]
    try:
        import PIL  # noqa: F401
        rgba = small.textures[0].rgba.copy()
        rgba[..., :3] = np.clip(rgba[..., :3].astype(int) +
                                np.random.default_rng(1).integers(-30, 31, rgba[..., :3].shape), 0, 255)
        sj = dataclasses.replace(small, textures=[dataclasses.replace(small.textures[0], rgba=rgba)] +
                                 list(small.textures[1:]))
        out.append(scenes.write_gltf(sj, os.path.join(tmp, "j", "small.gltf"), jpeg_quality=85))
    except ImportError:
        pass
    return out


def _to_glb(gltf_path, glb_path):
    doc = json.load(open(gltf_path))
    d = os.path.dirname(gltf_path)
    binb = open(os.path.join(d, doc["buffers"][0]["uri"]), "rb").read()
    del doc["buffers"][0]["uri"]
    js = json.dumps(doc).encode()
    js += b" " * (-len(js) % 4)
    binb += b"\0" * (-len(binb) % 4)
    body = struct.pack("<II", len(js), 0x4E4F534A) + js + struct.pack("<II", len(binb), 0x004E4942) + binb
    with open(glb_path, "wb") as f:
        f.write(b"glTF" + struct.pack("<II", 2, 12 + len(body)) + body)
    for im in doc.get("images", []):
        shutil.copy(os.path.join(d, im["uri"]), os.path.dirname(glb_path))


def _to_data_uri(gltf_path, out_path):
    doc = json.load(open(gltf_path))
    d = os.path.dirname(gltf_path)
    binb = open(os.path.join(d, doc["buffers"][0]["uri"]), "rb").read()
    doc["buffers"][0]["uri"] = "data:application/octet-stream;base64," + base64.b64encode(binb).decode()
    with open(out_path, "w") as f:
        json.dump(doc, f)
    for im in doc.get("images", []):
        shutil.copy(os.path.join(d, im["uri"]), os.path.dirname(out_path))


def _images(tmp):
    rng = np.random.default_rng(3)
    out = []
    img = rng.integers(0, 256, (19, 23, 4)).astype(np.uint8)
    for name, a in (("rgb.png", img[..., :3]), ("rgba.png", img)):
        p = os.path.join(tmp, name)
        pngio.write(p, a)
        out.append(p)
    try:
        from PIL import Image
    except ImportError:
        return out
    base = np.clip(np.add.outer(np.arange(24), np.arange(40))[..., None] * 5 +
                   rng.integers(-10, 11, (24, 40, 3)), 0, 255).astype(np.uint8)
    Image.fromarray(base[..., 0], "L").save(os.path.join(tmp, "gray.png"))
    Image.fromarray(base, "RGB").convert("P", palette=Image.ADAPTIVE, colors=16).save(os.path.join(tmp, "pal.png"))
    Image.fromarray(base[..., 0].astype(np.uint16) * 257).save(os.path.join(tmp, "g16.png"))
    out += [os.path.join(tmp, n) for n in ("gray.png", "pal.png", "g16.png")]
    for name, kw in (("b444.jpg", dict(quality=90, subsampling=0)), ("b420.jpg", dict(quality=75, subsampling=2)),
                     ("prog.jpg", dict(quality=80, subsampling=2, progressive=True)),
                     ("dri.jpg", dict(quality=70, subsampling=1, restart_marker_blocks=1))):
        p = os.path.join(tmp, name)
        Image.fromarray(base, "RGB").save(p, "JPEG", **kw)
        out.append(p)
    p = os.path.join(tmp, "gray.jpg")
    Image.fromarray(base[..., 0], "L").save(p, "JPEG", quality=85)
    out.append(p)
    return out


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_parsers_clean_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "parser_fuzz")
    srcs = [os.path.join(CSRC, f) for f in ("gltf.cpp", "png.cpp", "jpeg.cpp", "capi.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-ffp-contract=off",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I", os.path.join(ROOT, "include"), "-I", CSRC, *srcs,
                    os.path.join(ROOT, "tests", "cpp", "parser_fuzz.cpp"), "-o", exe, "-lz", "-pthread"],
                   check=True)
    seeds = []
    for g in _small_textured(str(tmp_path)):
        d = os.path.dirname(g)
        seeds.append(g)
        seeds += [os.path.join(d, f) for f in sorted(os.listdir(d)) if not f.endswith(".gltf")]
    glb_dir, uri_dir = tmp_path / "glb", tmp_path / "uri"
    glb_dir.mkdir()
    uri_dir.mkdir()
    _to_glb(seeds[0], str(glb_dir / "small.glb"))
    _to_data_uri(seeds[0], str(uri_dir / "small.gltf"))
    seeds += [str(glb_dir / "small.glb"), str(uri_dir / "small.gltf")]
    img_dir = tmp_path / "img"
    img_dir.mkdir()
    seeds += _images(str(img_dir))
    work = tmp_path / "work"
    work.mkdir()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:allocator_may_return_null=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, str(work), os.environ.get("ZRT_FUZZ_N", "1000"), *seeds], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(res)
    assert res["seed_failures"] == 0 and res["runs"] > 1500, res
