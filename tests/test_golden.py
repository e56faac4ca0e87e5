"""Committed golden fixtures (tests/golden/, made by tools/make_golden.py).

CPU: the oracle still reproduces every fixture bit for bit (guards the
checker itself).  GPU: the HIP path reproduces the build-mode fixtures
without consulting the oracle at run time.
"""
import os

import numpy as np
import pytest

from zig_raytracing_contest_amd import RenderScene, camera_for, native, scenes

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RENDERS = ["sphere", "cornell", "contest"]


def _load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def _ocam(orc, g, name):
    soup = scenes.get_scene(name)
    c = soup.camera(str(g["camera"]) or None)
    return orc.camera_from_matrix(c.matrix, c.yfov, c.aspect, None if c.aspect else int(g["w"]),
                                  int(g["h"]))


@pytest.mark.parametrize("name", RENDERS)
def test_oracle_reproduces_render_goldens(oracle_mod, name):
    g = _load(f"render_{name}.npz")
    sc = oracle_mod.OracleScene(scenes.get_scene(name))
    cam = _ocam(oracle_mod, g, name)
    rgb, lin, ctr = sc.render(cam, int(g["spp"]), int(g["max_bounce"]), oracle_mod.RNG_PATH, 0, 8)
    assert np.array_equal(rgb, g["rgb"]) and np.array_equal(lin, g["linear"])
    assert np.array_equal(ctr, g["counters"])
    rgb, lin, ctr = sc.render(cam, int(g["spp"]), int(g["max_bounce"]), oracle_mod.RNG_REF, 0, 4)
    assert np.array_equal(rgb, g["rgb_ref4"]) and np.array_equal(ctr, g["counters_ref4"])


def test_oracle_reproduces_vector_goldens(oracle_mod):
    v = _load("vectors.npz")
    for i in range(len(v["tri"])):
        t = v["tri"][i]
        h, r = oracle_mod.tri_intersect(t[:3], t[3:6], t[6:], v["tri_o"][i], v["tri_d"][i])
        assert h == bool(v["tri_hit"][i]) and np.array_equal(r, v["tri_tuv"][i])
    for i in range(len(v["dda_box"])):
        b = v["dda_box"][i]
        r = oracle_mod.grid_trace(b[:3], b[3:], tuple(v["dda_res"]), v["dda_o"][i], v["dda_d"][i], 64)
        k = int(v["dda_steps"][i])
        if r is None:
            assert k == -1
        else:
            assert len(r[2]) == k and np.array_equal(r[1], v["dda_cells"][i, :k])
            assert np.array_equal(r[2], v["dda_t"][i, :k])
    assert np.array_equal(np.stack([oracle_mod.to_rgb(x) for x in v["rgb_in"]]), v["rgb_out"])
    for k, f, z in zip(v["rng_keys"], v["rng_f32"], v["rng_norm"]):
        assert np.array_equal(oracle_mod.path_f32(int(k[0]), int(k[1]), int(k[2]), 16), f)
        assert np.array_equal(oracle_mod.path_norm(int(k[0]), int(k[1]), int(k[2]), 16), z)


@pytest.mark.gpu
@pytest.mark.parametrize("name", RENDERS)
def test_gpu_reproduces_render_goldens(name):
    g = _load(f"render_{name}.npz")
    soup = scenes.get_scene(name)
    cname = str(g["camera"]) or None
    c = soup.camera(cname)
    cam = camera_for(soup, cname, None if c.aspect else int(g["w"]), int(g["h"]))
    rs = RenderScene(soup)
    img, res = rs.render(cam, num_samples=int(g["spp"]), max_bounce=int(g["max_bounce"]),
                         stats=True, linear=True)
    rs.close()
    pix = native.tile_pixels(cam.w, cam.h)
    assert np.array_equal(img.reshape(-1, 3), g["rgb"])
    assert np.array_equal(res["linear"], g["linear"][pix])
    st = res["stats"]
    assert [st["segments"], st["cells_visited"], st["triangle_tests"], st["hits"]] == \
        [int(x) for x in g["counters"][:4]]


@pytest.mark.gpu
def test_gpu_reproduces_vector_goldens():
    v = _load("vectors.npz")
    n = len(v["tri"])
    inp = np.concatenate([v["tri"], v["tri_o"], v["tri_d"]], 1).astype(np.float32)
    out = native.probe(native.PROBE_TRIANGLE, inp, n, (n, 4))
    assert np.array_equal(out[:, 0].astype(np.uint8), v["tri_hit"])
    hit = v["tri_hit"].astype(bool)
    assert np.array_equal(out[hit, 1:], v["tri_tuv"][hit])
    m = len(v["dda_box"])
    inp = np.concatenate([v["dda_box"], v["dda_o"], v["dda_d"]], 1).astype(np.float32)
    out = native.probe(native.PROBE_DDA, inp, m, (m, native.DDA_PROBE_WIDTH), aux=v["dda_res"])
    for i in range(m):
        k = int(v["dda_steps"][i])
        assert int(out[i, 0]) == k
        if k > 0:
            got = out[i, 4:4 + 4 * k].reshape(k, 4)
            assert np.array_equal(got[:, :3].astype(np.uint32), v["dda_cells"][i, :k])
            assert np.array_equal(got[:, 3], v["dda_t"][i, :k])
    q = len(v["rgb_in"])
    out = native.probe(native.PROBE_TO_RGB, v["rgb_in"], q, (q, 3))
    assert np.array_equal(out.astype(np.uint8), v["rgb_out"])
    keys = v["rng_keys"]
    f = native.probe(native.PROBE_RNG_F32, keys, len(keys), (len(keys), 16))
    z = native.probe(native.PROBE_RNG_NORM, keys, len(keys), (len(keys), 16))
    assert np.array_equal(f, v["rng_f32"]) and np.array_equal(z, v["rng_norm"])


def test_frame_goldens_cover_every_benchmarked_config():
    """tests/golden/frames.json (tools/make_frame_golden.py) holds the whole
    frames of every config the bench and the configs log quote, made by the
    current oracle source (regenerate it when zrt_oracle.c changes)."""
    import hashlib
    import json
    with open(os.path.join(GOLD, "frames.json")) as fh:
        frames = json.load(fh)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "oracle", "zrt_oracle.c"), "rb") as fh:
        src = hashlib.sha1(fh.read()).hexdigest()
    for cfg in ("cfg2", "cfg3", "cfg4", "cfg5"):
        f = frames[cfg]
        d = scenes.CONFIGS[cfg]
        assert (f["scene"], f["spp"], f["max_bounce"], f["height"]) == (d["scene"], d["spp"], d["max_bounce"],
                                                                       d["height"])
        assert f["oracle_c_sha1"] == src, f"{cfg}: frames.json predates the oracle source"
        assert len(f["rgb8_sha1"]) == 40 and len(f["linear_sha1"]) == 40 and f["segments"] > 0


def test_oracle_reproduces_the_cfg2_frame_golden(oracle_mod):
    """The whole cfg2 frame (512^2, 64 spp: ~20 s on 8 CPUs) through the
    same script that made frames.json: its hashes and counters again."""
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tools"))
    import make_frame_golden
    with open(os.path.join(GOLD, "frames.json")) as fh:
        want = json.load(fh)["cfg2"]
    got = make_frame_golden.frame("cfg2", min(8, len(os.sched_getaffinity(0))))
    for k in ("rgb8_sha1", "linear_sha1", "segments", "cells_visited", "triangle_tests", "hits"):
        assert got[k] == want[k], k
