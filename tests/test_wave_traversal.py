"""Wave-shared triangle testing (render.hip trace_wave) emulated on the host
(tests/cpp/wave_emul.cpp) against the sequential traceRay walk: identical
nearest t, ref, u and v for every ray of a real baked scene, including rays
from inside the grid in random directions (the bounce rays' case)."""
import ctypes as C
import os
import shutil
import subprocess

import numpy as np
import pytest

from zig_raytracing_contest_amd import native, scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def emul(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    so = tmp_path_factory.mktemp("wave") / "libwave.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC",
                    "-I", os.path.join(ROOT, "zig_raytracing_contest_amd", "csrc"),
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "wave_emul.cpp"), "-o", str(so)], check=True)
    lib = C.CDLL(str(so))
    lib.wave_check.restype = C.c_int
    return lib


@pytest.mark.parametrize("name,res", [("cornell", (32, 32, 32)), ("sphere", (24, 16, 40)), ("contest", (128, 128, 128))])
def test_wave_shared_tests_match_sequential(emul, name, res):
    soup = scenes.get_scene(name)
    geo = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat, resolution=res)
    g = geo.scene.grid
    bmin = np.array(g.bbox_min, np.float32)
    bmax = np.array(g.bbox_max, np.float32)
    r = np.array(g.resolution, np.uint32)
    cs = np.array(g.cell_size, np.float32)
    cells = np.ascontiguousarray(geo.cells().reshape(-1), np.uint32)
    pos = np.ascontiguousarray(geo.tri_pos().reshape(-1), np.float32)
    rng = np.random.default_rng(7)
    n = 4096
    o = bmin + (bmax - bmin) * rng.random((n, 3), np.float32)
    o[: n // 4] = bmin - (bmax - bmin) * 0.5 + (bmax - bmin) * 2.0 * rng.random((n // 4, 3), np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.ascontiguousarray(np.concatenate([o, d], axis=1), np.float32)
    out_s = np.zeros((n, 4), np.float32)
    out_w = np.zeros((n, 4), np.float32)
    f = lambda a: a.ctypes.data_as(C.c_void_p)
    bad = emul.wave_check(f(bmin), f(bmax), f(r), f(cs), f(cells), f(pos), n, f(rays), f(out_s), f(out_w))
    hits = int(np.isfinite(out_s[:, 0]).sum())
    assert hits > n // 20
    assert bad == 0


@pytest.mark.parametrize("name,res", [("cornell", (32, 32, 32)), ("contest", (128, 128, 128)),
                                      ("sponza", (128, 128, 128)), ("contest", (37, 64, 101))])
def test_entry_face_skip_is_exact(emul, name, res):
    """The park kernel's entry-face skip (render.hip cell32_kernel): a ref
    whose (v0, e1, e2) bits equal a ref of the cell the ray just left is not
    tested again.  Sequential traceRay with and without the skip, random rays
    from inside and outside the grid: bit-identical nearest t, u, v and ref;
    and the skip removes a real share of the tests."""
    soup = scenes.get_scene(name)
    geo = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat, resolution=res)
    g = geo.scene.grid
    bmin = np.array(g.bbox_min, np.float32)
    bmax = np.array(g.bbox_max, np.float32)
    r = np.array(g.resolution, np.uint32)
    cs = np.array(g.cell_size, np.float32)
    cells = np.ascontiguousarray(geo.cells().reshape(-1), np.uint32)
    pos = np.ascontiguousarray(geo.tri_pos().reshape(-1), np.float32)
    rng = np.random.default_rng(11)
    n = 3000
    o = bmin + (bmax - bmin) * rng.random((n, 3), np.float32)
    o[: n // 4] = bmin - (bmax - bmin) * 0.5 + (bmax - bmin) * 2.0 * rng.random((n // 4, 3), np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.ascontiguousarray(np.concatenate([o, d], axis=1), np.float32)
    stats = np.zeros(2, np.uint64)
    f = lambda a: a.ctypes.data_as(C.c_void_p)
    emul.skip_check.restype = C.c_int
    bad = emul.skip_check(f(bmin), f(bmax), f(r), f(cs), f(cells), f(pos), n, f(rays), f(stats))
    assert bad == 0
    assert stats[1] < stats[0] * 0.9, stats
