"""ctypes binding for the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.  See
zrt_oracle.h for what each entry point restates (reference file:line).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

RNG_REF = 0
RNG_PATH = 1

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


class OrcCamera(C.Structure):
    _fields_ = [("w", C.c_uint32), ("h", C.c_uint32), ("origin", C.c_float * 3),
                ("llc", C.c_float * 3), ("right", C.c_float * 3), ("up", C.c_float * 3)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    L = C.CDLL(_LIB_PATH)
    L.orc_scene_build.restype = C.c_void_p
    L.orc_scene_build.argtypes = [_f32p, _f32p, _f32p, _u32p, C.c_uint32, _u32p]
    L.orc_scene_free.argtypes = [C.c_void_p]
    L.orc_scene_num_refs.restype = C.c_uint32
    L.orc_scene_num_refs.argtypes = [C.c_void_p]
    L.orc_scene_get.argtypes = [C.c_void_p, _f32p, _f32p, C.c_void_p, C.c_void_p]
    L.orc_scene_set_materials.argtypes = [C.c_void_p, C.c_uint32, _i32p, _f32p, C.c_uint64]
    L.orc_camera_from_matrix.argtypes = [_f32p, C.c_float, C.c_int, C.c_float, C.c_int, C.c_int,
                                         C.POINTER(OrcCamera)]
    L.orc_render.argtypes = [C.c_void_p, C.POINTER(OrcCamera), C.c_uint32, C.c_uint32, C.c_int,
                             C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                             C.c_void_p, _u64p]
    L.orc_render_pixels.argtypes = [C.c_void_p, C.POINTER(OrcCamera), C.c_uint32, C.c_uint32,
                                    C.c_int, C.c_uint64, C.c_uint32, _u32p, C.c_uint32, C.c_void_p,
                                    C.c_void_p, _u64p]
    L.orc_bbox_ray.argtypes = [_f32p, _f32p, _f32p, C.POINTER(C.c_float)]
    L.orc_grid_trace.argtypes = [_f32p, _u32p, _f32p, _f32p, _u32p, _f32p, C.c_int, _u32p]
    L.orc_grid_cell_bbox.argtypes = [_f32p, _u32p, C.c_uint32, C.c_uint32, C.c_uint32, _f32p]
    L.orc_tri_intersect.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, _f32p]
    L.orc_tri_aabb.argtypes = [_f32p, _f32p]
    L.orc_cross.argtypes = [_f32p, _f32p, _f32p]
    L.orc_length.restype = C.c_float
    L.orc_length.argtypes = [_f32p]
    L.orc_to_rgb.argtypes = [_f32p, _u8p]
    L.orc_powf.restype = C.c_float
    L.orc_powf.argtypes = [C.c_float, C.c_float]
    L.orc_exp.restype = C.c_double
    L.orc_exp.argtypes = [C.c_double]
    L.orc_log.restype = C.c_double
    L.orc_log.argtypes = [C.c_double]
    L.orc_env.argtypes = [_f32p, _f32p]
    L.orc_tex_sample.argtypes = [_f32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_int, C.c_float, C.c_float, _f32p]
    for name, p in (("orc_xoshiro_u64", _u64p), ("orc_splitmix_u64", _u64p), ("orc_xoshiro_f32", _f32p),
                    ("orc_xoshiro_norm", _f32p)):
        getattr(L, name).argtypes = [C.c_uint64, p, C.c_int]
    for name, p in (("orc_path_u64", _u64p), ("orc_path_f32", _f32p), ("orc_path_norm", _f32p)):
        getattr(L, name).argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, p, C.c_int]
    L.orc_zig_tables.argtypes = [_f64p, _f64p]
    _lib = L
    return L


def _f(a, n=None):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32).reshape(-1))
    if n is not None:
        assert a.size == n
    return a


# ---------------------------------------------------------------- unit calls
def bbox_ray(bbox_min, bbox_max, orig, dir_):
    t = C.c_float(0)
    hit = lib().orc_bbox_ray(_f(list(bbox_min) + list(bbox_max)), _f(orig, 3), _f(dir_, 3),
                             C.byref(t))
    return bool(hit), t.value


def grid_trace(bbox_min, bbox_max, res, orig, dir_, max_steps=4096):
    cells = np.zeros(3 * max_steps, np.uint32)
    ts = np.zeros(max_steps, np.float32)
    first = np.zeros(3, np.uint32)
    n = lib().orc_grid_trace(_f(list(bbox_min) + list(bbox_max)), np.asarray(res, np.uint32),
                             _f(orig, 3), _f(dir_, 3), cells, ts, max_steps, first)
    if n < 0:
        return None
    return tuple(int(x) for x in first), cells[:3 * n].reshape(n, 3).copy(), ts[:n].copy()


def grid_cell_bbox(bbox_min, bbox_max, res, x, y, z):
    out = np.zeros(6, np.float32)
    lib().orc_grid_cell_bbox(_f(list(bbox_min) + list(bbox_max)), np.asarray(res, np.uint32),
                             x, y, z, out)
    return out[:3].copy(), out[3:].copy()


def tri_intersect(v0, v1, v2, orig, dir_):
    out = np.zeros(3, np.float32)
    hit = lib().orc_tri_intersect(_f(v0, 3), _f(v1, 3), _f(v2, 3), _f(orig, 3), _f(dir_, 3), out)
    return bool(hit), out


def tri_aabb(tri9, bbox_min, bbox_max):
    return bool(lib().orc_tri_aabb(_f(tri9, 9), _f(list(bbox_min) + list(bbox_max))))


def cross(a, b):
    out = np.zeros(3, np.float32)
    lib().orc_cross(_f(a, 3), _f(b, 3), out)
    return out


def length(v):
    return lib().orc_length(_f(v, 3))


def to_rgb(v):
    out = np.zeros(3, np.uint8)
    lib().orc_to_rgb(_f(v, 3), out)
    return out


def env_color(d):
    out = np.zeros(3, np.float32)
    lib().orc_env(_f(d, 3), out)
    return out


def tex_sample(data, chans, w, h, u_min, u_max, v_min, v_max, u, v):
    out = np.zeros(chans, np.float32)
    lib().orc_tex_sample(_f(data), chans, w, h, u_min, u_max, v_min, v_max, u, v, out)
    return out


def xoshiro_u64(seed, n):
    out = np.zeros(n, np.uint64)
    lib().orc_xoshiro_u64(seed, out, n)
    return out


def splitmix_u64(seed, n):
    out = np.zeros(n, np.uint64)
    lib().orc_splitmix_u64(seed, out, n)
    return out


def path_u64(seed, pixel, sample, n):
    out = np.zeros(n, np.uint64)
    lib().orc_path_u64(seed, pixel, sample, out, n)
    return out


def path_f32(seed, pixel, sample, n):
    out = np.zeros(n, np.float32)
    lib().orc_path_f32(seed, pixel, sample, out, n)
    return out


def path_norm(seed, pixel, sample, n):
    out = np.zeros(n, np.float32)
    lib().orc_path_norm(seed, pixel, sample, out, n)
    return out


def xoshiro_f32(seed, n):
    out = np.zeros(n, np.float32)
    lib().orc_xoshiro_f32(seed, out, n)
    return out


def xoshiro_norm(seed, n):
    out = np.zeros(n, np.float32)
    lib().orc_xoshiro_norm(seed, out, n)
    return out


def zig_tables():
    x = np.zeros(257, np.float64)
    f = np.zeros(257, np.float64)
    lib().orc_zig_tables(x, f)
    return x, f


def camera_from_matrix(m16, yfov, aspect=None, width=None, height=None):
    cam = OrcCamera()
    rc = lib().orc_camera_from_matrix(_f(m16, 16), yfov, 0 if aspect is None else 1,
                                      0.0 if aspect is None else aspect,
                                      -1 if width is None else width,
                                      -1 if height is None else height, C.byref(cam))
    if rc != 0:
        raise ValueError({-1: "OutputImgSizeIsNotSpecified", -2: "CameraHasAspectRatio",
                          -3: "CameraHasntAspectRatio"}[rc])
    return cam


def camera_from_dict(d):
    cam = OrcCamera()
    cam.w, cam.h = int(d["w"]), int(d["h"])
    for k in ("origin", "llc", "right", "up"):
        getattr(cam, k)[:] = [float(x) for x in d[k]]
    return cam


# -------------------------------------------------------------------- scene
class OracleScene:
    """stage2.Geometry.build + bakeInto + stage1 materials (restated)."""

    def __init__(self, soup, res=(128, 128, 128)):
        L = lib()
        self.soup = soup
        self._h = L.orc_scene_build(_f(soup.pos), _f(soup.nrm), _f(soup.uv),
                                    np.ascontiguousarray(soup.mat, np.uint32),
                                    int(soup.num_triangles), np.asarray(res, np.uint32))
        self.res = tuple(int(r) for r in res)
        L.orc_scene_set_materials(self._h, int(soup.num_materials),
                                  np.ascontiguousarray(soup.tex_desc, np.int32).reshape(-1),
                                  _f(soup.texels), int(np.asarray(soup.texels).size))

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.orc_scene_free(self._h)
            self._h = None

    @property
    def num_refs(self):
        return int(lib().orc_scene_num_refs(self._h))

    def baked(self):
        gb = np.zeros(6, np.float32)
        cs = np.zeros(3, np.float32)
        ncells = self.res[0] * self.res[1] * self.res[2]
        cells = np.zeros(2 * ncells, np.uint32)
        idx = np.zeros(max(self.num_refs, 1), np.uint32)
        lib().orc_scene_get(self._h, gb, cs, cells.ctypes.data, idx.ctypes.data)
        return gb, cs, cells.reshape(ncells, 2), idx[:self.num_refs]

    def render(self, cam, spp, max_bounce, rng_mode=RNG_PATH, seed=0, num_threads=8,
               px_begin=0, px_end=None, want_linear=True):
        if px_end is None:
            px_end = cam.w * cam.h
        n = px_end - px_begin
        rgb = np.zeros(3 * n, np.uint8)
        lin = np.zeros(3 * n, np.float32) if want_linear else None
        ctr = np.zeros(5, np.uint64)
        rc = lib().orc_render(self._h, C.byref(cam), spp, max_bounce, rng_mode, seed, num_threads,
                              px_begin, px_end, rgb.ctypes.data,
                              None if lin is None else lin.ctypes.data, ctr)
        if rc != 0:
            raise RuntimeError("orc_render failed")
        return rgb.reshape(n, 3), (None if lin is None else lin.reshape(n, 3)), ctr

    def render_pixels(self, cam, spp, max_bounce, pixels, rng_mode=RNG_PATH, seed=0,
                      num_threads=8):
        pixels = np.ascontiguousarray(pixels, np.uint32)
        n = pixels.size
        rgb = np.zeros(3 * n, np.uint8)
        lin = np.zeros(3 * n, np.float32)
        ctr = np.zeros(5, np.uint64)
        rc = lib().orc_render_pixels(self._h, C.byref(cam), spp, max_bounce, rng_mode, seed,
                                     num_threads, pixels, n, rgb.ctypes.data, lin.ctypes.data, ctr)
        if rc != 0:
            raise RuntimeError("orc_render_pixels failed")
        return rgb.reshape(n, 3), lin.reshape(n, 3), ctr
