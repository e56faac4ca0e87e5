"""ctypes binding of libzrt.so (include/zrt.h) -- the product's C ABI.

No fallback: if the HIP library is missing the import of `lib()` raises, so a
GPU test can never pass on a silent CPU path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# ZRT_LIB: an alternative build of the library (tools/ tuning builds only)
LIB_PATH = os.environ.get("ZRT_LIB") or os.path.join(_HERE, "libzrt.so")
_lib = None

ZRT_OK = 0
STATUS = {0: "ok", -1: "invalid argument", -2: "no HIP device", -3: "HIP runtime error",
          -4: "out of memory", -5: "unsupported configuration", -6: "I/O error",
          -7: "parse error", -8: "not found", -9: "camera/output size rules violated"}
FLAG_COUNT_STATS, FLAG_LANE_WALK = 0x1, 0x2
FLAG_ESCAPE, FLAG_NO_ESCAPE = 0x40, 0x80
FLAG_FRUSTUM, FLAG_NO_FRUSTUM = 0x100, 0x200
FLAG_ONE_SET, FLAG_KERNEL_TIMES = 0x10, 0x20
FLAG_MT_EXACT = 0x400
FLAG_RELEASE, FLAG_NO_RELEASE = 0x800, 0x1000
# zrt_kernel_profile classes (include/zrt.h)
KERNEL_CLASSES = ("primary", "park", "shade", "bounce", "resolve", "count")

PROBE_TRIANGLE, PROBE_BBOX, PROBE_DDA, PROBE_TO_RGB = 0, 1, 2, 3
PROBE_RNG_F32, PROBE_RNG_NORM, PROBE_EXP_LOG, PROBE_TEXTURE = 4, 5, 6, 7
PROBE_TRIANGLE_FLAT = 8
PROBE_RECIP, PROBE_RECIP_SWEEP, PROBE_TRIANGLE_EXACT = 9, 10, 11
PROBE_QUOT, PROBE_QUOT_SWEEP = 12, 13
DDA_PROBE_WIDTH = 4 + 4 * 64      # floats per ray: steps, first cell, 64 x (cell, t)


class ZrtError(RuntimeError):
    def __init__(self, status, what=""):
        self.status = status
        super().__init__(f"{what}: {STATUS.get(status, status)} ({status})")


class Grid(C.Structure):
    _fields_ = [("bbox_min", C.c_float * 3), ("bbox_max", C.c_float * 3),
                ("resolution", C.c_uint32 * 3), ("cell_size", C.c_float * 3)]


class Texture(C.Structure):
    _fields_ = [("offset", C.c_uint64), ("w", C.c_int32), ("h", C.c_int32),
                ("u_min", C.c_int32), ("u_max", C.c_int32), ("v_min", C.c_int32),
                ("v_max", C.c_int32), ("_pad", C.c_int32)]


class Material(C.Structure):
    _fields_ = [("base_color", Texture), ("emissive", Texture), ("transparency", Texture)]


class Scene(C.Structure):
    _fields_ = [("grid", Grid), ("num_cells", C.c_uint32), ("cells", C.POINTER(C.c_uint32)),
                ("num_triangles", C.c_uint32), ("triangles_pos", C.POINTER(C.c_float)),
                ("triangles_data", C.POINTER(C.c_float)),
                ("triangles_material", C.POINTER(C.c_uint32)), ("num_materials", C.c_uint32),
                ("materials", C.POINTER(Material)), ("texels", C.POINTER(C.c_float)),
                ("num_texel_floats", C.c_uint64)]


class Camera(C.Structure):
    _fields_ = [("w", C.c_uint32), ("h", C.c_uint32), ("origin", C.c_float * 3),
                ("lower_left_corner", C.c_float * 3), ("right", C.c_float * 3),
                ("up", C.c_float * 3)]

    def as_dict(self):
        return {"w": self.w, "h": self.h, "origin": list(self.origin),
                "llc": list(self.lower_left_corner), "right": list(self.right), "up": list(self.up)}


class RenderConfig(C.Structure):
    _fields_ = [("num_samples", C.c_uint32), ("max_bounce", C.c_uint32), ("seed", C.c_uint64),
                ("device", C.c_int32), ("rank", C.c_uint32), ("num_ranks", C.c_uint32),
                ("tile_size", C.c_uint32), ("flags", C.c_uint32), ("samples_per_pass", C.c_uint32),
                ("num_devices", C.c_uint32), ("_reserved0", C.c_uint32),
                ("devices", C.POINTER(C.c_int32))]


class Stats(C.Structure):
    _fields_ = [("segments", C.c_uint64), ("cells_visited", C.c_uint64),
                ("triangle_tests", C.c_uint64), ("hits", C.c_uint64), ("samples", C.c_uint64),
                ("render_ms", C.c_double), ("trace_kernel_ms", C.c_double),
                ("trace_launches", C.c_uint32), ("_pad", C.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if not k.startswith("_")}


class KernelProfile(C.Structure):
    _fields_ = [("ms", C.c_double * 8), ("launches", C.c_uint32 * 8), ("passes", C.c_uint32),
                ("sets", C.c_uint32), ("primary_counts", C.c_uint64 * 4)]

    def as_dict(self):
        return {"kernels": {k: {"ms": self.ms[i], "launches": int(self.launches[i])}
                            for i, k in enumerate(KERNEL_CLASSES) if self.launches[i]},
                "passes": int(self.passes), "sets": int(self.sets),
                "primary": dict(zip(("segments", "cells_visited", "triangle_tests", "hits"),
                                    (int(x) for x in self.primary_counts)))}


class Outputs(C.Structure):
    _fields_ = [("rgb_image", C.c_void_p), ("rgb_packed", C.c_void_p),
                ("linear_packed", C.c_void_p), ("device_rgb_packed", C.c_void_p)]


EXPORTS = [
    "zrt_error_string", "zrt_abi_version", "zrt_device_count", "zrt_device_warmup", "zrt_geometry_build",
    "zrt_geometry_build_device",
    "zrt_geometry_scene", "zrt_geometry_indices", "zrt_geometry_free", "zrt_render",
    "zrt_context_create", "zrt_context_create_built", "zrt_context_grid_info", "zrt_context_render", "zrt_context_destroy", "zrt_tile_pixels",
    "zrt_gltf_load", "zrt_gltf_soup", "zrt_gltf_materials", "zrt_gltf_camera", "zrt_gltf_free",
    "zrt_camera_from_matrix", "zrt_probe", "zrt_timed_kernels", "zrt_context_profile",
    "zrt_group_create", "zrt_group_create_built", "zrt_group_render", "zrt_group_context", "zrt_group_destroy",
]


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libzrt.so not built at {LIB_PATH} (run `make` or "
                          "__graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    L.zrt_error_string.restype = C.c_char_p
    L.zrt_error_string.argtypes = [C.c_int]
    L.zrt_device_count.argtypes = [C.POINTER(C.c_int)]
    L.zrt_geometry_build.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                     C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_void_p)]
    L.zrt_geometry_build_device.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                            C.POINTER(C.c_uint32), C.c_int, C.POINTER(C.c_void_p)]
    L.zrt_geometry_scene.argtypes = [C.c_void_p, C.POINTER(Scene)]
    L.zrt_geometry_indices.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_uint32)),
                                       C.POINTER(C.c_uint32)]
    L.zrt_geometry_free.argtypes = [C.c_void_p]
    L.zrt_geometry_free.restype = None
    L.zrt_render.argtypes = [C.POINTER(Scene), C.POINTER(Camera), C.POINTER(RenderConfig),
                             C.c_void_p, C.POINTER(Stats)]
    L.zrt_context_create.argtypes = [C.POINTER(Scene), C.c_int, C.POINTER(C.c_void_p)]
    L.zrt_context_create_built.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                           C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(Material),
                                           C.POINTER(C.c_float), C.c_uint64, C.c_int,
                                           C.POINTER(C.c_void_p)]
    L.zrt_context_grid_info.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint32)]
    L.zrt_context_render.argtypes = [C.c_void_p, C.POINTER(Camera), C.POINTER(RenderConfig),
                                     C.POINTER(Outputs), C.POINTER(Stats)]
    L.zrt_context_profile.argtypes = [C.c_void_p, C.POINTER(KernelProfile)]
    L.zrt_context_destroy.argtypes = [C.c_void_p]
    L.zrt_context_destroy.restype = None
    if hasattr(L, "zrt_group_create"):      # ABI 2 (an ABI-1 build: tools/ A/B baselines only)
        L.zrt_group_create.argtypes = [C.POINTER(Scene), C.POINTER(C.c_int32), C.c_uint32, C.POINTER(C.c_void_p)]
        L.zrt_group_create_built.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                             C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(Material),
                                             C.POINTER(C.c_float), C.c_uint64, C.POINTER(C.c_int32), C.c_uint32,
                                             C.POINTER(C.c_void_p)]
        L.zrt_group_render.argtypes = [C.c_void_p, C.POINTER(Camera), C.POINTER(RenderConfig), C.c_void_p,
                                       C.POINTER(Stats)]
        L.zrt_group_context.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p)]
        L.zrt_group_destroy.argtypes = [C.c_void_p]
        L.zrt_group_destroy.restype = None
    L.zrt_tile_pixels.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                  C.c_void_p, C.POINTER(C.c_uint32)]
    L.zrt_camera_from_matrix.argtypes = [C.c_void_p, C.c_float, C.c_int, C.c_float, C.c_int32,
                                         C.c_int32, C.POINTER(Camera)]
    L.zrt_probe.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_int]
    L.zrt_timed_kernels.restype = C.c_char_p
    L.zrt_timed_kernels.argtypes = []
    if hasattr(L, "zrt_gltf_load"):
        L.zrt_gltf_load.argtypes = [C.c_char_p, C.c_uint32, C.POINTER(C.c_void_p)]
        L.zrt_gltf_soup.argtypes = [C.c_void_p] + [C.POINTER(C.c_void_p)] * 4 + [
            C.POINTER(C.c_uint32)]
        L.zrt_gltf_materials.argtypes = [C.c_void_p, C.POINTER(Scene)]
        L.zrt_gltf_camera.argtypes = [C.c_void_p, C.c_char_p, C.c_int32, C.c_int32,
                                      C.POINTER(Camera)]
        L.zrt_gltf_free.argtypes = [C.c_void_p]
        L.zrt_gltf_free.restype = None
    _lib = L
    return L


def check(rc, what):
    if rc != ZRT_OK:
        raise ZrtError(rc, what)


def device_count() -> int:
    n = C.c_int(0)
    rc = lib().zrt_device_count(C.byref(n))
    return n.value if rc == ZRT_OK else 0


def _ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def camera_from_matrix(m16, yfov, aspect=None, width=None, height=None) -> Camera:
    """stage1.zig:309-371 loadCamera through the C ABI."""
    cam = Camera()
    m = np.ascontiguousarray(m16, np.float32)
    rc = lib().zrt_camera_from_matrix(m.ctypes.data, float(yfov), 0 if aspect is None else 1,
                                      0.0 if aspect is None else float(aspect),
                                      -1 if width is None else int(width),
                                      -1 if height is None else int(height), C.byref(cam))
    check(rc, "zrt_camera_from_matrix")
    return cam


def tile_pixels(w, h, tile=64, rank=0, num_ranks=1) -> np.ndarray:
    n = C.c_uint32(0)
    check(lib().zrt_tile_pixels(w, h, tile, rank, num_ranks, None, C.byref(n)), "zrt_tile_pixels")
    out = np.zeros(max(n.value, 1), np.uint32)
    check(lib().zrt_tile_pixels(w, h, tile, rank, num_ranks, out.ctypes.data, C.byref(n)),
          "zrt_tile_pixels")
    return out[:n.value]


class Geometry:
    """stage2.Geometry: build (SAT binning) + bake, on host threads, or on
    GPU `device` (zrt_geometry_build_device: same arrays, bit for bit)."""

    def __init__(self, pos, nrm, uv, mat, resolution=(128, 128, 128), num_threads=0, device=None):
        self._keep = [np.ascontiguousarray(pos, np.float32), np.ascontiguousarray(nrm, np.float32),
                      np.ascontiguousarray(uv, np.float32), np.ascontiguousarray(mat, np.uint32)]
        n = self._keep[3].size
        res = (C.c_uint32 * 3)(*resolution)
        h = C.c_void_p()
        args = [k.ctypes.data for k in self._keep] + [n, res]
        if device is None:
            check(lib().zrt_geometry_build(*args, num_threads, C.byref(h)), "zrt_geometry_build")
        else:
            check(lib().zrt_geometry_build_device(*args, int(device), C.byref(h)),
                  "zrt_geometry_build_device")
        self._h = h
        self.scene = Scene()
        check(lib().zrt_geometry_scene(self._h, C.byref(self.scene)), "zrt_geometry_scene")

    def __del__(self):
        if getattr(self, "_h", None) is not None and _lib is not None:
            _lib.zrt_geometry_free(self._h)
            self._h = None

    @property
    def num_refs(self):
        return int(self.scene.num_triangles)

    def indices(self):
        p = C.POINTER(C.c_uint32)()
        n = C.c_uint32(0)
        check(lib().zrt_geometry_indices(self._h, C.byref(p), C.byref(n)), "zrt_geometry_indices")
        return np.ctypeslib.as_array(p, (n.value,)).copy() if n.value else np.zeros(0, np.uint32)

    def cells(self):
        n = self.scene.num_cells
        return np.ctypeslib.as_array(self.scene.cells, (n, 2)).copy()

    def tri_pos(self):
        return np.ctypeslib.as_array(self.scene.triangles_pos, (self.num_refs, 9)).copy()

    def tri_data(self):
        return np.ctypeslib.as_array(self.scene.triangles_data, (self.num_refs, 15)).copy()

    def tri_material(self):
        return np.ctypeslib.as_array(self.scene.triangles_material, (self.num_refs,)).copy()


def attach_materials(scene: Scene, tex_desc: np.ndarray, texels: np.ndarray, keep: list):
    """Fill the material fields of a zrt_scene from (nmat,3,7) descriptors."""
    td = np.asarray(tex_desc, np.int64).reshape(-1, 3, 7)
    mats = (Material * len(td))()
    for i, m in enumerate(td):
        for k, name in enumerate(("base_color", "emissive", "transparency")):
            t = getattr(mats[i], name)
            t.offset, t.w, t.h, t.u_min, t.u_max, t.v_min, t.v_max = (int(x) for x in m[k])
    tx = np.ascontiguousarray(texels, np.float32)
    keep += [mats, tx]
    scene.num_materials = len(td)
    scene.materials = C.cast(mats, C.POINTER(Material))
    scene.texels = _ptr(tx, C.c_float)
    scene.num_texel_floats = tx.size


class Context:
    """Device-resident scene (zrt_context): upload once, render many times."""

    def __init__(self, scene: Scene, device: int = -1):
        h = C.c_void_p()
        check(lib().zrt_context_create(C.byref(scene), device, C.byref(h)), "zrt_context_create")
        self._h = h

    @classmethod
    def built(cls, pos, nrm, uv, mat, materials: Scene, resolution=(128, 128, 128), device: int = -1):
        """zrt_context_create_built: grid built on the GPU straight into the
        context (materials/texels taken from `materials`' material fields)."""
        keep = [np.ascontiguousarray(pos, np.float32), np.ascontiguousarray(nrm, np.float32),
                np.ascontiguousarray(uv, np.float32), np.ascontiguousarray(mat, np.uint32)]
        res = (C.c_uint32 * 3)(*resolution)
        h = C.c_void_p()
        check(lib().zrt_context_create_built(*[k.ctypes.data for k in keep], keep[3].size, res,
                                             materials.num_materials, materials.materials,
                                             materials.texels, materials.num_texel_floats, device,
                                             C.byref(h)), "zrt_context_create_built")
        self = cls.__new__(cls)
        self._h = h
        return self

    def grid_info(self):
        """(num_refs, empty cells, min refs of a non-empty cell, max refs)."""
        info = (C.c_uint32 * 4)()
        check(lib().zrt_context_grid_info(self._h, None, info), "zrt_context_grid_info")
        return tuple(int(x) for x in info)

    def profile(self):
        """zrt_context_profile: per-kernel launches (and device ms with
        FLAG_KERNEL_TIMES) of the last render, primary-segment counts of a
        counting render."""
        kp = KernelProfile()
        check(lib().zrt_context_profile(self._h, C.byref(kp)), "zrt_context_profile")
        return kp.as_dict()

    def close(self):
        if getattr(self, "_h", None) is not None and _lib is not None:
            _lib.zrt_context_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def render(self, cam: Camera, spp: int, max_bounce: int, seed: int = 0, rank: int = 0,
               num_ranks: int = 1, tile: int = 64, stats: bool = False, image=None,
               packed=False, linear=False, device_ptr=None, samples_per_pass=0, flags=0):
        cfg = RenderConfig()
        cfg.num_samples, cfg.max_bounce, cfg.seed = spp, max_bounce, seed
        cfg.device, cfg.rank, cfg.num_ranks, cfg.tile_size = -1, rank, num_ranks, tile
        cfg.flags = (FLAG_COUNT_STATS if stats else 0) | flags
        cfg.samples_per_pass = samples_per_pass
        n = None
        out = Outputs()
        res = {}
        if image is not None:
            out.rgb_image = image.ctypes.data
        if packed or linear:
            n = int(tile_pixels(cam.w, cam.h, tile, rank, num_ranks).size)
        if packed:
            res["packed"] = np.zeros((n, 3), np.uint8)
            out.rgb_packed = res["packed"].ctypes.data
        if linear:
            res["linear"] = np.zeros((n, 3), np.float32)
            out.linear_packed = res["linear"].ctypes.data
        if device_ptr is not None:
            out.device_rgb_packed = device_ptr
        st = Stats()
        check(lib().zrt_context_render(self._h, C.byref(cam), C.byref(cfg), C.byref(out),
                                       C.byref(st)), "zrt_context_render")
        res["stats"] = st.as_dict()
        return res


def render_oneshot(scene: Scene, cam: Camera, spp: int, max_bounce: int, seed: int = 0,
                   device: int = -1, devices=None, num_devices=None):
    """zrt_render: the one-shot drop-in for Scene.render (stage3.zig:247) --
    upload, render the whole image, download, free.  `devices`: a list of
    HIP ordinals (repeats allowed) to split the image's tiles over
    (zrt_render_config.devices / num_devices).  Returns (h, w, 3) RGB8."""
    cfg = RenderConfig()
    cfg.num_samples, cfg.max_bounce, cfg.seed, cfg.device = spp, max_bounce, seed, device
    cfg.num_ranks = 1
    if devices is not None:
        dl = (C.c_int32 * len(devices))(*devices)
        cfg.num_devices, cfg.devices = len(devices), dl
    elif num_devices is not None:      # a count without a list (ABI-1 callers)
        cfg.num_devices = num_devices
    img = np.zeros((cam.h, cam.w, 3), np.uint8)
    st = Stats()
    check(lib().zrt_render(C.byref(scene), C.byref(cam), C.byref(cfg), img.ctypes.data, C.byref(st)),
          "zrt_render")
    return img, st.as_dict()


class Group:
    """zrt_group: one context per device of `devices` (repeats allowed), one
    render call splitting the image's tiles over them and gathering them over
    xGMI into one image (Scene.render's spawn + join, stage3.zig:247-256)."""

    def __init__(self, scene: Scene, devices):
        self._dev = (C.c_int32 * len(devices))(*devices)
        h = C.c_void_p()
        check(lib().zrt_group_create(C.byref(scene), self._dev, len(devices), C.byref(h)), "zrt_group_create")
        self._h = h
        self.devices = list(devices)

    @classmethod
    def built(cls, pos, nrm, uv, mat, materials: Scene, devices, resolution=(128, 128, 128)):
        """zrt_group_create_built: the grid built on every device."""
        keep = [np.ascontiguousarray(pos, np.float32), np.ascontiguousarray(nrm, np.float32),
                np.ascontiguousarray(uv, np.float32), np.ascontiguousarray(mat, np.uint32)]
        res = (C.c_uint32 * 3)(*resolution)
        self = cls.__new__(cls)
        self._dev = (C.c_int32 * len(devices))(*devices)
        self.devices = list(devices)
        h = C.c_void_p()
        check(lib().zrt_group_create_built(*[k.ctypes.data for k in keep], keep[3].size, res,
                                           materials.num_materials, materials.materials, materials.texels,
                                           materials.num_texel_floats, self._dev, len(devices), C.byref(h)),
              "zrt_group_create_built")
        self._h = h
        return self

    def render(self, cam: Camera, spp: int, max_bounce: int, seed: int = 0, rank: int = 0, num_ranks: int = 1,
               image=None, flags=0):
        """Returns ((h, w, 3) RGB8 with this process's pixels, stats dict)."""
        cfg = RenderConfig()
        cfg.num_samples, cfg.max_bounce, cfg.seed = spp, max_bounce, seed
        cfg.rank, cfg.num_ranks, cfg.flags = rank, num_ranks, flags
        img = np.zeros((cam.h, cam.w, 3), np.uint8) if image is None else image
        st = Stats()
        check(lib().zrt_group_render(self._h, C.byref(cam), C.byref(cfg), img.ctypes.data, C.byref(st)),
              "zrt_group_render")
        return img, st.as_dict()

    def close(self):
        if getattr(self, "_h", None) is not None and _lib is not None:
            _lib.zrt_group_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def timed_kernels():
    """Mangled-name substrings of the timed kernel instantiations (no HIP call)."""
    return lib().zrt_timed_kernels().decode().split(",")


# bytes per item the probe reads / writes (render.hip zrt_probe)
_PROBE_IO = {PROBE_TRIANGLE: (60, 16), PROBE_TRIANGLE_FLAT: (60, 16), PROBE_BBOX: (48, 8),
             PROBE_DDA: (48, 4 * DDA_PROBE_WIDTH), PROBE_TO_RGB: (12, 12), PROBE_RNG_F32: (12, 64),
             PROBE_RNG_NORM: (12, 64), PROBE_EXP_LOG: (8, 16), PROBE_TEXTURE: (8, 12),
             PROBE_RECIP: (4, 8), PROBE_RECIP_SWEEP: (8, 16), PROBE_TRIANGLE_EXACT: (60, 16),
             PROBE_QUOT: (8, 8), PROBE_QUOT_SWEEP: (8, 16)}


def probe(which, inp: np.ndarray, n: int, out_shape, out_dtype=np.float32, aux=None, device=-1):
    inp = np.ascontiguousarray(inp)
    out = np.zeros(out_shape, out_dtype)
    in_b, out_b = _PROBE_IO[which]
    if inp.nbytes < n * in_b or out.nbytes < n * out_b:
        raise ValueError(f"probe {which}: buffers too small for {n} items")
    auxp = None if aux is None else np.ascontiguousarray(aux).ctypes.data
    check(lib().zrt_probe(which, inp.ctypes.data, out.ctypes.data, n, auxp, device), "zrt_probe")
    return out


class Gltf:
    """stage1: glTF/GLB load through the C ABI (zrt_gltf_*)."""

    def __init__(self, path: str, num_threads: int = 0):
        h = C.c_void_p()
        check(lib().zrt_gltf_load(path.encode(), num_threads, C.byref(h)), f"zrt_gltf_load({path})")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None) is not None and _lib is not None:
            _lib.zrt_gltf_free(self._h)
            self._h = None

    def soup(self):
        ptrs = [C.c_void_p() for _ in range(4)]
        n = C.c_uint32(0)
        check(lib().zrt_gltf_soup(self._h, *[C.byref(p) for p in ptrs], C.byref(n)), "zrt_gltf_soup")
        k = n.value

        def arr(p, shape, ctype, dtype):
            if k == 0:
                return np.zeros(shape, dtype)
            return np.ctypeslib.as_array(C.cast(p, C.POINTER(ctype)), shape).copy()
        return (arr(ptrs[0], (k, 9), C.c_float, np.float32), arr(ptrs[1], (k, 9), C.c_float, np.float32),
                arr(ptrs[2], (k, 6), C.c_float, np.float32), arr(ptrs[3], (k,), C.c_uint32, np.uint32))

    def materials(self):
        s = Scene()
        check(lib().zrt_gltf_materials(self._h, C.byref(s)), "zrt_gltf_materials")
        desc = np.zeros((s.num_materials, 3, 7), np.int64)
        for i in range(s.num_materials):
            m = s.materials[i]
            for k, name in enumerate(("base_color", "emissive", "transparency")):
                t = getattr(m, name)
                desc[i, k] = (t.offset, t.w, t.h, t.u_min, t.u_max, t.v_min, t.v_max)
        tex = np.ctypeslib.as_array(s.texels, (s.num_texel_floats,)).copy()
        return desc, tex

    def camera(self, name=None, width=None, height=None) -> Camera:
        cam = Camera()
        check(lib().zrt_gltf_camera(self._h, None if name is None else name.encode(),
                                    -1 if width is None else width, -1 if height is None else height,
                                    C.byref(cam)), "zrt_gltf_camera")
        return cam
