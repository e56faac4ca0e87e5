"""MI355X-native render hot path of tigrazone/zig_raytracing_contest.

Host-side mirror of the reference's interface around the one accelerated
seam, `Scene.render(threads, camera, img)` (src/stage3.zig:247):

  * `Config`       -- main.zig:56-69 config.json (grid_resolution, num_threads,
                      num_samples, max_bounce), same keys, same file.
  * `RenderScene`  -- stage2 Geometry.build + bakeInto (host C++, libzrt) and
                      the device-resident scene; `.render(camera, img)` is the
                      drop-in for Scene.render (HIP kernels on gfx950).
  * `camera_for`   -- stage1.loadCamera rules (width/height/aspect ratio).

Everything computes through libzrt.so (include/zrt.h).  There is no CPU
fallback: without the HIP library or a GPU, rendering raises.
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Optional, Tuple

import numpy as np

from . import native

__all__ = ["Config", "RenderScene", "camera_for", "native"]


@dataclasses.dataclass
class Config:
    """main.zig:56-69; parsed strictly like std.json (unknown keys rejected)."""
    grid_resolution: Tuple[int, int, int] = (128, 128, 128)
    num_threads: Optional[int] = None
    num_samples: int = 3
    max_bounce: int = 4

    @classmethod
    def load(cls, path: str = "config.json") -> "Config":
        with open(path) as f:
            d = json.load(f)
        keys = {"grid_resolution", "num_threads", "num_samples", "max_bounce"}
        unknown = set(d) - keys
        if unknown:
            raise ValueError(f"UnknownField: {sorted(unknown)}")
        missing = {"grid_resolution", "num_samples", "max_bounce"} - set(d)
        if missing:
            raise ValueError(f"MissingField: {sorted(missing)}")
        gr = d["grid_resolution"]
        if not (isinstance(gr, list) and len(gr) == 3 and all(isinstance(x, int) and 0 <= x < 2**32
                                                              for x in gr)):
            raise ValueError("grid_resolution must be [u32, u32, u32]")
        nt = d.get("num_threads")
        if nt is not None and not (isinstance(nt, int) and 0 <= nt < 256):
            raise ValueError("num_threads must be null or u8")
        for k in ("num_samples", "max_bounce"):
            if not (isinstance(d[k], int) and 0 <= d[k] < 65536):
                raise ValueError(f"{k} must be u16")
        return cls(tuple(gr), nt, d["num_samples"], d["max_bounce"])


def camera_for(soup, name=None, width=None, height=None) -> native.Camera:
    """stage1.zig:309-371: find the camera by name, apply the size rules."""
    c = soup.camera(name)
    return native.camera_from_matrix(c.matrix, c.yfov, c.aspect, width, height)


class RenderScene:
    """Baked scene on one GPU; `render` mirrors stage3.Scene.render."""

    def __init__(self, soup, resolution=(128, 128, 128), device: int = -1, num_threads: int = 0,
                 device_build: bool = False):
        """device_build: stage 2 on the GPU straight into the context
        (zrt_context_create_built); otherwise host threads + upload."""
        self.soup = soup
        self._keep = []
        if device_build:
            self.geometry = None
            mats = native.Scene()
            native.attach_materials(mats, soup.tex_desc, soup.texels, self._keep)
            self.context = native.Context.built(soup.pos, soup.nrm, soup.uv, soup.mat, mats,
                                                resolution, device)
            return
        self.geometry = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat, resolution,
                                        num_threads)
        native.attach_materials(self.geometry.scene, soup.tex_desc, soup.texels, self._keep)
        self.context = native.Context(self.geometry.scene, device)

    def close(self):
        self.context.close()

    def render(self, camera: native.Camera, img: Optional[np.ndarray] = None, num_samples: int = 3,
               max_bounce: int = 4, seed: int = 0, rank: int = 0, num_ranks: int = 1,
               stats: bool = False, linear: bool = False, packed: bool = False,
               samples_per_pass: int = 0, flags: int = 0):
        """Fills img (h, w, 3) uint8 (this rank's pixels) and returns (img, extras)."""
        if img is None:
            img = np.zeros((camera.h, camera.w, 3), np.uint8)
        assert img.shape == (camera.h, camera.w, 3) and img.dtype == np.uint8 and \
            img.flags["C_CONTIGUOUS"]
        res = self.context.render(camera, num_samples, max_bounce, seed=seed, rank=rank,
                                  num_ranks=num_ranks, stats=stats, image=img, linear=linear,
                                  packed=packed, samples_per_pass=samples_per_pass, flags=flags)
        return img, res
