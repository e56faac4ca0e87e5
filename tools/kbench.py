#!/usr/bin/env python3
"""Variant sweep on one GPU: same frame, several env settings, one process.
Checks every variant's image is identical to the first (exactness guard)."""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zig_raytracing_contest_amd import camera_for, native, scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg3")
ap.add_argument("--spp", type=int, default=64, help="0: the config's own spp")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--cell-stats", action="store_true", help="one counting render first (ZRT_CELL_STATS)")
ap.add_argument("--var", action="append", default=[], help="ENV=VAL[,ENV=VAL] per variant")
a = ap.parse_args()
cfg = scenes.CONFIGS[a.config]
if a.spp == 0:
    a.spp = cfg["spp"]
soup = scenes.get_scene(cfg["scene"])
cam = camera_for(soup, cfg["camera"], cfg["width"], cfg["height"])
geo = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat)
keep = []
native.attach_materials(geo.scene, soup.tex_desc, soup.texels, keep)
ref = None
if a.cell_stats:
    os.environ["ZRT_CELL_STATS"] = "1"
    ctx = native.Context(geo.scene)
    r = ctx.render(cam, a.spp, cfg["max_bounce"], stats=True)
    print(json.dumps({"stats": {k: v for k, v in r["stats"].items()}}), flush=True)
    ctx.close()
for var in (a.var or [""]):
    env = dict(kv.split("=") for kv in var.split(",") if kv)
    flags = int(env.pop("FLAGS", "0"), 0)   # zrt_render_config.flags (ZRT_FLAG_*)
    spp_pass = int(env.pop("SPP_PASS", "0"))  # zrt_render_config.samples_per_pass (0 = auto)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    ctx = native.Context(geo.scene)
    img = np.zeros((cam.h, cam.w, 3), np.uint8)
    ctx.render(cam, a.spp, cfg["max_bounce"], image=img, flags=flags, samples_per_pass=spp_pass)   # warm
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        r = ctx.render(cam, a.spp, cfg["max_bounce"], image=img, flags=flags, samples_per_pass=spp_pass)
        ts.append(time.perf_counter() - t0)
    st = r["stats"]
    same = True if ref is None else bool(np.array_equal(ref, img))
    if ref is None:
        ref = img.copy()
    rec = {"var": var or "default", "mrays": round(st["segments"] / min(ts) / 1e6, 1),
           "kernel_ms": round(st["trace_kernel_ms"], 2), "wall_ms": round(min(ts) * 1e3, 2),
           "identical": same, "segments": int(st["segments"]),
           "img_sha1": hashlib.sha1(img.tobytes()).hexdigest()[:12]}
    if flags & native.FLAG_KERNEL_TIMES:   # per-kernel device ms of the last frame (one stream with FLAG_ONE_SET)
        rec["kernels_ms"] = {k: round(v["ms"], 2) for k, v in ctx.profile()["kernels"].items()}
    if not same:
        dif = np.any(ref != img, axis=2)
        rec["diff_pixels"] = int(dif.sum())
        rec["max_abs"] = int(np.abs(ref.astype(int) - img.astype(int)).max())
    print(json.dumps(rec), flush=True)
    ctx.close()
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
