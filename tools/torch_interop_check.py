#!/usr/bin/env python3
"""bench.py's N > 1 load order on one GPU: torch (and its bundled HIP runtime)
first, then libzrt through ctypes, rendering into a torch device buffer; the
packed RGB8 must equal the plain render's.  Prints which libamdhip64 is mapped."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zig_raytracing_contest_amd import RenderScene, camera_for, native, scenes  # noqa: E402

torch.cuda.set_device(0)
x = torch.ones(16, device="cuda:0")
soup = scenes.get_scene("cornell")
cam = camera_for(soup, None, 128, 96)
rs = RenderScene(soup, device=0)
P = native.tile_pixels(cam.w, cam.h, 64, 0, 1).size
buf = torch.zeros(P * 3, dtype=torch.uint8, device="cuda:0")
res = rs.context.render(cam, 4, 4, device_ptr=buf.data_ptr(), packed=True)
torch.cuda.synchronize()
dev = buf.cpu().numpy()
host = res["packed"].reshape(-1) if "packed" in res else None
maps = [l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l]
print({"hip_libs": sorted(set(maps)), "device_equals_host": bool(host is not None and (dev == host).all()),
       "nonzero": int((dev != 0).sum()), "x": float(x.sum())})
g = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat, device=0)
print({"device_grid_build_refs": g.num_refs})
