#!/usr/bin/env python3
"""Writes the host simulators' inputs (tools/walk_sim.cpp, tools/frustum_sim.cpp)
for a bench config: <out>/scene.bin (grid, cells, triangle positions, host
build) and <out>/cam.bin (origin, lower-left corner, right, up, w, h).
  python tools/dump_sim_inputs.py cfg3 /tmp/sim_cfg3"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zig_raytracing_contest_amd import camera_for, native, scenes  # noqa: E402


def main():
    cfg, out = sys.argv[1], sys.argv[2]
    os.makedirs(out, exist_ok=True)
    d = scenes.CONFIGS[cfg]
    soup = scenes.get_scene(d["scene"])
    cam = camera_for(soup, d["camera"], d["width"], d["height"])
    geo = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat)
    g = geo.scene.grid
    cells = geo.cells().astype(np.uint32)
    tp = geo.tri_pos().astype(np.float32)
    with open(os.path.join(out, "scene.bin"), "wb") as fh:
        np.array(list(g.bbox_min) + list(g.bbox_max), np.float32).tofile(fh)
        np.array(list(g.resolution), np.uint32).tofile(fh)
        np.array(list(g.cell_size), np.float32).tofile(fh)
        np.array([cells.shape[0], tp.shape[0]], np.uint32).tofile(fh)
        cells.tofile(fh)
        tp.tofile(fh)
    c = cam.as_dict()
    np.array(c["origin"] + c["llc"] + c["right"] + c["up"] + [c["w"], c["h"]], np.float32).tofile(
        os.path.join(out, "cam.bin"))
    print(cfg, "cells", cells.shape[0], "refs", tp.shape[0], "camera", c["w"], "x", c["h"])


if __name__ == "__main__":
    main()
