#!/usr/bin/env python3
"""Quick GPU check of the park kernel before the full suite: small renders
must equal the per-lane wf_kernel image (bit for bit)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zig_raytracing_contest_amd import RenderScene, camera_for, native, scenes  # noqa: E402

for name, cam_name, h, spp in (("cornell", None, 48, 4), ("sphere", None, 48, 4), ("contest", "Camera 1", 54, 2)):
    soup = scenes.get_scene(name)
    c = soup.camera(cam_name)
    cam = camera_for(soup, cam_name, None if c.aspect else h, h)
    rs = RenderScene(soup, device=0)
    ref, r0 = rs.render(cam, num_samples=spp, max_bounce=4, flags=native.FLAG_LANE_WALK)
    for mode, flags in (("bounces", 0),):
        img, r = rs.render(cam, num_samples=spp, max_bounce=4, flags=flags)
        print(json.dumps({"scene": name, "park": mode, "identical": bool(np.array_equal(ref, img)),
                          "segments": [r0["stats"]["segments"], r["stats"]["segments"]]}), flush=True)
    rs.close()
