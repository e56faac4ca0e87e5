#!/usr/bin/env python3
"""One rank's share of a frame on one GPU, for N = 1, 2, 4, 8 ranks: the
time an N-GPU run's ranks spend rendering (bench.py's step minus the gather),
and the strong-scaling efficiency that implies: t(1) / (N * max over ranks).
  python tools/rank_time.py [--config cfg3] [--reps 3]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zig_raytracing_contest_amd import RenderScene, camera_for, scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg3")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--ranks", default="1,2,4,8")
a = ap.parse_args()
cfg = scenes.CONFIGS[a.config]
soup = scenes.get_scene(cfg["scene"])
cam = camera_for(soup, cfg["camera"], cfg["width"], cfg["height"])
rs = RenderScene(soup, device=0)
ctx = rs.context
t1 = None
for n in [int(x) for x in a.ranks.split(",")]:
    per = {}
    for r in sorted({0, n - 1} | ({n // 2} if n > 2 else set())):
        ctx.render(cam, cfg["spp"], cfg["max_bounce"], rank=r, num_ranks=n)     # warm
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            st = ctx.render(cam, cfg["spp"], cfg["max_bounce"], rank=r, num_ranks=n)["stats"]
            ts.append(time.perf_counter() - t0)
        per[r] = (min(ts), st["segments"], st["trace_kernel_ms"])
    tmax = max(v[0] for v in per.values())
    if n == 1:
        t1 = tmax
    print(json.dumps({"ranks": n, "ms_per_rank": {r: round(v[0] * 1e3, 2) for r, v in per.items()},
                      "segments": {r: v[1] for r, v in per.items()},
                      "kernel_ms": {r: round(v[2], 2) for r, v in per.items()},
                      "efficiency": round(t1 / (n * tmax), 4) if t1 else None}), flush=True)
rs.close()
