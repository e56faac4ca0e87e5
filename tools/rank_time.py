#!/usr/bin/env python3
"""Every rank's share of a frame on one GPU, for N = 1, 2, 4, 8 ranks: the
time an N-GPU run's ranks spend rendering (bench.py's step minus the gather),
the balance of the interleaved 64x64 tiles (max / mean over ranks), and the
strong-scaling efficiency that implies: t(1) / (N * max over ranks).  The
segments of all ranks must add up to the one-rank frame's.
  python tools/rank_time.py [--config cfg3] [--reps 2] [--ranks 1,2,4,8]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zig_raytracing_contest_amd import RenderScene, camera_for, scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg3")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--ranks", default="1,2,4,8")
ap.add_argument("--tile", type=int, default=32, help="square tile edge (zrt_render_config.tile_size; bench.py: dist.TILE)")
ap.add_argument("--spp-pass", type=int, default=0, help="zrt_render_config.samples_per_pass (0 = automatic)")
a = ap.parse_args()
cfg = scenes.CONFIGS[a.config]
soup = scenes.get_scene(cfg["scene"])
cam = camera_for(soup, cfg["camera"], cfg["width"], cfg["height"])
rs = RenderScene(soup, device=0)
ctx = rs.context
t1 = seg1 = None
for n in [int(x) for x in a.ranks.split(",")]:
    per = {}
    for r in range(n):
        ctx.render(cam, cfg["spp"], cfg["max_bounce"], rank=r, num_ranks=n, tile=a.tile,
                   samples_per_pass=a.spp_pass)     # warm
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            st = ctx.render(cam, cfg["spp"], cfg["max_bounce"], rank=r, num_ranks=n, tile=a.tile,
                            samples_per_pass=a.spp_pass)["stats"]
            ts.append(time.perf_counter() - t0)
        prof = ctx.profile()
        per[r] = (min(ts), st["segments"], st["trace_kernel_ms"], prof["passes"], prof["sets"])
    tmax = max(v[0] for v in per.values())
    tmean = sum(v[0] for v in per.values()) / n
    segs = sum(v[1] for v in per.values())
    if n == 1:
        t1, seg1 = tmax, segs
    print(json.dumps({"config": a.config, "ranks": n, "tile": a.tile, "spp_pass": a.spp_pass,
                      "ms_per_rank": {r: round(v[0] * 1e3, 2) for r, v in per.items()},
                      "segments": {r: v[1] for r, v in per.items()},
                      "passes_sets": {r: [v[3], v[4]] for r, v in per.items()},
                      "max_over_mean": round(tmax / tmean, 4),
                      "segments_total_equal_one_rank": segs == seg1,
                      "predicted_mrays_per_s": round(segs / tmax / 1e6, 1),
                      "efficiency": round(t1 / (n * tmax), 4) if t1 else None}), flush=True)
rs.close()
