#!/usr/bin/env python3
"""Headline benchmark: Mrays/s of the render hot path on the contest config.

BASELINE.json metric "Mrays/sec + wall-clock to output.png on contest
config.json scene", configs[2]: contest scene, 1920x1080, 256 spp, 1 MI355X.
The contest round1.gltf is not in the container, so the scene is the
deterministic ~100k-triangle stand-in of zig_raytracing_contest_amd/scenes.py
("Camera 1", aspect 16:9, --height 1080), config.json max_bounce 4, grid 128^3.

A step = one full render of that frame (530,841,600 path samples) on the
device-resident scene: path-trace kernel + in-order sample resolve + RGB8, and
for N > 1 the RCCL gather of every rank's packed RGB8 tiles to rank 0.
Mrays = Scene.traceRay segments (primary + bounce + pass-through).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line.  Image tiles (64x64, interleaved t % N) shard the
frame: total work is fixed as N grows ("scaling": "strong").
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from zig_raytracing_contest_amd import RenderScene, camera_for, native, scenes  # noqa: E402
from zig_raytracing_contest_amd import dist as zdist  # noqa: E402

PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# algorithmic bytes: 8 B per visited Cell, 36 B per triangle
# test (v0, e1, e2 as 9 f32), per hit 64 B of Triangle.Data + 4 texels x
# (12 B base colour + 12 B emissive + 4 B transparency), 3 B per output pixel.
B_CELL, B_TRI, B_HIT, B_PIX = 8, 36, 64 + 4 * (12 + 12 + 4), 3


def traffic_for(config, kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary for this
    workload (tools/pmc_traffic.py over rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
    passes of this bench; gfx950 corrections there), or None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_traffic_{config}.json"))):
        try:
            with open(f) as fh:
                t = json.load(fh)
        except (OSError, ValueError):
            continue
        if t.get("kernel") == kernel:
            best = (t["bytes_per_launch"], os.path.relpath(f, ROOT))
    return best


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="cfg3", choices=sorted(scenes.CONFIGS))
    ap.add_argument("--spp", type=int, default=None, help="override spp (NOT the headline)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    return ap.parse_args()


def cpu_baseline(soup, cfg, target_s):
    """Oracle in REF mode (the reference's Xoshiro-per-thread, contiguous
    blocks, recursion) on a bounded, evenly spread sample of the same frame."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc   # test infrastructure: the CPU baseline leg only
    c = soup.camera(cfg["camera"])
    cam = orc.camera_from_matrix(c.matrix, c.yfov, c.aspect, cfg["width"], cfg["height"])
    osc = orc.OracleScene(soup)
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16,
                         len(os.sched_getaffinity(0))))
    npx = cam.w * cam.h

    def run(stride, spp):
        pixels = np.arange(0, npx, stride, dtype=np.uint32)
        t0 = time.perf_counter()
        _, _, ctr = osc.render_pixels(cam, spp, cfg["max_bounce"], pixels, orc.RNG_REF, 0, threads)
        return time.perf_counter() - t0, ctr, pixels.size

    dt, ctr, n = run(4096, 4)                   # calibration: ~500 pixels x 4 spp
    seg_rate = max(float(ctr[0]), 1.0) / max(dt, 1e-3)
    seg_per_sample = max(float(ctr[0]) / (n * 4), 1.0)
    want_samples = seg_rate * target_s / seg_per_sample
    spp = 4
    stride = max(1, int(npx * spp / max(want_samples, 1.0)))
    if stride == 1:                             # whole frame: raise spp instead
        spp = int(min(64, max(4, want_samples / npx)))
    dt, ctr, n = run(stride, spp)
    return {"value": round(float(ctr[0]) / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads,
            "kind": "port",
            "sample": f"{n} pixels (every {stride}th of {cam.w}x{cam.h}) x {spp} spp, "
                      f"{int(ctr[0])} segments in {dt:.1f}s; oracle REF mode (Xoshiro256++ per "
                      f"thread, contiguous blocks, recursion), gcc -O2, {threads} threads"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    cfgd = dict(scenes.CONFIGS[a.config])
    spp = a.spp or cfgd["spp"]
    soup = scenes.get_scene(cfgd["scene"])
    cam = camera_for(soup, cfgd["camera"], cfgd["width"], cfgd["height"])
    rs = RenderScene(soup, device=local)
    P = native.tile_pixels(cam.w, cam.h, 64, rank, world).size

    torch = None
    dev_buf = None
    if world > 1:
        import torch
        dev_buf = torch.zeros(zdist.max_packed(cam.w, cam.h, world) * 3, dtype=torch.uint8,
                              device=f"cuda:{local}")

    def step(stats=False):
        ptr = dev_buf.data_ptr() if dev_buf is not None else None
        res = rs.context.render(cam, spp, cfgd["max_bounce"], rank=rank, num_ranks=world,
                                stats=stats, device_ptr=ptr)
        if world > 1:   # RCCL gather of the packed RGB8 tiles to rank 0 (+ unpermute)
            zdist.gather_image(dev_buf, cam.w, cam.h, rank, world, dist)
        return res["stats"]

    # untimed counting run: exact algorithmic work of one step (same RNG ->
    # same paths as the timed kernel)
    cst = step(stats=True)
    for _ in range(a.warmup):
        step()

    def barrier():
        if world > 1:
            dist.barrier()
            torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    kern_ms, launches, segs = 0.0, 0, 0
    for _ in range(a.steps):
        st = step()
        kern_ms += st["trace_kernel_ms"]
        launches += st["trace_launches"]
        segs += st["segments"]
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed, float(segs)], dtype=torch.float64, device=f"cuda:{local}")
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, total_segs = float(tmax[0]), float(t[1])
    else:
        total_segs = float(segs)

    if rank == 0:
        assert cst["segments"] * a.steps == segs, "counting and timed kernels disagree"
        avg_launch_s = kern_ms / 1e3 / max(launches, 1)
        alg_bytes = (B_CELL * cst["cells_visited"] + B_TRI * cst["triangle_tests"] +
                     B_HIT * cst["hits"] + B_PIX * P)
        # the counting run takes the megakernel (1 launch/pass); the timed run
        # takes the wavefront path (max_bounce launches/pass): bytes per timed
        # launch = the step's bytes / the step's timed launches, so
        # achieved = sum(bytes) / sum(launch durations) over the step.
        per_launch = alg_bytes / max(launches / a.steps, 1)
        achieved = per_launch / avg_launch_s / 1e9
        mode = os.environ.get("ZRT_MODE", "wf")
        kname = {"mega": "trace_kernel", "split": "wf_trace_kernel"}.get(mode, "wf_kernel")
        out = {
            "metric": "Mrays/sec + wall-clock to output.png on contest config.json scene",
            "value": round(total_segs / elapsed / 1e6, 3),
            "unit": "Mrays/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{a.config}: {cfgd['scene']} stand-in "
                                   f"({soup.num_triangles} tris, {rs.geometry.num_refs} refs), "
                                   f"{cam.w}x{cam.h}, {spp} spp, max_bounce "
                                   f"{cfgd['max_bounce']}, grid 128^3",
                       "global_batch": cam.w * cam.h * spp, "parallelism": f"tiles{world}",
                       "segments_per_step": int(total_segs / a.steps)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
                         "traffic": None,
                         "kernel": kname, "avg_launch_ms": round(avg_launch_s * 1e3, 3),
                         "alg_bytes_per_launch": int(per_launch)},
            "work": {k: int(cst[k]) for k in ("segments", "cells_visited", "triangle_tests",
                                               "hits", "samples")},
        }
        tr = traffic_for(a.config, kname) if spp == cfgd["spp"] else None
        if tr:
            out["roofline"]["traffic"] = round(tr[0] / 1e9, 3)
            out["roofline"]["traffic_unit"] = "GB per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)"
            out["roofline"]["traffic_source"] = tr[1]
            out["roofline"]["alg_GB_per_launch"] = round(per_launch / 1e9, 3)
        if not a.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(soup, cfgd, a.cpu_seconds)
            out["gpu_over_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    rs.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
