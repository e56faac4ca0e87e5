#!/usr/bin/env python3
"""Headline benchmark: Mrays/s of the render hot path on the contest config,
plus the wall-clock to output.png.

BASELINE.json metric "Mrays/sec + wall-clock to output.png on contest
config.json scene", configs[2]: contest scene, 1920x1080, 256 spp, 1 MI355X.
The contest round1.gltf is not in the container, so the scene is the
deterministic ~100k-triangle stand-in of zig_raytracing_contest_amd/scenes.py
("Camera 1", aspect 16:9, --height 1080), config.json max_bounce 4, grid 128^3.

A step = one full render of that frame (530,841,600 path samples) on the
device-resident scene: path-trace kernels + in-order sample resolve + RGB8, and
for N > 1 the RCCL gather of every rank's packed RGB8 tiles to rank 0.
Mrays = Scene.traceRay segments (primary + bounce + pass-through).

Beside the timed loop (rank 0, N = 1, after it):
  * wall_clock_ms: the `zrt` CLI end to end on the same scene written as glTF
    with the repo's config.json (its num_samples), i.e. the reference's "Done
    in" (main.zig:78 -> :142: load, grid build, render, PNG save), and the CPU
    path's end-to-end time on the same input (cpu_wall_clock_ms);
  * cpu_baseline: the oracle's REF mode (the reference's schedule) on the
    host's CPUs over a bounded sample of the timed frame.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline] [--no-wall-clock]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line.  Image tiles (64x64, interleaved t % N) shard the
frame: total work is fixed as N grows ("scaling": "strong").
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# algorithmic bytes: 8 B per visited Cell, 36 B per triangle
# test (v0, e1, e2 as 9 f32), per hit 64 B of Triangle.Data + 4 texels x
# (12 B base colour + 12 B emissive + 4 B transparency), 3 B per output pixel.
B_CELL, B_TRI, B_HIT, B_PIX = 8, 36, 64 + 4 * (12 + 12 + 4), 3
CLI = os.path.join(ROOT, "zig_raytracing_contest_amd", "bin", "zrt")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--spp", type=int, default=None, help="override spp (NOT the headline)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-wall-clock", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=24.0)
    return ap.parse_args()


def traffic_for(config, kernel):
    """Memory-side bytes per launch of `kernel` from the newest committed PMC
    summary for this workload (tools/pmc_traffic.py over rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of this bench, gfx950 corrections there)."""
    best = None
    # newest round tag last: r01 < r01i < r02e < r02m < r02aj (length, then name)
    def tag_key(f):
        t = os.path.basename(f).split("_traffic_")[0]
        return (len(t), t)
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_traffic_{config}.json")), key=tag_key):
        try:
            with open(f) as fh:
                t = json.load(fh)
        except (OSError, ValueError):
            continue
        if kernel in t.get("kernel", ""):
            best = (t["bytes_per_launch"], os.path.relpath(f, ROOT))
    return best


def valu_for(config):
    """VALU issue fraction per launch type (SURVEY.md d3's secondary figure)
    from the newest committed SQ counter summary for this workload
    (tools/gpu_r2round.sh: SQ_INSTS_VALU x 2 cycles / SIMD cycles)."""
    files = glob.glob(os.path.join(ROOT, "profiles", "r02", f"r*_sq_counters_{config}_*.json"))
    if not files:
        return None
    f = max(files, key=lambda x: (len(os.path.basename(x).split("_")[0]), os.path.basename(x)))
    try:
        with open(f) as fh:
            d = json.load(fh)
        return {"per_kernel": {k.rstrip("( "): v.get("_valu_issue_frac") for k, v in d["kernels"].items()},
                "source": os.path.relpath(f, ROOT)}
    except (OSError, ValueError, KeyError):
        return None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_threads():
    """All CPUs this process may use (the reference's num_threads null =
    getCpuCount, main.zig:90), capped by OMP_NUM_THREADS when set: on the
    shared GPU host that is the CPU share of one GPU."""
    avail = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(avail, omp) if omp > 0 else avail), avail


def cpu_baseline(soup, cfg, target_s):
    """Oracle in REF mode (the reference's Xoshiro-per-thread, contiguous
    blocks, recursion; gcc -O3, no fast-math) on a bounded, evenly spread
    sample of the same frame."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc   # test infrastructure: the CPU baseline leg only
    c = soup.camera(cfg["camera"])
    cam = orc.camera_from_matrix(c.matrix, c.yfov, c.aspect, cfg["width"], cfg["height"])
    osc = orc.OracleScene(soup)
    threads, avail = cpu_threads()
    npx = cam.w * cam.h

    def run(stride, spp):
        pixels = np.arange(0, npx, stride, dtype=np.uint32)
        t0 = time.perf_counter()
        _, _, ctr = osc.render_pixels(cam, spp, cfg["max_bounce"], pixels, orc.RNG_REF, 0, threads)
        return time.perf_counter() - t0, ctr, pixels.size

    dt, ctr, n = run(1024, 4)                   # calibration: ~2000 pixels x 4 spp
    seg_rate = max(float(ctr[0]), 1.0) / max(dt, 1e-3)
    seg_per_sample = max(float(ctr[0]) / (n * 4), 1.0)
    want_samples = seg_rate * target_s / seg_per_sample
    spp = 4
    stride = max(1, int(npx * spp / max(want_samples, 1.0)))
    if stride == 1:                             # whole frame: raise spp instead
        spp = int(min(256, max(4, want_samples / npx)))
    dt, ctr, n = run(stride, spp)
    return {"value": round(float(ctr[0]) / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads,
            "cores_available": avail, "nproc": os.cpu_count(), "cpu_model": cpu_model(), "kind": "port",
            "sample": f"{n} pixels (every {stride}th of {cam.w}x{cam.h}) x {spp} spp, "
                      f"{int(ctr[0])} segments in {dt:.1f}s; oracle REF mode (Xoshiro256++ per "
                      f"thread, contiguous blocks, recursion), gcc -O3, {threads} threads "
                      f"({avail} in the affinity mask; OMP_NUM_THREADS caps it on the GPU host)"}


_DUR = re.compile(r"(\d+(?:\.\d+)?)(ms|us|ns|s|m|h)")


def parse_duration_ms(s):
    """The CLI's fmt_duration ("1m2.5s", "171.234ms") in milliseconds."""
    scale = {"h": 3.6e6, "m": 6e4, "s": 1e3, "ms": 1.0, "us": 1e-3, "ns": 1e-6}
    return sum(float(v) * scale[u] for v, u in _DUR.findall(s))


def wall_clock(soup, cfgd, reps=3, cpu=True):
    """glTF -> output.png: the product CLI (GPU), and the CPU path on the same
    files.  Returns a dict of the JSON fields."""
    from zig_raytracing_contest_amd import native, pngio, scenes
    tmp = tempfile.mkdtemp(prefix="zrt_wall_")
    try:
        scenes.write_gltf(soup, os.path.join(tmp, "contest.gltf"))
        shutil.copy(os.path.join(ROOT, "config.json"), tmp)
        with open(os.path.join(ROOT, "config.json")) as fh:
            conf = json.load(fh)
        args = [CLI, "--in", "contest.gltf", "--out", "output.png", "--height", str(cfgd["height"]),
                "--camera", cfgd["camera"]]
        done, wall, log = [], [], ""
        for _ in range(reps):
            t0 = time.perf_counter()
            p = subprocess.run(args, cwd=tmp, capture_output=True, text=True, timeout=600)
            wall.append((time.perf_counter() - t0) * 1e3)
            if p.returncode != 0:
                raise RuntimeError(f"zrt CLI failed ({p.returncode}): {p.stderr[-400:]}")
            log = p.stderr
            m = re.search(r"Done in (\S+)", log)
            done.append(parse_duration_ms(m.group(1)) if m else float("nan"))
        rays = re.search(r"Rays: .*", log)
        stages = {m.group(1).lower(): round(parse_duration_ms(m.group(2)), 2)
                  for m in re.finditer(r"info: (\w+) in (\S+)", log) if m.group(1) != "Done"}
        out = {"wall_clock_ms": round(min(done), 2),
               "wall_clock": {"what": f"zrt CLI, contest stand-in as glTF, --height {cfgd['height']} "
                                      f"--camera '{cfgd['camera']}', config.json num_samples "
                                      f"{conf['num_samples']} max_bounce {conf['max_bounce']}: "
                                      "'Done in' (main.zig:78 -> :142), min of "
                                      f"{reps} runs", "done_in_ms": [round(x, 2) for x in done],
                              "process_ms": [round(x, 2) for x in wall],
                              "cli_rays": rays.group(0) if rays else None,
                              "stages_ms_last_run": stages}}
        if cpu:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as orc   # test infrastructure: the CPU leg only
            threads, _ = cpu_threads()
            t = {}
            t0 = time.perf_counter()
            g = native.Gltf(os.path.join(tmp, "contest.gltf"), threads)
            pos, nrm, uv, mat = g.soup()
            desc, tex = g.materials()
            t["load"] = time.perf_counter() - t0
            c = soup.camera(cfgd["camera"])
            cam = orc.camera_from_matrix(c.matrix, c.yfov, c.aspect, None, cfgd["height"])
            t1 = time.perf_counter()

            class _Soup:   # the loaded glTF as the oracle's scene input
                pass
            s = _Soup()
            s.pos, s.nrm, s.uv, s.mat, s.tex_desc, s.texels = pos, nrm, uv, mat, desc[:, :, :7], tex
            s.num_triangles, s.num_materials = int(mat.size), int(desc.shape[0])
            osc = orc.OracleScene(s, tuple(conf["grid_resolution"]))
            t["build"] = time.perf_counter() - t1
            t2 = time.perf_counter()
            rgb, _, ctr = osc.render(cam, conf["num_samples"], conf["max_bounce"], orc.RNG_REF, 0, threads,
                                     want_linear=False)
            t["render"] = time.perf_counter() - t2
            t3 = time.perf_counter()
            pngio.write(os.path.join(tmp, "output_cpu.png"), rgb.reshape(cam.h, cam.w, 3))
            t["save"] = time.perf_counter() - t3
            total = sum(t.values()) * 1e3
            out["cpu_wall_clock_ms"] = round(total, 2)
            out["cpu_wall_clock"] = {
                "what": f"same glTF and config.json on the host: glTF load (zrt_gltf_load, {threads} threads), "
                        "grid build + bake (oracle, single-threaded as stage2.zig), render (oracle REF mode, "
                        f"{threads} threads), PNG save (zlib); Python process already running",
                "stages_ms": {k: round(v * 1e3, 2) for k, v in t.items()},
                "segments": int(ctr[0]), "cores": threads}
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = torch = None
    if world > 1:
        # torch first: libzrt then binds to torch's HIP runtime (one runtime
        # per process, so the RCCL buffers and libzrt share device memory)
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from zig_raytracing_contest_amd import RenderScene, camera_for, native, scenes
    from zig_raytracing_contest_amd import dist as zdist
    cfgd = dict(scenes.CONFIGS[a.config])
    spp = a.spp or cfgd["spp"]
    soup = scenes.get_scene(cfgd["scene"])
    cam = camera_for(soup, cfgd["camera"], cfgd["width"], cfgd["height"])
    rs = RenderScene(soup, device=local)
    P = native.tile_pixels(cam.w, cam.h, 64, rank, world).size
    dev_buf = None
    if world > 1:
        dev_buf = torch.zeros(zdist.max_packed(cam.w, cam.h, world) * 3, dtype=torch.uint8,
                              device=f"cuda:{local}")

    def step(stats=False):
        if world > 1:   # this rank's tiles into device memory + RCCL gather to rank 0
            return zdist.render_gathered(rs.context, cam, spp, cfgd["max_bounce"], rank, world, dist,
                                         dev_buf, stats=stats)[1]["stats"]
        return rs.context.render(cam, spp, cfgd["max_bounce"], stats=stats)["stats"]

    # untimed counting run: exact algorithmic work of one step (same RNG ->
    # same paths as the timed kernels)
    cst = step(stats=True)
    for _ in range(a.warmup):
        step()

    def barrier():
        if world > 1:
            dist.barrier()
            torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    kern_ms, gpu_ms, launches, segs = 0.0, 0.0, 0, 0
    for _ in range(a.steps):
        st = step()
        kern_ms += st["trace_kernel_ms"]
        gpu_ms += st["render_ms"]
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
        # two passes are in flight at once on two HIP streams (DESIGN.md
        # §5), so launches overlap: a launch's share of the machine is the
        # step's GPU time (HIP events from the first launch to the join of
        # both streams) over its launches, and achieved = the step's
        # algorithmic bytes over that GPU time.  The per-launch event
        # intervals (what rocprofv3 reports as kernel durations, overlapped)
        # are kept beside it.
        avg_launch_s = gpu_ms / 1e3 / max(launches, 1)
        overlapped_launch_s = kern_ms / 1e3 / max(launches, 1)
        alg_bytes = (B_CELL * cst["cells_visited"] + B_TRI * cst["triangle_tests"] +
                     B_HIT * cst["hits"] + B_PIX * P)
        per_launch = alg_bytes / max(launches / a.steps, 1)
        achieved = per_launch / avg_launch_s / 1e9
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
            # the roofline contract names hbm|mfma; this kernel is a pointer
            # chase: its achieved fraction is algorithmic bytes over launch
            # time, and the memory side (PMC bytes over launch time) is far
            # lower -- it is bound by the latency of dependent loads under
            # divergence, not by DRAM bandwidth (profiles/)
            "roofline": {"bound": "hbm", "limiter": "latency", "achieved": round(achieved, 1),
                         "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
                         "traffic": None,
                         "kernel": "trace launches: wf_kernel<7,true> (primary), wf_park_kernel + "
                                   "wf_shade_kernel (each bounce)",
                         "avg_launch_ms": round(avg_launch_s * 1e3, 3),
                         "avg_launch_ms_overlapped": round(overlapped_launch_s * 1e3, 3),
                         "gpu_ms_per_step": round(gpu_ms / a.steps, 3),
                         "launch_time": "step GPU time / launches: two passes run at once on two "
                                        "HIP streams, so launches overlap; avg_launch_ms_overlapped "
                                        "is the per-launch HIP-event interval (rocprofv3's durations)",
                         "alg_GB_per_launch": round(per_launch / 1e9, 3)},
            "work": {k: int(cst[k]) for k in ("segments", "cells_visited", "triangle_tests",
                                               "hits", "samples")},
            # SURVEY.md d1's companion rate: w*h*spp per second of the timed frames
            "msamples_per_s": round(cam.w * cam.h * spp * a.steps / elapsed / 1e6, 3),
        }
        vc = valu_for(a.config) if spp == cfgd["spp"] else None
        if vc:
            out["roofline"]["valu_issue"] = vc
        tr = traffic_for(a.config, "wf_shade_kernel") if spp == cfgd["spp"] else None
        if tr:
            mem_gbs = tr[0] / 1e9 / avg_launch_s
            out["roofline"]["traffic"] = round(tr[0] / 1e9, 3)
            out["roofline"]["traffic_unit"] = "GB per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)"
            out["roofline"]["traffic_source"] = tr[1]
            out["roofline"]["memory_side_GBps"] = round(mem_gbs, 1)
            out["roofline"]["frac_memory_side"] = round(mem_gbs / PEAK_HBM_GBS, 4)
        if world == 1 and not a.no_wall_clock:
            out.update(wall_clock(soup, cfgd, cpu=not a.no_cpu_baseline))
        if not a.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(soup, cfgd, a.cpu_seconds)
            out["gpu_over_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    rs.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
