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
         or plain `python bench.py --gpus N`: with no WORLD_SIZE in the
         environment the process (which has made no HIP call) starts the N
         ranks itself through torch.distributed.run, relays rank 0's line and
         exits with the launcher's status.  A WORLD_SIZE that disagrees with
         --gpus is an error (exit 2): the frame must not silently run on
         fewer GPUs than asked (the reference's partition, stage3.zig:228-229).

Rank 0 prints ONE JSON line, with the sha1 of the whole frame (img_sha1: the
same for any N, asserted equal to the untimed counting frame's and to the CPU
oracle's whole-frame hash in tests/golden/frames.json: oracle_frame_match).
Image tiles (32x32 over several ranks, interleaved t % N) shard the frame: total work is fixed as N grows
("scaling": "strong").  The roofline block is the dominant kernel's, from one
extra frame on one HIP stream (exclusive kernel durations).
"""
from __future__ import annotations

import argparse
import glob
import hashlib
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
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--one-set", action="store_true",
                    help="time frames on one pass set (exclusive kernel durations: the rocprofv3 "
                         "profile of the roofline, NOT the headline schedule)")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="N > 1 process group; gloo (tests only) gathers host copies, ranks may share a GPU")
    return ap.parse_args()


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
    """The reference's thread count: config.json num_threads null means
    getCpuCount (main.zig:90), and stage3.zig:248-252 spawns that many -- every
    CPU in this process's affinity mask.  Also returns the OMP_NUM_THREADS cap
    (on the shared GPU host, the CPU share of one GPU) for the secondary
    figure."""
    avail = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return avail, (min(avail, omp) if omp > 0 else avail)


def cgroup_cpu_quota():
    """cgroup v2 cpu.max as CPUs (None: unlimited or unreadable): what the
    all-core run can really use on a shared host."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def effective_cpus(threads):
    """CPUs the threads can really run on at once: min(affinity mask, cgroup
    cpu.max quota rounded up).  256 threads under a 16-CPU quota share 16."""
    q = cgroup_cpu_quota()
    return max(1, min(threads, int(-(-q // 1)))) if q else threads


def cpu_baseline(soup, cfg, target_s):
    """Oracle in REF mode (the reference's Xoshiro-per-thread, contiguous
    blocks, recursion; gcc -O3, no fast-math) on a bounded, evenly spread
    sample of the same frame, on getCpuCount threads (all CPUs of the
    affinity mask); the OMP_NUM_THREADS-capped run beside it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc   # test infrastructure: the CPU baseline leg only
    c = soup.camera(cfg["camera"])
    cam = orc.camera_from_matrix(c.matrix, c.yfov, c.aspect, cfg["width"], cfg["height"])
    osc = orc.OracleScene(soup)
    threads, capped = cpu_threads()
    npx = cam.w * cam.h

    def run(stride, spp, nthr):
        pixels = np.arange(0, npx, stride, dtype=np.uint32)
        t0 = time.perf_counter()
        _, _, ctr = osc.render_pixels(cam, spp, cfg["max_bounce"], pixels, orc.RNG_REF, 0, nthr)
        return time.perf_counter() - t0, ctr, pixels.size

    def measure(nthr, secs):
        dt, ctr, n = run(1024, 4, nthr)            # calibration: ~2000 pixels x 4 spp
        seg_rate = max(float(ctr[0]), 1.0) / max(dt, 1e-3)
        seg_per_sample = max(float(ctr[0]) / (n * 4), 1.0)
        want_samples = seg_rate * secs / seg_per_sample
        spp = 4
        stride = max(1, int(npx * spp / max(want_samples, 1.0)))
        if stride == 1:                             # whole frame: raise spp instead
            spp = int(min(256, max(4, want_samples / npx)))
        dt, ctr, n = run(stride, spp, nthr)
        if stride == 1 and dt < secs / 2 and spp < 256:   # the calibration under-shot (thread start-up)
            spp = int(min(256, max(spp + 1, spp * secs / max(dt, 1e-3))))
            dt, ctr, n = run(stride, spp, nthr)
        return float(ctr[0]) / dt / 1e6, (f"{n} pixels (every {stride}th of {cam.w}x{cam.h}) x {spp} spp, "
                                          f"{int(ctr[0])} segments in {dt:.1f}s")

    v, sample = measure(threads, target_s)
    eff = effective_cpus(threads)
    out = {"value": round(v, 3), "unit": "Mrays/s", "cores": eff, "effective_cpus": eff,
           "threads": threads, "value_per_effective_cpu": round(v / eff, 4),
           "cgroup_cpu_quota": cgroup_cpu_quota(), "affinity_cpus": threads, "nproc": os.cpu_count(),
           "cpu_model": cpu_model(), "kind": "port",
           "sample": f"{sample}; oracle REF mode (Xoshiro256++ per thread, contiguous blocks, "
                     f"recursion), gcc -O3, {threads} threads = every CPU of the affinity mask "
                     "(num_threads null -> getCpuCount, main.zig:90), sharing "
                     f"{eff} effective CPUs (min of the affinity mask and the cgroup quota)"}
    if capped < threads:
        vc, sc = measure(capped, target_s / 2)
        out["omp_capped"] = {"value": round(vc, 3), "cores": capped, "sample": sc,
                             "what": "the same on OMP_NUM_THREADS threads (the GPU host's CPU share of one GPU)"}
    return out


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
                              "done_in_median_ms": round(sorted(done)[len(done) // 2], 2),
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
                "segments": int(ctr[0]), "threads": threads, "cores": effective_cpus(threads),
                "effective_cpus": effective_cpus(threads),
                "render_mrays_per_effective_cpu": round(int(ctr[0]) / t["render"] / 1e6
                                                        / effective_cpus(threads), 4)}
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def frame_golden(config):
    """The CPU oracle's whole-frame hashes of a BASELINE config
    (tests/golden/frames.json, written by tools/make_frame_golden.py in the
    build container); None when the config has none."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "frames.json")) as fh:
            return json.load(fh).get(config)
    except (OSError, ValueError):
        return None


def roofline_profile_for(config, one_set_kernel="wf_park_kernel"):
    """The newest committed per-kernel counter profile of this workload
    (tools/roofline_profile.py over rocprofv3 passes of `bench.py --one-set`:
    exclusive kernel durations, SQ VALU counts, PMC HBM bytes per launch)."""
    files = glob.glob(os.path.join(ROOT, "profiles", "r*", f"*_roofline_{config}.json"))
    if not files:
        return None
    def order(x):                      # round, then tag: r03zm < r04a < r04ab
        tag = os.path.basename(x).split("_")[0]
        return (int(tag[1:3]) if tag[1:3].isdigit() else 0, len(tag), tag)
    f = max(files, key=order)
    try:
        with open(f) as fh:
            d = json.load(fh)
        return d, os.path.relpath(f, ROOT)
    except (OSError, ValueError):
        return None


# MI355X_MICROARCH.md: 256 CUs x 4 SIMDs, a wave64 VALU instruction issues over
# 2 cycles (32 lanes per cycle), 2.4 GHz peak engine clock: 78.6 T lane-ops/s
# (the 157.3 TF f32 vector peak counts an FMA as 2 flops)
PEAK_VALU_GLANE = 256 * 4 * 32 * 2.4


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_cmd(n, argv, port):
    """The torch.distributed.run command that starts this bench on n ranks
    of one node (the driver's own N > 1 form), with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__)] + list(argv)


def world_check(gpus, env):
    """(world size to run at here, or None: spawn the ranks first).  Raises
    SystemExit(2) when the launcher's WORLD_SIZE disagrees with --gpus."""
    if "WORLD_SIZE" not in env:
        return None if gpus > 1 else 1
    world = int(env["WORLD_SIZE"])
    if world != gpus:
        print(f"bench.py: --gpus {gpus} but WORLD_SIZE={world} (the launcher started a different number "
              "of ranks)", file=sys.stderr, flush=True)
        raise SystemExit(2)
    return world


def spawn_ranks(n, argv):
    """No launcher around us and --gpus n > 1: start the n ranks (this
    process has made no HIP or torch-device call), relay rank 0's JSON line on
    stdout (everything else to stderr), return the launcher's exit status
    (non-zero when any rank failed)."""
    cmd = launcher_cmd(n, argv, free_port())
    print("bench.py: starting %d ranks: %s" % (n, " ".join(cmd)), file=sys.stderr, flush=True)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    for line in p.stdout:
        if line.startswith("{") and '"metric"' in line:
            sys.stdout.write(line)
            sys.stdout.flush()
        else:
            sys.stderr.write(line)
    return p.wait()


def main():
    a = parse()
    world = world_check(a.gpus, os.environ)
    if world is None:
        sys.exit(spawn_ranks(a.gpus, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = torch = None
    gloo = a.backend == "gloo"
    if world > 1:
        # torch first: libzrt then binds to torch's HIP runtime (one runtime
        # per process, so the RCCL buffers and libzrt share device memory)
        import torch
        import torch.distributed as dist
        if gloo:   # tests only: host copies gathered over gloo; ranks may share device 0
            local = local % max(torch.cuda.device_count(), 1)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from zig_raytracing_contest_amd import RenderScene, camera_for, native, scenes
    from zig_raytracing_contest_amd import dist as zdist
    cfgd = dict(scenes.CONFIGS[a.config])
    spp = a.spp or cfgd["spp"]
    soup = scenes.get_scene(cfgd["scene"])
    cam = camera_for(soup, cfgd["camera"], cfgd["width"], cfgd["height"])
    rs = RenderScene(soup, device=local)
    TILE = zdist.TILE                # the multi-rank tile edge (any tiling gives the same image)
    P = native.tile_pixels(cam.w, cam.h, TILE, rank, world).size
    dev_buf = None
    if world > 1 and not gloo:
        dev_buf = torch.zeros(zdist.max_packed(cam.w, cam.h, world) * 3, dtype=torch.uint8,
                              device=f"cuda:{local}")
    tflags = native.FLAG_ONE_SET if a.one_set else 0

    def step(stats=False, flags=tflags):
        """One frame; returns (stats dict, image handle: the assembled frame on
        rank 0 -- packed RGB8 at N = 1 -- or None)."""
        if world > 1 and not gloo:   # this rank's tiles into device memory + RCCL gather to rank 0
            img, res = zdist.render_gathered(rs.context, cam, spp, cfgd["max_bounce"], rank, world, dist,
                                             dev_buf, stats=stats)
            return res["stats"], img
        res = rs.context.render(cam, spp, cfgd["max_bounce"], rank=rank, num_ranks=world, stats=stats,
                                packed=True, flags=flags, tile=TILE)
        if world > 1:                # gloo: host copies
            buf = torch.zeros(zdist.max_packed(cam.w, cam.h, world) * 3, dtype=torch.uint8)
            buf[: res["packed"].size] = torch.from_numpy(res["packed"].reshape(-1))
            return res["stats"], zdist.gather_image(buf, cam.w, cam.h, rank, world, dist)
        return res["stats"], res["packed"]

    def frame_sha1(img):
        """sha1 of the whole w x h x 3 RGB8 frame (row-major): the same for any N."""
        if img is None:
            return None
        if world == 1:
            full = np.zeros((cam.w * cam.h, 3), np.uint8)
            full[native.tile_pixels(cam.w, cam.h, TILE)] = img
            return hashlib.sha1(full.tobytes()).hexdigest()
        return hashlib.sha1(img.cpu().numpy().tobytes()).hexdigest()

    # untimed counting run: exact algorithmic work of one step (same RNG ->
    # same paths as the timed kernels), and the frame every timed frame must equal
    cst, cimg = step(stats=True)
    cprof = rs.context.profile()
    count_sha1 = frame_sha1(cimg) if rank == 0 else None
    for _ in range(a.warmup):
        step()

    def barrier():
        if world > 1:
            dist.barrier()
            if not gloo:
                torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    kern_ms, gpu_ms, launches, segs, img = 0.0, 0.0, 0, 0, None
    for _ in range(a.steps):
        st, img = step()
        kern_ms += st["trace_kernel_ms"]
        gpu_ms += st["render_ms"]
        launches += st["trace_launches"]
        segs += st["segments"]
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dev = "cpu" if gloo else f"cuda:{local}"
        t = torch.tensor([elapsed, float(segs)], dtype=torch.float64, device=dev)
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, total_segs = float(tmax[0]), float(t[1])
    else:
        total_segs = float(segs)

    if rank == 0:
        assert cst["segments"] * a.steps == segs, "counting and timed kernels disagree"
        img_sha1 = frame_sha1(img)
        assert img_sha1 == count_sha1, "the timed frame differs from the counting frame"
        # the whole frame against the CPU oracle's (tools/make_frame_golden.py:
        # every pixel of the frame through oracle/zrt_oracle.c, the
        # reference's renderWorker restated, in the counter-RNG mode)
        golden = frame_golden(a.config) if spp == cfgd["spp"] else None
        oracle_match = None
        if golden is not None:
            oracle_match = (img_sha1 == golden["rgb8_sha1"] and
                            int(total_segs / a.steps) == golden["segments"])
            assert oracle_match, (f"frame differs from the oracle's: sha1 {img_sha1} vs {golden['rgb8_sha1']}, "
                                  f"segments {int(total_segs / a.steps)} vs {golden['segments']}")
        # ---- roofline of the dominant kernel.  The timed frames run two
        # pass sets on two HIP streams, so their kernels overlap and no
        # kernel's duration is its own.  One more frame (after the timed
        # region) runs the same passes on ONE stream with HIP events around
        # every launch: exclusive per-kernel durations (what the committed
        # rocprofv3 profile of `bench.py --one-set` reports).
        rres = rs.context.render(cam, spp, cfgd["max_bounce"], rank=rank, num_ranks=world, packed=True,
                                 flags=native.FLAG_ONE_SET | native.FLAG_KERNEL_TIMES, tile=TILE)
        rprof = rs.context.profile()
        if world == 1:
            assert frame_sha1(rres["packed"]) == img_sha1, "the one-stream frame differs"
        else:   # this rank's tiles only (no collective here: the other ranks wait at the barrier)
            assert rres["stats"]["segments"] == cst["segments"]
        kt = rprof["kernels"]
        dom = max(kt, key=lambda k: kt[k]["ms"])
        dom_name = {"primary": "wf_kernel (primary)", "park": "wf_park_kernel", "shade": "wf_shade_kernel",
                    "bounce": "wf_kernel (bounce)", "resolve": "wf_resolve_kernel"}[dom]
        launch_s = kt[dom]["ms"] / 1e3 / kt[dom]["launches"]
        # algorithmic work of the dominant kernel's launches:
        # the park kernel traces the bounce segments = all - primary
        pc = cprof["primary"]
        if dom == "park":
            cells = cst["cells_visited"] - pc["cells_visited"]
            tests = cst["triangle_tests"] - pc["triangle_tests"]
            alg = B_CELL * cells + B_TRI * tests
        else:
            alg = (B_CELL * cst["cells_visited"] + B_TRI * cst["triangle_tests"] + B_HIT * cst["hits"] + B_PIX * P)
        alg_per_launch = alg / kt[dom]["launches"]
        roof = {"bound": "issue", "kernel": dom_name,
                "launch_ms": round(launch_s * 1e3, 3), "launches_per_frame": kt[dom]["launches"],
                "launch_time": "exclusive: HIP events around each launch of one extra frame whose passes "
                               "run on one stream (the timed frames overlap two streams)",
                "per_kernel_ms_one_stream": {k: round(v["ms"], 3) for k, v in kt.items()},
                "limiter": "VALU issue in the walk, dependent-load latency in the test rounds; "
                           "not DRAM bandwidth (memory_side below)",
                "achieved": None, "peak": round(PEAK_VALU_GLANE, 1), "unit": "Glane-op/s", "frac": None,
                "traffic": None}
        rp = roofline_profile_for(a.config) if spp == cfgd["spp"] and world == 1 else None
        if rp:
            d, src = rp
            kk = d["kernels"].get({"park": "wf_park_kernel", "shade": "wf_shade_kernel"}.get(dom, dom_name))
            if kk:
                lane_ops = kk["valu_insts_per_launch"] * 64 * kk["lane_util"]
                roof["achieved"] = round(lane_ops / launch_s / 1e9, 1)
                roof["frac"] = round(roof["achieved"] / PEAK_VALU_GLANE, 4)
                roof["lane_ops_per_launch"] = lane_ops
                roof["profile"] = src
                roof["profile_launch_ms"] = kk.get("avg_ms")
                roof["profile_valu_issue_frac"] = kk.get("valu_issue_frac")
                roof["profile_lane_util"] = kk.get("lane_util")
                if kk.get("hbm_bytes_per_launch"):
                    tb = kk["hbm_bytes_per_launch"]
                    roof["traffic"] = round(tb / 1e9, 3)
                    roof["traffic_unit"] = "GB per launch (PMC FETCH_SIZE x2 + WRITE_SIZE, gfx950 corrections)"
                    roof["memory_side"] = {"achieved": round(tb / launch_s / 1e9, 1), "peak": PEAK_HBM_GBS,
                                           "unit": "GB/s", "frac": round(tb / launch_s / 1e9 / PEAK_HBM_GBS, 4)}
        roof["algorithmic"] = {
            "what": "SURVEY.md d4 bytes of the kernel's work (8 B per visited cell, 36 B per triangle test"
                    + ("" if dom == "park" else ", hit data + texels, 3 B per pixel") +
                    ") per second: a work rate in HBM-equivalent bytes, NOT DRAM traffic (empty cells are "
                    "answered from LDS, re-reads hit L2)",
            "GB_per_launch": round(alg_per_launch / 1e9, 3),
            "achieved": round(alg_per_launch / launch_s / 1e9, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(alg_per_launch / launch_s / 1e9 / PEAK_HBM_GBS, 4)}
        # the whole frame's d4 bytes over the timed (two-stream) frames: the
        # reference's memory work per second (every cell it visits, every
        # triangle it tests).  A work rate, not a fraction of HBM: the GPU
        # answers most of those cells from LDS and the escape / frustum tables
        # without reading them, so no peak fraction is given.
        frame_alg = (B_CELL * cst["cells_visited"] + B_TRI * cst["triangle_tests"] + B_HIT * cst["hits"] + B_PIX * P)
        roof["reference_equivalent_rate"] = {
            "what": "SURVEY.md d4 bytes of the reference's whole-frame work (8 B per cell visited, 36 B per "
                    "triangle test, hit data + texels, 3 B per pixel) per second of the timed frames; "
                    "NOT DRAM traffic and not comparable with the HBM peak",
            "GB_per_frame": round(frame_alg / 1e9, 1),
            "GBps": round(frame_alg * a.steps / (gpu_ms / 1e3) / 1e9, 1),
            "gpu_ms_per_step": round(gpu_ms / a.steps, 3),
            "avg_launch_ms_overlapped": round(kern_ms / max(launches, 1), 3)}
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
                       "segments_per_step": int(total_segs / a.steps),
                       "schedule": "one pass set (profiling)" if a.one_set else
                                   f"{cprof['passes']} counting passes; timed: default pass sets"},
            "img_sha1": img_sha1,
            "oracle_frame_match": oracle_match,
            "oracle_frame": None if golden is None else {
                "rgb8_sha1": golden["rgb8_sha1"], "segments": golden["segments"],
                "source": "tests/golden/frames.json (tools/make_frame_golden.py: the CPU oracle over every "
                          "pixel, RNG_PATH mode)"},
            "roofline": roof,
            "work": {k: int(cst[k]) for k in ("segments", "cells_visited", "triangle_tests",
                                               "hits", "samples")},
            "work_primary": pc,
            # SURVEY.md d1's companion rate: w*h*spp per second of the timed frames
            "msamples_per_s": round(cam.w * cam.h * spp * a.steps / elapsed / 1e6, 3),
        }
        if world > 1:
            out["backend"] = a.backend
        if world == 1 and not a.no_wall_clock:
            out.update(wall_clock(soup, cfgd, cpu=not a.no_cpu_baseline))
        if not a.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(soup, cfgd, a.cpu_seconds)
            out["gpu_over_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
    rs.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
