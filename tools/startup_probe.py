#!/usr/bin/env python3
"""Where the zrt CLI's "Done in" goes before the render.

Writes the contest stand-in as glTF (as bench.py's wall_clock does), runs the
CLI N times with ZRT_TIMING=1 (cli.cpp: when the HIP warm-up thread ran, how
long the first GPU use waited for it, group_create_built, grid info) and
tools/bin/hip_init_probe N times (hipGetDeviceCount, context creation,
dlopen(libzrt.so), the grid-build module, the rest of zrt_device_warmup).
Prints one JSON line per run and a summary of medians.

  python tools/startup_probe.py [--runs 5] [--height 1080]
"""
import argparse
import json
import os
import re
import shutil
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from zig_raytracing_contest_amd import scenes  # noqa: E402

CLI = os.path.join(ROOT, "zig_raytracing_contest_amd", "bin", "zrt")
PROBE = os.path.join(ROOT, "tools", "bin", "hip_init_probe")
_DUR = re.compile(r"([0-9.]+)(h|ms|us|ns|m|s)")


def ms(s):
    scale = {"h": 3.6e6, "m": 6e4, "s": 1e3, "ms": 1.0, "us": 1e-3, "ns": 1e-6}
    return sum(float(v) * scale[u] for v, u in _DUR.findall(s))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--height", type=int, default=1080)
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="zrt_start_")
    try:
        scenes.write_gltf(scenes.get_scene("contest"), os.path.join(tmp, "contest.gltf"))
        shutil.copy(os.path.join(ROOT, "config.json"), tmp)
        rows = []
        for _ in range(a.runs):
            env = dict(os.environ, ZRT_TIMING="1")
            p = subprocess.run([CLI, "--in", "contest.gltf", "--out", "o.png", "--height", str(a.height),
                                "--camera", "Camera 1"], cwd=tmp, capture_output=True, text=True, timeout=300,
                               env=env)
            if p.returncode != 0:
                raise SystemExit(p.stderr[-500:])
            st = {m.group(1).lower(): ms(m.group(2)) for m in re.finditer(r"info: (\w+) in (\S+)", p.stderr)}
            t = re.search(r"timing: warm-up thread (\S+) \.\. (\S+) \((\S+)\), joined at (\S+) after waiting (\S+), "
                          r"group_create_built (\S+), grid info (\S+)", p.stderr)
            row = {"stages_ms": {k: round(v, 2) for k, v in st.items()}}
            if t:
                row.update({"warm_begin_ms": ms(t.group(1)), "warm_end_ms": ms(t.group(2)),
                            "warm_ms": ms(t.group(3)), "joined_at_ms": ms(t.group(4)),
                            "join_wait_ms": ms(t.group(5)), "group_create_built_ms": ms(t.group(6)),
                            "grid_info_ms": ms(t.group(7))})
            rows.append(row)
            print(json.dumps({"cli": row}), flush=True)
        probes = []
        if os.path.exists(PROBE):
            for _ in range(a.runs):
                p = subprocess.run([PROBE, os.path.join(ROOT, "zig_raytracing_contest_amd", "libzrt.so")],
                                   capture_output=True, text=True, timeout=120)
                if p.returncode == 0:
                    probes.append(json.loads(p.stdout))
                    print(json.dumps({"hip_init_probe": probes[-1]}), flush=True)
        med = lambda xs: round(statistics.median(xs), 2) if xs else None  # noqa: E731
        summ = {k: med([r[k] for r in rows if k in r]) for k in
                ("warm_ms", "joined_at_ms", "join_wait_ms", "group_create_built_ms", "grid_info_ms")}
        for k in ("loaded", "compiled", "rendered", "saved", "done"):
            summ[k] = med([r["stages_ms"].get(k) for r in rows if k in r["stages_ms"]])
        for k in (probes[0].keys() if probes else []):
            summ["probe_" + k] = med([p[k] for p in probes])
        print(json.dumps({"summary": summ}), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
