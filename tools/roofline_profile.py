#!/usr/bin/env python3
"""Per-kernel roofline profile of one bench command (bench.py reads it).

  python tools/roofline_profile.py gpurun_out/<tag> --config cfg3 --out profiles/r03/<tag>_roofline_cfg3.json

<dir> holds the rocprofv3 runs of tools/gpu_roofline.sh, all of the SAME
command (`bench.py --one-set ...`: every pass on one HIP stream, so each
kernel's duration is its own):
  prof/      --kernel-trace --stats      -> average duration per kernel
  pmc_sq1/   --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY
             SQ_INSTS_SALU GRBM_GUI_ACTIVE
  pmc_l2/    --pmc TCC_HIT_sum TCC_MISS_sum
  pmc_FETCH_SIZE/, pmc_WRITE_SIZE/  (one TCC byte counter per pass)

Per kernel and launch (counters summed over the per-XCD rows of a dispatch,
averaged over the kernel's dispatches):
  valu_insts_per_launch  SQ_INSTS_VALU
  lane_util              SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU)
  valu_issue_frac        2 SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
                         (a wave64 VALU instruction occupies its SIMD 2 cycles;
                         GRBM_GUI_ACTIVE is summed over the 8 XCDs)
  wait_frac              SQ_WAIT_ANY / SQ_WAVE_CYCLES
  hbm_bytes_per_launch   FETCH_SIZE KiB x 1024 x 2 + WRITE_SIZE KiB x 1024
                         (MI355X_MICROARCH.md's gfx950 corrections)
"""
import argparse
import collections
import csv
import glob
import json
import os
import re

KERNELS = (("wf_park_kernel", r"wf_park2?_kernel"), ("wf_shade_kernel", r"wf_shade_kernel"),
           ("wf_kernel (primary)", r"wf_kernel<\d+, true"), ("wf_kernel (bounce)", r"wf_kernel<\d+, false"),
           ("wf_resolve_kernel", r"wf_resolve_kernel"), ("trace_kernel", r"trace_kernel"))


def kname(raw):
    for k, rx in KERNELS:
        if re.search(rx, raw):
            return k
    return None


def counters(path):
    """{kernel: {counter: sum over dispatches}}, {kernel: dispatches}"""
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if k:
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((f, r["Dispatch_Id"]))
    return tot, {k: len(v) for k, v in disp.items()}


def kernel_stats(path):
    out = {}
    for f in glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r["Name"])
            if k:
                calls, tot = int(r["Calls"]), float(r["TotalDurationNs"])
                o = out.setdefault(k, {"calls": 0, "total_ns": 0.0})
                o["calls"] += calls
                o["total_ns"] += tot
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--command", default="")
    ap.add_argument("--out")
    a = ap.parse_args()
    ks = kernel_stats(os.path.join(a.dir, "prof"))
    res = {}
    for k, _ in KERNELS:
        if k not in ks:
            continue
        r = {"avg_ms": round(ks[k]["total_ns"] / ks[k]["calls"] / 1e6, 3), "calls": ks[k]["calls"]}
        res[k] = r
    sq, nsq = counters(os.path.join(a.dir, "pmc_sq1"))
    l2, _ = counters(os.path.join(a.dir, "pmc_l2"))
    fe, nfe = counters(os.path.join(a.dir, "pmc_FETCH_SIZE"))
    wr, nwr = counters(os.path.join(a.dir, "pmc_WRITE_SIZE"))
    for k in list(res):
        r = res[k]
        c = sq.get(k)
        if c and nsq.get(k):
            n = nsq[k]
            r["pmc_dispatches"] = n
            r["valu_insts_per_launch"] = c["SQ_INSTS_VALU"] / n
            r["salu_insts_per_launch"] = c.get("SQ_INSTS_SALU", 0.0) / n
            if c.get("SQ_ACTIVE_INST_VALU"):
                r["lane_util"] = round(c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"]), 4)
            if c.get("GRBM_GUI_ACTIVE"):
                r["valu_issue_frac"] = round(2 * c["SQ_INSTS_VALU"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
            if c.get("SQ_WAVE_CYCLES"):
                r["wait_frac"] = round(c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 4)
            for key in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_WAVE_CYCLES",
                        "SQ_WAIT_ANY", "SQ_INSTS_SALU", "GRBM_GUI_ACTIVE"):
                if key in c:
                    r.setdefault("counters_total", {})[key] = c[key]
        h = l2.get(k)
        if h and (h.get("TCC_HIT_sum", 0) + h.get("TCC_MISS_sum", 0)):
            r["l2_hit"] = round(h["TCC_HIT_sum"] / (h["TCC_HIT_sum"] + h["TCC_MISS_sum"]), 4)
        if fe.get(k) and wr.get(k):
            fb = 2.0 * 1024.0 * fe[k]["FETCH_SIZE"] / nfe[k]
            wb = 1024.0 * wr[k]["WRITE_SIZE"] / nwr[k]
            r["fetch_bytes_per_launch"] = fb
            r["write_bytes_per_launch"] = wb
            r["hbm_bytes_per_launch"] = fb + wb
    out = {"config": a.config, "command": a.command, "source": os.path.basename(os.path.normpath(a.dir)),
           "note": "every run is the same `bench.py --one-set` command: passes on one HIP stream, so a "
                   "kernel's duration is exclusive; counters per launch = sum over a kernel's dispatches / "
                   "dispatches", "kernels": res}
    s = json.dumps(out, indent=1)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as fh:
            fh.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
