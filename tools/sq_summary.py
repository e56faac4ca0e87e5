#!/usr/bin/env python3
"""Per-kernel SQ / TCC / GRBM counter summary of the counter passes that
tools/gpu_r2round.sh runs (kbench cfg3 64 spp, all dispatches incl. warm-up).

  python tools/sq_summary.py gpurun_out/<tag> [--out profiles/r02/<tag>_sq_counters_cfg3_64spp.json]

Derived fields (gfx950: 256 CUs x 4 SIMDs, 8 XCDs; GRBM_GUI_ACTIVE is summed
over the XCDs; a wave64 VALU instruction occupies its SIMD 2 cycles):
  _dur_s            summed dispatch time of the kernel
  _clock_GHz        GRBM_GUI_ACTIVE / 8 / _dur_s
  _valu_issue_frac  2 * SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
  _lane_util_valu   SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)
  _wait_any_frac    SQ_WAIT_ANY / SQ_WAVE_CYCLES
  _wait_inst_frac   SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  _l2_hit           TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
"""
import argparse
import collections
import csv
import glob
import json
import os
import re

KERNELS = (("wf_kernel<6, true>", r"wf_kernel<\d, true"), ("wf_park_kernel", r"wf_park_kernel"),
           ("wf_shade_kernel", r"wf_shade_kernel"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    tot = {k: collections.defaultdict(float) for k, _ in KERNELS}
    dur = {k: {} for k, _ in KERNELS}
    for f in sorted(glob.glob(os.path.join(a.dir, "sq", "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            for k, rx in KERNELS:
                if re.search(rx, r["Kernel_Name"]):
                    tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                    key = (f, r["Dispatch_Id"])
                    dur[k][key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
    res = {}
    for k, _ in KERNELS:
        c = dict(sorted(tot[k].items()))
        if not c:
            continue
        passes = len({f for f, _ in dur[k]})
        d = sum(dur[k].values()) / max(passes, 1)
        gui = c.get("GRBM_GUI_ACTIVE", 0.0) / 8
        c["_dur_s"] = round(d, 4)
        if gui:
            c["_clock_GHz"] = round(gui / d / 1e9, 4)
            c["_valu_issue_frac"] = round(2 * c.get("SQ_INSTS_VALU", 0.0) / (gui * 1024), 4)
        if c.get("SQ_ACTIVE_INST_VALU"):
            c["_lane_util_valu"] = round(c.get("SQ_THREAD_CYCLES_VALU", 0.0) / (64 * c["SQ_ACTIVE_INST_VALU"]), 4)
        if c.get("SQ_WAVE_CYCLES"):
            c["_wait_any_frac"] = round(c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 4)
            c["_wait_inst_frac"] = round(c.get("SQ_WAIT_INST_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 4)
        h, m = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        if h + m:
            c["_l2_hit"] = round(h / (h + m), 4)
        res[k] = c
    tag = os.path.basename(os.path.normpath(a.dir))
    out = {"workload": "tools/kbench.py --config cfg3 --spp 64 --reps 1 (all dispatches incl. warm-up), "
                       f"3 rocprofv3 --pmc passes (tools/gpu_r2round.sh {tag})", "kernels": res}
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
