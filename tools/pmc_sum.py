#!/usr/bin/env python3
"""Sum PMC counters over the last K dispatches of a kernel (name substring)
across the pass directories of a tools/gpu_pmc_kb.sh run.
  python tools/pmc_sum.py gpurun_out/pmc/TAG KERNEL_SUBSTR [K]"""
import collections
import csv
import glob
import json
import os
import sys

d, kern = sys.argv[1], sys.argv[2]
K = int(sys.argv[3]) if len(sys.argv) > 3 else 4
tot = collections.defaultdict(float)
dur = None
for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    ts = {}
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        i = int(r["Dispatch_Id"])
        agg[i][r["Counter_Name"]] += float(r["Counter_Value"])
        ts[i] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    last = sorted(agg)[-K:]
    for i in last:
        for k, v in agg[i].items():
            tot[k] += v
    if dur is None and last:
        dur = sum((ts[i][1] - ts[i][0]) / 1e9 for i in last)
out = {k: v for k, v in sorted(tot.items())}
out["_dur_s"] = dur
if "GRBM_GUI_ACTIVE" in tot and dur:
    cyc = tot["GRBM_GUI_ACTIVE"] / 8
    out["_clock_GHz"] = cyc / dur / 1e9
    simd_cyc = cyc * 1024
    if "SQ_INSTS_VALU" in tot:
        out["_valu_issue_frac"] = 2 * tot["SQ_INSTS_VALU"] / simd_cyc
    if "TD_TD_BUSY_sum" in tot:
        out["_td_busy"] = tot["TD_TD_BUSY_sum"] / (cyc * 256)
    if "TA_TA_BUSY_sum" in tot:
        out["_ta_busy"] = tot["TA_TA_BUSY_sum"] / (cyc * 256)
print(json.dumps({k: (round(v, 4) if isinstance(v, float) and v < 100 else v) for k, v in out.items()}, indent=0))
