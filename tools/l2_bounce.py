#!/usr/bin/env python3
"""Per-dispatch L2 hit rate and duration of one rocprofv3 --pmc TCC_HIT_sum
TCC_MISS_sum --kernel-trace run (tools/gpu_l2_bounce.sh), in dispatch order,
so the park launches read bounce by bounce.
  python tools/l2_bounce.py gpurun_out/<tag>/l2_cfg5/pmc_l2"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from roofline_profile import kname  # noqa: E402


def main():
    d = sys.argv[1]
    hit = collections.defaultdict(float)
    miss = collections.defaultdict(float)
    name = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            i = int(r["Dispatch_Id"])
            name[i] = r["Kernel_Name"]
            (hit if r["Counter_Name"].startswith("TCC_HIT") else miss)[i] += float(r["Counter_Value"])
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    seen = collections.Counter()
    print("dispatch kernel launch# ms l2_hit hit+miss(M)")
    for i in sorted(name):
        k = kname(name[i])
        if not k:
            continue
        seen[k] += 1
        tot = hit[i] + miss[i]
        print(f"{i} {k.replace(' ', '_')} {seen[k]} {dur.get(i, float('nan')):.3f} "
              f"{hit[i] / tot if tot else float('nan'):.3f} {tot / 1e6:.1f}")


if __name__ == "__main__":
    main()
