#!/usr/bin/env python3
"""HBM traffic per launch of the dominant kernel from rocprofv3 --pmc passes.

  python tools/pmc_traffic.py gpurun_out/<tag> [--kernel REGEX] [--out profiles/x.json]

Reads <dir>/pmc_FETCH_SIZE/*counter_collection.csv and <dir>/pmc_WRITE_SIZE/...
(one counter per pass, as MI355X_MICROARCH.md's TCC budget requires), sums
each dispatch's per-XCD rows, and applies that guide's gfx950 corrections:
FETCH_SIZE (KiB) counts 64 B per 128 B request -> x2; WRITE_SIZE (KiB) as is.
Prints / writes {"bytes_per_launch", "launches", "fetch_bytes", "write_bytes", ...}.
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def per_dispatch(path, kernel):
    files = glob.glob(os.path.join(path, "*counter_collection.csv"))
    if not files:
        raise SystemExit(f"no counter_collection.csv under {path}")
    agg = collections.OrderedDict()
    for r in csv.DictReader(open(files[0])):
        if re.search(kernel, r["Kernel_Name"]):
            k = int(r["Dispatch_Id"])
            agg[k] = agg.get(k, 0.0) + float(r["Counter_Value"])
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default=r"wf_kernel|wf_park_kernel|wf_shade_kernel",
                    help="regex over the demangled kernel names: the kernels inside the timed launches")
    ap.add_argument("--launches", default=r"wf_kernel|wf_park_kernel",
                    help="regex of the kernel that opens each timed launch (the per-launch divisor; a "
                         "split park launch is wf_park_kernel + wf_shade_kernel)")
    ap.add_argument("--out")
    ap.add_argument("--workload", default="")
    a = ap.parse_args()
    f = per_dispatch(os.path.join(a.dir, "pmc_FETCH_SIZE"), a.kernel)
    w = per_dispatch(os.path.join(a.dir, "pmc_WRITE_SIZE"), a.kernel)
    assert f and len(f) == len(w), (len(f), len(w))
    n = len(per_dispatch(os.path.join(a.dir, "pmc_FETCH_SIZE"), a.launches))
    fetch = 2.0 * 1024.0 * sum(f.values())      # gfx950: FETCH_SIZE is half the bytes
    write = 1024.0 * sum(w.values())
    res = {"kernel": a.kernel, "launches": n, "dispatches": len(f), "fetch_bytes": fetch, "write_bytes": write,
           "bytes_per_launch": (fetch + write) / n, "workload": a.workload,
           "source": os.path.basename(os.path.normpath(a.dir)),
           "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count), WRITE_SIZE KiB x1024"}
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
