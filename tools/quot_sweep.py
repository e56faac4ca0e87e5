#!/usr/bin/env python3
"""Exhaustive check of dda_init_fq's quotient (zrt_math.h quot_rn: q0 = a y,
r = fma(-b, q0, a), q = fma(r, y, q0) with y the short reciprocal of b)
against the IEEE f32 division on the device, for EVERY pair of significands
(a, b in [1, 2): 2^46 pairs), in chunks of b significands
(ZRT_PROBE_QUOT_SWEEP).  Power-of-two scaling carries the result to the whole
operand range quot_rn is used on.

  python tools/quot_sweep.py [--chunk 131072] [--first 0] [--count 8388608]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zig_raytracing_contest_amd import native  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--chunk", type=int, default=1 << 17)
ap.add_argument("--first", type=int, default=0)
ap.add_argument("--count", type=int, default=1 << 23)
a = ap.parse_args()
t0 = time.time()
bad = 0
first = None
s = a.first
end = min(1 << 23, a.first + a.count)
while s < end:
    n = min(a.chunk, end - s)
    out = native.probe(native.PROBE_QUOT_SWEEP, np.array([[s, n]], np.uint32), 1, (1, 4), np.uint32)[0]
    bad += int(out[0])
    if out[0] and first is None:
        first = (hex(int(out[2])), hex(int(out[3])))
    s += n
    print(json.dumps({"b_significands_done": s - a.first, "pairs": (s - a.first) << 23, "mismatches": bad,
                      "seconds": round(time.time() - t0, 1)}), flush=True)
print(json.dumps({"quot_sweep": {"b_significands": [a.first, end], "pairs": (end - a.first) << 23,
                                 "mismatches": bad, "first_mismatch_a_b_bits": first,
                                 "seconds": round(time.time() - t0, 1)}}), flush=True)
