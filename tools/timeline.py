#!/usr/bin/env python3
"""Kernel timeline of one rendered frame from a rocprofv3 kernel trace, with
the frame's critical path attributed per kernel.

  python tools/timeline.py <run_kernel_trace.csv> [--frame N] [--out file.json]

A frame is the run of dispatches from one frustum_kernel launch (every timed
render of 2^23 samples or more starts with one) to the next; --frame picks
which (0 = the first such frame, e.g. bench.py's first timed frame with
--warmup 0).  Streams are the HIP queues (Queue_Id).

Critical path: walk back from the frame's last kernel to finish; each step
goes to the dispatch whose end is the latest at or before the current one's
start (what it waited for: its own stream's predecessor or, across streams,
the event it waited on).  Per kernel name the report gives the summed
duration, the time it ran with no other kernel beside it ("alone"), and its
time on the critical path; the critical path's gaps are launch gaps.
"""
import argparse
import collections
import csv
import json
import re


def short(name):
    n = re.sub(r"^void\s+", "", name).replace("(anonymous namespace)::", "")
    n = re.sub(r"^zrt::", "", n)
    n = re.sub(r"\(.*$", "", n)
    return n.replace("__amd_rocclr_", "")


def base(name):
    return re.sub(r"<.*$", "", name)


def load(path):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append({"kernel": short(r["Kernel_Name"]), "stream": int(r["Queue_Id"]),
                         "t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"])})
    rows.sort(key=lambda r: r["t0"])
    return rows


def frames(rows):
    idx = [i for i, r in enumerate(rows) if base(r["kernel"]) == "frustum_kernel"]
    out = []
    for k, i in enumerate(idx):
        j = idx[k + 1] if k + 1 < len(idx) else len(rows)
        fr = rows[i:j]
        # the frame ends with its last resolve (later dispatches: copies of the next call)
        last = max((n for n, r in enumerate(fr) if base(r["kernel"]) == "wf_resolve_kernel"), default=len(fr) - 1)
        out.append(fr[:last + 1])
    return out


def analyse(fr):
    t0 = min(r["t0"] for r in fr)
    t1 = max(r["t1"] for r in fr)
    span = (t1 - t0) / 1e6
    # sweep: time each kernel name ran alone
    ev = sorted([(r["t0"], 1, i) for i, r in enumerate(fr)] + [(r["t1"], -1, i) for i, r in enumerate(fr)])
    active, alone, busy, last_t = set(), collections.Counter(), 0.0, None
    for t, kind, i in ev:
        if last_t is not None and t > last_t:
            if len(active) == 1:
                alone[base(fr[next(iter(active))]["kernel"])] += (t - last_t) / 1e6
            if active:
                busy += (t - last_t) / 1e6
        if kind == 1:
            active.add(i)
        else:
            active.discard(i)
        last_t = t
    # critical path, backwards
    cur = max(range(len(fr)), key=lambda i: fr[i]["t1"])
    crit, gaps, path = collections.Counter(), 0.0, []
    while True:
        r = fr[cur]
        crit[base(r["kernel"])] += (r["t1"] - r["t0"]) / 1e6
        path.append(cur)
        prev = [i for i in range(len(fr)) if fr[i]["t1"] <= r["t0"] + 2000 and i != cur and i not in path]
        if not prev:
            break
        nxt = max(prev, key=lambda i: fr[i]["t1"])
        gaps += max(0, r["t0"] - fr[nxt]["t1"]) / 1e6
        cur = nxt
    summed = collections.Counter()
    count = collections.Counter()
    for r in fr:
        summed[base(r["kernel"])] += (r["t1"] - r["t0"]) / 1e6
        count[base(r["kernel"])] += 1
    names = sorted(summed, key=lambda k: -summed[k])
    return {
        "frame_ms": round(span, 3), "busy_ms": round(busy, 3),
        "per_kernel": {k: {"launches": count[k], "summed_ms": round(summed[k], 3),
                           "alone_ms": round(alone[k], 3), "critical_path_ms": round(crit[k], 3)}
                       for k in names},
        "critical_path_gaps_ms": round(gaps, 3),
        "critical_path": [{"kernel": base(fr[i]["kernel"]), "stream": fr[i]["stream"],
                           "start_ms": round((fr[i]["t0"] - t0) / 1e6, 3),
                           "end_ms": round((fr[i]["t1"] - t0) / 1e6, 3)} for i in reversed(path)],
        "timeline": [{"kernel": base(r["kernel"]), "stream": r["stream"], "start_ms": round((r["t0"] - t0) / 1e6, 3),
                      "end_ms": round((r["t1"] - t0) / 1e6, 3)} for r in fr],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--frame", type=int, default=0)
    ap.add_argument("--out")
    ap.add_argument("--command", default=None)
    ap.add_argument("--all", action="store_true", help="one summary line per frame of the trace")
    a = ap.parse_args()
    fr = frames(load(a.trace))
    if a.all:
        for k, f in enumerate(fr):
            res = analyse(f)
            print(json.dumps({"frame": k, "frame_ms": res["frame_ms"], "busy_ms": res["busy_ms"],
                              "gaps_ms": res["critical_path_gaps_ms"],
                              "critical_ms": {n: v["critical_path_ms"] for n, v in res["per_kernel"].items()},
                              "summed_ms": {n: v["summed_ms"] for n, v in res["per_kernel"].items()},
                              "alone_ms": {n: v["alone_ms"] for n, v in res["per_kernel"].items()}}))
        return
    res = analyse(fr[a.frame])
    res["frames_in_trace"] = len(fr)
    res["frame_index"] = a.frame
    if a.command:
        res["command"] = a.command
    s = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s + "\n")
    summary = {k: v for k, v in res.items() if k not in ("timeline", "critical_path")}
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
