#!/usr/bin/env python3
"""Itemise bench.py's timed windows: lay the host timestamps the bench writes
with --window-log beside a rocprofv3 --kernel-trace of the same run and split each window into
  launch    t0 -> the first kernel's start (the host's launch calls + the dispatch)
  kernel    oc_step_n_kernel's duration (all of them, when the window has several launches)
  gap       the step kernel's end -> the all-gather kernel's start
  gather    the RCCL all-gather kernel(s)
  seen      the last kernel's end -> t1 (the completion seen by the host's synchronize)
Usage:  python tools/window_split.py WINDOW_LOG.rank0.json KERNEL_TRACE.csv [OUT.json]
The trace's timestamps are matched to the host clock whose value brackets the step kernel
(CLOCK_MONOTONIC or CLOCK_BOOTTIME; both are logged).  Under the profiler every launch carries
the tracer's own cost, so the split is of a traced run; the bench's untraced windows are the
headline."""
import csv
import json
import sys


def main():
    log = json.load(open(sys.argv[1]))["events"]
    rows = list(csv.DictReader(open(sys.argv[2])))
    kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    kern.sort()
    wins = {}
    for tag, mono, boot in log:
        w, what = tag.split(":", 1)
        wins.setdefault(w, {})[what] = (mono, boot)
    out = {}
    for w, ev in wins.items():
        if "t0" not in ev or "t1" not in ev:
            continue
        best = None
        for ci, clock in enumerate(("CLOCK_MONOTONIC", "CLOCK_BOOTTIME")):
            t0, t1 = ev["t0"][ci], ev["t1"][ci]
            inside = [k for k in kern if k[0] >= t0 and k[1] <= t1]
            if any("oc_step_n_kernel" in k[2] for k in inside) and (best is None or len(inside) > len(best[2])):
                best = (clock, ci, inside, t0, t1)
        if best is None:
            out[w] = {"error": "no oc_step_n_kernel inside the window on either clock"}
            continue
        clock, ci, inside, t0, t1 = best
        steps = [k for k in inside if "oc_step_n_kernel" in k[2]]
        gathers = [k for k in inside if "nccl" in k[2].lower() or "rccl" in k[2].lower()]
        others = [k for k in inside if k not in steps and k not in gathers]
        first, last = inside[0], max(inside, key=lambda k: k[1])
        d = {"clock": clock, "window_us": (t1 - t0) / 1e3,
             "launch_us": (first[0] - t0) / 1e3,
             "kernel_us": sum(k[1] - k[0] for k in steps) / 1e3,
             "step_launches": len(steps),
             "gap_us": ((gathers[0][0] - steps[-1][1]) / 1e3) if gathers else None,
             "gather_us": (sum(k[1] - k[0] for k in gathers) / 1e3) if gathers else None,
             "gather_kernels": [k[2][:60] for k in gathers],
             "seen_us": (t1 - last[1]) / 1e3,
             "other_kernels": [k[2][:60] for k in others]}
        rets = sorted((v[ci] - t0) / 1e3 for what, v in ev.items() if what.endswith("_returned"))
        d["host_launch_calls_returned_us"] = rets
        out[w] = d
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
