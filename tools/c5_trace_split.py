#!/usr/bin/env python3
"""Per-measurement means of the C5 kernels from a rocprofv3 kernel trace of bench.py.

bench.py times each C5 kernel as runs of back-to-back launches of one pre-bound launcher
(time_launches: 3 untimed + reps timed launches).  The trace lists every dispatch; this
splits each kernel's dispatches, in order, into those runs and prints, per run, the mean
kernel duration of its timed launches, next to the bench line's own ms_per_launch.
  python tools/c5_trace_split.py TRACE_CSV BENCH_JSON > out.json"""
import csv
import json
import sys

# kernel -> [(bench field, launches in the run incl. the 3 untimed)] in bench.py's order
RUNS = {
    "oc_rollout_kernel": [("rollout.random_order", 203), ("rollout", 203)],
    "oc_likelihood_compact_kernel": [("rollout.likelihood", 43), ("rollout.likelihood.random_order", 43)],
    "oc_bounds_kernel": [("rollout.subtask_bounds", 63)],
}


def bench_ms(line, field):
    d = line
    parts = field.split(".")
    for p in parts:
        d = d[p]
    return d["ms_per_launch"] if isinstance(d, dict) else d


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    with open(bench) as f:
        line = json.loads([x for x in f if x.startswith("{")][-1])
    durs = {k: [] for k in RUNS}
    with open(trace) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            for k in RUNS:
                if k + "<" in name:
                    durs[k].append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
    out = {}
    for k, runs in RUNS.items():
        ds = [d for _, d in sorted(durs[k])]
        i = 0
        for field, n in runs:
            seg = ds[i + 3:i + n]
            i += n
            mean_us = sum(seg) / len(seg) / 1e3 if seg else None
            b_us = bench_ms(line, field) * 1e3
            out[field] = {"kernel": k, "trace_mean_us": mean_us, "timed_launches": len(seg), "bench_us": b_us,
                          "bench_over_trace": b_us / mean_us if mean_us else None}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
