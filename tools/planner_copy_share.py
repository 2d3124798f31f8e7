#!/usr/bin/env python3
"""Share of the planner's GPU time spent in copies, from a rocprofv3 --kernel-trace
--memory-copy-trace --stats run of tools/planner_probe.py (the r01
planner spent 35 % of its GPU time in __amd_rocclr_copyBuffer kernels and 17 % in torch
direct_copy kernels).  Usage: planner_copy_share.py OUT_DIR  (prints JSON)."""
import csv
import glob
import json
import os
import re
import sys

COPY_KERNELS = ("copyBuffer", "direct_copy", "copy_kernel", "CopyKernel", "fillBuffer")


def short(name):
    m = re.search(r"(oc_\w+_kernel<[^>]*>|__amd_rocclr_\w+|at::native::\w+)", name)
    return m.group(1) if m else name[:80]


def stats(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])))
    return rows


def main(out):
    ks = glob.glob(os.path.join(out, "**", "*kernel_stats.csv"), recursive=True)
    ms = glob.glob(os.path.join(out, "**", "*memory_copy_stats.csv"), recursive=True)
    kern = stats(ks[0]) if ks else []
    mcp = stats(ms[0]) if ms else []
    k_total = sum(t for _, _, t in kern)
    k_copy = sum(t for n, _, t in kern if any(c in n for c in COPY_KERNELS))
    m_total = sum(t for _, _, t in mcp)
    gpu = k_total + m_total
    res = {
        "kernel_ns": k_total,
        "copy_kernel_ns": k_copy,
        "copy_kernel_calls": sum(c for n, c, _ in kern if any(x in n for x in COPY_KERNELS)),
        "memory_copy_ns": m_total,
        "memory_copy_calls": sum(c for _, c, _ in mcp),
        "copy_share_of_gpu_time": (k_copy + m_total) / gpu if gpu else None,
        "kernels": [{"name": short(n), "calls": c, "total_ns": t} for n, c, t in
                    sorted(kern, key=lambda x: -x[2])[:12]],
        "memory_copies": [{"name": n, "calls": c, "total_ns": t} for n, c, t in mcp],
    }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
