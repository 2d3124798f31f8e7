#!/usr/bin/env python3
"""Where the planner.batch and bayes lines' time goes on the GPU box: bench.py's own workloads
(measure_plan_batch, measure_bayes' batched call) with the expander's launches timed apart
from the host search (the searches' Python + _brtdp time).  One JSON line per workload.
  python tools/prof_plan_gpu.py [--B 1024]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cooking_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from gym_cooking_amd import planner as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1024)
    args = ap.parse_args()
    dev = "cuda:0"
    acc = {"launch_s": 0.0, "launches": 0, "rows": 0}
    orig = P._Expander._launch

    def timed_launch(self, chunk, subs):
        t0 = time.perf_counter()
        try:
            return orig(self, chunk, subs)
        finally:
            acc["launch_s"] += time.perf_counter() - t0
            acc["launches"] += 1
            acc["rows"] += sum(len(r[1]) for r, _ in chunk)

    P._Expander._launch = timed_launch
    bench.measure_plan_batch(dev, B=64)  # warm: library, expander, caches
    acc.update(launch_s=0.0, launches=0, rows=0)
    r = bench.measure_plan_batch(dev, B=args.B)
    print(json.dumps({"workload": "plan_batch", "B": args.B, "seconds": r["seconds"], "plans_per_s": r["plans_per_s"],
                      "launch_s": acc["launch_s"], "host_s": r["seconds"] - acc["launch_s"],
                      "launches": acc["launches"], "rows": acc["rows"],
                      "us_per_launch": acc["launch_s"] / max(1, acc["launches"]) * 1e6}), flush=True)
    from gym_cooking_amd.delegation import bayes_update_batch
    make, calls, fx = bench.bayes_jobs(dev)
    warm = [make(c) for c in calls]
    bayes_update_batch([w[0] for w in warm], [w[1] for w in warm], [w[2] for w in warm], fx["beta"])
    jobs = [make(calls[i % len(calls)]) for i in range(256)]
    acc.update(launch_s=0.0, launches=0, rows=0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bayes_update_batch([j[0] for j in jobs], [j[1] for j in jobs], [j[2] for j in jobs], fx["beta"])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"workload": "bayes", "updates": 256, "value": 256 / dt, "seconds": dt,
                      "launch_s": acc["launch_s"], "host_s": dt - acc["launch_s"], "launches": acc["launches"],
                      "rows": acc["rows"]}), flush=True)


if __name__ == "__main__":
    main()
