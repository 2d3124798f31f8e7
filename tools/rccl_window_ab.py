"""What the RCCL summary all-gather costs inside the bench window at world size 1.

The bench's window is one oc_step_n launch (20 steps, 2^20 envs, in-launch statistics fold)
followed by the all-gather of the rank's summary row and a synchronize.  Modes, timed
interleaved (median wall time from a synchronised start to the host seeing completion):
  none      the launch alone (what round 2 timed: the all-gather was a Python early return)
  copy      all_gather_into_tensor(out, row) with row a separate buffer (RCCL copies it)
  inplace   row is this rank's slice of out (RCCL's in-place all-gather: no local copy)
  direct    in place through gym_cooking_amd.dist.RcclComm: ncclAllGather via the librccl C
            API on the launch stream (no process-group event record / wait around it)
Usage: python tools/rccl_window_ab.py [--reps 300]"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from gym_cooking_amd import dist as ocdist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--n", type=int, default=20)
    args = ap.parse_args()
    ocdist.init("nccl")
    from gym_cooking_amd.engine import OvercookedBatch
    dev = torch.device("cuda:0")
    eb = OvercookedBatch("partial-divider_salad", 2, 1 << 20, max_T=100, device=dev)
    P, A, S, n = eb.pitch, eb.A, eb.layout.state_bytes, args.n
    acts = torch.empty((n, A * P), dtype=torch.uint8, device=dev)
    for i in range(n):
        eb.gen_actions(acts[i], step=i, seed=0)
    traj = torch.empty(n * S, dtype=torch.uint8, device=dev)
    ex = torch.empty(n * A * P, dtype=torch.uint8, device=dev)
    coll = torch.empty(n * P, dtype=torch.uint8, device=dev)
    s_a, stats = eb.new_state(), eb.new_stats()
    eb.reset(s_a)
    world, rank = dist.get_world_size(), dist.get_rank()
    out_copy = torch.zeros(world * 8, dtype=torch.int64, device=dev)
    row_copy = torch.zeros(8, dtype=torch.int64, device=dev)
    out_in = torch.zeros((world, 8), dtype=torch.int64, device=dev)
    row_in = out_in[rank]
    launch = {m: eb.step_n_launcher(s_a, traj[(n - 1) * S:n * S], acts.reshape(-1), n, traj[:n * S], ex, coll,
                                    stats, r[:5]) for m, r in (("none", row_copy), ("copy", row_copy),
                                                               ("inplace", row_in), ("direct", row_in))}
    gather = {"none": lambda: None,
              "copy": lambda: dist.all_gather_into_tensor(out_copy, row_copy),
              "inplace": lambda: dist.all_gather_into_tensor(out_in.view(-1), row_in),
              "direct": lambda: ocdist.rccl().all_gather_rows(out_in)}
    xs = {m: [] for m in launch}
    for rep in range(args.reps + 20):
        for m in launch:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            launch[m]()
            gather[m]()
            torch.cuda.synchronize()
            if rep >= 20:
                xs[m].append((time.perf_counter() - t0) * 1e6)
    res = {m: {"median_us": statistics.median(v), "p10_us": sorted(v)[len(v) // 10]} for m, v in xs.items()}
    res["check"] = {"copy": out_copy.tolist()[:5], "inplace": out_in.view(-1).tolist()[:5]}
    print(json.dumps(res), flush=True)
    ocdist.shutdown()


if __name__ == "__main__":
    main()
