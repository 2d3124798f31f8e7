#!/usr/bin/env python3
"""Workload for rocprofv3 --pmc passes (run under the profiler, one counter group per pass).

Dispatches, on the bench workload (partial-divider_salad, 2 agents, 2^20 envs):
  oc_reset_kernel     x3  -- writes exactly state_bytes with dword stores (WRITE_SIZE calibration)
  oc_checksum_kernel  x3  -- reads exactly 17 planes x B bytes with oc_step's dword pattern
                             (FETCH_SIZE calibration for this access width)
  oc_step_kernel      x20 -- the headline kernel (eager launches)
  oc_step_n_kernel    x3 with 20 steps, then x3 with 100 steps (bench.py's launch lengths: the
                             driver's --steps 20 and the default 100-step cap), trajectory + exec +
                             coll written, state_out = the trajectory's last state and statistics
                             folded in-launch (as bench.py's launches)
tools/pmc_report.py turns the counter CSVs into profiles/pmc_traffic.json.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))

import torch  # noqa: E402

from gym_cooking_amd.engine import OvercookedBatch  # noqa: E402

B = 1 << 20
NFUSED = (20, 100)  # bench.py's launch lengths, in dispatch order (pmc_report.py relies on it)
eb = OvercookedBatch("partial-divider_salad", 2, B, max_T=100, device="cuda:0")
a, b = eb.new_state(), eb.new_state()
NMAX = max(NFUSED)
acts = torch.empty((NMAX, eb.A * eb.pitch), dtype=torch.uint8, device="cuda:0")
for i in range(NMAX):
    eb.gen_actions(acts[i], step=i, seed=0)
exe, coll, stats = eb.new_exec(), eb.new_coll(), eb.new_stats()
for _ in range(3):
    eb.reset(a)
for _ in range(3):
    eb.checksum(a)
for i in range(20):
    eb.step(a, b, acts[i], exe, coll, stats)
    a, b = b, a
S = eb.layout.state_bytes
totals = torch.zeros(5, dtype=torch.int64, device="cuda:0")
for n in NFUSED:
    traj = torch.empty(n * S, dtype=torch.uint8, device="cuda:0")
    exn = torch.empty(n * eb.A * eb.pitch, dtype=torch.uint8, device="cuda:0")
    colln = torch.empty(n * eb.pitch, dtype=torch.uint8, device="cuda:0")
    flat = acts[:n].reshape(-1)
    for _ in range(3):
        eb.step_n(a, traj[(n - 1) * S:], flat, n, traj, exn, colln, stats, totals)
    torch.cuda.synchronize()
    del traj, exn, colln
torch.cuda.synchronize()
print("pmc probe done")
