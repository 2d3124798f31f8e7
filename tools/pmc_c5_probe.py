#!/usr/bin/env python3
"""Workload for the C5 kernels' rocprofv3 --pmc passes (tools/profile_c5.sh runs one counter
group per pass; tools/pmc_c5_report.py reads them).

Dispatches, on bench.py's C5 rows (full-divider_salad, 4 agents, 2^18 mid-episode states,
64 Salad (subtask, agents) configurations, random allocation and joint action per row; rows in
random order, or configuration-major with OC_C5_ORDER=grouped as bench.py times them):
  oc_rollout_kernel     x4
  oc_rollout_group_kernel x4 (the planner's launch: 4,096 rows of a second batch, configuration-major)
  oc_bounds_kernel      x4
  oc_likelihood_kernel  x3
  oc_checksum_kernel    x3   (read calibration of FETCH_SIZE on the same batch)
  oc_step_n_kernel      x3   (the headline kernel at 2 agents / 2^20 envs / 20 steps, for contrast)
"""
import itertools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import SALAD_SUBTASKS  # noqa: E402
from gym_cooking_amd import capi  # noqa: E402
from gym_cooking_amd.engine import OvercookedBatch  # noqa: E402

dev = torch.device("cuda", 0)
A, rows = 4, 1 << 18
eb = OvercookedBatch("full-divider_salad", A, rows, max_T=100, device=dev)
s, s2 = eb.new_state(), eb.new_state()
eb.reset(s)
a = eb.new_actions()
for t in range(37):
    eb.gen_actions(a, t, 11)
    eb.step(s, s2, a)
    s, s2 = s2, s
agent_sets = [(i,) for i in range(A)] + list(itertools.combinations(range(A), 2))
table = [capi.subtask(k, ags, st, g, 0) for (k, st, g) in SALAD_SUBTASKS for ags in agent_sets][:capi.MAX_SUBTASKS]
gen = torch.Generator(device=dev)
gen.manual_seed(5)
alloc = torch.randint(0, len(table), (eb.pitch,), dtype=torch.uint8, device=dev, generator=gen)
ORDER = os.environ.get("OC_C5_ORDER", "random")  # "grouped": configuration-major rows, as bench.py
if ORDER == "grouped":
    alloc = torch.sort(alloc)[0].contiguous()
eb.gen_actions(a, 99, 12)
out = eb.new_state()
flags = torch.empty(eb.pitch, dtype=torch.uint8, device=dev)
lb = torch.empty(eb.pitch, dtype=torch.float32, device=dev)
for _ in range(4):
    eb.rollout(s, out, a, table, alloc, flags, lb)
eb4 = OvercookedBatch("full-divider_salad", A, 4096, max_T=100, device=dev)
s4, s42, a4 = eb4.new_state(), eb4.new_state(), eb4.new_actions()
eb4.reset(s4)
for t in range(37):
    eb4.gen_actions(a4, t, 11)
    eb4.step(s4, s42, a4)
    s4, s42 = s42, s4
alloc4 = torch.sort(torch.randint(0, len(table), (eb4.pitch,), dtype=torch.uint8, device=dev, generator=gen))[0].contiguous()
eb4.gen_actions(a4, 99, 12)
out4 = eb4.new_state()
for _ in range(4):
    eb4.rollout(s4, out4, a4, table, alloc4)
blb = torch.empty((len(table), eb.pitch), dtype=torch.float32, device=dev)
bok = torch.empty((len(table), eb.pitch), dtype=torch.uint8, device=dev)
for _ in range(4):
    eb.subtask_bounds(s, table, blb, bok)
for _ in range(3):
    eb.nav_likelihood(s, a, table, 0, 1.3, 0.5, alloc)
for _ in range(3):
    eb.checksum(s)
torch.cuda.synchronize()

B, n = 1 << 20, 20
e2 = OvercookedBatch("partial-divider_salad", 2, B, max_T=100, device=dev)
x, y = e2.new_state(), e2.new_state()
e2.reset(x)
acts = torch.empty((n, e2.A * e2.pitch), dtype=torch.uint8, device=dev)
for i in range(n):
    e2.gen_actions(acts[i], step=i, seed=0)
S = e2.layout.state_bytes
traj = torch.empty(n * S, dtype=torch.uint8, device=dev)
exn = torch.empty(n * e2.A * e2.pitch, dtype=torch.uint8, device=dev)
colln = torch.empty(n * e2.pitch, dtype=torch.uint8, device=dev)
stats, totals = e2.new_stats(), torch.zeros(5, dtype=torch.int64, device=dev)
for _ in range(3):
    e2.step_n(x, y, acts.reshape(-1), n, traj, exn, colln, stats, totals)
torch.cuda.synchronize()
print("pmc c5 probe done (%s rows): rollout rows %d, configurations %d, state planes %d"
      % (ORDER, rows, len(table), eb.layout.num_planes))
