#!/usr/bin/env python3
"""Workload for the C3 step kernel's rocprofv3 --pmc passes (tools/profile_c5.sh with
PROBE="python3 tools/pmc_c3_probe.py"): bench.py's C3 line -- full-divider_tl, 3 agents, 2^20
envs, 100-step oc_step_n launches with the trajectory (state_out its last state), executed
actions and collision masks written -- x3, plus oc_checksum_kernel x3 on a 4-agent
full-divider_salad batch of 2^18 envs (tools/pmc_c5_report.py calibrates FETCH_SIZE on it)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))

import torch  # noqa: E402

from gym_cooking_amd.engine import OvercookedBatch  # noqa: E402

dev = torch.device("cuda", 0)
n = 100
eb = OvercookedBatch("full-divider_tl", 3, 1 << 20, max_T=100, device=dev)
P, A, S = eb.pitch, eb.A, eb.layout.state_bytes
acts = torch.empty((n, A * P), dtype=torch.uint8, device=dev)
for i in range(n):
    eb.gen_actions(acts[i], step=i, seed=3)
traj = torch.empty(n * S, dtype=torch.uint8, device=dev)
ex, coll = torch.empty(n * A * P, dtype=torch.uint8, device=dev), torch.empty(n * P, dtype=torch.uint8, device=dev)
s = eb.new_state()
stats = eb.new_stats()
for _ in range(3):
    eb.reset(s)
    eb.step_n(s, traj[(n - 1) * S:], acts.reshape(-1), n, traj, ex, coll, stats)
torch.cuda.synchronize()
del traj, ex, coll, acts
e4 = OvercookedBatch("full-divider_salad", 4, 1 << 18, max_T=100, device=dev)
x = e4.new_state()
e4.reset(x)
for _ in range(3):
    e4.checksum(x)
torch.cuda.synchronize()
print("pmc c3 probe done")
