#!/usr/bin/env python3
"""Workload for the render kernel's rocprofv3 --pmc passes (tools/profile_c5.sh with
PROBE="python3 tools/pmc_render_probe.py"): bench.py's render line -- 1,024 mid-episode states of
partial-divider_salad with 2 agents, 560x560x3 images -- oc_render_kernel x4, plus
oc_checksum_kernel x3 on a 4-agent full-divider_salad batch of 2^18 envs (tools/pmc_c5_report.py
calibrates FETCH_SIZE on that kernel's known bytes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))

import torch  # noqa: E402

from gym_cooking_amd.engine import OvercookedBatch  # noqa: E402
from gym_cooking_amd.render import Renderer  # noqa: E402

dev = torch.device("cuda", 0)
eb = OvercookedBatch("partial-divider_salad", 2, 1024, max_T=100, device=dev)
s, s2, a = eb.new_state(), eb.new_state(), eb.new_actions()
eb.reset(s)
for t in range(37):
    eb.gen_actions(a, t, 11)
    eb.step(s, s2, a)
    s, s2 = s2, s
rd = Renderer(eb)
out = rd.new_images()
for _ in range(4):
    rd.render(s, out)
e4 = OvercookedBatch("full-divider_salad", 4, 1 << 18, max_T=100, device=dev)
x = e4.new_state()
e4.reset(x)
for _ in range(3):
    e4.checksum(x)
torch.cuda.synchronize()
print("pmc render probe done")
