#!/usr/bin/env python3
"""Workload for the planner's rocprofv3 kernel / memory-copy trace (where its GPU time goes):
bench.py's plan_batch line at 256 searches (open-divider_salad, Chop(Tomato) by agent-1 from
random-play states) and its bayes line at 64 delegators (full-divider_salad, 4 agents, the
reference's recorded Level-1 updates in one bayes_update_batch call).  Run on the GPU box:
  rocprofv3 --kernel-trace --memory-copy-trace --stats -d OUT -o planner -- python3 tools/planner_probe.py
then tools/planner_copy_share.py OUT."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
pb = bench.measure_plan_batch(dev, B=256)
by = bench.measure_bayes(dev, 1, n_updates=64, n_seq=1)
print(json.dumps({"plan_batch": pb, "bayes": {k: v for k, v in by.items() if not isinstance(v, (list, dict))}}))
