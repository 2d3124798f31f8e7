"""cProfile of bench.py's plan_batch workload on the GPU (1,024 Level-0 searches sharing
oc_rollout launches): where the host time per launch goes.  Run from the repo root on a GPU box:
python tools/prof_planbatch.py [B]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
bench.measure_plan_batch("cuda:0", B=64)  # warm: extension loads, first launches
pr = cProfile.Profile()
pr.enable()
out = bench.measure_plan_batch("cuda:0", B=B)
pr.disable()
print({k: v for k, v in out.items() if k != "workload"})
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
