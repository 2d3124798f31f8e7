#!/usr/bin/env python3
"""Generate the fixtures for a narrow kitchen (at most 255 cells: byte cell ids) whose
reachability graph has more than 390 nodes, from the reference itself (SURVEY 8(f) #3:
load_level has no size limit, overcooked_environment.py:144-198; until round 5 the planner
kernels kept a narrow level's all-pairs node distances in LDS, which held 390 nodes):
  * dense-15x17_salad  (255 cells, Salad, 4 items, a 417-node graph: counter islands with a
                        Floor square on every side).
Same records as gen_widegraph.py (densegraph.json / .npz, bounds_densegraph.npz,
rollout_densegraph.npz).  Runs ONLY in the build container (the reference is imported with
gen_golden.py's stubs).
Usage:  PYTHONHASHSEED=0 python tests/golden/gen_densegraph.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_widegraph  # noqa: E402

LEVELS = ["dense-15x17_salad"]
BOUND_CONFIGS = [("dense-15x17_salad", 3, 1, 9300)]
ROLL_CONFIGS = [("dense-15x17_salad", 2, 1, 9400)]

if __name__ == "__main__":
    gen_widegraph.generate(LEVELS, BOUND_CONFIGS, ROLL_CONFIGS, "densegraph", pair_seed=417, gid0=13700)
