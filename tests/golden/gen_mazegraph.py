#!/usr/bin/env python3
"""Generate the fixtures for a maze kitchen whose reachability graph has BFS distances of 255
and more, from the reference itself (load_level has no size limit,
overcooked_environment.py:144-198; the BFS of make_reachability_graph, utils/world.py:67-108,
has none either; until round 5 the engine kept node distances in bytes and refused such a
graph):
  * maze-31x31_salad  (961 cells, Salad, a serpentine of 15 corridors: the food and the
                       cutboards at its top, the plates and the Delivery at its far end,
                       about 450 edges away).
Same records as gen_widegraph.py (mazegraph.json / .npz, bounds_mazegraph.npz,
rollout_mazegraph.npz).  Runs ONLY in the build container (the reference is imported with
gen_golden.py's stubs).
Usage:  PYTHONHASHSEED=0 python tests/golden/gen_mazegraph.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_widegraph  # noqa: E402

LEVELS = ["maze-31x31_salad"]
BOUND_CONFIGS = [("maze-31x31_salad", 4, 1, 9500)]
ROLL_CONFIGS = [("maze-31x31_salad", 2, 1, 9600)]

if __name__ == "__main__":
    gen_widegraph.generate(LEVELS, BOUND_CONFIGS, ROLL_CONFIGS, "mazegraph", pair_seed=961, gid0=14700)
