#!/usr/bin/env python3
"""Generate the fixtures for a kitchen whose BFS distances pass 255 while staying below the
level's perimeter, from the reference itself (load_level and
make_reachability_graph have no size limits, overcooked_environment.py:144-198, utils/world.py:
67-108):
  * corridor-204x5_salad  (1,020 cells: two 202-square lanes joined at the right end, a U;
                           the food at the top lane's left end, the cutboards and the Delivery
                           at the bottom lane's left end, about 406 edges apart; perimeter 418).
get_lower_bound_between_helper starts from perimeter + 1 (utils/world.py:148-264), so on the
31x31 maze (perimeter 124) every distance past 124 saturates the bound; here a Chop by an agent
of the top lane has an exact bound of about 407, which a byte distance table could not give.
Same records as gen_widegraph.py (corridorgraph.json / .npz, bounds_corridorgraph.npz,
rollout_corridorgraph.npz).  Runs ONLY in the build container (the reference is imported with
gen_golden.py's stubs).
Usage:  PYTHONHASHSEED=0 python tests/golden/gen_corridorgraph.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_widegraph  # noqa: E402

LEVELS = ["corridor-204x5_salad"]
BOUND_CONFIGS = [("corridor-204x5_salad", 4, 1, 9700)]
ROLL_CONFIGS = [("corridor-204x5_salad", 2, 1, 9800)]

if __name__ == "__main__":
    gen_widegraph.generate(LEVELS, BOUND_CONFIGS, ROLL_CONFIGS, "corridorgraph", pair_seed=1020, gid0=15700)
