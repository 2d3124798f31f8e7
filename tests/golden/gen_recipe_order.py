#!/usr/bin/env python3
"""Record the iteration order of each reference recipe's ``actions`` set (recipe_planner/
recipe.py:6-197) under five PYTHONHASHSEEDs.

``generate_graph`` (recipe_planner/stripsworld.py:50-70) adds one networkx edge per (state,
next state) pair while it walks ``recipe.actions``, so of two actions with one transition the
one iterated last is kept; recipes._HASH0_KEPT restates that choice for PYTHONHASHSEED=0 and
tests/test_recipes.py checks it against this fixture.  Runs ONLY in the build container
(the reference is imported with gen_golden.py's stubs).  Output: tests/golden/recipe_order.json.

Usage:  python tests/golden/gen_recipe_order.py
"""
from __future__ import annotations

import json
import os
import platform
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SEEDS = ("0", "1", "3", "7", "11")
RECIPES = ("SimpleTomato", "SimpleLettuce", "Salad", "OnionSalad")

CHILD = r"""
import json, sys
sys.path.insert(0, %r)
import gen_golden as gg
gg.load_reference()
import recipe_planner.recipe as R
print("JSON" + json.dumps({n: [str(a) for a in getattr(R, n)().actions] for n in %r}))
"""


def main():
    out = {}
    for seed in SEEDS:
        env = dict(os.environ, PYTHONHASHSEED=seed, PYTHONDONTWRITEBYTECODE="1")
        res = subprocess.run([sys.executable, "-c", CHILD % (HERE, RECIPES)], env=env, capture_output=True,
                             text=True, check=True, cwd="/tmp")
        line = [ln for ln in res.stdout.splitlines() if ln.startswith("JSON")][-1]
        out[seed] = json.loads(line[4:])
    with open(os.path.join(HERE, "recipe_order.json"), "w") as f:
        json.dump(dict(python=platform.python_version(), orders=out), f, indent=1, sort_keys=True)
    print("recorded", {s: {r: len(v) for r, v in d.items()} for s, d in out.items()})


if __name__ == "__main__":
    main()
