#!/usr/bin/env python3
"""Record ``env.all_subtasks`` (run_recipes, gym_cooking/envs/overcooked_environment.py:396-473)
of every builtin level from the reference itself, under five PYTHONHASHSEEDs.

Runs ONLY in the build container (the reference is read from /root/reference, imported with
gen_golden.py's stubs).  The reference returns, per recipe, a Python *set* of STRIPS actions
flattened into a list, so its order follows string hashing.  The content depends on it too:
``generate_graph`` adds one networkx edge per (state, next state) pair
(recipe_planner/stripsworld.py:50-70), so of two actions with the same transition --
``Merge(Tomato, Lettuce)`` and ``Merge(Lettuce, Tomato)`` -- only the one iterated last
survives.  The fixture stores, per level, every sorted variant seen and the seed that gave
it.  Output: tests/golden/subtasks.json.

Usage:  python tests/golden/gen_subtasks.py
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SEEDS = ("0", "1", "3", "7", "11")

CHILD = r"""
import contextlib, io, json, sys
sys.path.insert(0, %r)
import gen_golden as gg
ref = gg.load_reference()
out = {}
for name in gg.LEVEL_NAMES:
    env = gg.RefEnv(ref, name, 2, 100).env
    out[name] = [str(s) for s in env.all_subtasks]
print("JSON" + json.dumps(out))
"""


def main():
    runs = {}
    for seed in SEEDS:
        env = dict(os.environ, PYTHONHASHSEED=seed, PYTHONDONTWRITEBYTECODE="1")
        res = subprocess.run([sys.executable, "-c", CHILD % HERE], env=env, capture_output=True, text=True,
                             check=True, cwd="/tmp")
        line = [ln for ln in res.stdout.splitlines() if ln.startswith("JSON")][-1]
        runs[seed] = json.loads(line[4:])
    variants = {}
    for seed in SEEDS:
        for k, v in runs[seed].items():
            variants.setdefault(k, {}).setdefault(json.dumps(sorted(v)), []).append(seed)
    out = {k: [dict(sorted=json.loads(v), seeds=seeds) for v, seeds in sorted(d.items())]
           for k, d in variants.items()}
    with open(os.path.join(HERE, "subtasks.json"), "w") as f:
        json.dump(dict(hash_seeds=list(SEEDS), variants=out), f, indent=1, sort_keys=True)
    for k in sorted(out):
        print(k, [(len(v["sorted"]), v["seeds"]) for v in out[k]])


if __name__ == "__main__":
    main()
