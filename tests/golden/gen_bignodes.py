#!/usr/bin/env python3
"""Generate the fixtures of the planner tables on a reachability graph past 255 nodes (node
ids no longer fit a byte): the 255-cell kitchen tests/golden/levels/big-15x17_salad.txt.

Runs ONLY in the build container (the reference is imported with gen_golden.py's stubs and
never travels to the GPU box); the level file is copied into a scratch ``utils/levels/`` that
becomes the working directory, as gen_biglevels.py does.

Recorded:
  * reach_big.json       -- the level's ``world.reachability_graph``
                            (World.make_reachability_graph, utils/world.py:67-108) as sorted node
                            and edge lists, the reach.json format;
  * bounds_bignodes.npz  -- gen_bounds.record_state rows (get_lower_bound_for_subtask_given_objs
                            and subtask_alloc_is_doable on full states) along goal-directed
                            episodes with 2 and 4 agents, gen_biglevels.bounds_rows' format.
Usage:  PYTHONHASHSEED=0 python tests/golden/gen_bignodes.py
"""
from __future__ import annotations

import json
import os
import shutil
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_biglevels as gbl  # noqa: E402
import gen_golden as gg  # noqa: E402

LEVEL = "big-15x17_salad"
CONFIGS = [(LEVEL, 2, 2, 5500), (LEVEL, 4, 1, 5600)]


def main():
    ref = gg.load_reference()
    scratch = tempfile.mkdtemp(prefix="oc_levels_")
    os.makedirs(os.path.join(scratch, "utils", "levels"))
    shutil.copy(os.path.join(gbl.LEVEL_DIR, LEVEL + ".txt"), os.path.join(scratch, "utils", "levels"))
    os.chdir(scratch)
    from delegation_planner.bayesian_delegator import BayesianDelegator  # noqa: E402
    _, nav_utils, _ = ref

    env = gg.RefEnv(ref, LEVEL, 4, 100)
    g = env.env.world.reachability_graph

    def key(n):
        (x, y), a = n
        return [[int(x), int(y)], [int(a[0]), int(a[1])]]

    reach = {LEVEL: {"nodes": sorted(key(n) for n in g.nodes()),
                     "edges": sorted(sorted([key(u), key(v)]) for u, v in g.edges())}}
    with open(os.path.join(HERE, "reach_big.json"), "w") as f:
        json.dump(reach, f, separators=(",", ":"))
    print("%s: %d nodes, %d edges" % (LEVEL, g.number_of_nodes(), g.number_of_edges()))

    info = {LEVEL: gbl.level_info(env.env)}
    goals = []
    for st in env.env.all_subtasks:
        if type(st).__name__ == "Deliver":
            m = gg.content_mask(nav_utils.get_subtask_obj(st)[1])
            if m not in goals:
                goals.append(int(m))
    info[LEVEL]["goals"] = sorted(goals)
    gbl.bounds_rows(ref, nav_utils, BayesianDelegator, info, CONFIGS, "bounds_bignodes.npz", 4)
    shutil.rmtree(scratch)


if __name__ == "__main__":
    main()
