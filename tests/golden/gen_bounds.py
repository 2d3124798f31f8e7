#!/usr/bin/env python3
"""Generate tests/golden/bounds.npz: subtask lower bounds and allocation feasibility recorded
from the reference on FULL environment states (no planner Level-0 view).

Runs ONLY in the build container (the reference is imported with gen_golden.py's stubs; it
never travels to the GPU box).

For sampled states of goal-directed episodes on several (level, A) configs, for every subtask
in ``env.all_subtasks`` plus None, and every ordered 1- and 2-agent subtask-agent set, the row
records
  * lb      -- ``env.get_lower_bound_for_subtask_given_objs(subtask, agents, start_obj,
               goal_obj, subtask_action_obj)`` (overcooked_environment.py:594-664 ->
               get_AB_locs_given_objs :480-589 -> world.py:115-283), with the objects from
               nav_utils.get_subtask_obj / get_subtask_action_obj (navigation_planner/utils.py:154-246)
  * doable  -- ``BayesianDelegator.subtask_alloc_is_doable(env, subtask, agents)``
               (delegation_planner/bayesian_delegator.py:98-156: None -> True, else the
               get_lower_bound_between distance < world.perimeter)
The subtask is stored as (kind, agent indices, start masks, goal mask).

It also writes tests/golden/reach.json: every builtin level's ``world.reachability_graph``
(World.make_reachability_graph, utils/world.py:67-108) as sorted node and edge lists.

Usage:  python tests/golden/gen_bounds.py
"""
from __future__ import annotations

import contextlib
import io
import itertools
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as gg  # noqa: E402

CONFIGS = [  # (level, A, episodes, seed base)
    ("full-divider_salad", 4, 3, 2500),
    ("partial-divider_salad", 2, 3, 2600),
    ("open-divider_tl", 3, 3, 2700),
    ("full-divider_tl", 3, 2, 2800),
    ("partial-divider_tomato", 2, 2, 2900),
]
SAMPLE_EVERY, MAX_T = 3, 60
LEVELS = ["%s-divider_%s" % (d, r) for d in ("open", "partial", "full") for r in ("salad", "tl", "tomato")]
KIND = {"Chop": 1, "Merge": 2, "Deliver": 3}


def main():
    ref = gg.load_reference()
    _, nav_utils, _ = ref
    from delegation_planner.bayesian_delegator import BayesianDelegator  # noqa: E402

    rows = {k: [] for k in ("state", "kind", "agents", "start", "goal_mask", "lb", "doable")}
    states = []  # (cfg index, canonical agents, items, t)
    for ci, (level, A, n_eps, seed0) in enumerate(CONFIGS):
        info = gg.RefEnv(ref, level, 4, 100).level_info()
        for e in range(n_eps):
            env = gg.RefEnv(ref, level, A, 100)
            pol = gg.GoalPolicy(info, A, seed=seed0 + e, eps=0.2)
            st = env.canon(0)
            for T in range(MAX_T):
                if T % SAMPLE_EVERY == 0:
                    si = len(states)
                    states.append((ci, st["agents"].copy(), st["items"].copy(), int(st["t"])))
                    record_state(rows, nav_utils, BayesianDelegator, env.env, A, si)
                st, _, _ = env.step(pol.act(st))
                if env.err or st["flags"] & 1:
                    break
    out = {k: np.array(v) for k, v in rows.items()}
    np.savez_compressed(
        os.path.join(HERE, "bounds.npz"),
        cfg_level=np.array([c[0] for c in CONFIGS]), cfg_A=np.array([c[1] for c in CONFIGS], np.int32),
        st_cfg=np.array([s[0] for s in states], np.int32), st_agents=np.array([s[1] for s in states], np.uint8),
        st_items=np.array([s[2] for s in states], np.uint8), st_t=np.array([s[3] for s in states], np.int32),
        **out)
    print("wrote %d bound rows over %d states; doable %d" % (len(out["lb"]), len(states), int(out["doable"].sum())))
    reach = {}
    for level in LEVELS:
        g = gg.RefEnv(ref, level, 2, 100).env.world.reachability_graph
        key = lambda n: (tuple(int(v) for v in n[0]), tuple(int(v) for v in n[1]))  # noqa: E731
        reach[level] = {"nodes": sorted(key(n) for n in g.nodes()),
                        "edges": sorted(tuple(sorted((key(u), key(v)))) for u, v in g.edges())}
    with open(os.path.join(HERE, "reach.json"), "w") as f:
        json.dump(reach, f, separators=(",", ":"))
    print("wrote reachability graphs of %d levels" % len(reach))


def record_state(rows, nav_utils, BayesianDelegator, env, A, si):
    names = [a.name for a in env.sim_agents]
    subtasks = [None] + [s for s in env.all_subtasks if type(s).__name__ in KIND]
    for st in subtasks:
        kind = 0 if st is None else KIND[type(st).__name__]
        start_obj, goal_obj = nav_utils.get_subtask_obj(subtask=st)
        action_obj = nav_utils.get_subtask_action_obj(subtask=st)
        start = [] if start_obj is None else (start_obj if isinstance(start_obj, list) else [start_obj])
        start_m = [gg.content_mask(o) for o in start] + [0] * (2 - len(start))
        goal_m = 0 if goal_obj is None else gg.content_mask(goal_obj)
        for size in (1, 2):
            for sub in itertools.combinations(range(A), size):
                sub_names = tuple(names[i] for i in sub)
                with contextlib.redirect_stdout(io.StringIO()):
                    lb = float(env.get_lower_bound_for_subtask_given_objs(
                        subtask=st, subtask_agent_names=sub_names, start_obj=start_obj, goal_obj=goal_obj,
                        subtask_action_obj=action_obj))
                    doable = bool(BayesianDelegator.subtask_alloc_is_doable(None, env, st, sub_names))
                ag = np.full(2, gg.PAD, np.uint8)
                ag[:size] = sub
                rows["state"].append(si)
                rows["kind"].append(kind)
                rows["agents"].append(ag)
                rows["start"].append(np.array(start_m, np.uint8))
                rows["goal_mask"].append(goal_m)
                rows["lb"].append(lb)
                rows["doable"].append(int(doable))


if __name__ == "__main__":
    main()
