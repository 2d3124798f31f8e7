#!/usr/bin/env python3
"""Generate tests/golden/brtdp_level1.json: the reference navigation planner's decisions at
Level 1 -- E2E_BRTDP.get_next_action with other_agent_planners, the call Bayesian-delegation
agents make (utils/agent.py:244-264).  The other agents' planners are built the way
BayesianDelegator.get_other_agent_planners builds them (bayesian_delegator.py:375-433): a
shallow copy of the agent's own planner (so all of them share one pair of value tables),
set up with set_settings for that agent's subtask.  Here each other agent gets a doable
single-agent subtask drawn at random.

Runs ONLY in the build container.  Same record format as gen_brtdp.py, plus "others": the
other planners as [agent index, subtask, kind, start masks, goal mask] in dict order.

Usage:  PYTHONHASHSEED=0 python tests/golden/gen_brtdp_level1.py
"""
from __future__ import annotations

import contextlib
import copy
import io
import itertools
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_brtdp as gb  # noqa: E402
import gen_golden as gg  # noqa: E402

CONFIGS = [  # (level, A, seed, steps): goal-directed episodes
    ("open-divider_salad", 2, 5100, 30),
    ("partial-divider_salad", 2, 5200, 30),
    ("open-divider_tl", 3, 5300, 24),
]
SAMPLE_EVERY = 6
PARAMS = dict(gb.PARAMS)  # main.py defaults


def main():
    ref = gg.load_reference()
    _, nav_utils, _ = ref
    from navigation_planner.planners.e2e_brtdp import E2E_BRTDP  # noqa: E402
    from delegation_planner.bayesian_delegator import BayesianDelegator  # noqa: E402

    calls = []
    t0 = time.time()
    for ci, (level, A, seed0, steps) in enumerate(CONFIGS):
        info = gg.RefEnv(ref, level, 4, 100).level_info()
        env = gg.RefEnv(ref, level, A, 100)
        pol = gg.GoalPolicy(info, A, seed=seed0, eps=0.2)
        rng = np.random.default_rng(seed0)
        st = env.canon(0)
        for T in range(steps):
            if T % SAMPLE_EVERY == 0:
                names = [a.name for a in env.env.sim_agents]
                doable = {}
                for sub in env.env.all_subtasks:
                    if type(sub).__name__ not in gb.KIND:
                        continue
                    for i in range(A):
                        with contextlib.redirect_stdout(io.StringIO()):
                            if BayesianDelegator.subtask_alloc_is_doable(None, env.env, sub, (names[i],)):
                                doable.setdefault(i, []).append(sub)
                for i in sorted(doable):
                    sub = doable[i][int(rng.integers(len(doable[i])))]
                    others = [j for j in range(A) if j != i and j in doable]
                    if not others:
                        continue
                    p = E2E_BRTDP(**PARAMS)
                    oplans, orec = {}, []
                    for j in others:
                        osub = doable[j][int(rng.integers(len(doable[j])))]
                        op = copy.copy(p)
                        with contextlib.redirect_stdout(io.StringIO()):
                            op.set_settings(env=copy.copy(env.env), subtask=osub, subtask_agent_names=(names[j],))
                        oplans[names[j]] = op
                        so, go = nav_utils.get_subtask_obj(subtask=osub)
                        so = so if isinstance(so, list) else [so]
                        orec.append([j, str(osub), gb.KIND[type(osub).__name__],
                                     [gg.content_mask(o) for o in so] + [0] * (2 - len(so)), gg.content_mask(go)])
                    seed = int(rng.integers(0, 2**31 - 1))
                    rec = record(p, env, sub, i, names, nav_utils, seed, ci, T, oplans)
                    rec["others"] = orec
                    calls.append(rec)
                    print("  call %d: cfg %d t %d %s %s others %s -> %s (%.1f s, %d states)" % (
                        len(calls), ci, T, sub, names[i], [o[1] for o in orec], rec["action"], rec["ref_seconds"],
                        rec["n_states"]), flush=True)
            st, _, _ = env.step(pol.act(st))
            if env.err or st["flags"] & 1:
                break
        save(calls)
    save(calls)
    print("wrote %d planner calls in %.0f s" % (len(calls), time.time() - t0))


def record(p, env, sub, i, names, nav_utils, seed, ci, T, oplans):
    canon = env.canon(0)
    groups = sorted(env.env.world.objects.keys())
    start_obj, goal_obj = nav_utils.get_subtask_obj(subtask=sub)
    start = start_obj if isinstance(start_obj, list) else [start_obj]
    np.random.seed(seed)
    obs = copy.copy(env.env)
    t = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        action = p.get_next_action(env=obs, subtask=sub, subtask_agent_names=(names[i],), other_agent_planners=oplans)
    dt = time.time() - t
    srepr = p.cur_state.get_repr()
    return {
        "cfg": ci, "episode": 0, "t": T, "mode": "level1",
        "agents": canon["agents"].tolist(), "items": canon["items"].tolist(), "env_t": int(canon["t"]),
        "groups": groups, "subtask": str(sub), "kind": gb.KIND[type(sub).__name__], "sub_agents": [i],
        "start": [gg.content_mask(o) for o in start] + [0] * (2 - len(start)), "goal_mask": gg.content_mask(goal_obj),
        "seed": seed, "action": None if action is None else gb.code_of(action), "goal_count": int(p.cur_obj_count),
        "v_l": p.v_l[(srepr, sub)], "v_u": p.v_u[(srepr, sub)], "n_states": len(p.v_l), "ref_seconds": dt,
    }


def save(calls):
    out = {"configs": [{"level": c[0], "A": c[1]} for c in CONFIGS], "params": PARAMS, "calls": calls}
    with open(os.path.join(HERE, "brtdp_level1.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
