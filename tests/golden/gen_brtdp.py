#!/usr/bin/env python3
"""Generate tests/golden/brtdp.json: the reference navigation planner's decisions,
E2E_BRTDP.get_next_action at Level 0 (other_agent_planners = {}, the greedy agents' call,
utils/agent.py:239-264), recorded with the planner hyper-parameters main.py defaults to
(alpha 0.01, tau 2, cap 75, main_cap 100).

Runs ONLY in the build container (the reference is imported with gen_golden.py's stubs; it
never travels to the GPU box).

Two kinds of runs, on sampled states of goal-directed episodes:
  "fresh"  -- a new planner per call;
  "chain"  -- one planner kept across the calls of an episode (agents keep theirs, so its
              v_l / v_u dictionaries carry over from call to call).
Every call is preceded by np.random.seed(seed) (the planner's argmin tie-breaks draw from
numpy's global generator, e2e_brtdp.py:27-36).  A call records the state (canonical agents /
items, the names of the env's object groups, which are part of every state repr), the
subtask (kind, agents, start / goal masks), the seed, and the outcome: the returned action,
the planner's cur_obj_count, v_l / v_u of the start state and the number of states the
planner has initialised (len(v_l)).

The reference planner takes up to minutes per joint call here; the committed file was
written under a 50-minute budget, so the last config (partial-divider_tl) has no calls (the
file is saved after every finished episode).

Usage:  PYTHONHASHSEED=0 python tests/golden/gen_brtdp.py
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
import gen_golden as gg  # noqa: E402

CONFIGS = [  # (level, A, episodes, seed base, steps)
    ("open-divider_salad", 2, 2, 3100, 40),
    ("partial-divider_salad", 2, 1, 3200, 40),
    ("full-divider_salad", 3, 1, 3300, 32),
    ("partial-divider_tl", 3, 1, 3400, 32),
]
SAMPLE_EVERY = 8
PICKS = 2
KIND = {"Chop": 1, "Merge": 2, "Deliver": 3}
PARAMS = dict(alpha=0.01, tau=2, cap=75, main_cap=100)


def code_of(action):
    if isinstance(action[0], int):
        return [gg.CODE[tuple(action)]]
    return [gg.CODE[tuple(a)] for a in action]


def main():
    ref = gg.load_reference()
    _, nav_utils, _ = ref
    from navigation_planner.planners.e2e_brtdp import E2E_BRTDP  # noqa: E402
    from delegation_planner.bayesian_delegator import BayesianDelegator  # noqa: E402

    calls = []
    t0 = time.time()
    for ci, (level, A, n_eps, seed0, steps) in enumerate(CONFIGS):
        info = gg.RefEnv(ref, level, 4, 100).level_info()
        for e in range(n_eps):
            env = gg.RefEnv(ref, level, A, 100)
            pol = gg.GoalPolicy(info, A, seed=seed0 + e, eps=0.2)
            rng = np.random.default_rng(seed0 + e)
            chain = {}  # (subtask str, agents) -> persistent planner
            st = env.canon(0)
            for T in range(steps):
                if T % SAMPLE_EVERY == 0:
                    names = [a.name for a in env.env.sim_agents]
                    cand = []
                    for sub in env.env.all_subtasks:
                        if type(sub).__name__ not in KIND:
                            continue
                        for size in (1, 2):
                            for ags in itertools.combinations(range(A), size):
                                agn = tuple(names[i] for i in ags)
                                with contextlib.redirect_stdout(io.StringIO()):
                                    ok = BayesianDelegator.subtask_alloc_is_doable(None, env.env, sub, agn)
                                if ok:
                                    cand.append((sub, ags, agn))
                    if cand:
                        picks = [cand[int(i)] for i in rng.choice(len(cand), size=min(PICKS, len(cand)), replace=False)]
                        for k, (sub, ags, agn) in enumerate(picks):
                            for mode in ("fresh", "chain"):
                                key = (str(sub), agn)
                                if mode == "fresh":
                                    p = E2E_BRTDP(**PARAMS)
                                else:
                                    p = chain.setdefault(key, E2E_BRTDP(**PARAMS))
                                seed = int(rng.integers(0, 2**31 - 1))
                                rec = record_call(p, env, sub, ags, agn, nav_utils, seed, ci, e, T, mode)
                                calls.append(rec)
                                print("  call %d: cfg %d ep %d t %d %s %s %s -> %s (%.1f s, %d states)" % (
                                    len(calls), ci, e, T, mode, sub, agn, rec["action"], rec["ref_seconds"],
                                    rec["n_states"]), flush=True)
                st, _, _ = env.step(pol.act(st))
                if env.err or st["flags"] & 1:
                    break
            print("config %d episode %d: %d calls so far, %.0f s" % (ci, e, len(calls), time.time() - t0),
                  flush=True)
            save(calls)
    save(calls)
    print("wrote %d planner calls in %.0f s" % (len(calls), time.time() - t0))


def save(calls):
    out = {"configs": [{"level": c[0], "A": c[1]} for c in CONFIGS], "params": PARAMS, "calls": calls}
    with open(os.path.join(HERE, "brtdp.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))


def record_call(p, env, sub, ags, agn, nav_utils, seed, ci, e, T, mode):
    canon = env.canon(0)
    groups = sorted(env.env.world.objects.keys())
    start_obj, goal_obj = nav_utils.get_subtask_obj(subtask=sub)
    start = start_obj if isinstance(start_obj, list) else [start_obj]
    start_m = [gg.content_mask(o) for o in start] + [0] * (2 - len(start))
    np.random.seed(seed)
    obs = copy.copy(env.env)
    t = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        action = p.get_next_action(env=obs, subtask=sub, subtask_agent_names=agn, other_agent_planners={})
    dt = time.time() - t
    srepr = p.cur_state.get_repr()
    return {
        "cfg": ci, "episode": e, "t": T, "mode": mode,
        "agents": canon["agents"].tolist(), "items": canon["items"].tolist(), "env_t": int(canon["t"]),
        "groups": groups,
        "subtask": str(sub), "kind": KIND[type(sub).__name__], "sub_agents": list(ags), "start": start_m,
        "goal_mask": gg.content_mask(goal_obj), "seed": seed,
        "action": None if action is None else code_of(action), "goal_count": int(p.cur_obj_count),
        "v_l": p.v_l[(srepr, sub)], "v_u": p.v_u[(srepr, sub)], "n_states": len(p.v_l),
        "ref_seconds": dt,
    }


if __name__ == "__main__":
    main()
