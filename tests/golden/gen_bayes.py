#!/usr/bin/env python3
"""Generate tests/golden/bayes.json: the reference's Bayesian-delegation posterior update,
BayesianDelegator.bayes_update(obs_tm1, actions_tm1, beta) (delegation_planner/
bayesian_delegator.py:1026-1072) with the "bd" model: prune the allocations that are not
doable, then multiply every allocation by sum over its (subtask, agents) of
len(agents) * prob_nav_actions(..., no_level_1=False) -- Level-1 inverse planning with the
other agents' planners taken from the delegator's own beliefs (get_other_agent_planners,
:375-433) -- and normalise.

Runs ONLY in the build container.  For sampled steps of goal-directed episodes, a delegator
for one agent is built with a fresh E2E_BRTDP (main.py's defaults) and the "bd" allocation
set of set_priors(obs_tm1, env.all_subtasks, "uniform") (get_subtask_alloc_probs and
prune_subtask_allocs, :262-294), each allocation's prior multiplied by a random factor (so that select_subtask's argmax is mostly unique); then
random.seed / np.random.seed and one bayes_update on env.obs_tm1 / env.agent_actions.
Records the state, the actions, the allocations and their probabilities before and after.

Usage:  PYTHONHASHSEED=0 python tests/golden/gen_bayes.py
"""
from __future__ import annotations

import contextlib
import copy
import io
import json
import os
import random
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_brtdp as gb  # noqa: E402
import gen_golden as gg  # noqa: E402

CONFIGS = [  # (level, A, seed, steps)
    ("open-divider_salad", 2, 6100, 30),
    ("partial-divider_tomato", 2, 6200, 30),
    ("open-divider_tl", 3, 6300, 18),
    ("partial-divider_salad", 3, 6500, 24),
    ("full-divider_salad", 4, 6400, 16),
]
SAMPLE_EVERY = 2
BETA, NONE_P = 1.3, 0.5


def sub_rec(t):
    return [None if t.subtask is None else str(t.subtask), list(t.subtask_agent_names)]


def main():
    ref = gg.load_reference()
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
            pre = env.canon(0)
            st, _, _ = env.step(pol.act(st))
            if env.err or st["flags"] & 1:
                break
            if T % SAMPLE_EVERY != SAMPLE_EVERY - 1:
                continue
            e = env.env
            names = [a.name for a in e.sim_agents]
            me = names[int(rng.integers(A))]
            d = BayesianDelegator(me, names, "bd", E2E_BRTDP(**gb.PARAMS), NONE_P)
            with contextlib.redirect_stdout(io.StringIO()):  # allocations + prune (:262-294), uniform weights
                d.set_priors(obs=copy.copy(e.obs_tm1), incomplete_subtasks=list(e.all_subtasks),
                             priors_type="uniform")
            for k in d.probs.enumerate_subtask_allocs():
                d.probs.update(k, float(rng.uniform(0.5, 1.5)))
            d.probs.normalize()
            before = [[[sub_rec(t) for t in k], p] for k, p in d.probs.get_list()]
            obs = copy.copy(e.obs_tm1)  # as the agent passes it (utils/agent.py:200-203)
            acts = {n: list(a) for n, a in e.agent_actions.items()}
            s_py, s_np = int(rng.integers(0, 2**31 - 1)), int(rng.integers(0, 2**31 - 1))
            random.seed(s_py)
            np.random.seed(s_np)
            t = time.time()
            try:
                with contextlib.redirect_stdout(io.StringIO()):
                    d.bayes_update(obs_tm1=obs, actions_tm1=e.agent_actions, beta=BETA)
                raised = None
            except Exception as ex:  # an assert inside prob_nav_actions: recorded, the test expects it
                raised = type(ex).__name__
            dt = time.time() - t
            after = None if raised else [[[sub_rec(t) for t in k], p] for k, p in d.probs.get_list()]
            obs_groups = sorted(obs.world.objects.keys())
            calls.append({
                "cfg": ci, "t": T, "self": me, "agents": pre["agents"].tolist(), "items": pre["items"].tolist(),
                "env_t": int(pre["t"]), "groups": obs_groups, "actions": acts, "random_seed": s_py,
                "np_seed": s_np, "before": before, "after": after, "raised": raised, "ref_seconds": dt,
            })
            print("  call %d: cfg %d t %d self %s, %d allocations -> %s (%.1f s)" % (
                len(calls), ci, T, me, len(before), raised or "%d allocations" % len(after), dt), flush=True)
        save(calls)
    save(calls)
    print("wrote %d updates in %.0f s" % (len(calls), time.time() - t0))


def save(calls):
    out = {"configs": [{"level": c[0], "A": c[1]} for c in CONFIGS], "params": gb.PARAMS, "beta": BETA,
           "none_action_prob": NONE_P, "calls": calls}
    with open(os.path.join(HERE, "bayes.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
