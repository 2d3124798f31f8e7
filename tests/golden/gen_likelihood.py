#!/usr/bin/env python3
"""Generate tests/golden/likelihood.npz: Bayesian-delegation action likelihoods recorded
from the reference.

Runs ONLY in the build container (the reference is imported with gen_golden.py's stubs).

For sampled steps of goal-directed episodes on several (level, A) configs, with
obs_tm1 = env.obs_tm1 (the pre-execution state, overcooked_environment.py:273) and
actions_tm1 = env.agent_actions (the post-collision executed actions, :770), every
delegating agent ("self", the first two agents), every subtask in env.all_subtasks plus
None, and every ordered 1- and 2-agent subtask-agent set, the row records
    BayesianDelegator.prob_nav_actions(obs_tm1, actions_tm1, subtask, agents, beta=1.3,
                                       no_level_1=True)      (bayesian_delegator.py:461-689)
with none_action_prob = 0.5 (utils/agent.py:45), computed on a FRESH E2E_BRTDP per call, so
that every planner value is value_init's (e2e_brtdp.py:678-729).  Rows where the reference
raises (the executed action is not in get_actions -> AssertionError; a joint T co-location
AssertionError; None with no movable action -> ZeroDivisionError) are flagged.

Usage:  python tests/golden/gen_likelihood.py
"""
from __future__ import annotations

import contextlib
import copy
import io
import itertools
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as gg  # noqa: E402

CONFIGS = [  # (level, A, episodes, seed base)
    ("full-divider_salad", 4, 2, 1500),
    ("partial-divider_salad", 2, 3, 1600),
    ("open-divider_tl", 3, 2, 1700),
    ("open-divider_salad", 2, 2, 1800),
]
SAMPLE_EVERY, MAX_T = 3, 40
KIND = {"Chop": 1, "Merge": 2, "Deliver": 3}
BETA, NONE_P = 1.3, 0.5
NAV_UTILS = None


def main():
    global NAV_UTILS
    ref = gg.load_reference()
    NAV_UTILS = ref[1]
    from navigation_planner.planners.e2e_brtdp import E2E_BRTDP  # noqa: E402
    from delegation_planner.bayesian_delegator import BayesianDelegator  # noqa: E402

    rows = {k: [] for k in ("state", "self_agent", "kind", "agents", "start", "goal_mask", "goal_count",
                            "taken", "value", "raised")}
    states = []
    for ci, (level, A, n_eps, seed0) in enumerate(CONFIGS):
        info = gg.RefEnv(ref, level, 4, 100).level_info()
        for e in range(n_eps):
            env = gg.RefEnv(ref, level, A, 100)
            pol = gg.GoalPolicy(info, A, seed=seed0 + e, eps=0.2)
            st = env.canon(0)
            for T in range(MAX_T):
                prev = st
                st, _, _ = env.step(pol.act(st))
                if env.err:
                    break
                if T % SAMPLE_EVERY == 0:
                    obs_tm1 = env.env.obs_tm1
                    acts = dict(env.env.agent_actions)
                    names = [a.name for a in obs_tm1.sim_agents]
                    taken = np.full(4, 4, np.uint8)
                    for i, n in enumerate(names):
                        taken[i] = gg.CODE[tuple(acts[n])]
                    si = len(states)
                    states.append((ci, prev["agents"].copy(), prev["items"].copy(), int(prev["t"]), taken))
                    record(rows, E2E_BRTDP, BayesianDelegator, obs_tm1, acts, names, A, si)
                if st["flags"] & 1:
                    break
    out = {k: np.array(v) for k, v in rows.items()}
    np.savez_compressed(
        os.path.join(HERE, "likelihood.npz"),
        cfg_level=np.array([c[0] for c in CONFIGS]), cfg_A=np.array([c[1] for c in CONFIGS], np.int32),
        st_cfg=np.array([s[0] for s in states], np.int32), st_agents=np.array([s[1] for s in states], np.uint8),
        st_items=np.array([s[2] for s in states], np.uint8), st_t=np.array([s[3] for s in states], np.int32),
        st_taken=np.array([s[4] for s in states], np.uint8), beta=BETA, none_action_prob=NONE_P, **out)
    ok = out["raised"] == 0
    print("wrote %d likelihood rows over %d states; %d computed, %d raised; value range %.3g..%.3g" % (
        len(out["value"]), len(states), int(ok.sum()), int((~ok).sum()), out["value"][ok].min(),
        out["value"][ok].max()))


def record(rows, E2E_BRTDP, BayesianDelegator, obs_tm1, acts, names, A, si):
    subtasks = list(obs_tm1.all_subtasks) + [None]
    for self_i in range(min(A, 2)):
        for st in subtasks:
            kind = 0 if st is None else KIND.get(type(st).__name__)
            if kind is None:
                continue
            for size in ((1,) if st is None else (1, 2)):
                for sub in itertools.combinations(range(A), size):
                    sub_names = tuple(names[i] for i in sub)
                    p = E2E_BRTDP(alpha=0.01, tau=2, cap=75, main_cap=100)
                    d = BayesianDelegator(agent_name=names[self_i], all_agent_names=names, model_type="bd",
                                          planner=p, none_action_prob=NONE_P)
                    raised, value = 0, 0.0
                    try:
                        with contextlib.redirect_stdout(io.StringIO()):
                            value = float(d.prob_nav_actions(obs_tm1=copy.copy(obs_tm1), actions_tm1=acts,
                                                             subtask=st, subtask_agent_names=sub_names,
                                                             beta=BETA, no_level_1=True))
                    except AssertionError:
                        raised = 1
                    except ZeroDivisionError:
                        raised = 2
                    start_m, goal_m, count = [0, 0], 0, 0
                    if st is not None:
                        s_obj, g_obj = NAV_UTILS.get_subtask_obj(st)
                        start = s_obj if isinstance(s_obj, list) else [s_obj]
                        start_m = [gg.content_mask(o) for o in start] + [0] * (2 - len(start))
                        goal_m = gg.content_mask(g_obj)
                        count = int(getattr(p, "cur_obj_count", 0))
                        if not hasattr(p, "goal_obj"):
                            raised = 3  # raised before the planner was configured
                    ag = np.full(2, gg.PAD, np.uint8)
                    ag[:size] = sub
                    rows["state"].append(si)
                    rows["self_agent"].append(self_i)
                    rows["kind"].append(kind)
                    rows["agents"].append(ag)
                    rows["start"].append(np.array(start_m, np.uint8))
                    rows["goal_mask"].append(goal_m)
                    rows["goal_count"].append(count)
                    rows["taken"].append(np.array([gg.CODE[tuple(acts[n])] for n in sub_names] + [4] * (2 - size),
                                                  np.uint8))
                    rows["value"].append(value)
                    rows["raised"].append(raised)


if __name__ == "__main__":
    main()
