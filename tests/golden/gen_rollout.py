#!/usr/bin/env python3
"""Generate tests/golden/rollout.npz: planner-rollout rows recorded from the reference's own
navigation planner.

Runs ONLY in the build container (the reference is imported from /root/reference with the
stub modules of gen_golden.py; it never travels to the GPU box).

For sampled states of goal-directed episodes on several (level, agent count) configs, and
for every subtask in ``env.all_subtasks`` x every ordered subtask-agent set of size 1 and 2,
an ``E2E_BRTDP`` is configured exactly as the agents do (``set_settings`` on a copy of the
env: Level-0 view, e2e_brtdp.py:582-652), and for EVERY navigation action (5 single / 25
joint) the row records:
  * legal   -- the action is in ``get_actions(state_repr)`` (e2e_brtdp.py:151-206)
  * assert  -- ``T`` raised the joint co-location AssertionError (e2e_brtdp.py:143)
  * next    -- canonical state of ``T(state_repr, action)`` (e2e_brtdp.py:103-149),
               agents indexed by their original number (removed agents = PAD rows)
  * goal    -- ``is_goal_state`` of the next state (e2e_brtdp.py:435-566)
  * lb      -- ``get_lower_bound_for_subtask_given_objs`` of the next state
               (overcooked_environment.py:594-664 -> world.py:115-283)
  * v_l/v_u -- the planner's value_init of the next state (e2e_brtdp.py:678-729)
The subtask is stored as (kind, agent indices, start masks, goal mask, cur_obj_count).

With --level1 the planners are configured at Level 1 (a non-empty other_agent_planners:
every agent stays in the planner's env, e2e_brtdp.py:383-392; the other planners themselves
are only consulted by get_next_action, never by T / get_actions / value_init) and the rows go
to tests/golden/rollout_level1.npz.

Usage:  python tests/golden/gen_rollout.py [--level1]
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
    ("full-divider_salad", 4, 3, 500),     # C5
    ("partial-divider_salad", 2, 3, 600),
    ("open-divider_tl", 3, 3, 700),
    ("open-divider_salad", 2, 3, 800),
    ("full-divider_tl", 2, 2, 900),
]
SAMPLE_EVERY, MAX_T = 4, 48
KIND = {"Chop": 1, "Merge": 2, "Deliver": 3}


LEVEL1 = "--level1" in sys.argv


def main():
    ref = gg.load_reference()
    from navigation_planner.planners.e2e_brtdp import E2E_BRTDP  # noqa: E402

    rows = {k: [] for k in ("cfg", "state", "kind", "agents", "start", "goal_mask", "goal_count",
                            "action", "legal", "assert_", "copy_raise", "next", "goal", "lb", "v_l", "v_u")}
    states = []  # (cfg index, canonical agents, items, t)
    for ci, (level, A, n_eps, seed0) in enumerate(CONFIGS):
        info = gg.RefEnv(ref, level, 4, 100).level_info()
        for e in range(n_eps):
            env = gg.RefEnv(ref, level, A, 100)
            pol = gg.GoalPolicy(info, A, seed=seed0 + e, eps=0.2)
            st = env.canon(0)
            for T in range(MAX_T):
                if T % SAMPLE_EVERY == 0:
                    snap = copy.copy(env.env)
                    si = len(states)
                    states.append((ci, st["agents"].copy(), st["items"].copy(), int(st["t"])))
                    record_state(rows, E2E_BRTDP, ref, snap, A, ci, si)
                st, _, _ = env.step(pol.act(st))
                if env.err or st["flags"] & 1:
                    break
    n = len(rows["cfg"])
    out = {k: np.array(v) for k, v in rows.items()}
    np.savez_compressed(
        os.path.join(HERE, "rollout_level1.npz" if LEVEL1 else "rollout.npz"),
        cfg_level=np.array([c[0] for c in CONFIGS]), cfg_A=np.array([c[1] for c in CONFIGS], np.int32),
        st_cfg=np.array([s[0] for s in states], np.int32), st_agents=np.array([s[1] for s in states], np.uint8),
        st_items=np.array([s[2] for s in states], np.uint8), st_t=np.array([s[3] for s in states], np.int32),
        **out)
    print("wrote %d rollout rows over %d states; legal %d, assert %d, goal %d" % (
        n, len(states), int(out["legal"].sum()), int(out["assert_"].sum()), int(out["goal"].sum())))


def record_state(rows, E2E_BRTDP, ref, env, A, ci, si):
    _, nav_utils, recipe = ref
    names = [a.name for a in env.sim_agents]
    for st in env.all_subtasks:
        kind = KIND.get(type(st).__name__)
        if kind is None:
            continue
        for size in (1, 2):
            for sub in itertools.combinations(range(A), size):
                sub_names = tuple(names[i] for i in sub)
                p = E2E_BRTDP(alpha=0.01, tau=2, cap=75, main_cap=100)
                with contextlib.redirect_stdout(io.StringIO()):
                    others = {n: None for n in names if n not in sub_names} if LEVEL1 else {}
                    p.set_settings(env=copy.copy(env), subtask=st, subtask_agent_names=sub_names,
                                   other_agent_planners=others)
                srepr = p.start.get_repr()
                with contextlib.redirect_stdout(io.StringIO()):
                    legal = set(p.get_actions(srepr))
                start = p.start_obj if isinstance(p.start_obj, list) else [p.start_obj]
                start_m = [gg.content_mask(o) for o in start] + [0] * (2 - len(start))
                goal_m = gg.content_mask(p.goal_obj)
                acts = list(itertools.product(range(5), repeat=size))
                for codes in acts:
                    action = gg.NAV[codes[0]] if size == 1 else tuple(gg.NAV[c] for c in codes)
                    nxt_canon = np.full((4, 3), gg.PAD, np.uint8), np.full((4, 4), gg.PAD, np.uint8)
                    asserted, copy_raise, goal, lb, v_l, v_u = 0, 0, 0, -1.0, 0.0, 0.0
                    try:
                        with contextlib.redirect_stdout(io.StringIO()):
                            nxt = p.T(srepr, action)
                    except AssertionError:
                        asserted = 1
                    except AttributeError:
                        # Level 1 only, actions outside get_actions: an agent steps onto another
                        # agent's Floor and both hold items; T's repr_init copy raises as
                        # env.step's does (overcooked_environment.py:108-113 -> world.py:417)
                        copy_raise = 1
                    else:
                        nxt_canon = canon(nxt, names)
                        nrepr = nxt.get_repr()
                        goal = int(bool(p.is_goal_state(nrepr)))
                        with contextlib.redirect_stdout(io.StringIO()):
                            lb = float(nxt.get_lower_bound_for_subtask_given_objs(
                                subtask=st, subtask_agent_names=sub_names, start_obj=p.start_obj,
                                goal_obj=p.goal_obj, subtask_action_obj=p.subtask_action_obj))
                        v_l, v_u = p.v_l[(nrepr, st)], p.v_u[(nrepr, st)]
                    ag = np.full(2, gg.PAD, np.uint8)
                    ag[:size] = sub
                    ac = np.full(2, gg.PAD, np.uint8)
                    ac[:size] = codes
                    rows["cfg"].append(ci)
                    rows["state"].append(si)
                    rows["kind"].append(kind)
                    rows["agents"].append(ag)
                    rows["start"].append(np.array(start_m, np.uint8))
                    rows["goal_mask"].append(goal_m)
                    rows["goal_count"].append(int(p.cur_obj_count))
                    rows["action"].append(ac)
                    rows["legal"].append(int(action in legal))
                    rows["assert_"].append(asserted)
                    rows["copy_raise"].append(copy_raise)
                    rows["next"].append(np.concatenate([nxt_canon[0].reshape(-1), nxt_canon[1].reshape(-1)]))
                    rows["goal"].append(goal)
                    rows["lb"].append(lb)
                    rows["v_l"].append(v_l)
                    rows["v_u"].append(v_u)


def canon(env, all_names):
    """Canonical (agents by original index, items sorted) of a Level-0 planner env."""
    from utils.core import Object
    agents = np.full((4, 3), gg.PAD, np.uint8)
    for ag in env.sim_agents:
        i = all_names.index(ag.name)
        agents[i] = (ag.location[0], ag.location[1], 0 if ag.holding is None else gg.content_mask(ag.holding))
    items = []
    for objs in env.world.objects.values():
        for o in objs:
            if isinstance(o, Object):
                items.append((gg.content_mask(o), o.location[0], o.location[1], int(bool(o.is_held))))
    items.sort()
    assert len(items) <= 4
    it = np.full((4, 4), gg.PAD, np.uint8)
    for i, r in enumerate(items):
        it[i] = r
    return agents, it


if __name__ == "__main__":
    main()
