#!/usr/bin/env python3
"""Generate the fixtures for kitchens with a Floor square on the grid's border (SURVEY 8(f) #3:
arbitrary user levels) from the reference itself.

The reference loads such a map (load_level, overcooked_environment.py:144-198) and resets it
(make_reachability_graph clamps with World.inbounds, world.py:67-108).  A step then behaves in
one of two ways when an agent on a border Floor acts towards the outside:
  * with two or more agents, check_collisions -> is_collision looks the unclamped next square
    up (:692-700) and get_gridsquare_at's `assert len(gss) == 1` fails (world.py:429): step
    raises AssertionError after t += 1 and before anything moves;
  * with one agent there is no pair to check, and interact clamps the square with inbounds
    (interact.py:22): the agent stays where it is.
Levels (tests/golden/levels/): edge-7x6_salad (Floor gaps on the top and left borders, Salad)
and edge-8x7_tl (gaps on the right and bottom borders, SimpleTomato + SimpleLettuce).

Runs ONLY in the build container (the reference is imported with gen_golden.py's stubs).
Recorded, in gen_golden's formats (presence masks, MAXK = 4):
  * edgelevels.json   per level: the tables load_level / reset built, env.all_subtasks;
  * edgelevels.npz    episodes with 1-3 agents (uniform counter-RNG and goal-directed actions);
                      a step that raises is recorded with flags DONE | ERR (0x05) and the
                      reference's state after the raise (t advanced, nothing moved);
  * bounds_edge.npz / rollout_edge.npz   gen_bounds / gen_rollout rows along goal episodes.
Usage:  PYTHONHASHSEED=0 python tests/golden/gen_edgelevels.py
"""
from __future__ import annotations

import contextlib
import copy
import io
import json
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_bounds as gb  # noqa: E402
import gen_duplevels as gd  # noqa: E402
import gen_golden as gg  # noqa: E402
import gen_rollout as gr  # noqa: E402

LEVELS = ["edge-7x6_salad", "edge-8x7_tl"]
BOUND_CONFIGS = [("edge-7x6_salad", 3, 3, 7700), ("edge-8x7_tl", 2, 3, 7800)]
ROLL_CONFIGS = [("edge-7x6_salad", 2, 2, 7900), ("edge-8x7_tl", 3, 2, 8000)]


class EdgeRefEnv(gg.RefEnv):
    """gen_golden.RefEnv whose step also records the off-grid raise of check_collisions."""

    def step(self, codes):
        env = self.env
        t_before = env.t
        locs = [ag.location for ag in env.sim_agents]
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                _, reward, done, _ = env.step({ag.name: gg.NAV[c] for ag, c in zip(env.sim_agents, codes)})
        except AssertionError as ex:
            assert "gridsquares at" in str(ex), ex  # get_gridsquare_at, world.py:429
            assert env.t == t_before + 1 and [ag.location for ag in env.sim_agents] == locs
            self.err = True
            return self.canon(0x05), np.full(gg.MAXA, gg.PAD, np.uint8), 0
        except Exception:
            self.err = True
            held = [ag.location for ag in env.sim_agents if ag.holding is not None]
            assert len(held) != len(set(held)), "unexpected reference exception"
            return self.canon(0x05), np.full(gg.MAXA, gg.PAD, np.uint8), 0
        flags = (1 if done else 0) | (2 if reward == 1 else 0)
        ex = np.full(gg.MAXA, gg.PAD, np.uint8)
        for i, ag in enumerate(env.sim_agents):
            ex[i] = gg.CODE[tuple(env.agent_actions[ag.name])]
        names = [ag.name for ag in env.sim_agents]
        pairs = [(i, j) for i in range(self.A) for j in range(i + 1, self.A)]
        coll = 0
        for c in env.collisions:
            if c.time == env.t:
                i, j = names.index(c.agent_names[0]), names.index(c.agent_names[1])
                coll |= 1 << pairs.index((i, j))
        return self.canon(flags), ex, coll


def goal_states(ref, info, configs, every, max_T, visit):
    states = []
    for ci, (name, A, n_eps, seed0) in enumerate(configs):
        for e in range(n_eps):
            env = EdgeRefEnv(ref, name, A, 100)
            pol = gg.GoalPolicy(info[name], A, seed=seed0 + e, eps=0.0)
            st = env.canon(0)
            for T in range(max_T):
                if T % every == 0:
                    states.append((ci, st["agents"].copy(), st["items"].copy(), int(st["t"])))
                    visit(ci, env, st, A, len(states) - 1)
                st, _, _ = env.step(pol.act(st))
                if env.err or st["flags"] & 1:
                    break
    return states


def main():
    ref = gg.load_reference()
    gr.canon = gd.canon_k
    scratch = tempfile.mkdtemp(prefix="oc_edge_")
    os.makedirs(os.path.join(scratch, "utils", "levels"))
    for name in LEVELS:
        shutil.copy(os.path.join(HERE, "levels", name + ".txt"), os.path.join(scratch, "utils", "levels"))
    os.chdir(scratch)
    from delegation_planner.bayesian_delegator import BayesianDelegator  # noqa: E402
    from navigation_planner.planners.e2e_brtdp import E2E_BRTDP  # noqa: E402
    _, nav_utils, _ = ref

    info = {name: gd.level_info(gg.RefEnv(ref, name, 4, 100), nav_utils) for name in LEVELS}
    with open(os.path.join(HERE, "edgelevels.json"), "w") as f:
        json.dump(info, f, indent=1, sort_keys=True, default=int)

    gg.LEVEL_NAMES = list(LEVELS)
    gg.RefEnv = EdgeRefEnv  # Recorder.run builds its envs through gg.RefEnv
    rec = gg.Recorder()
    gid = 9700
    for name in LEVELS:
        for A in (1, 2, 3):
            for e in range(3):
                seed, g = 4400 + e, gid
                rec.run(ref, name, A, 60, "uniform", seed,
                        lambda T, st, s=seed, g=g, A=A: [gg.rng_action(s, g, T, a) for a in range(A)])
                gid += 1
            for e in range(5):
                pol = gg.GoalPolicy(info[name], A, seed=17 * gid + e, eps=0.25)
                rec.run(ref, name, A, 100, "goal", gid, lambda T, st, p=pol: p.act(st))
                gid += 1
    gg.LEVEL_NAMES = ["levels/%s.txt" % n for n in LEVELS]
    rec.save(os.path.join(HERE, "edgelevels.npz"), ["uniform", "goal"])
    fl = np.array(rec.S["flags"])
    print("wrote %d episodes / %d steps; done-success %d, err %d" % (
        len(rec.eps), len(rec.act), int(((fl & 3) == 3).sum()), int(((fl & 4) != 0).sum())))

    rows = {k: [] for k in ("state", "kind", "agents", "start", "goal_mask", "lb", "doable")}

    def visit_bounds(ci, env, st, A, si):
        with contextlib.redirect_stdout(io.StringIO()):
            gb.record_state(rows, nav_utils, BayesianDelegator, env.env, A, si)
    states = goal_states(ref, info, BOUND_CONFIGS, 4, 60, visit_bounds)
    out = gd.save_states(os.path.join(HERE, "bounds_edge.npz"), BOUND_CONFIGS, states, rows)
    print("wrote %d bound rows over %d states" % (len(out["lb"]), len(states)))

    rrows = {k: [] for k in ("cfg", "state", "kind", "agents", "start", "goal_mask", "goal_count",
                             "action", "legal", "assert_", "copy_raise", "next", "goal", "lb", "v_l", "v_u")}

    def visit_roll(ci, env, st, A, si):
        gr.record_state(rrows, E2E_BRTDP, ref, copy.copy(env.env), A, ci, si)
    states = goal_states(ref, info, ROLL_CONFIGS, 6, 48, visit_roll)
    width = 12 + 4 * gg.MAXK
    rrows["next"] = [np.concatenate([n, np.full(width - len(n), gg.PAD, np.uint8)]) for n in rrows["next"]]
    out = gd.save_states(os.path.join(HERE, "rollout_edge.npz"), ROLL_CONFIGS, states, rrows)
    print("wrote %d rollout rows over %d states; legal %d, goal %d" % (
        len(out["lb"]), len(states), int(out["legal"].sum()), int(out["goal"].sum())))
    shutil.rmtree(scratch)


if __name__ == "__main__":
    main()
