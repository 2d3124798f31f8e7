#!/usr/bin/env python3
"""Generate the fixtures for kitchens of more than 255 cells (arbitrary user
levels; the engine's wide-cell layout, u16 item cells) from the reference itself.

load_level puts no limit on the grid (overcooked_environment.py:144-198); these kitchens are
past the byte cell ids of the narrow layout:
  * wide-17x17_salad  (289 cells, Salad, 4 items);
  * wide-23x13_tl     (299 cells, SimpleTomato + SimpleLettuce, 5 items: 8 item slots, two
                       Delivery squares).

Runs ONLY in the build container (the reference is imported with gen_golden.py's stubs).
Recorded, in gen_golden's formats (presence masks, canonical states with MAXK = 8 item rows,
x / y coordinates, so independent of the cell-id width):
  * widelevels.json   per level: the tables load_level / reset built, env.all_subtasks;
  * widelevels.npz    episodes with 1-4 agents (uniform counter-RNG and goal-directed);
  * bounds_wide.npz / rollout_wide.npz   gen_bounds / gen_rollout rows along goal episodes.
Usage:  PYTHONHASHSEED=0 python tests/golden/gen_widelevels.py
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

LEVELS = ["wide-17x17_salad", "wide-23x13_tl"]
BOUND_CONFIGS = [("wide-17x17_salad", 3, 2, 8700), ("wide-23x13_tl", 2, 2, 8800)]
ROLL_CONFIGS = [("wide-17x17_salad", 2, 2, 8900), ("wide-23x13_tl", 3, 2, 9000)]


class WidePolicy(gg.GoalPolicy):
    """gen_golden.GoalPolicy with targets kept for 60 steps: the paths across these kitchens
    are longer than the 20 steps a target lives on the 7x7 ones."""
    TTL = 60

    def act(self, st):
        codes = []
        for i in range(self.A):
            if self.rng.random() < self.eps:
                codes.append(self.rng.randrange(5))
                continue
            if self.target[i] is None or self.ttl[i] <= 0:
                self.target[i] = self.pick_target(i, st)
                self.ttl[i] = self.TTL
            self.ttl[i] -= 1
            ag = st["agents"][i]
            c = self.path_action((int(ag[0]), int(ag[1])), self.target[i])
            tx, ty = int(ag[0]) + gg.NAV[c][0], int(ag[1]) + gg.NAV[c][1]
            if c != 4 and tx + ty * self.W == self.target[i]:
                self.target[i] = None
            codes.append(c)
        return codes


def goal_states(ref, info, configs, every, max_T, visit):
    states = []
    for ci, (name, A, n_eps, seed0) in enumerate(configs):
        for e in range(n_eps):
            env = gg.RefEnv(ref, name, A, 400)
            pol = WidePolicy(info[name], A, seed=seed0 + e, eps=0.05)
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
    gg.MAXK = 8
    gr.canon = gd.canon_k
    scratch = tempfile.mkdtemp(prefix="oc_wide_")
    os.makedirs(os.path.join(scratch, "utils", "levels"))
    for name in LEVELS:
        shutil.copy(os.path.join(HERE, "levels", name + ".txt"), os.path.join(scratch, "utils", "levels"))
    os.chdir(scratch)
    from delegation_planner.bayesian_delegator import BayesianDelegator  # noqa: E402
    from navigation_planner.planners.e2e_brtdp import E2E_BRTDP  # noqa: E402
    _, nav_utils, _ = ref

    info = {name: gd.level_info(gg.RefEnv(ref, name, 4, 100), nav_utils) for name in LEVELS}
    for name in LEVELS:
        env = gg.RefEnv(ref, name, 4, 100)
        g = env.env.world.reachability_graph
        info[name]["graph_nodes"] = g.number_of_nodes()
    with open(os.path.join(HERE, "widelevels.json"), "w") as f:
        json.dump(info, f, indent=1, sort_keys=True, default=int)

    gg.LEVEL_NAMES = list(LEVELS)
    rec = gg.Recorder()
    gid = 11700
    for name in LEVELS:
        for A in (1, 2, 3, 4):
            for e in range(2):
                seed, g = 4700 + e, gid
                rec.run(ref, name, A, 80, "uniform", seed,
                        lambda T, st, s=seed, g=g, A=A: [gg.rng_action(s, g, T, a) for a in range(A)])
                gid += 1
            for e in range(5):
                pol = WidePolicy(info[name], A, seed=17 * gid + e, eps=0.03)
                rec.run(ref, name, A, 400, "goal", gid, lambda T, st, p=pol: p.act(st))
                gid += 1
    gg.LEVEL_NAMES = ["levels/%s.txt" % n for n in LEVELS]
    rec.save(os.path.join(HERE, "widelevels.npz"), ["uniform", "goal"])
    fl = np.array(rec.S["flags"])
    print("wrote %d episodes / %d steps; done-success %d, err %d" % (
        len(rec.eps), len(rec.act), int(((fl & 3) == 3).sum()), int(((fl & 4) != 0).sum())))

    rows = {k: [] for k in ("state", "kind", "agents", "start", "goal_mask", "lb", "doable")}

    def visit_bounds(ci, env, st, A, si):
        with contextlib.redirect_stdout(io.StringIO()):
            gb.record_state(rows, nav_utils, BayesianDelegator, env.env, A, si)
    states = goal_states(ref, info, BOUND_CONFIGS, 12, 240, visit_bounds)
    out = gd.save_states(os.path.join(HERE, "bounds_wide.npz"), BOUND_CONFIGS, states, rows)
    print("wrote %d bound rows over %d states" % (len(out["lb"]), len(states)))

    rrows = {k: [] for k in ("cfg", "state", "kind", "agents", "start", "goal_mask", "goal_count",
                             "action", "legal", "assert_", "copy_raise", "next", "goal", "lb", "v_l", "v_u")}

    def visit_roll(ci, env, st, A, si):
        gr.record_state(rrows, E2E_BRTDP, ref, copy.copy(env.env), A, ci, si)
    states = goal_states(ref, info, ROLL_CONFIGS, 16, 240, visit_roll)
    width = 12 + 4 * gg.MAXK
    rrows["next"] = [np.concatenate([n, np.full(width - len(n), gg.PAD, np.uint8)]) for n in rrows["next"]]
    out = gd.save_states(os.path.join(HERE, "rollout_wide.npz"), ROLL_CONFIGS, states, rrows)
    print("wrote %d rollout rows over %d states; legal %d, goal %d" % (
        len(out["lb"]), len(states), int(out["legal"].sum()), int(out["goal"].sum())))
    shutil.rmtree(scratch)


if __name__ == "__main__":
    main()
