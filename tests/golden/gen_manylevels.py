#!/usr/bin/env python3
"""Generate the fixtures for kitchens of more than 8 objects (arbitrary user
levels), which the engine runs with 16 item slots (include/oc_engine.h OC_MAX_ITEMS), from the
reference itself.

The reference puts no limit on how many t/l/o/p characters a level holds (load_level,
overcooked_environment.py:158-165, one Object each).  Levels (tests/golden/levels/):
  many-11x10_salad9    Tomato, Lettuce, 7 Plates: 9 objects, presence encoding (no food
                       type repeats), 110 cells, Salad
  many-12x11_onion2    2 each of Tomato / Lettuce / Onion, 5 Plates: 11 objects, counts
                       encoding, 132 cells (full-byte cell path), OnionSalad twice
  many-13x12_full16    3 each of Tomato / Lettuce / Onion, 7 Plates: 16 objects (the slot
                       limit), counts encoding, 156 cells, OnionSalad + Salad

Runs ONLY in the build container, with gen_golden.py's stubs (the reference never travels to
the GPU box).  Item masks are recorded in each level's own encoding: the presence masks of
gen_golden.content_mask, or the counts masks of gen_duplevels.content_mask_counts.  Rows are
MAXK = 16 wide.  Recorded, in gen_duplevels.py's formats:
  * manylevels.json   per level: tables load_level / reset built, env.all_subtasks;
  * manylevels.npz    72 episodes (uniform counter-RNG and goal-directed actions, 2-4 agents);
  * bounds_many.npz   gen_bounds.record_state rows along goal episodes;
  * rollout_many.npz  gen_rollout.record_state rows along goal episodes.
Usage:  PYTHONHASHSEED=0 python tests/golden/gen_manylevels.py
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

LEVEL_DIR = os.path.join(HERE, "levels")
LEVELS = {"many-11x10_salad9": "presence", "many-12x11_onion2": "counts", "many-13x12_full16": "counts"}
BOUND_CONFIGS = [("many-11x10_salad9", 3, 3, 7100), ("many-12x11_onion2", 2, 3, 7200), ("many-13x12_full16", 4, 2, 7300)]
ROLL_CONFIGS = [("many-11x10_salad9", 2, 2, 7400), ("many-13x12_full16", 3, 2, 7500)]

_presence_mask = gg.content_mask
_enc = {"cur": "presence"}


def content_mask(obj) -> int:
    """The mask of a reference Object in the encoding of the level being recorded."""
    return (gd.content_mask_counts if _enc["cur"] == "counts" else _presence_mask)(obj)


def policy(info, name, A, seed, eps=0.15):
    cls = gd.CountsGoalPolicy if LEVELS[name] == "counts" else gg.GoalPolicy
    return cls(info[name], A, seed=seed, eps=eps)


def goal_states(ref, info, configs, every, max_T, visit):
    """gen_duplevels.goal_states with the policy and mask encoding of each config's level."""
    states = []
    for ci, (name, A, n_eps, seed0) in enumerate(configs):
        _enc["cur"] = LEVELS[name]
        for e in range(n_eps):
            env = gg.RefEnv(ref, name, A, 100)
            pol = policy(info, name, A, seed0 + e, eps=0.2)
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
    gg.content_mask = content_mask
    gg.MAXK = 16
    gr.canon = gd.canon_k
    scratch = tempfile.mkdtemp(prefix="oc_many_")
    os.makedirs(os.path.join(scratch, "utils", "levels"))
    for name in LEVELS:
        shutil.copy(os.path.join(LEVEL_DIR, name + ".txt"), os.path.join(scratch, "utils", "levels"))
    os.chdir(scratch)
    from delegation_planner.bayesian_delegator import BayesianDelegator  # noqa: E402
    from navigation_planner.planners.e2e_brtdp import E2E_BRTDP  # noqa: E402
    _, nav_utils, _ = ref

    info = {}
    for name in LEVELS:
        _enc["cur"] = LEVELS[name]
        info[name] = gd.level_info(gg.RefEnv(ref, name, 4, 100), nav_utils)
        info[name]["encoding"] = LEVELS[name]
    with open(os.path.join(HERE, "manylevels.json"), "w") as f:
        json.dump(info, f, indent=1, sort_keys=True, default=int)

    gg.LEVEL_NAMES = list(LEVELS)
    rec = gg.Recorder()
    gid = 9500
    for name in LEVELS:
        _enc["cur"] = LEVELS[name]
        for A in (2, 3, 4):
            for e in range(2):
                seed, g = 4300 + e, gid
                rec.run(ref, name, A, 100, "uniform", seed,
                        lambda T, st, s=seed, g=g, A=A: [gg.rng_action(s, g, T, a) for a in range(A)])
                gid += 1
            for e in range(6):
                pol = policy(info, name, A, 17 * gid + e)
                rec.run(ref, name, A, 100, "goal", gid, lambda T, st, p=pol: p.act(st))
                gid += 1
    gg.LEVEL_NAMES = ["levels/%s.txt" % n for n in LEVELS]
    rec.save(os.path.join(HERE, "manylevels.npz"), ["uniform", "goal"])
    fl = np.array(rec.S["flags"])
    items = np.array(rec.S["items"])
    print("wrote %d episodes / %d steps; done-success %d, err %d; max live objects %d" % (
        len(rec.eps), len(rec.act), int(((fl & 3) == 3).sum()), int((fl & 4).sum()),
        int((items[..., 0] != gg.PAD).sum(-1).max())))

    rows = {k: [] for k in ("state", "kind", "agents", "start", "goal_mask", "lb", "doable")}

    def visit_bounds(ci, env, st, A, si):
        with contextlib.redirect_stdout(io.StringIO()):
            gb.record_state(rows, nav_utils, BayesianDelegator, env.env, A, si)
    states = goal_states(ref, info, BOUND_CONFIGS, 4, 60, visit_bounds)
    out = gd.save_states(os.path.join(HERE, "bounds_many.npz"), BOUND_CONFIGS, states, rows)
    print("wrote %d bound rows over %d states" % (len(out["lb"]), len(states)))

    rrows = {k: [] for k in ("cfg", "state", "kind", "agents", "start", "goal_mask", "goal_count",
                             "action", "legal", "assert_", "copy_raise", "next", "goal", "lb", "v_l", "v_u")}

    def visit_roll(ci, env, st, A, si):
        gr.record_state(rrows, E2E_BRTDP, ref, copy.copy(env.env), A, ci, si)
    states = goal_states(ref, info, ROLL_CONFIGS, 6, 48, visit_roll)
    width = 12 + 4 * gg.MAXK
    rrows["next"] = [np.concatenate([n, np.full(width - len(n), gg.PAD, np.uint8)]) for n in rrows["next"]]
    out = gd.save_states(os.path.join(HERE, "rollout_many.npz"), ROLL_CONFIGS, states, rrows)
    print("wrote %d rollout rows over %d states; legal %d, goal %d" % (
        len(out["lb"]), len(states), int(out["legal"].sum()), int(out["goal"].sum())))
    shutil.rmtree(scratch)


if __name__ == "__main__":
    main()
