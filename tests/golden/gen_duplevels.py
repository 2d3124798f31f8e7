#!/usr/bin/env python3
"""Generate the repeated-food-type fixtures (arbitrary user levels) from the
reference itself: kitchens whose map holds a food type more than once, which the engine
runs in the OC_ENC_COUNTS item encoding (include/oc_engine.h).

The reference's load_level makes one Object per t/l/o/p character with no uniqueness check
(overcooked_environment.py:158-165); two chopped foods of one type merge into one object
(mergeable / Object.merge, core.py:194-241), whose identity is the sorted multiset of its
contents' full names (core.py:143-171).  Levels (tests/golden/levels/):
  dup-7x7_tomato2     2 Tomatoes, 2 Plates (4 item slots), SimpleTomato
  dup-9x8_tomato2     2 Tomatoes, 3 Plates (8 slots), SimpleTomato twice (all_subtasks repeats)
  dup-12x12_salad3t   3 Tomatoes, 1 Lettuce, 4 Plates (8 slots, 144 cells: the engine's
                      full-byte cell path), Salad + SimpleTomato

Runs ONLY in the build container (the reference is imported with gen_golden.py's stubs and
never travels to the GPU box).  Item masks are recorded in the counts encoding: 2-bit Tomato /
Lettuce / Onion counts in bits 0-1 / 2-3 / 4-5, Plate 0x40, Fresh 0x80.
Recorded:
  * duplevels.json   per level: what load_level / reset built (tiles, items, spawns, goal
                     masks, perimeter) and env.all_subtasks as printed;
  * duplevels.npz    episodes in gen_golden.Recorder's format with 8 canonical item rows
                     (uniform counter-RNG actions and goal-directed ones, 2-4 agents);
  * bounds_dup.npz   gen_bounds.record_state rows (subtask lower bounds, allocation
                     feasibility) along goal episodes;
  * rollout_dup.npz  gen_rollout.record_state rows (planner T, get_actions, goal test, lower
                     bound, value_init at Level 0) along goal episodes.
Usage:  PYTHONHASHSEED=0 python tests/golden/gen_duplevels.py
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
import gen_golden as gg  # noqa: E402
import gen_rollout as gr  # noqa: E402

LEVEL_DIR = os.path.join(HERE, "levels")
LEVELS = ["dup-7x7_tomato2", "dup-9x8_tomato2", "dup-12x12_salad3t"]
UNIT = {"Tomato": 0x01, "Lettuce": 0x04, "Onion": 0x10}
PLATE, FRESH = 0x40, 0x80
BOUND_CONFIGS = [("dup-9x8_tomato2", 3, 3, 6100), ("dup-12x12_salad3t", 2, 3, 6200), ("dup-7x7_tomato2", 4, 2, 6300)]
ROLL_CONFIGS = [("dup-9x8_tomato2", 2, 2, 6400), ("dup-12x12_salad3t", 3, 2, 6500)]


def content_mask_counts(obj) -> int:
    """OC_ENC_COUNTS mask of a reference Object."""
    m, fresh = 0, False
    for c in obj.contents:
        if c.name == "Plate":
            assert not m & PLATE
            m |= PLATE
            continue
        assert (m // UNIT[c.name]) & 3 < 3
        m += UNIT[c.name]
        fresh |= c.get_state() == "Fresh"
    if fresh:
        assert len(obj.contents) == 1, "a fresh food inside a merged object"
        m |= FRESH
    return m


def _single(m):  # at most one content
    x = m & 0x7F
    return x in (0, 0x01, 0x04, 0x10, 0x40)


class CountsGoalPolicy(gg.GoalPolicy):
    """gen_golden.GoalPolicy reading counts-encoded masks: chop fresh foods, deliver merged
    objects, merge chopped things (two of one food included) and plates."""

    def pick_target(self, i, st):
        ag = st["agents"][i]
        held = int(ag[2])
        items = [tuple(r) for r in st["items"] if r[0] != gg.PAD and not r[3]]
        deliv = [c for c, t in enumerate(self.tiles) if t == 3]
        cuts = [c for c, t in enumerate(self.tiles) if t == 2]
        counters = [c for c, t in enumerate(self.tiles) if t != 0]
        cell_of = lambda r: int(r[2]) * self.W + int(r[1])  # noqa: E731
        r = self.rng.random()
        if held:
            if held & FRESH and r < 0.8:
                return self.rng.choice(cuts)
            if not _single(held) and (held in self.goals or r < 0.3) and r < 0.85:
                return self.rng.choice(deliv)
            merge_ok = [cell_of(it) for it in items if cell_of(it) not in deliv and not (held & it[0] & PLATE)
                        and not ((held | it[0]) & FRESH)]
            if merge_ok and r < 0.7:
                return self.rng.choice(merge_ok)
            return self.rng.choice(counters)
        cand = [cell_of(it) for it in items if cell_of(it) not in deliv]
        if cand and r < 0.85:
            return self.rng.choice(cand)
        return self.rng.choice(counters)


def canon_k(env, all_names):
    """gen_rollout.canon with gg.MAXK item rows."""
    from utils.core import Object
    agents = np.full((4, 3), gg.PAD, np.uint8)
    for ag in env.sim_agents:
        agents[all_names.index(ag.name)] = (ag.location[0], ag.location[1],
                                            0 if ag.holding is None else gg.content_mask(ag.holding))
    items = sorted((gg.content_mask(o), o.location[0], o.location[1], int(bool(o.is_held)))
                   for objs in env.world.objects.values() for o in objs if isinstance(o, Object))
    assert len(items) <= gg.MAXK
    it = np.full((gg.MAXK, 4), gg.PAD, np.uint8)
    for i, row in enumerate(items):
        it[i] = row
    return agents, it


def level_info(env, nav_utils):
    info = env.level_info()
    info["all_subtasks"] = [str(s) for s in env.env.all_subtasks]
    return info


def goal_states(ref, info, configs, every, max_T, visit):
    """Walk CountsGoalPolicy episodes of `configs` and call visit(ci, env, st, A) every
    `every` steps; returns the list of (cfg, agents, items, t) states visited."""
    states = []
    for ci, (name, A, n_eps, seed0) in enumerate(configs):
        for e in range(n_eps):
            env = gg.RefEnv(ref, name, A, 100)
            pol = CountsGoalPolicy(info[name], A, seed=seed0 + e, eps=0.2)
            st = env.canon(0)
            for T in range(max_T):
                if T % every == 0:
                    states.append((ci, st["agents"].copy(), st["items"].copy(), int(st["t"])))
                    visit(ci, env, st, A, len(states) - 1)
                st, _, _ = env.step(pol.act(st))
                if env.err or st["flags"] & 1:
                    break
    return states


def save_states(path, configs, states, rows):
    out = {k: np.array(v) for k, v in rows.items()}
    np.savez_compressed(
        path, cfg_level=np.array(["levels/%s.txt" % c[0] for c in configs]),
        cfg_A=np.array([c[1] for c in configs], np.int32),
        st_cfg=np.array([s[0] for s in states], np.int32), st_agents=np.array([s[1] for s in states], np.uint8),
        st_items=np.array([s[2] for s in states], np.uint8), st_t=np.array([s[3] for s in states], np.int32),
        **out)
    return out


def main():
    ref = gg.load_reference()
    gg.content_mask = content_mask_counts  # every recorder below reads masks through it
    gg.MAXK = 8
    gr.canon = canon_k
    scratch = tempfile.mkdtemp(prefix="oc_dup_")
    os.makedirs(os.path.join(scratch, "utils", "levels"))
    for name in LEVELS:
        shutil.copy(os.path.join(LEVEL_DIR, name + ".txt"), os.path.join(scratch, "utils", "levels"))
    os.chdir(scratch)
    from delegation_planner.bayesian_delegator import BayesianDelegator  # noqa: E402
    from navigation_planner.planners.e2e_brtdp import E2E_BRTDP  # noqa: E402
    _, nav_utils, _ = ref

    info = {name: level_info(gg.RefEnv(ref, name, 4, 100), nav_utils) for name in LEVELS}
    with open(os.path.join(HERE, "duplevels.json"), "w") as f:
        json.dump(info, f, indent=1, sort_keys=True, default=int)

    gg.LEVEL_NAMES = list(LEVELS)
    rec = gg.Recorder()
    gid = 9000
    for name in LEVELS:
        for A in (2, 3, 4):
            for e in range(2):
                seed, g = 4200 + e, gid
                rec.run(ref, name, A, 100, "uniform", seed,
                        lambda T, st, s=seed, g=g, A=A: [gg.rng_action(s, g, T, a) for a in range(A)])
                gid += 1
            for e in range(6):
                pol = CountsGoalPolicy(info[name], A, seed=17 * gid + e)
                rec.run(ref, name, A, 100, "goal", gid, lambda T, st, p=pol: p.act(st))
                gid += 1
    gg.LEVEL_NAMES = ["levels/%s.txt" % n for n in LEVELS]
    rec.save(os.path.join(HERE, "duplevels.npz"), ["uniform", "goal"])
    fl = np.array(rec.S["flags"])
    items = np.array(rec.S["items"])
    m = items[..., 0].astype(np.int64)
    doubled = ((m != gg.PAD) & (((m & 3) >= 2) | (((m >> 2) & 3) >= 2))).any(-1)
    print("wrote %d episodes / %d steps; done-success %d, err %d; states with two of one food in an object: %d" % (
        len(rec.eps), len(rec.act), int(((fl & 3) == 3).sum()), int((fl & 4).sum()), int(doubled.sum())))

    rows = {k: [] for k in ("state", "kind", "agents", "start", "goal_mask", "lb", "doable")}

    def visit_bounds(ci, env, st, A, si):
        with contextlib.redirect_stdout(io.StringIO()):
            gb.record_state(rows, nav_utils, BayesianDelegator, env.env, A, si)
    states = goal_states(ref, info, BOUND_CONFIGS, 4, 60, visit_bounds)
    out = save_states(os.path.join(HERE, "bounds_dup.npz"), BOUND_CONFIGS, states, rows)
    print("wrote %d bound rows over %d states" % (len(out["lb"]), len(states)))

    rrows = {k: [] for k in ("cfg", "state", "kind", "agents", "start", "goal_mask", "goal_count",
                             "action", "legal", "assert_", "copy_raise", "next", "goal", "lb", "v_l", "v_u")}

    def visit_roll(ci, env, st, A, si):
        gr.record_state(rrows, E2E_BRTDP, ref, copy.copy(env.env), A, ci, si)
    states = goal_states(ref, info, ROLL_CONFIGS, 6, 48, visit_roll)
    width = 12 + 4 * gg.MAXK  # rows where T asserted carry gen_rollout's 4-row placeholder
    rrows["next"] = [np.concatenate([n, np.full(width - len(n), gg.PAD, np.uint8)]) for n in rrows["next"]]
    out = save_states(os.path.join(HERE, "rollout_dup.npz"), ROLL_CONFIGS, states, rrows)
    print("wrote %d rollout rows over %d states; legal %d, goal %d" % (
        len(out["lb"]), len(states), int(out["legal"].sum()), int(out["goal"].sum())))
    shutil.rmtree(scratch)


if __name__ == "__main__":
    main()
