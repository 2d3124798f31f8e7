#!/usr/bin/env python3
"""Generate the custom-level fixtures (tests/golden/biglevels.npz, biglevels.json,
bounds_big.npz) from the reference itself, for user levels outside the nine shipped 7x7
kitchens: larger grids (10x12 = 120 cells, 13x13 = 169 cells with two Delivery squares,
15x17 = 255 cells, the engine's maximum) and ragged maps.

Runs ONLY in the build container (the reference is imported with gen_golden.py's stubs and
never travels to the GPU box).  The level files are committed under tests/golden/levels/;
the reference's load_level opens ``utils/levels/<name>.txt`` relative to the working
directory (overcooked_environment.py:146), so they are copied into a scratch directory
that becomes the working directory after the reference is imported.

Recorded:
  * biglevels.json  -- per level: what load_level / reset built (gg.RefEnv.level_info, with
                       squares past the world width skipped), or the exception reset raised
                       (type and argument) for a map with missing squares;
  * biglevels.npz   -- episodes in gen_golden.Recorder's format (uniform counter-RNG actions
                       and gen_golden.GoalPolicy episodes, 2-4 agents), level_names holding
                       the level file paths relative to tests/golden;
  * bounds_big.npz  -- gen_bounds.record_state rows (subtask lower bounds and allocation
                       feasibility on full states) along goal episodes of the 120- and
                       169-cell kitchens; cfg_level holds the level file paths;
  * biglevels_k8.npz, bounds_k8.npz -- the same for a 9x9 OnionSalad kitchen of 6 items
                       (Tomato, Lettuce, Onion, 3 Plates: the engine's 8-slot layout), canonical
                       states with 8 item rows.
Usage:  PYTHONHASHSEED=0 python tests/golden/gen_biglevels.py
(the order of env.all_subtasks, and so of the bound rows, follows the hash seed; the tests
match rows by content)
"""
from __future__ import annotations

import contextlib
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

LEVEL_DIR = os.path.join(HERE, "levels")
# stepped levels (episodes recorded); the ragged maps are recorded as the exceptions the
# reference raises: ragged-short (a row shorter than the last) at reset, ragged-long (rows
# longer than the last) at every step, after the step's actions were executed
STEP_LEVELS = ["big-10x12_salad", "big-13x13_tl", "big-15x17_salad"]
# a kitchen of 6 items (Tomato, Lettuce, Onion, 3 Plates): 8 item slots in the engine
K8_LEVELS = ["onion-9x9_onionsalad"]
RAISE_LEVELS = ["ragged-short_salad"]
STEP_RAISE_LEVELS = ["ragged-long_salad"]
BOUND_CONFIGS = [("big-10x12_salad", 3, 2, 5100), ("big-13x13_tl", 4, 2, 5200), ("big-13x13_tl", 2, 1, 5300)]
BOUND_CONFIGS_K8 = [("onion-9x9_onionsalad", 3, 2, 5400)]


def level_info(env):
    """gg.RefEnv.level_info for maps whose rows may be longer than the last one: squares past
    the world width exist in world.objects but are skipped here (the engine ignores them)."""
    w = env.world
    cls = {"Floor": 0, "Counter": 1, "Cutboard": 2, "Delivery": 3}
    tiles = [[None] * w.width for _ in range(w.height)]
    for key, objs in w.objects.items():
        for o in objs:
            if type(o).__name__ in cls:
                x, y = o.location
                if x < w.width:
                    assert tiles[y][x] is None
                    tiles[y][x] = cls[type(o).__name__]
    from utils.core import Object
    items = []
    for key, objs in w.objects.items():
        for o in objs:
            if isinstance(o, Object) and o.location[0] < w.width:
                items.append((o.location[1] * w.width + o.location[0], gg.content_mask(o)))
    items.sort()
    return dict(width=w.width, height=w.height, tiles=[t for row in tiles for t in row], items=items,
                spawns=[list(a.location) for a in env.sim_agents], perimeter=w.perimeter)


def bounds_rows(ref, nav_utils, BayesianDelegator, info, configs, fname, maxk):
    """gen_bounds.record_state rows along goal episodes of `configs`, canonical states with
    `maxk` item rows."""
    gg.MAXK = maxk
    rows = {k: [] for k in ("state", "kind", "agents", "start", "goal_mask", "lb", "doable")}
    states = []
    for ci, (name, A, n_eps, seed0) in enumerate(configs):
        for e in range(n_eps):
            env = gg.RefEnv(ref, name, A, 100)
            pol = gg.GoalPolicy(info[name], A, seed=seed0 + e, eps=0.2)
            st = env.canon(0)
            for T in range(60):
                if T % 4 == 0:
                    si = len(states)
                    states.append((ci, st["agents"].copy(), st["items"].copy(), int(st["t"])))
                    with contextlib.redirect_stdout(io.StringIO()):
                        gb.record_state(rows, nav_utils, BayesianDelegator, env.env, A, si)
                st, _, _ = env.step(pol.act(st))
                if env.err or st["flags"] & 1:
                    break
    out = {k: np.array(v) for k, v in rows.items()}
    np.savez_compressed(
        os.path.join(HERE, fname),
        cfg_level=np.array(["levels/%s.txt" % c[0] for c in configs]),
        cfg_A=np.array([c[1] for c in configs], np.int32),
        st_cfg=np.array([s[0] for s in states], np.int32), st_agents=np.array([s[1] for s in states], np.uint8),
        st_items=np.array([s[2] for s in states], np.uint8), st_t=np.array([s[3] for s in states], np.int32),
        **out)
    gg.MAXK = 4
    print("wrote %d bound rows over %d states -> %s" % (len(out["lb"]), len(states), fname))


def main():
    ref = gg.load_reference()
    scratch = tempfile.mkdtemp(prefix="oc_levels_")
    os.makedirs(os.path.join(scratch, "utils", "levels"))
    for name in STEP_LEVELS + RAISE_LEVELS + STEP_RAISE_LEVELS + K8_LEVELS:
        shutil.copy(os.path.join(LEVEL_DIR, name + ".txt"), os.path.join(scratch, "utils", "levels"))
    os.chdir(scratch)
    from delegation_planner.bayesian_delegator import BayesianDelegator  # noqa: E402
    _, nav_utils, _ = ref

    info = {}
    for name in STEP_LEVELS + STEP_RAISE_LEVELS + K8_LEVELS:
        env = gg.RefEnv(ref, name, 4, 100)
        info[name] = level_info(env.env)
        goals = []
        for st in env.env.all_subtasks:
            if type(st).__name__ == "Deliver":
                m = gg.content_mask(nav_utils.get_subtask_obj(st)[1])
                if m not in goals:
                    goals.append(int(m))
        info[name]["goals"] = sorted(goals)
    for name in RAISE_LEVELS:
        try:
            gg.RefEnv(ref, name, 2, 100)
            info[name] = {"raises": None}
        except Exception as exc:  # the reference's own exception at reset
            info[name] = {"raises": type(exc).__name__, "arg": list(exc.args[0]) if exc.args else None}
    for name in STEP_RAISE_LEVELS:
        env = gg.RefEnv(ref, name, 2, 100)
        before = [ag.location for ag in env.env.sim_agents]
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                env.env.step({ag.name: a for ag, a in zip(env.env.sim_agents, [(1, 0), (-1, 0)])})
            info[name]["step_raises"] = None
        except Exception as exc:
            info[name]["step_raises"] = type(exc).__name__
        info[name]["step_probe"] = {"actions": [[1, 0], [-1, 0]], "before": [list(l) for l in before],
                                    "after": [list(ag.location) for ag in env.env.sim_agents], "t": env.env.t}
    with open(os.path.join(HERE, "biglevels.json"), "w") as f:
        json.dump(info, f, indent=1, sort_keys=True, default=int)

    # episodes: Recorder keys levels by their index in gg.LEVEL_NAMES
    gg.LEVEL_NAMES = list(STEP_LEVELS)
    kinds = ["uniform", "goal"]
    rec = gg.Recorder()
    gid = 7000
    for name in STEP_LEVELS:
        for A in (2, 3, 4):
            for e in range(2):
                seed, g = 4000 + e, gid
                rec.run(ref, name, A, 100, "uniform", seed,
                        lambda T, st, s=seed, g=g, A=A: [gg.rng_action(s, g, T, a) for a in range(A)])
                gid += 1
            for e in range(4):
                pol = gg.GoalPolicy(info[name], A, seed=17 * gid + e)
                rec.run(ref, name, A, 100, "goal", gid, lambda T, st, p=pol: p.act(st))
                gid += 1
    gg.LEVEL_NAMES = ["levels/%s.txt" % n for n in STEP_LEVELS]  # what Recorder.save writes
    rec.save(os.path.join(HERE, "biglevels.npz"), kinds)
    fl = np.array(rec.S["flags"])
    print("wrote %d episodes / %d steps; done-success %d, err %d" % (
        len(rec.eps), len(rec.act), int(((fl & 3) == 3).sum()), int((fl & 4).sum())))

    # the 8-slot kitchen: canonical states with 8 item rows (biglevels_k8.npz)
    gg.MAXK = 8
    gg.LEVEL_NAMES = list(K8_LEVELS)
    rec8 = gg.Recorder()
    for name in K8_LEVELS:
        for A in (2, 3, 4):
            for e in range(2):
                seed, g = 4100 + e, gid
                rec8.run(ref, name, A, 100, "uniform", seed,
                         lambda T, st, s=seed, g=g, A=A: [gg.rng_action(s, g, T, a) for a in range(A)])
                gid += 1
            for e in range(5):
                pol = gg.GoalPolicy(info[name], A, seed=17 * gid + e)
                rec8.run(ref, name, A, 100, "goal", gid, lambda T, st, p=pol: p.act(st))
                gid += 1
    gg.LEVEL_NAMES = ["levels/%s.txt" % n for n in K8_LEVELS]
    rec8.save(os.path.join(HERE, "biglevels_k8.npz"), kinds)
    fl = np.array(rec8.S["flags"])
    print("wrote %d 8-slot episodes / %d steps; done-success %d, err %d" % (
        len(rec8.eps), len(rec8.act), int(((fl & 3) == 3).sum()), int((fl & 4).sum())))
    gg.MAXK = 4

    # subtask bounds on full states of the 120- and 169-cell kitchens
    rows = {k: [] for k in ("state", "kind", "agents", "start", "goal_mask", "lb", "doable")}
    states = []
    for ci, (name, A, n_eps, seed0) in enumerate(BOUND_CONFIGS):
        for e in range(n_eps):
            env = gg.RefEnv(ref, name, A, 100)
            pol = gg.GoalPolicy(info[name], A, seed=seed0 + e, eps=0.2)
            st = env.canon(0)
            for T in range(60):
                if T % 4 == 0:
                    si = len(states)
                    states.append((ci, st["agents"].copy(), st["items"].copy(), int(st["t"])))
                    with contextlib.redirect_stdout(io.StringIO()):
                        gb.record_state(rows, nav_utils, BayesianDelegator, env.env, A, si)
                st, _, _ = env.step(pol.act(st))
                if env.err or st["flags"] & 1:
                    break
    out = {k: np.array(v) for k, v in rows.items()}
    np.savez_compressed(
        os.path.join(HERE, "bounds_big.npz"),
        cfg_level=np.array(["levels/%s.txt" % c[0] for c in BOUND_CONFIGS]),
        cfg_A=np.array([c[1] for c in BOUND_CONFIGS], np.int32),
        st_cfg=np.array([s[0] for s in states], np.int32), st_agents=np.array([s[1] for s in states], np.uint8),
        st_items=np.array([s[2] for s in states], np.uint8), st_t=np.array([s[3] for s in states], np.int32),
        **out)
    print("wrote %d bound rows over %d states" % (len(out["lb"]), len(states)))
    bounds_rows(ref, nav_utils, BayesianDelegator, info, BOUND_CONFIGS_K8, "bounds_k8.npz", 8)
    shutil.rmtree(scratch)


if __name__ == "__main__":
    main()
