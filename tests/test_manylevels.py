"""Kitchens of more than 8 objects, on the CPU.

The reference's load_level makes one Object per t/l/o/p character and puts no limit on their
number (overcooked_environment.py:158-165); the engine gives such levels 16 item slots
(include/oc_engine.h OC_MAX_ITEMS; capi.item_slots picks 4, 8 or 16).  Pinned to the
reference's own runs of the same level files (tests/golden/gen_manylevels.py):
  * levels.parse_level_text builds the reference's tables, in the presence encoding for a
    9-object kitchen without repeated foods and the counts encoding for 11- and 16-object ones;
  * the CPU oracle and the host build of the device SWAR step replay all 72 recorded episodes
    (7,003 steps, up to 16 live objects, the 128+-cell full-byte path) bit for bit;
  * the host build of the planner row (oc_rollout.h) and the oracle reproduce the reference
    planner's rollout rows and subtask-bound rows;
  * random play and random subtask tables agree between the oracle and the host builds."""
import json
import os

import numpy as np
import pytest

import oc_testlib as tl
import test_bounds_host as tb
import test_rollout_host as th
import test_swar_host as ts
from gym_cooking_amd import capi, levels, recipes

from oracle import oracle

MANY = ["many-11x10_salad9", "many-12x11_onion2", "many-13x12_full16"]
ENC = {"presence": levels.ENC_PRESENCE, "counts": levels.ENC_COUNTS}


def _info():
    with open(os.path.join(tl.GOLDEN, "manylevels.json")) as f:
        return json.load(f)


def _path(name):
    return os.path.join(tl.GOLDEN, "levels", name + ".txt")


@pytest.mark.parametrize("name", MANY)
def test_many_level_files_match_reference_loader(name):
    ref = _info()[name]
    lv = levels.load_level(_path(name))
    assert lv.encoding == ENC[ref["encoding"]]
    assert (lv.width, lv.height) == (ref["width"], ref["height"])
    assert lv.tiles == ref["tiles"]
    assert sorted(lv.items) == sorted(tuple(x) for x in ref["items"])
    assert len(lv.items) > 8 and capi.item_slots(lv) == 16
    assert [list(s) for s in lv.spawns] == ref["spawns"]
    assert sorted(lv.goals) == ref["goals"]
    assert sorted(str(s) for s in recipes.all_subtasks(lv)) == sorted(ref["all_subtasks"])
    lv.validate(4)


def test_seventeen_objects_are_refused():
    text = "\n".join(["--ttt-lll-ooo", "/           p", "/     -     p", "-     -     p", "*     -     p",
                      "-     -     p", "-           p", "-------p-p---"]) + "\n\nSalad\n\n2 1\n4 1\n"
    lv = levels.parse_level_text(text, "seventeen")
    assert len(lv.items) == 17
    with pytest.raises(ValueError):
        lv.validate(2)


@pytest.mark.parametrize("impl", ["oracle", "swar_host"])
def test_many_level_episodes_match_reference(impl):
    fx = tl.load_fixture("manylevels.npz")
    groups = tl.episode_groups(fx)
    assert sum(g.B for g in groups) == 72
    assert {g.K for g in groups} == {16}
    for g in groups:
        if impl == "oracle":
            ob = oracle.OracleBatch(g.level, g.A, g.max_T, g.B)
            from test_oracle_golden import _oracle_step_fn as mk
        else:
            ts._load()
            ob = ts.SwarHostBatch(g.level, g.A, g.max_T, g.B)
            mk = ts._step_fn
        s = ob.new_state()
        ob.reset(s)
        g.relocate(s, ob.pitch)
        errs = tl.compare_group(g, mk(ob), s, ob.pitch, g.level.width)
        assert not errs, "%s A=%d: %s" % (g.level.name, g.A, "\n".join(errs[:10]))


def test_many_fixtures_reach_sixteen_objects_and_merges():
    fx = tl.load_fixture("manylevels.npz")
    items = fx["items"][..., 0].astype(np.int64)
    live = (items != tl.PAD).sum(-1)
    assert live.max() == 16 and (live > 8).mean() > 0.9
    # merged objects (a plate with a chopped food, or two foods) occur in every level
    names = [str(n) for n in fx["level_names"]]
    lvl = fx["ep_level"][np.searchsorted(fx["ep_state_off"], np.arange(len(items)), side="right") - 1]
    for i, n in enumerate(names):
        enc = levels.load_level(os.path.join(tl.GOLDEN, n)).encoding
        m = items[lvl == i]
        m = m[m != tl.PAD]
        merged = [x for x in np.unique(m) if len(levels.mask_contents(int(x), enc)) > 1]
        assert merged, n


@pytest.mark.parametrize("name", MANY)
@pytest.mark.parametrize("A", [2, 4])
def test_many_level_swar_matches_oracle_random(name, A):
    ts._load()
    B, steps, max_T = 1001, 90, 40
    lv = levels.load_level(_path(name))
    ob = oracle.OracleBatch(lv, A, max_T, B)
    sb = ts.SwarHostBatch(lv, A, max_T, B)
    assert ob.K == 16
    s, s2 = ob.new_state(), ob.new_state()
    ob.reset(s)
    h, h2 = s.copy(), s.copy()
    act = ob.new_actions()
    for t in range(steps):
        ob.gen_actions(act, 0, t, 91)
        ob.step(s, s2, act)
        sb.step(h, h2, act)
        s, s2, h, h2 = s2, s, h2, h
        assert np.array_equal(tl.env_view(s, A, ob.K, ob.pitch, B), tl.env_view(h, A, ob.K, ob.pitch, B)), t


@pytest.mark.parametrize("cfg", range(3))
def test_many_level_bounds_match_reference_rows(cfg):
    rows = tl.BoundRows(tl.load_fixture("bounds_many.npz"), cfg)
    ob = oracle.OracleBatch(rows.level, rows.A, 100, rows.B)
    assert ob.K == 16
    st = rows.state(ob.pitch)
    lb, doable = tb.host_bounds(ob, st, rows.subtasks)
    errs = rows.compare(lb, doable)
    assert not errs, "\n".join(errs[:20])
    o_lb, o_ok = ob.subtask_bounds(st, rows.subtasks)
    errs = rows.compare(o_lb, o_ok)
    assert not errs, "oracle: " + "\n".join(errs[:20])


@pytest.mark.parametrize("cfg", range(2))
@pytest.mark.parametrize("impl", ["oracle", "host"])
def test_many_level_rollout_matches_reference_rows(cfg, impl):
    fx = tl.load_fixture("rollout_many.npz")
    n = 0
    for rows in tl.RolloutRows(fx, cfg).split(capi.MAX_SUBTASKS):
        ob = oracle.OracleBatch(rows.level, rows.A, 100, rows.B)
        sin = tl.state_from_canonical(rows.level, rows.A, ob.K, ob.pitch, rows.agents, rows.items, rows.t)
        alloc = np.zeros(ob.pitch, np.uint8)
        alloc[:rows.B] = rows.alloc
        if impl == "oracle":
            sout = ob.new_state()
            flags, lb = ob.rollout(sin, sout, rows.actions(ob.pitch), rows.subtasks, alloc)
        else:
            sout, flags, lb = th.host_rollout(ob, sin, rows.actions(ob.pitch), rows.subtasks, alloc)
        errs = rows.compare(sout, flags, lb, ob.pitch)
        assert not errs, "\n".join(errs[:20])
        n += rows.B
    assert n == int((fx["cfg"] == cfg).sum())


# masks the objects of these kitchens can take, per encoding
_CAND = {levels.ENC_PRESENCE: [0x01, 0x02, 0x11, 0x22, 0x33, 0x08, 0x19, 0x2A, 0x3B],
         levels.ENC_COUNTS: [0x81, 0x84, 0x90, 0x01, 0x04, 0x10, 0x02, 0x05, 0x15, 0x2A, 0x40, 0x41, 0x45, 0x55,
                             0x46, 0x6A]}


def many_rollout_case(name, A, B, seed):
    """Random mid-episode states x random subtask tables over masks the level can take."""
    rng = np.random.default_rng(seed)
    lv = levels.load_level(_path(name))
    ob = oracle.OracleBatch(lv, A, 1000, B)
    s, s2 = ob.new_state(), ob.new_state()
    ob.reset(s)
    act = ob.new_actions()
    for t in range(int(rng.integers(5, 60))):
        ob.gen_actions(act, 0, t, seed)
        ob.step(s, s2, act)
        s, s2 = s2, s
    cand = sorted(set(_CAND[lv.encoding]) | {m for _, m in lv.items} | set(lv.goals))
    subs = []
    for i in range(int(rng.integers(1, capi.MAX_SUBTASKS + 1))):
        n = int(rng.integers(1, 3)) if A >= 2 else 1
        ags = sorted(rng.choice(A, n, replace=False).tolist())
        subs.append(capi.subtask(int(rng.integers(0, 4)), ags, [int(rng.choice(cand)), int(rng.choice(cand))],
                                 int(rng.choice(cand)), int(rng.integers(0, 3)), int(rng.integers(0, 2))))
    alloc = rng.integers(0, len(subs), ob.pitch).astype(np.uint8)
    acts = rng.integers(0, 7, A * ob.pitch).astype(np.uint8)
    return ob, s, acts, subs, alloc


@pytest.mark.parametrize("name", MANY)
@pytest.mark.parametrize("A", [2, 3])
def test_many_level_host_rollout_and_bounds_match_oracle_random(name, A):
    ob, s, acts, subs, alloc = many_rollout_case(name, A, 3000, seed=A * 23 + len(name))
    o_out = ob.new_state()
    o_fl, o_lb = ob.rollout(s, o_out, acts, subs, alloc)
    h_out, h_fl, h_lb = th.host_rollout(ob, s, acts, subs, alloc)
    assert np.array_equal(o_fl, h_fl) and np.array_equal(o_lb, h_lb)
    assert np.array_equal(tl.env_view(o_out, A, ob.K, ob.pitch, ob.B), tl.env_view(h_out, A, ob.K, ob.pitch, ob.B))
    subs0 = [capi.subtask(x.kind, list(x.agent[:x.num_agents]), list(x.start_mask), x.goal_mask, 0) for x in subs]
    lb, ok = tb.host_bounds(ob, s, subs0)
    o_lb2, o_ok2 = ob.subtask_bounds(s, subs0)
    assert np.array_equal(lb, o_lb2) and np.array_equal(ok, o_ok2)
