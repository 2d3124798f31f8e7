"""Kitchens with a Floor square on the grid's border, on the CPU.

The reference loads and resets such a map; a step where an agent on a border Floor acts
towards the outside raises AssertionError in check_collisions when there are two or more
agents (is_collision looks the unclamped square up, overcooked_environment.py:692-700 ->
get_gridsquare_at, world.py:429), and clamps the move away with World.inbounds when there is
one (interact.py:22).  The engine gives the raise OC_FLAG_DONE | OC_FLAG_ERR with the state
unchanged but t (include/oc_engine.h).  Pinned to the reference's own runs of the same level
files (tests/golden/gen_edgelevels.py): the parser against load_level's tables, the CPU
oracle and the host build of the device SWAR step against all recorded episodes (1-3 agents,
raises included), the planner row and the oracle against the reference planner's rollout and
subtask-bound rows, and random play between the oracle and the host build."""
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

EDGE = ["edge-7x6_salad", "edge-8x7_tl"]


def _info():
    with open(os.path.join(tl.GOLDEN, "edgelevels.json")) as f:
        return json.load(f)


def _path(name):
    return os.path.join(tl.GOLDEN, "levels", name + ".txt")


@pytest.mark.parametrize("name", EDGE)
def test_edge_level_files_match_reference_loader(name):
    ref = _info()[name]
    lv = levels.load_level(_path(name))
    assert lv.edge
    assert (lv.width, lv.height) == (ref["width"], ref["height"])
    assert lv.tiles == ref["tiles"]
    assert sorted(lv.items) == sorted(tuple(x) for x in ref["items"])
    assert [list(s) for s in lv.spawns] == ref["spawns"]
    assert sorted(lv.goals) == ref["goals"]
    assert sorted(str(s) for s in recipes.all_subtasks(lv)) == sorted(ref["all_subtasks"])
    lv.validate(4)


def off_grid_step(fx, e, s):
    """Recorded step s of episode e has an agent acting off the grid (two or more agents:
    the reference's step raises in check_collisions)."""
    A = int(fx["ep_A"][e])
    lv = levels.load_level(os.path.join(tl.GOLDEN, str(fx["level_names"][fx["ep_level"][e]])))
    pre, codes = fx["agents"][int(fx["ep_state_off"][e]) + s], fx["act"][int(fx["ep_act_off"][e]) + s]
    return A >= 2 and any(lv.off_grid(int(pre[a][0]), int(pre[a][1]), int(codes[a])) for a in range(A))


def _raise_steps(fx):
    """(episode, step) of every recorded step that raised off the grid; each is recorded as
    DONE | ERR with the agents where they were."""
    out = []
    for e in range(len(fx["ep_T"])):
        off = int(fx["ep_state_off"][e])
        for s in range(int(fx["ep_T"][e])):
            if off_grid_step(fx, e, s):
                assert fx["flags"][off + s + 1] & 5 == 5
                assert np.array_equal(fx["agents"][off + s + 1], fx["agents"][off + s])
                out.append((e, s))
    return out


def test_edge_fixtures_hold_raises_and_clamps():
    fx = tl.load_fixture("edgelevels.npz")
    assert len(_raise_steps(fx)) >= 5
    # one-agent episodes where the agent acted off the grid from a border Floor and stayed
    clamps = 0
    for e in range(len(fx["ep_T"])):
        if int(fx["ep_A"][e]) != 1:
            continue
        lv = levels.load_level(os.path.join(tl.GOLDEN, str(fx["level_names"][fx["ep_level"][e]])))
        off, aoff = int(fx["ep_state_off"][e]), int(fx["ep_act_off"][e])
        for s in range(int(fx["ep_T"][e])):
            x, y = (int(v) for v in fx["agents"][off + s][0][:2])
            if lv.off_grid(x, y, int(fx["act"][aoff + s][0])):
                assert tuple(fx["agents"][off + s + 1][0][:2]) == (x, y)
                clamps += 1
    assert clamps >= 3


@pytest.mark.parametrize("impl", ["oracle", "swar_host"])
def test_edge_level_episodes_match_reference(impl):
    fx = tl.load_fixture("edgelevels.npz")
    groups = tl.episode_groups(fx)
    assert sum(g.B for g in groups) == 48
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


@pytest.mark.parametrize("name", EDGE)
@pytest.mark.parametrize("A", [1, 2, 3])
def test_edge_level_swar_matches_oracle_random(name, A):
    ts._load()
    B, steps, max_T = 1001, 90, 40
    lv = levels.load_level(_path(name))
    ob = oracle.OracleBatch(lv, A, max_T, B)
    sb = ts.SwarHostBatch(lv, A, max_T, B)
    s, s2 = ob.new_state(), ob.new_state()
    ob.reset(s)
    h, h2 = s.copy(), s.copy()
    act = ob.new_actions()
    P = ob.pitch
    ex_o, ex_h = np.zeros(A * P, np.uint8), np.zeros(A * P, np.uint8)
    c_o, c_h = np.zeros(P, np.uint8), np.zeros(P, np.uint8)
    errs = 0
    for t in range(steps):
        ob.gen_actions(act, 0, t, 93)
        ob.step(s, s2, act, ex_o, c_o)
        sb.step(h, h2, act, ex_h, c_h)
        s, s2, h, h2 = s2, s, h2, h
        assert np.array_equal(tl.env_view(s, A, ob.K, P, B), tl.env_view(h, A, ob.K, P, B)), t
        assert np.array_equal(ex_o.reshape(A, P)[:, :B], ex_h.reshape(A, P)[:, :B]), t
        assert np.array_equal(c_o[:B], c_h[:B]), t
        errs += int((tl.planes_view(s, A, ob.K, P)["fl"][:B] & 4).sum() > 0)
    if A >= 2:
        assert errs > 0  # the off-grid raise occurs in random play


@pytest.mark.parametrize("cfg", range(2))
def test_edge_level_bounds_match_reference_rows(cfg):
    rows = tl.BoundRows(tl.load_fixture("bounds_edge.npz"), cfg)
    ob = oracle.OracleBatch(rows.level, rows.A, 100, rows.B)
    st = rows.state(ob.pitch)
    lb, doable = tb.host_bounds(ob, st, rows.subtasks)
    errs = rows.compare(lb, doable)
    assert not errs, "\n".join(errs[:20])
    o_lb, o_ok = ob.subtask_bounds(st, rows.subtasks)
    errs = rows.compare(o_lb, o_ok)
    assert not errs, "oracle: " + "\n".join(errs[:20])


@pytest.mark.parametrize("cfg", range(2))
@pytest.mark.parametrize("impl", ["oracle", "host"])
def test_edge_level_rollout_matches_reference_rows(cfg, impl):
    fx = tl.load_fixture("rollout_edge.npz")
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
