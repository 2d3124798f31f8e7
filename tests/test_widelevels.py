"""Kitchens of more than 255 cells (user levels past the byte cell ids) on the
CPU: the engine's wide layout (u16 item cells, include/oc_engine.h oc_layout.cell_bytes) and
its scalar step (oc_rollout.h RowOps::env_step), pinned to the reference's own runs of the same
level files (tests/golden/gen_widelevels.py: a 17x17 Salad kitchen of 289 cells, a 23x13
two-recipe kitchen of 299 cells with 5 items and two Delivery squares):

* the parser against load_level / reset's tables and the reachability graph's node count;
* the CPU oracle and oc_cpu_step (the product library's host pass of the scalar step) against
  every recorded episode (1-4 agents, uniform and goal-directed);
* oc_cpu_step against the oracle in random play (timeouts, auto-resets, ERR ends, collisions),
  with the window statistics;
* the planner row (host build of oc_rollout.h) and the oracle against the reference planner's
  rollout and subtask-bound rows on the wide kitchens, and against each other on random rows
  (rollout, bounds, likelihoods)."""
import ctypes
import json
import os

import numpy as np
import pytest

import oc_testlib as tl
import test_bounds_host as tb
import test_rollout_host as th
from gym_cooking_amd import capi, levels, recipes
from gym_cooking_amd.engine import CpuStepper

from oracle import oracle

WIDE = ["wide-17x17_salad", "wide-23x13_tl"]


def _info():
    with open(os.path.join(tl.GOLDEN, "widelevels.json")) as f:
        return json.load(f)


def _path(name):
    return os.path.join(tl.GOLDEN, "levels", name + ".txt")


def _graph_nodes(lv):
    """Node count of the engine's reachability graph (oc_reachability; host tables, no GPU)."""
    lib = capi.load_library()
    d = capi.level_desc(lv, 2)
    h = ctypes.c_void_p()
    capi.check(lib.oc_create(ctypes.byref(d), 2, 100, 0, ctypes.byref(h)))
    n = ctypes.c_int32()
    try:
        capi.check(lib.oc_reachability(h, ctypes.byref(n), None, 0, None, 0))
    finally:
        lib.oc_destroy(h)
    return n.value


@pytest.mark.parametrize("name", WIDE)
def test_wide_level_files_match_reference_loader(name):
    ref = _info()[name]
    lv = levels.load_level(_path(name))
    assert lv.ncells > levels.MAX_NARROW_CELLS and capi.is_wide(lv)
    assert (lv.width, lv.height) == (ref["width"], ref["height"])
    assert lv.tiles == ref["tiles"]
    assert sorted(lv.items) == sorted(tuple(x) for x in ref["items"])
    assert [list(s) for s in lv.spawns] == ref["spawns"]
    assert sorted(lv.goals) == ref["goals"]
    assert sorted(str(s) for s in recipes.all_subtasks(lv)) == sorted(ref["all_subtasks"])
    lv.validate(4)
    assert _graph_nodes(lv) == ref["graph_nodes"]


def test_wide_layout():
    lv = levels.load_level(_path("wide-23x13_tl"))
    cs = CpuStepper(lv, 3, 10)
    L = cs.layout
    assert (L.cell_bytes, cs.K) == (2, 8)
    assert (L.plane_item_loc, L.plane_item_loc_hi, L.plane_item_mask) == (9, 17, 25)
    assert (L.plane_t, L.plane_flags, L.num_planes) == (33, 35, 36)
    assert capi.layout_planes(3, 8, True)["num_planes"] == 36
    narrow = CpuStepper("open-divider_salad", 3, 10).layout
    assert (narrow.cell_bytes, narrow.plane_item_loc_hi, narrow.num_planes) == (1, -1, 20)


def _cpu_step_fn(cs):
    def fn(state, acts):
        a = np.full(cs.A * cs.pitch, 4, np.uint8)
        a.reshape(cs.A, cs.pitch)[:, :cs.B] = acts
        out = np.zeros_like(state)
        ex = np.zeros(cs.A * cs.pitch, np.uint8)
        coll = np.zeros(cs.pitch, np.uint8)
        cs.step(state, out, a, ex, coll)
        return out, ex.reshape(cs.A, cs.pitch)[:, :cs.B], coll[:cs.B]
    return fn


@pytest.mark.parametrize("impl", ["oracle", "cpu_step"])
def test_wide_level_episodes_match_reference(impl):
    fx = tl.load_fixture("widelevels.npz")
    groups = tl.episode_groups(fx)
    assert sum(g.B for g in groups) == len(fx["ep_T"]) >= 48
    for g in groups:
        ob = oracle.OracleBatch(g.level, g.A, g.max_T, g.B)
        s = ob.new_state()
        ob.reset(s)
        g.relocate(s, ob.pitch)
        if impl == "oracle":
            from test_oracle_golden import _oracle_step_fn
            fn = _oracle_step_fn(ob)
        else:
            fn = _cpu_step_fn(CpuStepper(g.level, g.A, g.B, g.max_T, nthreads=2))
        errs = tl.compare_group(g, fn, s, ob.pitch, g.level.width)
        assert not errs, "%s A=%d: %s" % (g.level.name, g.A, "\n".join(errs[:10]))


def test_wide_fixtures_reach_deliveries_and_items_past_cell_255():
    fx = tl.load_fixture("widelevels.npz")
    fl = fx["flags"]
    assert int(((fl & 3) == 3).sum()) >= 3, "no delivered episode recorded"
    W = {str(n): levels.load_level(os.path.join(tl.GOLDEN, str(n))).width for n in fx["level_names"]}
    it = fx["items"]
    cells = it[..., 2].astype(int) * 23 + it[..., 1].astype(int)  # a lower bound for both widths
    assert (cells[it[..., 0] != tl.PAD] > 255).any()
    assert min(W.values()) >= 17


@pytest.mark.parametrize("name", WIDE)
@pytest.mark.parametrize("A", [1, 2, 3, 4])
def test_wide_cpu_step_matches_oracle_random(name, A):
    lv = levels.load_level(_path(name))
    B, steps, max_T = 1003, 120, 45
    ob = oracle.OracleBatch(lv, A, max_T, B)
    cs = CpuStepper(lv, A, B, max_T, nthreads=3)
    P = ob.pitch
    s1, n1 = ob.new_state(), ob.new_state()
    ob.reset(s1)
    assert np.array_equal(tl.env_view(cs.new_state(), A, cs.K, P, B), tl.env_view(s1, A, ob.K, P, B))
    s2, n2 = s1.copy(), s1.copy()
    act = ob.new_actions()
    e1, e2 = np.zeros(A * P, np.uint8), np.zeros(A * P, np.uint8)
    c1, c2 = np.zeros(P, np.uint8), np.zeros(P, np.uint8)
    tot, want = np.zeros(5, np.uint64), np.zeros(5, np.int64)
    for t in range(steps):
        ob.gen_actions(act, 0, t, 31 * A + 7)
        fl_in = tl.planes_view(s1, A, ob.K, P)["fl"].copy()
        ob.step(s1, n1, act, e1, c1)
        cs.step(s2, n2, act, e2, c2, tot)
        s1, n1, s2, n2 = n1, s1, n2, s2
        want += tl.window_totals(fl_in, s1, c1, A, ob.K, P, B)
        v1, v2 = tl.env_view(s1, A, ob.K, P, B), tl.env_view(s2, A, ob.K, P, B)
        if not np.array_equal(v1, v2):
            bad = np.argwhere(v1 != v2)
            raise AssertionError("step %d: %d bytes differ, first (plane, env) %s" % (t, len(bad), bad[:5].tolist()))
        assert np.array_equal(e1.reshape(A, -1)[:, :B], e2.reshape(A, -1)[:, :B]), t
        assert np.array_equal(c1[:B], c2[:B]), t
    assert np.array_equal(tot.astype(np.int64), want), (tot, want)
    assert want[0] >= B  # the timeouts
    if A >= 2:
        assert want[3] > 0  # collisions


@pytest.mark.parametrize("cfg", range(2))
@pytest.mark.parametrize("impl", ["oracle", "host"])
def test_wide_level_bounds_match_reference_rows(cfg, impl):
    rows = tl.BoundRows(tl.load_fixture("bounds_wide.npz"), cfg)
    ob = oracle.OracleBatch(rows.level, rows.A, 100, rows.B)
    st = rows.state(ob.pitch)
    for c0 in range(0, len(rows.subtasks), capi.MAX_SUBTASKS):
        subs = rows.subtasks[c0:c0 + capi.MAX_SUBTASKS]
        lb, ok = tb.host_bounds(ob, st, subs) if impl == "host" else ob.subtask_bounds(st, subs)
        errs = rows.compare(lb, ok, sub0=c0)
        assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("cfg", range(2))
@pytest.mark.parametrize("impl", ["oracle", "host"])
def test_wide_level_rollout_matches_reference_rows(cfg, impl):
    fx = tl.load_fixture("rollout_wide.npz")
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


@pytest.mark.parametrize("name", WIDE)
@pytest.mark.parametrize("A", [2, 4])
def test_wide_host_rows_match_oracle_random(name, A):
    """Random states x random configuration tables (Level 0 and 1): the host build of the
    row code against the oracle, for rollout, subtask bounds and likelihood rows."""
    B = 1500
    ob, s, acts, subs, alloc = th.random_rollout_case(_path(name), A, B, seed=B + A, planner_levels=(0, 1))
    o_out = ob.new_state()
    o_fl, o_lb = ob.rollout(s, o_out, acts, subs, alloc)
    h_out, h_fl, h_lb = th.host_rollout(ob, s, acts, subs, alloc)
    assert np.array_equal(o_fl, h_fl)
    assert np.array_equal(o_lb, h_lb)
    assert np.array_equal(tl.env_view(o_out, A, ob.K, ob.pitch, B), tl.env_view(h_out, A, ob.K, ob.pitch, B))
    subs0 = [capi.subtask(x.kind, list(x.agent[:x.num_agents]), list(x.start_mask), x.goal_mask, x.goal_count, 0)
             for x in subs]
    o_b, o_ok = ob.subtask_bounds(s, subs0)
    h_b, h_ok = tb.host_bounds(ob, s, subs0)
    assert np.array_equal(o_b, h_b) and np.array_equal(o_ok, h_ok)
    o_v, o_f = ob.nav_likelihood(s, acts, subs0, alloc, 0, 1.3, 0.5)
    h_v, h_f = th.host_likelihood(ob, s, acts, subs0, alloc, 0, 1.3, 0.5)
    assert np.array_equal(o_f, h_f)
    ok = o_f == capi.LIK_OK
    assert ok.sum() > 20
    np.testing.assert_allclose(h_v[ok], o_v[ok], rtol=1e-12)


def _variant(kind):
    """wide-17x17_salad edited into the level kinds the wide SWAR step (ocsw::step4w) has
    branches for: `edge` opens two border squares to Floor (an action can point off the grid);
    `counts` repeats the foods (OC_ENC_COUNTS masks, 8 item slots); `many` has 10 objects (16)."""
    rows, rest = open(_path("wide-17x17_salad")).read().split("\n\n", 1)
    grid = [list(r) for r in rows.split("\n")]
    if kind == "edge":
        grid[0][3] = " "
        grid[10][16] = " "
    if kind in ("counts", "many"):
        grid[16][3], grid[0][12] = "t", "l"
    if kind == "many":
        grid[3][16], grid[16][12], grid[0][14], grid[8][0] = "p", "p", "o", "t"
    return levels.parse_level_text("\n".join("".join(r) for r in grid) + "\n\n" + rest, "wide-17x17-" + kind)


@pytest.mark.parametrize("kind,A", [("edge", 1), ("edge", 3), ("counts", 2), ("counts", 4), ("many", 3)])
def test_wide_swar_step_variants_match_oracle(kind, A):
    """The wide SWAR step's wave-uniform branches (Floor on the border with one agent, where
    interact clamps the square, and with several, where check_collisions raises; repeated foods
    in the counts encoding; 16 item slots) on oc_cpu_step, the host pass of the kernel's code,
    against the oracle over random play with timeouts and resets."""
    lv = _variant(kind)
    assert capi.is_wide(lv)
    B, steps, max_T = 1003, 150, 37
    ob = oracle.OracleBatch(lv, A, max_T, B)
    cs = CpuStepper(lv, A, B, max_T, nthreads=3)
    assert cs.K == {"edge": 4, "counts": 8, "many": 16}[kind] and lv.encoding == (0 if kind == "edge" else 1)
    P = ob.pitch
    s1, n1 = ob.new_state(), ob.new_state()
    ob.reset(s1)
    s2, n2 = s1.copy(), s1.copy()
    act = ob.new_actions()
    e1, e2 = np.zeros(A * P, np.uint8), np.zeros(A * P, np.uint8)
    c1, c2 = np.zeros(P, np.uint8), np.zeros(P, np.uint8)
    tot, want = np.zeros(5, np.uint64), np.zeros(5, np.int64)
    for t in range(steps):
        ob.gen_actions(act, 0, t, 53 * A + 11)
        fl_in = tl.planes_view(s1, A, ob.K, P)["fl"].copy()
        ob.step(s1, n1, act, e1, c1)
        cs.step(s2, n2, act, e2, c2, tot)
        s1, n1, s2, n2 = n1, s1, n2, s2
        want += tl.window_totals(fl_in, s1, c1, A, ob.K, P, B)
        v1, v2 = tl.env_view(s1, A, ob.K, P, B), tl.env_view(s2, A, ob.K, P, B)
        assert np.array_equal(v1, v2), (t, np.argwhere(v1 != v2)[:5].tolist())
        assert np.array_equal(e1.reshape(A, -1)[:, :B], e2.reshape(A, -1)[:, :B]), t
        assert np.array_equal(c1[:B], c2[:B]), t
    assert np.array_equal(tot.astype(np.int64), want), (tot, want)
    if kind == "edge" and A > 1:
        assert want[4] > 0  # off-grid raises (ERR ends)
