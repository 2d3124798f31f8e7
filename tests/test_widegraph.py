"""Kitchens whose reachability graph has more than the 360 nodes whose distance table a
narrow level's planner kernels hold in LDS:
  * widegraph-24x24_salad: 576 cells (wide: u16 cell ids), a 605-node graph;
  * dense-15x17_salad: 255 cells (narrow: byte cell ids), a 417-node graph (round 5; round 4
    refused it with OC_ELEVEL);
  * maze-31x31_salad: 961 cells (wide), a serpentine whose BFS distances pass 255 (about 450
    edges end to end): u16 distance tables (round 6; round 5 refused it with OC_ELEVEL);
  * corridor-204x5_salad: 1,020 cells, two lanes joined at one end (a U), distances to about 410
    below its perimeter (418), so its subtask bounds past 255 are exact values, not the
    perimeter + 1 the maze's saturate to (round 6).
Their planner kernels stage the level's other tables in LDS and read the distance table from
device memory (oc_rollout.h, RollLevel.dist_global).  Pinned on the CPU to the reference's own
runs of the level files (tests/golden/gen_widegraph.py, gen_densegraph.py, gen_mazegraph.py,
gen_corridorgraph.py):

* the parser and the engine's graph (node count, and the BFS distance of 400 random node pairs
  against the reference's nx.shortest_path_length);
* the CPU oracle and oc_cpu_step against the recorded episodes (2-4 agents);
* the host build of the planner rows and the oracle against the reference's subtask-bound and
  rollout rows, and against each other on random rows."""
import ctypes
import json
import os

import numpy as np
import pytest

import oc_testlib as tl
import test_bounds_host as tb
import test_rollout_host as th
import test_widelevels as tw
from gym_cooking_amd import capi, levels, recipes

from oracle import oracle

NAME = "widegraph-24x24_salad"
# kitchen -> (fixture prefix, wide layout)
KITCHENS = {"widegraph-24x24_salad": ("widegraph", True), "dense-15x17_salad": ("densegraph", False),
            "maze-31x31_salad": ("mazegraph", True), "corridor-204x5_salad": ("corridorgraph", True)}
LONG = ("maze-31x31_salad", "corridor-204x5_salad")  # BFS distances of 255 and more: u16 tables


def _info(name=NAME):
    with open(os.path.join(tl.GOLDEN, KITCHENS[name][0] + ".json")) as f:
        return json.load(f)[name]


def _graph(lv):
    """The engine's graph (oc_reachability16, a host-only handle): node count, node_of
    [cells * 5], dist [n * n] (u16, 0xFFFF = no path)."""
    lib = capi.load_library()
    d = capi.level_desc(lv, 2)
    h = ctypes.c_void_p()
    capi.check(lib.oc_create(ctypes.byref(d), 2, 100, capi.OC_DEVICE_HOST, ctypes.byref(h)))
    try:
        n = ctypes.c_int32()
        capi.check(lib.oc_reachability16(h, ctypes.byref(n), None, 0, None, 0))
        node_of = np.zeros(lv.ncells * 5, np.uint16)
        dist = np.zeros(n.value * n.value, np.uint16)
        capi.check(lib.oc_reachability16(h, ctypes.byref(n), node_of.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)),
                                         len(node_of), dist.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)),
                                         len(dist)))
    finally:
        lib.oc_destroy(h)
    return n.value, node_of, dist.reshape(n.value, n.value)


_NAV = {(0, 1): 0, (0, -1): 1, (-1, 0): 2, (1, 0): 3, (0, 0): 4}  # World.NAV_ACTIONS order + (0, 0)


KIT = pytest.mark.parametrize("name", sorted(KITCHENS))


def _fx(name, kind=""):
    return tl.load_fixture(kind + KITCHENS[name][0] + ".npz")


@KIT
def test_widegraph_level_matches_reference_graph(name):
    ref = _info(name)
    lv = levels.load_level(tw._path(name))
    assert (lv.width, lv.height) == (ref["width"], ref["height"]) and capi.is_wide(lv) == KITCHENS[name][1]
    assert lv.tiles == ref["tiles"]
    assert sorted(str(s) for s in recipes.all_subtasks(lv)) == sorted(ref["all_subtasks"])
    n, node_of, dist = _graph(lv)
    assert n == ref["graph_nodes"] > 360
    checked = 0
    for (ux, uy), ud, (vx, vy), vd, d in ref["dist_pairs"]:
        u = int(node_of[(uy * lv.width + ux) * 5 + _NAV[tuple(ud)]])
        v = int(node_of[(vy * lv.width + vx) * 5 + _NAV[tuple(vd)]])
        assert u != 0xFFFF and v != 0xFFFF
        got = int(dist[u, v])
        assert (got if got != 0xFFFF else -1) == d, ((ux, uy), ud, (vx, vy), vd, got, d)
        checked += 1
    assert checked == 400
    if name in LONG:  # the reason for these kitchens: distances a byte cannot hold
        assert max(p[4] for p in ref["dist_pairs"]) >= 255 and int(dist.max(initial=0, where=dist != 0xFFFF)) >= 255


def test_u8_reachability_refuses_only_the_long_graph():
    """oc_reachability's u8 table holds every graph whose BFS distances stay below 255 (the
    same bytes as oc_reachability16's low bytes there); on the maze it refuses the table with
    OC_ELEVEL (the node count and node ids still come back), and oc_reachability16 gives it."""
    lib = capi.load_library()
    for name in sorted(KITCHENS):
        lv = levels.load_level(tw._path(name))
        d = capi.level_desc(lv, 2)
        h = ctypes.c_void_p()
        capi.check(lib.oc_create(ctypes.byref(d), 2, 100, capi.OC_DEVICE_HOST, ctypes.byref(h)))
        try:
            n = ctypes.c_int32()
            capi.check(lib.oc_reachability(h, ctypes.byref(n), None, 0, None, 0))
            d8 = np.zeros(n.value * n.value, np.uint8)
            rc = lib.oc_reachability(h, ctypes.byref(n), None, 0, d8.ctypes.data, len(d8))
            _, _, d16 = _graph(lv)
            if name in LONG:
                assert rc == capi.OC_ELEVEL and b"oc_reachability16" in lib.oc_last_error()
            else:
                assert rc == 0 and int(d16[d16 != 0xFFFF].max()) < 255
                assert np.array_equal(d8.reshape(d16.shape), np.where(d16 == 0xFFFF, 0xFF, d16).astype(np.uint8))
        finally:
            lib.oc_destroy(h)


@KIT
@pytest.mark.parametrize("impl", ["oracle", "cpu_step"])
def test_widegraph_episodes_match_reference(name, impl):
    fx = _fx(name)
    groups = tl.episode_groups(fx)
    assert sum(g.B for g in groups) == len(fx["ep_T"]) >= 6
    for g in groups:
        ob = oracle.OracleBatch(g.level, g.A, g.max_T, g.B)
        s = ob.new_state()
        ob.reset(s)
        g.relocate(s, ob.pitch)
        if impl == "oracle":
            from test_oracle_golden import _oracle_step_fn
            fn = _oracle_step_fn(ob)
        else:
            from gym_cooking_amd.engine import CpuStepper
            fn = tw._cpu_step_fn(CpuStepper(g.level, g.A, g.B, g.max_T, nthreads=2))
        errs = tl.compare_group(g, fn, s, ob.pitch, g.level.width)
        assert not errs, "%s A=%d: %s" % (g.level.name, g.A, "\n".join(errs[:10]))


@KIT
@pytest.mark.parametrize("impl", ["oracle", "host"])
def test_widegraph_bounds_match_reference_rows(name, impl):
    rows = tl.BoundRows(_fx(name, "bounds_"), 0)
    assert rows.B > 0
    ob = oracle.OracleBatch(rows.level, rows.A, 100, rows.B)
    st = rows.state(ob.pitch)
    for c0 in range(0, len(rows.subtasks), capi.MAX_SUBTASKS):
        subs = rows.subtasks[c0:c0 + capi.MAX_SUBTASKS]
        lb, ok = tb.host_bounds(ob, st, subs) if impl == "host" else ob.subtask_bounds(st, subs)
        errs = rows.compare(lb, ok, sub0=c0)
        assert not errs, "\n".join(errs[:20])


@KIT
@pytest.mark.parametrize("impl", ["oracle", "host"])
def test_widegraph_rollout_matches_reference_rows(name, impl):
    fx = _fx(name, "rollout_")
    n = 0
    for rows in tl.RolloutRows(fx, 0).split(capi.MAX_SUBTASKS):
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
    assert n == len(fx["cfg"]) > 0


@KIT
@pytest.mark.parametrize("A", [2, 4])
def test_widegraph_host_rows_match_oracle_random(name, A):
    B = 1200
    ob, s, acts, subs, alloc = th.random_rollout_case(tw._path(name), A, B, seed=B + 7 * A, planner_levels=(0, 1))
    o_out = ob.new_state()
    o_fl, o_lb = ob.rollout(s, o_out, acts, subs, alloc)
    h_out, h_fl, h_lb = th.host_rollout(ob, s, acts, subs, alloc)
    assert np.array_equal(o_fl, h_fl) and np.array_equal(o_lb, h_lb)
    assert np.array_equal(tl.env_view(o_out, A, ob.K, ob.pitch, B), tl.env_view(h_out, A, ob.K, ob.pitch, B))
    subs0 = [capi.subtask(x.kind, list(x.agent[:x.num_agents]), list(x.start_mask), x.goal_mask, x.goal_count, 0)
             for x in subs]
    o_b, o_ok = ob.subtask_bounds(s, subs0)
    h_b, h_ok = tb.host_bounds(ob, s, subs0)
    assert np.array_equal(o_b, h_b) and np.array_equal(o_ok, h_ok)
