#!/usr/bin/env python3
"""Generate the fixtures for a kitchen whose reachability graph has more than 390 nodes (SURVEY
8(f) #3: load_level has no size limit, overcooked_environment.py:144-198; the planner kernels
keep a narrow level's distance table in LDS, which holds 390 nodes, and read a wide level's
from device memory) from the reference itself:
  * widegraph-24x24_salad  (576 cells, Salad, 4 items, a 605-node graph).

Runs ONLY in the build container (the reference is imported with gen_golden.py's stubs).
Recorded, in gen_widelevels' formats:
  * widegraph.json      the tables load_level / reset built, env.all_subtasks, the graph's node
                        count, and the reference's BFS distance (nx.shortest_path_length) of
                        400 random (node, node) pairs of its reachability graph;
  * widegraph.npz       episodes with 2-4 agents (uniform counter-RNG, 40 steps, and
                        goal-directed, 120: the reference steps this kitchen slowly);
  * bounds_widegraph.npz / rollout_widegraph.npz   gen_bounds / gen_rollout rows along goal
                        episodes.
Usage:  PYTHONHASHSEED=0 python tests/golden/gen_widegraph.py
"""
from __future__ import annotations

import contextlib
import copy
import io
import json
import os
import random
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
import gen_widelevels as gw  # noqa: E402

LEVELS = ["widegraph-24x24_salad"]
BOUND_CONFIGS = [("widegraph-24x24_salad", 3, 1, 9100)]
ROLL_CONFIGS = [("widegraph-24x24_salad", 2, 1, 9200)]


def main():
    generate(LEVELS, BOUND_CONFIGS, ROLL_CONFIGS, "widegraph", pair_seed=605, gid0=12700)


_DIST_MEMO = {}


def _cache_distances_bfs(self):
    """OvercookedEnvironment.cache_distances (overcooked_environment.py:775-821) with one BFS per
    source node (nx.single_source_shortest_path_length) instead of one nx.shortest_path_length
    per (source, destination, approach pair): the same dict, entry for entry and in the same
    insertion order (on an unweighted graph shortest_path_length is the BFS distance; a missing
    node or no path leaves the pair out of the min, np.inf when none is left; a source's own
    entry is overwritten by the loop, as in the reference), computed once per level.  Every
    reset() calls it; the original makes ~W^2 H^2 BFS calls, hours on a 961-cell kitchen.  The
    reference only caches and copies env.distances (:105, world.py:39): no recorded value reads it."""
    import networkx as nx
    from utils.world import World
    key = self.arglist.level
    if key not in _DIST_MEMO:
        g = self.world.reachability_graph
        names = [n for n in self.world.objects if "Supply" in n or "Counter" in n or "Delivery" in n or "Cut" in n]
        src = copy.copy(self.world.objects["Floor"])
        for n in names:
            src += copy.copy(self.world.objects[n])
        edges = lambda o: [(0, 0)] if not o.collidable else World.NAV_ACTIONS  # noqa: E731
        bfs = {}
        for o in src:
            for e in edges(o):
                node = (o.location, e)
                bfs[node] = nx.single_source_shortest_path_length(g, node) if node in g else {}
        dist = {}
        for s_ in src:
            dist[s_.location] = {s_.location: 0}
            for d_ in src:
                best = np.inf
                for se in edges(s_):
                    row = bfs[(s_.location, se)]
                    for de in edges(d_):
                        v = row.get((d_.location, de))
                        if v is not None and v < best:
                            best = v
                dist[s_.location][d_.location] = best
        _DIST_MEMO[key] = dist
    self.distances = _DIST_MEMO[key]
    self.world.distances = self.distances


def generate(LEVELS, BOUND_CONFIGS, ROLL_CONFIGS, prefix, pair_seed, gid0):
    """Record <prefix>.json (tables, graph size, 400 reference BFS distances), <prefix>.npz
    (episodes), bounds_<prefix>.npz and rollout_<prefix>.npz for the kitchens LEVELS."""
    ref = gg.load_reference()
    ref[0].cache_distances = _cache_distances_bfs
    gg.MAXK = 8
    gr.canon = gd.canon_k
    scratch = tempfile.mkdtemp(prefix="oc_%s_" % prefix)
    os.makedirs(os.path.join(scratch, "utils", "levels"))
    for name in LEVELS:
        shutil.copy(os.path.join(HERE, "levels", name + ".txt"), os.path.join(scratch, "utils", "levels"))
    os.chdir(scratch)
    from delegation_planner.bayesian_delegator import BayesianDelegator  # noqa: E402
    from navigation_planner.planners.e2e_brtdp import E2E_BRTDP  # noqa: E402
    import networkx as nx  # noqa: E402
    _, nav_utils, _ = ref

    info = {name: gd.level_info(gg.RefEnv(ref, name, 4, 100), nav_utils) for name in LEVELS}
    rng = random.Random(pair_seed)
    for name in LEVELS:
        env = gg.RefEnv(ref, name, 4, 100)
        g = env.env.world.reachability_graph
        info[name]["graph_nodes"] = g.number_of_nodes()
        nodes = sorted(g.nodes(), key=lambda v: (v[0][1], v[0][0], v[1]))
        pairs = []
        for _ in range(400):
            u, v = rng.choice(nodes), rng.choice(nodes)
            try:
                d = nx.shortest_path_length(g, u, v)
            except nx.NetworkXNoPath:
                d = -1
            # a node is ((x, y), (dx, dy)): the square and the side it is approached from
            pairs.append([list(u[0]), list(u[1]), list(v[0]), list(v[1]), d])
        info[name]["dist_pairs"] = pairs
    with open(os.path.join(HERE, prefix + ".json"), "w") as f:
        json.dump(info, f, indent=1, sort_keys=True, default=int)

    gg.LEVEL_NAMES = list(LEVELS)
    rec = gg.Recorder()
    gid = gid0
    for name in LEVELS:
        for A in (2, 3, 4):
            seed, g_ = 4800, gid
            rec.run(ref, name, A, 40, "uniform", seed,
                    lambda T, st, s=seed, g=g_, A=A: [gg.rng_action(s, g, T, a) for a in range(A)])
            gid += 1
            pol = gw.WidePolicy(info[name], A, seed=17 * gid, eps=0.03)
            rec.run(ref, name, A, 120, "goal", gid, lambda T, st, p=pol: p.act(st))
            gid += 1
            print("episodes A=%d done" % A, flush=True)
    gg.LEVEL_NAMES = ["levels/%s.txt" % n for n in LEVELS]
    rec.save(os.path.join(HERE, prefix + ".npz"), ["uniform", "goal"])
    fl = np.array(rec.S["flags"])
    print("wrote %d episodes / %d steps; done-success %d, err %d" % (
        len(rec.eps), len(rec.act), int(((fl & 3) == 3).sum()), int(((fl & 4) != 0).sum())))

    rows = {k: [] for k in ("state", "kind", "agents", "start", "goal_mask", "lb", "doable")}

    def visit_bounds(ci, env, st, A, si):
        with contextlib.redirect_stdout(io.StringIO()):
            gb.record_state(rows, nav_utils, BayesianDelegator, env.env, A, si)
    states = gw.goal_states(ref, info, BOUND_CONFIGS, 15, 120, visit_bounds)
    out = gd.save_states(os.path.join(HERE, "bounds_" + prefix + ".npz"), BOUND_CONFIGS, states, rows)
    print("wrote %d bound rows over %d states" % (len(out["lb"]), len(states)))

    rrows = {k: [] for k in ("cfg", "state", "kind", "agents", "start", "goal_mask", "goal_count",
                             "action", "legal", "assert_", "copy_raise", "next", "goal", "lb", "v_l", "v_u")}

    def visit_roll(ci, env, st, A, si):
        gr.record_state(rrows, E2E_BRTDP, ref, copy.copy(env.env), A, ci, si)
    states = gw.goal_states(ref, info, ROLL_CONFIGS, 20, 120, visit_roll)
    width = 12 + 4 * gg.MAXK
    rrows["next"] = [np.concatenate([n, np.full(width - len(n), gg.PAD, np.uint8)]) for n in rrows["next"]]
    out = gd.save_states(os.path.join(HERE, "rollout_" + prefix + ".npz"), ROLL_CONFIGS, states, rrows)
    print("wrote %d rollout rows over %d states; legal %d, goal %d" % (
        len(out["lb"]), len(states), int(out["legal"].sum()), int(out["goal"].sum())))
    shutil.rmtree(scratch)


if __name__ == "__main__":
    main()
