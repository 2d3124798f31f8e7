#!/usr/bin/env python3
"""How much of the C5 kernels' time is wave divergence between rows of different planner
configurations?  Times oc_rollout / oc_nav_likelihood on bench.py's C5 rows (full-divider_salad,
4 agents, 2^18 mid-episode states, 64 Salad configurations) with the same multiset of
allocation ids in three orders:
  random    each row an independent random configuration (bench.py's workload)
  grouped   the same ids sorted, so the rows of one configuration are contiguous (how the
            reference's delegator iterates: for each allocation, for each agent)
  single    every row configuration 0
and a table of the one-agent configurations only, configuration-major (the likelihood
kernel's 8-lane groups; tables with a two-agent configuration take 32-lane groups).
Usage: python tools/c5_order_probe.py
"""
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import SALAD_SUBTASKS  # noqa: E402
from gym_cooking_amd import capi  # noqa: E402
from gym_cooking_amd.engine import OvercookedBatch  # noqa: E402


def timed(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda", 0)
    A, rows = 4, 1 << 18
    eb = OvercookedBatch("full-divider_salad", A, rows, max_T=100, device=dev)
    s, s2 = eb.new_state(), eb.new_state()
    eb.reset(s)
    a = eb.new_actions()
    for t in range(37):
        eb.gen_actions(a, t, 11)
        eb.step(s, s2, a)
        s, s2 = s2, s
    agent_sets = [(i,) for i in range(A)] + list(itertools.combinations(range(A), 2))
    table = [capi.subtask(k, ags, st, g, 0) for (k, st, g) in SALAD_SUBTASKS for ags in agent_sets]
    table = table[:capi.MAX_SUBTASKS]
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    rnd = torch.randint(0, len(table), (eb.pitch,), dtype=torch.uint8, device=dev, generator=gen)
    orders = {"random": rnd, "grouped": torch.sort(rnd)[0].contiguous(),
              "single": torch.zeros_like(rnd)}
    eb.gen_actions(a, 99, 12)
    out = eb.new_state()
    flags = torch.empty(eb.pitch, dtype=torch.uint8, device=dev)
    lb = torch.empty(eb.pitch, dtype=torch.float32, device=dev)
    res = {}
    for name, al in orders.items():
        r_ms = timed(lambda: eb.rollout(s, out, a, table, al, flags, lb), 20)
        l_ms = timed(lambda: eb.nav_likelihood(s, a, table, 0, 1.3, 0.5, al), 5)
        res[name] = {"rollout_ms": r_ms, "likelihood_ms": l_ms}
    # a table of one-agent configurations only (the likelihood kernel's 8-lane groups)
    singles = [i for i, t in enumerate(table) if t.num_agents == 1]
    t1 = [table[i] for i in singles]
    al1 = torch.sort(torch.randint(0, len(t1), (eb.pitch,), dtype=torch.uint8, device=dev, generator=gen))[0]
    res["one_agent_table_grouped"] = {"likelihood_ms": timed(lambda: eb.nav_likelihood(s, a, t1, 0, 1.3, 0.5, al1), 5)}
    bl = torch.empty((len(table), eb.pitch), dtype=torch.float32, device=dev)
    bo = torch.empty((len(table), eb.pitch), dtype=torch.uint8, device=dev)
    res["bounds_ms"] = timed(lambda: eb.subtask_bounds(s, table, bl, bo), 10)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
