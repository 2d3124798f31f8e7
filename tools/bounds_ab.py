#!/usr/bin/env python3
"""A/B of the C5 kernels between builds of liboc_engine.so, on one box: bench.py's C5 rows
(full-divider_salad, 4 agents, 2^18 mid-episode states, the 64 Salad (subtask, agents)
configurations), each build in a fresh process, alternating.  Per build: the mean
oc_subtask_bounds / oc_rollout / oc_nav_likelihood launch (HIP events around back-to-back
launches, bench.time_launches) and a digest of every output byte, so that the builds' outputs
can be compared.
  python tools/bounds_ab.py --libs A.so B.so [--rounds 3]
Prints one JSON line per (round, lib)."""
import argparse
import hashlib
import itertools
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cooking_amd")]
    import torch
    from gym_cooking_amd import capi
    capi.load_library(lib)
    import bench
    from gym_cooking_amd.engine import OvercookedBatch
    dev = "cuda:0"
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
    table = [capi.subtask(k, ags, st, g, 0) for (k, st, g) in bench.SALAD_SUBTASKS for ags in agent_sets]
    table = table[:capi.MAX_SUBTASKS]
    lb = torch.empty((len(table), eb.pitch), dtype=torch.float32, device=dev)
    ok = torch.empty((len(table), eb.pitch), dtype=torch.uint8, device=dev)
    ms_b = bench.time_launches(eb.subtask_bounds_launcher(s, table, lb, ok), 60, dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    alloc = torch.sort(torch.randint(0, len(table), (eb.pitch,), dtype=torch.uint8, device=dev, generator=gen))[0]
    alloc = alloc.contiguous()
    eb.gen_actions(a, 99, 12)
    out = eb.new_state()
    flags = torch.empty(eb.pitch, dtype=torch.uint8, device=dev)
    rlb = torch.empty(eb.pitch, dtype=torch.float32, device=dev)
    ms_r = bench.time_launches(eb.rollout_launcher(s, out, a, table, alloc, flags, rlb), 200, dev)
    # the planner's launch size: the first 4,096 rows (configuration-major)
    eb4 = OvercookedBatch("full-divider_salad", A, 4096, max_T=100, device=dev)
    NP = eb.layout.num_planes
    s4 = s.view(NP, eb.pitch)[:, :4096].contiguous().view(-1)
    a4 = a.view(A, eb.pitch)[:, :4096].contiguous().view(-1)
    o4, f4 = eb4.new_state(), torch.empty(eb4.pitch, dtype=torch.uint8, device=dev)
    l4 = torch.empty(eb4.pitch, dtype=torch.float32, device=dev)
    ms_r4 = bench.time_launches(eb4.rollout_launcher(s4, o4, a4, table, alloc[:4096].contiguous(), f4, l4), 400, dev)
    v = torch.empty(eb.pitch, dtype=torch.float64, device=dev)
    f = torch.empty(eb.pitch, dtype=torch.uint8, device=dev)
    ms_l = bench.time_launches(eb.nav_likelihood_launcher(s, a, table, 0, 1.3, 0.5, alloc, v, f), 40, dev)
    # the likelihood again with the rows in random configuration order, and with a table of
    # one-agent configurations only (8-lane groups)
    perm = torch.randperm(eb.pitch, device=dev, generator=gen)
    alloc_r = alloc[perm].contiguous()
    vr = torch.empty_like(v)
    fr = torch.empty_like(f)
    ms_lr = bench.time_launches(eb.nav_likelihood_launcher(s, a, table, 0, 1.3, 0.5, alloc_r, vr, fr), 40, dev)
    table1 = [capi.subtask(k, ags, st, g, 0) for (k, st, g) in bench.SALAD_SUBTASKS for ags in agent_sets
              if len(ags) == 1][:capi.MAX_SUBTASKS]
    alloc1 = (alloc % len(table1)).contiguous()
    v1 = torch.empty_like(v)
    f1 = torch.empty_like(f)
    ms_l1 = bench.time_launches(eb.nav_likelihood_launcher(s, a, table1, 0, 1.3, 0.5, alloc1, v1, f1), 40, dev)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in (lb[:, :rows], ok[:, :rows], out, flags[:rows], rlb[:rows], v[:rows], f[:rows], vr[:rows], fr[:rows],
              v1[:rows], f1[:rows], o4, f4[:4096], l4[:4096]):
        h.update(t.contiguous().cpu().numpy().tobytes())
    print(json.dumps({"lib": os.path.basename(lib), "bounds_ms": ms_b, "rollout_ms": ms_r, "rollout_4096_ms": ms_r4,
                      "likelihood_ms": ms_l,
                      "likelihood_random_ms": ms_lr, "likelihood_single_ms": ms_l1, "lik_ok": int((f[:rows] == 1).sum()),
                      "doable": int(ok[:, :rows].sum()), "digest": h.hexdigest()[:16]}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--child")
    a = ap.parse_args()
    if a.child:
        return child(a.child)
    for r in range(a.rounds):
        for lib in a.libs:
            out = subprocess.run([sys.executable, __file__, "--child", os.path.abspath(lib)], capture_output=True,
                                 text=True, timeout=300)
            line = [x for x in out.stdout.splitlines() if x.startswith("{")]
            if out.returncode != 0 or not line:
                print(out.stderr[-2000:], file=sys.stderr)
                return 1
            d = json.loads(line[0])
            d["round"] = r
            print(json.dumps(d), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
