#!/usr/bin/env python3
"""A/B of oc_step_n's final-state store, interleaved in one process on the bench workload
(partial-divider_salad, 2 agents, 2^20 envs, trajectory + exec + coll + in-launch totals):
  separate  state_out is its own buffer: the final state is stored twice (trajectory + state_out)
  alias     state_out is the trajectory's last state: stored once (bench.py's launches)
For each launch length, HIP events around 100 back-to-back launches of one variant, the
variants alternating for 7 rounds; prints min / median us per launch."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))

import torch  # noqa: E402

from gym_cooking_amd.engine import OvercookedBatch  # noqa: E402

B = 1 << 20
eb = OvercookedBatch("partial-divider_salad", 2, B, max_T=100, device="cuda:0")
S, P, A = eb.layout.state_bytes, eb.pitch, eb.A
for n in (20, 100):
    acts = torch.empty((n, A * P), dtype=torch.uint8, device="cuda:0")
    for i in range(n):
        eb.gen_actions(acts[i], step=i, seed=0)
    s0, out = eb.new_state(), eb.new_state()
    eb.reset(s0)
    traj = torch.empty(n * S, dtype=torch.uint8, device="cuda:0")
    ex = torch.empty(n * A * P, dtype=torch.uint8, device="cuda:0")
    coll = torch.empty(n * P, dtype=torch.uint8, device="cuda:0")
    stats, tot = eb.new_stats(), torch.zeros(5, dtype=torch.int64, device="cuda:0")
    flat = acts.reshape(-1)
    var = {"separate": eb.step_n_launcher(s0, out, flat, n, traj, ex, coll, stats, tot),
           "alias": eb.step_n_launcher(s0, traj[(n - 1) * S:], flat, n, traj, ex, coll, stats, tot)}
    res = {k: [] for k in var}
    reps = 100 if n == 20 else 25
    for f in var.values():
        for _ in range(10):
            f()
    for _ in range(7):
        for k, f in var.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1e3 / reps)
    for k, v in res.items():
        print("n=%3d %-9s min %8.2f  median %8.2f us/launch" % (n, k, min(v), statistics.median(v)))

# bench.py's default window: 200 steps as 2 chained launches of 100 (actions of all 200 steps
# resident, 400 MB), replayed back-to-back; separate = state buffers ping-pong (round-2 bench),
# alias = each launch's state_out is its trajectory's last state
K, n = 200, 100
acts = torch.empty((K, A * P), dtype=torch.uint8, device="cuda:0")
for i in range(K):
    eb.gen_actions(acts[i], step=i, seed=0)
outs = [(torch.empty(n * S, dtype=torch.uint8, device="cuda:0"), torch.empty(n * A * P, dtype=torch.uint8, device="cuda:0"),
         torch.empty(n * P, dtype=torch.uint8, device="cuda:0")) for _ in range(2)]
sa, sb = eb.new_state(), eb.new_state()
stats, tot = eb.new_stats(), torch.zeros(5, dtype=torch.int64, device="cuda:0")


def chain(alias):
    fs, src, dst = [], sa, sb
    for li in range(2):
        tr, ex, co = outs[li]
        d = tr[(n - 1) * S:] if alias else dst
        fs.append(eb.step_n_launcher(src, d, acts[li * n:(li + 1) * n].reshape(-1), n, tr, ex, co, stats,
                                     tot if li == 1 else None))
        src, dst = (d, src) if alias else (dst, src)
    return fs


for name, alias in (("separate", False), ("alias", True)):
    fs = chain(alias)
    eb.reset(sa)
    for _ in range(3):
        for f in fs:
            f()
    torch.cuda.synchronize()
    v = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            for f in fs:
                f()
        e1.record()
        torch.cuda.synchronize()
        v.append(e0.elapsed_time(e1) * 1e3 / 20)
    print("200 steps as 2 x 100, %-9s min %8.2f  median %8.2f us/launch" % (name, min(v), statistics.median(v)))

# each launch of the chain repeated on its own: L1 starts from the reset state, L2 from L1's
# final state (every env at max_T: DONE, so L2's first step resets them all)
fs = chain(True)
eb.reset(sa)
for f in fs:
    f()
torch.cuda.synchronize()
for li, name in ((0, "L1 alone"), (1, "L2 alone")):
    v = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fs[li]()
        e1.record()
        torch.cuda.synchronize()
        v.append(e0.elapsed_time(e1) * 1e3 / 10)
    print("200 steps as 2 x 100, alias, %-9s min %8.2f  median %8.2f us/launch" % (name, min(v), statistics.median(v)))

# the chain with ONE output set for both launches (state buffers ping-pong): is it the
# alternation between two 2.1 GB output sets that costs?
fs = []
for li, (src, dst) in enumerate(((sa, sb), (sb, sa))):
    tr, ex, co = outs[0]
    fs.append(eb.step_n_launcher(src, dst, acts[li * n:(li + 1) * n].reshape(-1), n, tr, ex, co, stats,
                                 tot if li == 1 else None))
eb.reset(sa)
for _ in range(3):
    for f in fs:
        f()
torch.cuda.synchronize()
v = []
for _ in range(7):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        for f in fs:
            f()
    e1.record()
    torch.cuda.synchronize()
    v.append(e0.elapsed_time(e1) * 1e3 / 20)
print("200 steps as 2 x 100, one output set  min %8.2f  median %8.2f us/launch" % (min(v), statistics.median(v)))
