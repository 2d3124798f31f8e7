#!/usr/bin/env python3
"""oc_step_n launch time against launch length on the bench workload (partial-divider_salad,
2 agents, 2^20 envs, bench.py's outputs: trajectory with state_out its last state, exec, coll,
in-launch totals): HIP events around back-to-back launches of each length, the lengths
interleaved for 5 rounds.  The fit t(n) = t0 + n * t_step separates the per-launch fixed cost
(state read, ramp, statistics fold, drain) from the per-step cost."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_cooking_amd.engine import OvercookedBatch  # noqa: E402

B = 1 << 20
NS = (1, 2, 5, 10, 20, 40, 100)
eb = OvercookedBatch("partial-divider_salad", 2, B, max_T=100, device="cuda:0")
S, P, A = eb.layout.state_bytes, eb.pitch, eb.A
NMAX = max(NS)
acts = torch.empty((NMAX, A * P), dtype=torch.uint8, device="cuda:0")
for i in range(NMAX):
    eb.gen_actions(acts[i], step=i, seed=0)
s0 = eb.new_state()
eb.reset(s0)
traj = torch.empty(NMAX * S, dtype=torch.uint8, device="cuda:0")
ex = torch.empty(NMAX * A * P, dtype=torch.uint8, device="cuda:0")
coll = torch.empty(NMAX * P, dtype=torch.uint8, device="cuda:0")
stats, tot = eb.new_stats(), torch.zeros(5, dtype=torch.int64, device="cuda:0")
fns = {n: eb.step_n_launcher(s0, traj[(n - 1) * S:n * S], acts[:n].reshape(-1), n, traj[:n * S], ex[:n * A * P],
                             coll[:n * P], stats, tot) for n in NS}
res = {n: [] for n in NS}
for f in fns.values():
    for _ in range(5):
        f()
for _ in range(5):
    for n, f in fns.items():
        reps = max(5, 2000 // n)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        res[n].append(e0.elapsed_time(e1) * 1e3 / reps)
med = {n: statistics.median(v) for n, v in res.items()}
for n in NS:
    print("n=%3d  median %8.2f us/launch  %6.2f us/step" % (n, med[n], med[n] / n))
x = np.array(NS, float)
y = np.array([med[n] for n in NS])
k, c = np.polyfit(x[3:], y[3:], 1)
print("fit over n >= 10: t0 = %.2f us per launch, %.3f us per step" % (c, k))

# which part of the launch is fixed: outputs and statistics switched off one at a time
out = eb.new_state()
variants = {
    "bench (alias, traj+exec+coll, stats+totals)": lambda n: fns[n],
    "stats, no totals": lambda n: eb.step_n_launcher(s0, traj[(n - 1) * S:n * S], acts[:n].reshape(-1), n,
                                                     traj[:n * S], ex[:n * A * P], coll[:n * P], stats, None),
    "no stats": lambda n: eb.step_n_launcher(s0, traj[(n - 1) * S:n * S], acts[:n].reshape(-1), n, traj[:n * S],
                                             ex[:n * A * P], coll[:n * P], None, None),
    "state only (no traj/exec/coll/stats)": lambda n: eb.step_n_launcher(s0, out, acts[:n].reshape(-1), n),
}
vres = {}
for name, mk in variants.items():
    for n in (1, 20):
        vres[(name, n)] = (mk(n), [])
for _ in range(5):
    for (name, n), (f, v) in vres.items():
        reps = 200 if n == 1 else 50
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        v.append(e0.elapsed_time(e1) * 1e3 / reps)
for (name, n), (f, v) in vres.items():
    print("%-46s n=%3d median %8.2f us/launch" % (name, n, statistics.median(v)))
a2, b2 = eb.new_state(), eb.new_state()
eb.reset(a2)
ex1, coll1, st1 = eb.new_exec(), eb.new_coll(), eb.new_stats()
v = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(200):
        eb.step(a2, b2, acts[i % NMAX], ex1, coll1, st1)
    e1.record()
    torch.cuda.synchronize()
    v.append(e0.elapsed_time(e1) * 1e3 / 200)
print("%-46s       median %8.2f us/launch" % ("oc_step (one step, exec+coll+stats)", statistics.median(v)))
