#!/usr/bin/env python3
"""One step per launch, two kernels, interleaved in one process on the bench workload
(partial-divider_salad, 2 agents, 2^20 envs, ping-pong state buffers, executed actions +
collision mask + statistics written, 20 consecutive steps per timed batch):
  oc_step    oc_step_kernel (128-thread blocks, one chunk per lane, sc1 stores)
  step_n(1)  oc_step_n with n = 1 (persistent grid of <= 5 blocks per CU, nt stores)
each both as eager back-to-back launches and replayed from a hipGraph."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))

import torch  # noqa: E402

from gym_cooking_amd.engine import OvercookedBatch  # noqa: E402

B, N = 1 << 20, 20
eb = OvercookedBatch("partial-divider_salad", 2, B, max_T=100, device="cuda:0")
A, P = eb.A, eb.pitch
acts = torch.empty((N, A * P), dtype=torch.uint8, device="cuda:0")
for i in range(N):
    eb.gen_actions(acts[i], step=i, seed=0)
sa, sb = eb.new_state(), eb.new_state()
ex, coll, stats = eb.new_exec(), eb.new_coll(), eb.new_stats()
eb.reset(sa)


def run_step():
    for i in range(N):
        src, dst = (sa, sb) if i % 2 == 0 else (sb, sa)
        eb.step(src, dst, acts[i], ex, coll, stats)


def run_step_n1():
    for i in range(N):
        src, dst = (sa, sb) if i % 2 == 0 else (sb, sa)
        eb.step_n(src, dst, acts[i], 1, None, ex, coll, stats)


# outputs agree
run_step()
ref = sa.clone()
eb.reset(sa)
run_step_n1()
torch.cuda.synchronize()
print("outputs identical" if torch.equal(ref, sa) else "OUTPUTS DIFFER")
variants = {"oc_step eager": run_step, "step_n(1) eager": run_step_n1}
s = torch.cuda.Stream()
for name, fn in list(variants.items()):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            fn()
    variants[name.replace("eager", "graph")] = g.replay
res = {k: [] for k in variants}
for _ in range(7):
    for k, f in variants.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        res[k].append(e0.elapsed_time(e1) * 1e3 / (5 * N))
for k, v in res.items():
    print("%-18s min %6.2f  median %6.2f us/step" % (k, min(v), statistics.median(v)))
