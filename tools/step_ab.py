"""A/B of the step_n kernel between two builds of liboc_engine.so, on one box.

Each measurement runs in a fresh process (the binding caches its library), alternating the
builds: per configuration the mean oc_step_n launch time of back-to-back launches (HIP
events on the launch stream), the same launch shape as bench.py (every step's state,
executed actions and collision mask written; the statistics folded into totals).
  python tools/step_ab.py --libs A.so B.so [--rounds 3] [--per-step]
With --per-step: hipGraphs of 20 oc_step launches (bench.py's per_step_launch shape).
Prints one JSON line per (round, lib, config)."""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = [("partial-divider_salad", 2, 20), ("partial-divider_salad", 2, 100), ("full-divider_tl", 3, 100),
           ("full-divider_salad", 4, 100)]
PER_STEP_CONFIGS = [("partial-divider_salad", 2, 20), ("full-divider_tl", 3, 20)]


def child(lib, level, A, n, B, reps):
    sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))
    import torch
    from gym_cooking_amd import capi
    capi.load_library(lib)
    from gym_cooking_amd.engine import OvercookedBatch
    eb = OvercookedBatch(level, A, B, max_T=100, device="cuda:0")
    P, S = eb.pitch, eb.layout.state_bytes
    acts = torch.empty((n, A * P), dtype=torch.uint8, device="cuda:0")
    for i in range(n):
        eb.gen_actions(acts[i], step=i, seed=0)
    traj = torch.empty(n * S, dtype=torch.uint8, device="cuda:0")
    ex = torch.empty(n * A * P, dtype=torch.uint8, device="cuda:0")
    coll = torch.empty(n * P, dtype=torch.uint8, device="cuda:0")
    s0, stats = eb.new_state(), eb.new_stats()
    tot = torch.zeros(5, dtype=torch.int64, device="cuda:0")
    eb.reset(s0)
    f = eb.step_n_launcher(s0, traj[(n - 1) * S:], acts.reshape(-1), n, traj, ex, coll, stats, tot)
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nS = eb.layout.num_planes
    gbs = (nS + n * (nS + 2 * A + 1)) * B / (ms * 1e-3) / 1e9
    print(json.dumps({"lib": os.path.basename(lib), "level": level, "A": A, "n": n, "ms": ms,
                      "us_per_step": ms * 1e3 / n, "frac": gbs / 8000.0, "totals": tot.tolist()}), flush=True)


def child_per_step(lib, level, A, n, B, reps):
    """bench.py's per_step_launch shape: a hipGraph of n oc_step launches (ping-pong states,
    executed actions, collision mask and statistics written), replayed `reps` times."""
    sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))
    import torch
    from gym_cooking_amd import capi
    capi.load_library(lib)
    from gym_cooking_amd.engine import OvercookedBatch
    eb = OvercookedBatch(level, A, B, max_T=100, device="cuda:0")
    acts = torch.empty((n, A * eb.pitch), dtype=torch.uint8, device="cuda:0")
    for i in range(n):
        eb.gen_actions(acts[i], step=i, seed=0)
    s_a, s_b = eb.new_state(), eb.new_state()
    eb.reset(s_a)
    exe, coll, stats = eb.new_exec(), eb.new_coll(), eb.new_stats()

    def run_steps():
        for i in range(n):
            src, dst = (s_a, s_b) if i % 2 == 0 else (s_b, s_a)
            eb.step(src, dst, acts[i], exe, coll, stats)

    run_steps()
    torch.cuda.synchronize()
    graph, cap = torch.cuda.CUDAGraph(), torch.cuda.Stream(device="cuda:0")
    cap.wait_stream(torch.cuda.current_stream("cuda:0"))
    with torch.cuda.graph(graph, stream=cap):
        run_steps()
    torch.cuda.synchronize()
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        graph.replay()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    gbs = (2 * eb.layout.num_planes + 3 * A + 1) * B / (ms / n * 1e-3) / 1e9
    print(json.dumps({"lib": os.path.basename(lib), "mode": "per_step_graph", "level": level, "A": A, "n": n, "ms": ms,
                      "us_per_step": ms * 1e3 / n, "frac": gbs / 8000.0,
                      "checksum": int(eb.checksum(s_a)) if hasattr(eb, "checksum") else None}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--child", nargs=4)
    ap.add_argument("--agents", type=int, nargs="*", help="only the configurations with these agent counts")
    ap.add_argument("--per-step", action="store_true", help="time hipGraphs of 20 oc_step launches instead")
    a = ap.parse_args()
    if a.child:
        lib, level, A, n = a.child
        if a.per_step:
            return child_per_step(lib, level, int(A), int(n), a.batch, a.reps)
        return child(lib, level, int(A), int(n), a.batch, a.reps)
    for r in range(a.rounds):
        for level, A, n in (PER_STEP_CONFIGS if a.per_step else CONFIGS):
            if a.agents and A not in a.agents:
                continue
            for lib in a.libs:
                out = subprocess.run([sys.executable, __file__, "--batch", str(a.batch), "--reps", str(a.reps)] +
                                     (["--per-step"] if a.per_step else []) +
                                     ["--child", os.path.abspath(lib), level, str(A), str(n)],
                                     capture_output=True, text=True, timeout=300)
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
