#!/usr/bin/env python3
"""What the in-launch statistics fold costs the headline kernel: bench.py's driver shape
(partial-divider_salad, 2 agents, 2^20 envs, 20-step oc_step_n launches with trajectory,
executed actions and collision masks), timed back to back (bench.time_launches) with
  fold    stats + totals (the bench's last launch of a window: partial rows, tickets, the fold)
  stats   the partial rows only (no totals: no tickets, no fold)
  none    no statistics
  python tools/fold_probe.py [--libs A.so B.so] [--rounds 3]
One JSON line per (round, lib, mode)."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cooking_amd")]
    import torch
    from gym_cooking_amd import capi
    if lib:
        capi.load_library(lib)
    import bench
    from gym_cooking_amd.engine import OvercookedBatch
    dev = "cuda:0"
    B, A, n = 1 << 20, 2, 20
    eb = OvercookedBatch("partial-divider_salad", A, B, max_T=100, device=dev)
    s = eb.new_state()
    eb.reset(s)
    S = s.numel()
    acts = eb.new_actions(n)
    for t in range(n):
        eb.gen_actions(acts[t], t, 7)
    traj = torch.empty(n * S, dtype=torch.uint8, device=dev)
    ex = torch.empty(n * A * eb.pitch, dtype=torch.uint8, device=dev)
    coll = torch.empty(n * eb.pitch, dtype=torch.uint8, device=dev)
    stats = eb.new_stats()
    tot = torch.zeros(8, dtype=torch.int64, device=dev)
    out = {}
    for mode in ("fold", "stats", "none"):
        st = stats if mode != "none" else None
        tt = tot[:5] if mode == "fold" else None
        f = eb.step_n_launcher(s, traj[(n - 1) * S:], acts.reshape(-1), n, traj, ex, coll, st, tt)
        out[mode] = bench.time_launches(f, 400, dev) * 1e3
    print(json.dumps({"lib": os.path.basename(lib) if lib else "in-tree", **{k + "_us": v for k, v in out.items()}}),
          flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="*", default=[""])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--child")
    a = ap.parse_args()
    if a.child is not None:
        return child(a.child)
    for r in range(a.rounds):
        for lib in a.libs:
            p = subprocess.run([sys.executable, __file__, "--child", os.path.abspath(lib) if lib else ""],
                               capture_output=True, text=True, timeout=300)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            if p.returncode != 0 or not line:
                print(p.stderr[-2000:], file=sys.stderr)
                return 1
            d = json.loads(line[0])
            d["round"] = r
            print(json.dumps(d), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
