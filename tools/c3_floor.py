"""C3 floors: the 3-agent step_n launch (full-divider_tl, 2^20 envs, 100 steps) with every
output written (bench shape), with no per-step output (trajectory, executed actions and
collision masks absent: their stores are dropped), and the 2-agent headline level beside it.
Back-to-back launches timed with HIP events on the launch stream.  One JSON line per case."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))
import torch  # noqa: E402

from gym_cooking_amd.engine import OvercookedBatch  # noqa: E402


def run(level, A, n, outputs, B=1 << 20, reps=20):
    eb = OvercookedBatch(level, A, B, max_T=100, device="cuda:0")
    P, S = eb.pitch, eb.layout.state_bytes
    acts = torch.empty((n, A * P), dtype=torch.uint8, device="cuda:0")
    for i in range(n):
        eb.gen_actions(acts[i], step=i, seed=0)
    s0, s1 = eb.new_state(), eb.new_state()
    eb.reset(s0)
    if outputs:
        traj = torch.empty(n * S, dtype=torch.uint8, device="cuda:0")
        ex = torch.empty(n * A * P, dtype=torch.uint8, device="cuda:0")
        coll = torch.empty(n * P, dtype=torch.uint8, device="cuda:0")
        f = eb.step_n_launcher(s0, traj[(n - 1) * S:], acts.reshape(-1), n, traj, ex, coll)
    else:
        f = eb.step_n_launcher(s0, s1, acts.reshape(-1), n)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(json.dumps({"level": level, "A": A, "n": n, "outputs": outputs, "us_per_step": ms * 1e3 / n}), flush=True)


for rnd in range(2):
    for lv, A in (("full-divider_tl", 3), ("partial-divider_salad", 2), ("full-divider_salad", 4)):
        for out in (True, False):
            run(lv, A, 100, out)
