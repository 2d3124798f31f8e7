"""Child process of tests/test_rccl_gpu.py (a fresh interpreter, started before it touches the
GPU): RCCL at world size 1 exactly as bench.py uses it.

It joins a world-1 "nccl" process group through gym_cooking_amd.dist.init (TCP store on
127.0.0.1), steps B envs of the metric level with oc_step_n and the in-launch statistics fold,
all-gathers the summary row (totals + PCI id) through RCCL and max-reduces a float, then
prints one JSON line: the gathered row, reduce_stats of the partial buffer, and the CPU
oracle's totals for the same workload."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oc_testlib as tl  # noqa: E402
from gym_cooking_amd import dist as ocdist  # noqa: E402
from oracle import oracle  # noqa: E402

LEVEL, A, MAX_T = "partial-divider_salad", 2, 100


def main() -> int:
    B, steps, n, seed = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), 31
    for k in ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    ocdist.init("nccl")
    dev = torch.device("cuda", 0)
    from gym_cooking_amd.engine import OvercookedBatch
    eb = OvercookedBatch(LEVEL, A, B, max_T=MAX_T, device=dev)
    P = eb.pitch
    s, s2, stats = eb.new_state(), eb.new_state(), eb.new_stats()
    eb.reset(s)
    out_rows, row = ocdist.summary_rows(8, dev)  # bench.py's in-place summary buffer
    row[5:] = ocdist.device_ident(dev).to(dev)
    acts = torch.empty((n, A * P), dtype=torch.uint8, device=dev)
    for i0 in range(0, steps, n):
        m = min(n, steps - i0)
        for r in range(m):
            eb.gen_actions(acts[r], step=i0 + r, seed=seed)
        eb.step_n(s, s2, acts[:m].reshape(-1), m, None, None, None, stats, row[:5])
        s, s2 = s2, s
    gathered = ocdist.gather_summaries(row, out_rows).clone()  # ncclAllGather on this stream
    via_pg = ocdist.gather_summaries(row)  # torch's process group (all_gather_into_tensor)
    mx = ocdist.max_over_ranks(3.5, dev)
    torch.cuda.synchronize()
    reduced = eb.reduce_stats(stats).cpu().tolist()

    ob = oracle.OracleBatch(eb.level, A, MAX_T, B)
    c, c2 = ob.new_state(), ob.new_state()
    ob.reset(c)
    cact, ccoll = ob.new_actions(), np.zeros(ob.pitch, np.uint8)
    tot = np.zeros(5, np.int64)
    for t in range(steps):
        ob.gen_actions(cact, 0, t, seed)
        fl_in = tl.planes_view(c, A, ob.K, ob.pitch)["fl"].copy()
        ob.step(c, c2, cact, None, ccoll, nthreads=8)
        c, c2 = c2, c
        tot += tl.window_totals(fl_in, c, ccoll, A, ob.K, ob.pitch, B)
    state_equal = bool(np.array_equal(s.cpu().numpy()[:c.size], c))
    out = {"backend": dist.get_backend(), "world": dist.get_world_size(), "rccl_ranks": ocdist.rccl_ranks(),
           "direct": ocdist.rccl() is not None, "gathered": gathered.cpu().tolist(),
           "via_process_group": via_pg.cpu().tolist(), "reduced": reduced, "oracle": tot.tolist(), "max": mx,
           "state_equal": state_equal, "summary": ocdist.summarize(gathered)}
    ocdist.shutdown()
    print("RESULT " + json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
