#!/usr/bin/env python3
"""Benchmark: batched Overcooked env-steps/s on MI355X (BASELINE.json metric).

Workload (BASELINE configs[1]/[3]): partial-divider_salad, 2 agents, 2^20 envs per GPU,
synthetic i.i.d. uniform actions from the counter RNG (materialised in HBM before the timed
region, one buffer per step), max_T = 100 with next-step auto-reset.  A "step" = one
oc_step launch over the whole per-GPU batch: reads the 17-B state + 2 action bytes per env,
writes the next state, the executed actions, the collision mask and per-block episode
statistics.  The K timed steps are replayed from a hipGraph (launch-bound loop), bracketed by
a barrier + synchronize; the episode summaries are all-gathered (RCCL) inside the window.

Run:  python bench.py [--gpus N --steps K --warmup W]
      (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))

import torch  # noqa: E402

from gym_cooking_amd import dist as ocdist  # noqa: E402
from gym_cooking_amd import levels  # noqa: E402

METRIC = "env-steps/sec (whole node), 2-agent partial-divider_salad, batch=2^20"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def algorithmic_bytes_per_env_step(A: int, K: int = 4) -> int:
    """B_step = 2*S + 2A + 1, S = 3A + 2K + 3 (state read + write, actions in,
    executed actions out, collision mask)."""
    S = 3 * A + 2 * K + 3
    return 2 * S + 2 * A + 1


def cpu_baseline(level_name: str, A: int, B: int, max_T: int, budget_s: float, threads: int) -> dict:
    """The CPU oracle (a scalar C restatement of the reference step, oracle/oc_oracle.c) on a
    bounded sample of the same workload, threaded over `threads` host cores."""
    sys.path.insert(0, ROOT)
    from oracle import oracle  # cpu_baseline leg only
    lv = levels.load_level(level_name)
    ob = oracle.OracleBatch(lv, A, max_T, B)
    s, s2 = ob.new_state(), ob.new_state()
    ob.reset(s)
    act = ob.new_actions()
    steps, t_step = 0, 0.0
    t_begin = time.perf_counter()
    while time.perf_counter() - t_begin < budget_s and steps < 2000:
        ob.gen_actions(act, 0, steps, 0)  # untimed, like the GPU side
        t0 = time.perf_counter()
        ob.step(s, s2, act, None, None, nthreads=threads)
        t_step += time.perf_counter() - t0
        s, s2 = s2, s
        steps += 1
    return {"value": B * steps / t_step, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": "%d envs x %d steps of %s %d-agent (oracle/oc_oracle.c, %d threads)"
                      % (B, steps, level_name, A, threads)}


def measure_fused(eb, acts, n, dev, world) -> dict:
    """Secondary line: the same n steps as ONE oc_step_n call (state kept in registers between
    steps), still writing every step's full state (trajectory), executed actions and collision
    mask.  Algorithmic bytes per env-step: S/n (state in) + S (trajectory) + A (actions in) +
    A (exec) + 1 (coll)."""
    P, S, A = eb.pitch, eb.layout.state_bytes, eb.A
    s0, out = eb.new_state(), eb.new_state()
    eb.reset(s0)
    traj = torch.empty(n * S, dtype=torch.uint8, device=dev)
    ex = torch.empty(n * A * P, dtype=torch.uint8, device=dev)
    coll = torch.empty(n * P, dtype=torch.uint8, device=dev)
    stats = eb.new_stats()
    flat = acts.reshape(-1)
    eb.step_n(s0, out, flat, n, traj, ex, coll, stats)  # warm
    torch.cuda.synchronize()
    ocdist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eb.step_n(s0, out, flat, n, traj, ex, coll, stats)
    e1.record()
    torch.cuda.synchronize()
    ms = ocdist.max_over_ranks(e0.elapsed_time(e1) * 1e-3, dev) * 1e3
    nS = eb.layout.num_planes  # bytes per env of state = planes (t counts 2)
    bytes_env_step = nS / n + nS + 2 * A + 1
    gbs = bytes_env_step * eb.B * n / (ms * 1e-3) / 1e9
    del traj, ex, coll
    return {"value": world * eb.B * n / (ms * 1e-3), "unit": "env-steps/s", "steps": n, "ms_per_step": ms / n,
            "kernel": "oc_step_n_kernel<%d,%d>" % (A, eb.K), "algorithmic_bytes_per_env_step": bytes_env_step,
            "achieved_GBs": gbs, "frac": gbs / HBM_PEAK_GBS,
            "outputs": "every step's state (trajectory), executed actions and collision mask written"}


# Salad recipe subtasks (recipe_planner: Chop x2, Merge x6, Deliver) as oc_subtask masks:
# (kind, start masks, goal mask); agents are filled in per allocation.
SALAD_SUBTASKS = [(1, (0x01, 0), 0x11), (1, (0x02, 0), 0x22),
                  (2, (0x11, 0x22), 0x33), (2, (0x11, 0x08), 0x19), (2, (0x22, 0x08), 0x2A),
                  (2, (0x33, 0x08), 0x3B), (2, (0x19, 0x22), 0x3B), (2, (0x2A, 0x11), 0x3B),
                  (3, (0x3B, 0), 0x3B)]


def measure_rollout(dev, world, rows: int = 1 << 18, reps: int = 20) -> dict:
    """Secondary line, config C5: navigation-planner rollout rows (oc_rollout) on
    full-divider_salad with 4 agents.  Row states are mid-episode random-play states; each
    row gets a random (subtask, 1-2 agent) allocation out of the Salad subtasks x every agent
    set, and a random joint action.  Algorithmic bytes per row: 2S(4) + 4 actions
    + 1 alloc id + 4 f32 bound = 55 (+1 flags byte written)."""
    import itertools
    from gym_cooking_amd import capi
    from gym_cooking_amd.engine import OvercookedBatch
    A = 4
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
    alloc = torch.randint(0, len(table), (eb.pitch,), dtype=torch.uint8, device=dev, generator=gen)
    eb.gen_actions(a, 99, 12)
    out = eb.new_state()
    flags = torch.empty(eb.pitch, dtype=torch.uint8, device=dev)
    lb = torch.empty(eb.pitch, dtype=torch.float32, device=dev)
    for _ in range(2):
        eb.rollout(s, out, a, table, alloc, flags, lb)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        eb.rollout(s, out, a, table, alloc, flags, lb)
    e1.record()
    torch.cuda.synchronize()
    ms = ocdist.max_over_ranks(e0.elapsed_time(e1) / reps * 1e-3, dev) * 1e3
    nbytes = 55 * rows
    legal = int((flags[:rows] & capi.ROLL_LEGAL).ne(0).sum())
    return {"value": world * rows / (ms * 1e-3), "unit": "rollout rows/s", "rows_per_gpu": rows,
            "ms_per_launch": ms, "kernel": "oc_rollout_kernel<4,4>",
            "workload": "C5: full-divider_salad 4 agents, %d Salad (subtask, agents) configs, random joint actions"
                        % len(table),
            "algorithmic_bytes_per_row": 55, "achieved_GBs": nbytes / (ms * 1e-3) / 1e9,
            "frac_hbm": nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "legal_rows": legal}


def load_traffic(path: str):
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    except (OSError, ValueError):
        return None, None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--level", default="partial-divider_salad")
    ap.add_argument("--agents", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1 << 20, help="envs per GPU")
    ap.add_argument("--max-T", type=int, default=100)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of a hipGraph")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of CPU-baseline sampling")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fused", action="store_true", help="skip the secondary oc_step_n measurement")
    ap.add_argument("--no-rollout", action="store_true", help="skip the secondary oc_rollout (C5) measurement")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    args = ap.parse_args()

    rank, world, local = ocdist.world_from_env()
    if world != args.gpus:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    ocdist.init("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from gym_cooking_amd.engine import OvercookedBatch  # raises without liboc_engine.so

    sh = ocdist.shard(args.batch, rank, world, local)
    eb = OvercookedBatch(args.level, args.agents, sh.batch, max_T=args.max_T, device=dev)
    K, W = args.steps, args.warmup
    s_a, s_b = eb.new_state(), eb.new_state()
    eb.reset(s_a)
    exe, coll, stats = eb.new_exec(), eb.new_coll(), eb.new_stats()
    n_act = K + (K % 2)  # even ring: the graph ends on the buffer it started from
    acts = torch.empty((n_act, eb.A * eb.pitch), dtype=torch.uint8, device=dev)
    for i in range(n_act):
        eb.gen_actions(acts[i], step=i, seed=args.seed, env_offset=sh.env_offset)

    def run_steps(n, events=None):
        for i in range(n):
            src, dst = (s_a, s_b) if i % 2 == 0 else (s_b, s_a)
            if events is not None:
                events[i][0].record()
            eb.step(src, dst, acts[i % n_act], exe, coll, stats)
            if events is not None:
                events[i][1].record()

    # warmup (eager), even count so the state is back in s_a
    run_steps(W + (W % 2))
    torch.cuda.synchronize()

    graph = None
    if not args.no_graph:
        graph = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(device=dev)
        cap.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.graph(graph, stream=cap):
            run_steps(n_act)
        torch.cuda.synchronize()
        graph.replay()  # one untimed replay
        torch.cuda.synchronize()
    # warm the summary path (reduce kernel + all-gather) so no first-use cost lands in the window
    ocdist.gather_summaries(eb.reduce_stats(stats))
    torch.cuda.synchronize()
    stats.zero_()

    # ---------------- timed region ----------------
    ocdist.barrier()
    torch.cuda.synchronize()
    ev0, ev1, ev2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    t0 = time.perf_counter()
    ev0.record()
    if graph is not None:
        graph.replay()
    else:
        run_steps(n_act)
    ev1.record()
    totals = eb.reduce_stats(stats)
    gathered = ocdist.gather_summaries(totals)
    ev2.record()
    torch.cuda.synchronize()
    ocdist.barrier()
    elapsed = time.perf_counter() - t0
    # ----------------------------------------------
    elapsed_max = ocdist.max_over_ranks(elapsed, dev)
    gpu_ms = ev0.elapsed_time(ev2)
    steps_ms = ev0.elapsed_time(ev1)
    summary = ocdist.summarize(gathered)

    # Dominant-kernel duration, live: HIP events on the launch stream bracket the K step
    # kernels of the timed window (graph replay: kernels back to back, no host gaps), so
    # window / K is the mean oc_step_kernel duration.  Eager mode also reports per-launch
    # event pairs (which add the event packets' own ~2 us).
    kern_ms = steps_ms / n_act
    kern_ms_pairs = None
    if graph is None:
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_act)]
        run_steps(n_act, evs)
        torch.cuda.synchronize()
        durs = sorted(a.elapsed_time(b) for a, b in evs)
        kern_ms_pairs = durs[len(durs) // 2]

    steps_done = n_act
    value = world * sh.batch * steps_done / elapsed_max
    bytes_step = algorithmic_bytes_per_env_step(args.agents, eb.K)
    achieved_gbs = bytes_step * sh.batch / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = load_traffic(args.traffic_json)
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": steps_done,
        "warmup": W,
        "ms_per_step": elapsed_max * 1e3 / steps_done,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (counter-RNG uniform actions; level template broadcast)",
        "config": {
            "workload": "%s %d-agent env step, %d envs per GPU, max_T %d, next-step auto-reset"
                        % (args.level, args.agents, sh.batch, args.max_T),
            "level": args.level, "num_agents": args.agents, "batch_per_gpu": sh.batch,
            "global_batch": world * sh.batch, "parallelism": "dp%d (env shards, no data-path collective)" % world,
            "launch": "eager" if graph is None else "hipGraph of %d steps" % n_act,
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
            "kernel": "oc_step_kernel<2,4>", "algorithmic_bytes_per_env_step": bytes_step,
            "kernel_ms_mean": kern_ms, "kernel_ms_event_pairs_median": kern_ms_pairs,
            "traffic_source": traffic_src,
        },
        "gpu_ms_timed_region": gpu_ms,
        "episodes": summary,
    }
    if not args.no_fused:
        line["fused_multi_step"] = measure_fused(eb, acts, n_act, dev, world)
    if not args.no_rollout:
        line["rollout"] = measure_rollout(dev, world)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        line["cpu_baseline"] = cpu_baseline(args.level, args.agents, sh.batch, args.max_T, args.cpu_budget, threads)
    elif rank == 0:
        line["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(line), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
