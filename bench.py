#!/usr/bin/env python3
"""Benchmark: batched Overcooked env-steps/s on MI355X (BASELINE.json metric).

Workload (BASELINE configs[1]/[3]): partial-divider_salad, 2 agents, 2^20 envs per GPU,
synthetic i.i.d. uniform actions from the counter RNG (materialised in HBM before the timed
region, one buffer per step), max_T = 100 with next-step auto-reset.

A "step" is one pass of the env transition over the whole per-GPU batch.  Every step reads
that step's actions and writes the step's full next state, executed actions and collision
mask to HBM, and accumulates the episode statistics.  The headline runs the K timed steps as
multi-step launches (oc_step_n, <= 100 steps per launch; the state stays in registers
between the steps of a launch, SURVEY 8(d) "a multi-step launch that still writes every
step's state"), with its own algorithmic bytes per env-step S*launches/K + S + 2A + 1.
The one-launch-per-step path (oc_step in a hipGraph, 2S + 2A + 1 bytes) is reported beside it
as "per_step_launch".  The timed region is bracketed by a barrier + synchronize on both
sides (timed_window: the closing barrier follows the rank's clock read); the per-GPU episode
summaries are all-gathered (RCCL) inside it, and `value` uses the max over ranks.

Run:  python bench.py [--gpus N --steps K --warmup W]
      N>1 starts N ranks itself (child processes joining a TCPStore this process hosts on
      127.0.0.1); under an external torchrun (WORLD_SIZE set) it runs as the given rank.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
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


# Salad recipe subtasks (recipe_planner: Chop x2, Merge x6, Deliver) as oc_subtask masks:
# (kind, start masks, goal mask); agents are filled in per allocation.
SALAD_SUBTASKS = [(1, (0x01, 0), 0x11), (1, (0x02, 0), 0x22),
                  (2, (0x11, 0x22), 0x33), (2, (0x11, 0x08), 0x19), (2, (0x22, 0x08), 0x2A),
                  (2, (0x33, 0x08), 0x3B), (2, (0x19, 0x22), 0x3B), (2, (0x2A, 0x11), 0x3B),
                  (3, (0x3B, 0), 0x3B)]


def time_launches(launch, reps: int, dev) -> float:
    """Mean duration (ms, max over ranks) of one kernel launch: `reps` launches of a pre-bound
    launcher (engine.*_launcher: one ctypes call each, no per-call validation or table
    packing) back to back between two HIP events on the launch stream.  The host enqueues a
    launch in a few microseconds, faster than the kernels run, so the queue never drains and
    the events bracket kernel time (rocprofv3's kernel-trace mean agrees: profiles/r04/c5/)."""
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    return ocdist.max_over_ranks(e0.elapsed_time(e1) / reps * 1e-3, dev) * 1e3


def measure_rollout(dev, world, rows: int = 1 << 18, reps: int = 200) -> dict:
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
    # Rows are configuration-major (the ids sorted: each configuration's rows contiguous), the
    # order in which the reference's delegator evaluates them (bayesian_delegator.py:1026-1072:
    # for each subtask allocation, for each agent) and in which planner.py / delegation.py batch
    # them.  The same ids in random row order are timed beside it ("random_order"): waves then
    # mix configurations and diverge (profiles/r02/pmc_c5.json: 17 % active lanes per VALU op).
    rnd = torch.randint(0, len(table), (eb.pitch,), dtype=torch.uint8, device=dev, generator=gen)
    alloc = torch.sort(rnd)[0].contiguous()
    eb.gen_actions(a, 99, 12)
    out = eb.new_state()
    flags = torch.empty(eb.pitch, dtype=torch.uint8, device=dev)
    lb = torch.empty(eb.pitch, dtype=torch.float32, device=dev)

    def time_rollout(al):
        return time_launches(eb.rollout_launcher(s, out, a, table, al, flags, lb), reps, dev)

    ms_rnd = time_rollout(rnd)
    ms = time_rollout(alloc)
    nbytes = 55 * rows
    legal = int((flags[:rows] & capi.ROLL_LEGAL).ne(0).sum())
    # the planner's own launch shape: planner.py / delegation.py send at most 4,096 rows per
    # oc_rollout launch (64 waves); the first 4,096 C5 rows, configuration-major
    small = 4096
    eb4 = OvercookedBatch("full-divider_salad", A, small, max_T=100, device=dev)
    NP = eb.layout.num_planes
    s4 = s.view(NP, eb.pitch)[:, :small].contiguous().view(-1)
    a4 = a.view(A, eb.pitch)[:, :small].contiguous().view(-1)
    al4 = torch.sort(rnd[:small])[0].contiguous()
    o4, f4 = eb4.new_state(), torch.empty(eb4.pitch, dtype=torch.uint8, device=dev)
    lb4 = torch.empty(eb4.pitch, dtype=torch.float32, device=dev)
    ms_small = time_launches(eb4.rollout_launcher(s4, o4, a4, table, al4, f4, lb4), 400, dev)
    lik = measure_likelihood(eb, s, a, table, alloc, dev, world)
    lik["random_order"] = measure_likelihood(eb, s, a, table, rnd, dev, world)["ms_per_launch"]
    bnd = measure_bounds(eb, s, table, dev, world)
    return {"value": world * rows / (ms * 1e-3), "unit": "rollout rows/s", "rows_per_gpu": rows, "likelihood": lik,
            "subtask_bounds": bnd,
            "ms_per_launch": ms, "kernel": "oc_rollout_kernel<4,4>",
            "workload": "C5: full-divider_salad 4 agents, %d Salad (subtask, agents) configs, random joint actions, "
                        "rows configuration-major" % len(table),
            "algorithmic_bytes_per_row": 55, "achieved_GBs": nbytes / (ms * 1e-3) / 1e9,
            "frac_hbm": nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "legal_rows": legal,
            "random_order": {"ms_per_launch": ms_rnd, "value": world * rows / (ms_rnd * 1e-3)},
            "planner_shape": {"rows": small, "ms_per_launch": ms_small,
                              "note": "the planner's launch size (<= 4,096 rows), back-to-back launches"}}


def measure_likelihood(eb, states, taken, table, alloc, dev, world, reps: int = 40) -> dict:
    """C5's consumer: Bayesian-delegation likelihoods (oc_nav_likelihood, prob_nav_actions with
    value_init values) of the same rows -- every legal candidate action of a row is a rollout."""
    from gym_cooking_amd import capi
    v = torch.empty(eb.pitch, dtype=torch.float64, device=dev)
    f = torch.empty(eb.pitch, dtype=torch.uint8, device=dev)
    ms = time_launches(eb.nav_likelihood_launcher(states, taken, table, 0, 1.3, 0.5, alloc, v, f), reps, dev)
    ok = int((f[:eb.B] == capi.LIK_OK).sum())
    return {"value": world * eb.B / (ms * 1e-3), "unit": "likelihood rows/s", "ms_per_launch": ms,
            "kernel": "oc_likelihood_compact_kernel<4,4>", "rows_computed": ok, "bound": "divergence + latency "
            "(the wave's candidate rollouts one per lane, compacted; the rollouts' own paths differ; DESIGN.md 3.4)"}


def measure_bounds(eb, states, table, dev, world, reps: int = 60) -> dict:
    """C5's prior setup: full-state subtask bounds + allocation feasibility (oc_subtask_bounds,
    get_lower_bound_for_subtask_given_objs / subtask_alloc_is_doable) of every env x every
    configuration of the table.  Algorithmic bytes per env: S(4) = 23 state bytes read + 5 B
    (f32 bound, u8 doable) written per configuration."""
    lb = torch.empty((len(table), eb.pitch), dtype=torch.float32, device=dev)
    ok = torch.empty((len(table), eb.pitch), dtype=torch.uint8, device=dev)
    ms = time_launches(eb.subtask_bounds_launcher(states, table, lb, ok), reps, dev)
    cells = eb.B * len(table)
    nbytes = eb.B * (23 + 5 * len(table))
    return {"value": world * cells / (ms * 1e-3), "unit": "(env, configuration) bounds/s", "ms_per_launch": ms,
            "kernel": "oc_bounds_kernel<4,4>", "envs": eb.B, "configurations": len(table),
            "doable": int(ok[:, :eb.B].sum()), "achieved_GBs": nbytes / (ms * 1e-3) / 1e9,
            "bound": "compute (LDS distance-table walk per configuration)"}


def measure_render(dev, world, level: str, A: int, B: int = 1024, reps: int = 10) -> dict:
    """Secondary line, SURVEY 8(f) #4: image observations (oc_render, GameImage.get_image_obs)
    of B mid-episode random-play states.  Algorithmic bytes per image: the u8 [H*80, W*80, 3]
    output plus the env's state bytes (the static level image and sprites are L2-resident
    and read by every env)."""
    from gym_cooking_amd.engine import OvercookedBatch
    from gym_cooking_amd.render import Renderer
    eb = OvercookedBatch(level, A, B, max_T=100, device=dev)
    s, s2 = eb.new_state(), eb.new_state()
    eb.reset(s)
    a = eb.new_actions()
    for t in range(37):
        eb.gen_actions(a, t, 13)
        eb.step(s, s2, a)
        s, s2 = s2, s
    rd = Renderer(eb)
    out = rd.new_images()
    for _ in range(2):
        rd.render(s, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        rd.render(s, out)
    e1.record()
    torch.cuda.synchronize()
    ms = ocdist.max_over_ranks(e0.elapsed_time(e1) / reps * 1e-3, dev) * 1e3
    img_bytes = out[0].numel()
    nbytes = B * (img_bytes + eb.layout.num_planes)
    gbs = nbytes / (ms * 1e-3) / 1e9
    return {"value": world * B / (ms * 1e-3), "unit": "images/s", "envs_per_gpu": B, "ms_per_launch": ms,
            "kernel": "oc_render_kernel<%d,%d>" % (A, eb.K), "image_shape": list(out.shape[1:]),
            "algorithmic_bytes_per_image": img_bytes + eb.layout.num_planes, "achieved_GBs": gbs,
            "frac_hbm": gbs / HBM_PEAK_GBS, "bound": "hbm (writes)"}


def load_traffic(path: str, kernel: str = "oc_step_n_kernel", steps_per_launch=None, algorithmic=None):
    """Calibrated HBM bytes per launch of `kernel` (tools/pmc_report.py's output) for the timed
    launch shape: the PMC record of exactly `steps_per_launch` steps when profiles/ holds one,
    else the nearest recorded shape's traffic/algorithmic ratio applied to this launch's
    algorithmic bytes (the source says so).  Returns (bytes or None, source)."""
    try:
        with open(path) as f:
            d = json.load(f)
        k = d[kernel]
    except (OSError, ValueError, KeyError):
        return None, None
    src = os.path.relpath(path, ROOT)
    if steps_per_launch is None:
        return k["hbm_bytes_per_launch"], src
    shapes = {int(n): v for n, v in k.get("by_steps_per_launch", {}).items()}
    if steps_per_launch in shapes:
        return shapes[steps_per_launch]["hbm_bytes_per_launch"], "%s [%s, %d steps/launch]" % (src, kernel,
                                                                                               steps_per_launch)
    if not shapes or algorithmic is None:
        return None, None
    n0 = min(shapes, key=lambda n: abs(n - steps_per_launch))
    return (shapes[n0]["ratio"] * algorithmic,
            "%s [%s, ratio of the %d-step record x this launch's algorithmic bytes]" % (src, kernel, n0))


def measure_bayes(dev, world, n_updates: int = 256, n_seq: int = 8) -> dict:
    """Secondary line, C5's consumer: Bayesian-delegation belief updates (delegation.bayes_update,
    Level-1 inverse planning over oc_rollout, doability over oc_subtask_bounds) on the C5 layout
    (full-divider_salad, 4 agents).  The workload is the reference's own: the 4-agent updates
    recorded from it (tests/golden/bayes.json: states, executed actions, the 18 allocations of
    set_priors and their probabilities), replicated to `n_updates` delegators with their own
    planners, all updated in ONE bayes_update_batch call; `n_seq` of them are also updated one
    at a time (bayes_update) for comparison."""
    from gym_cooking_amd.delegation import bayes_update_batch
    make, calls, fx = bayes_jobs(dev)
    warm = [make(c) for c in calls]  # first use of the level: expander, library, caches
    bayes_update_batch([w[0] for w in warm], [w[1] for w in warm], [w[2] for w in warm], fx["beta"])
    jobs = [make(calls[i % len(calls)]) for i in range(n_updates)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    errs = bayes_update_batch([j[0] for j in jobs], [j[1] for j in jobs], [j[2] for j in jobs], fx["beta"])
    torch.cuda.synchronize()
    dt = ocdist.max_over_ranks(time.perf_counter() - t0, dev)
    seq = [make(calls[i % len(calls)]) for i in range(n_seq)]
    t1 = time.perf_counter()
    for d, env, acts in seq:
        d.bayes_update(obs_tm1=env, actions_tm1=acts, beta=fx["beta"])
    dts = time.perf_counter() - t1
    exp = jobs[0][0].planner._exp
    return {"value": world * n_updates / dt, "unit": "belief updates/s", "updates_per_gpu": n_updates,
            "seconds": dt, "raised": sum(e is not None for e in errs),
            "sequential": {"updates": n_seq, "value": n_seq / dts, "unit": "belief updates/s"},
            "rollout_launches_per_batch": None if exp is None else exp.launches,
            "workload": "C5 layout: full-divider_salad 4 agents, the reference's recorded 4-agent bayes_update "
                        "calls (18 allocations each, Level-1 inverse planning) replicated, one batched call"}


def bayes_jobs(dev, **planner_kw):
    """(make, calls, fixture) of the bayes line: make(call) -> (delegator, PlanEnv, executed
    actions) of one recorded 4-agent update (tests/golden/bayes.json) with a fresh planner;
    `planner_kw` goes to E2E_BRTDP (tools/prof_host_search.py passes a CPU expander)."""
    import random as _random
    import re
    import numpy as np
    from gym_cooking_amd import capi, levels as _lv, recipes
    from gym_cooking_amd.delegation import BayesianDelegator, SubtaskAllocation, SubtaskAllocDistribution
    from gym_cooking_amd.planner import E2E_BRTDP, PlanEnv
    with open(os.path.join(ROOT, "tests", "golden", "bayes.json")) as f:
        fx = json.load(f)
    cfg4 = [i for i, c in enumerate(fx["configs"]) if c["A"] == 4]
    calls = [c for c in fx["calls"] if c["cfg"] in cfg4 and c["raised"] is None]
    static = {"Counter", "Floor", "Delivery", "Cutboard"}

    def subtask(text):
        m = re.fullmatch(r"(\w+)\((.*)\)", text)
        cls = {"Chop": recipes.Chop, "Merge": recipes.Merge, "Deliver": recipes.Deliver}[m.group(1)]
        return cls(*[a.strip() for a in m.group(2).split(",")])

    def make(c):
        cfg = fx["configs"][c["cfg"]]
        lv = _lv.load_level(cfg["level"])
        A, K, P = cfg["A"], capi.item_slots(lv), capi.pitch_for(1)
        s = np.zeros(capi.layout_planes(A, K)["num_planes"], np.uint8)
        L = capi.layout_planes(A, K)
        ag, it = np.array(c["agents"], np.uint8), np.array(c["items"], np.uint8)
        s[:] = 0
        s[L["agent_x"]:L["agent_x"] + A], s[L["agent_y"]:L["agent_y"] + A] = ag[:A, 0], ag[:A, 1]
        s[L["agent_hold"]:L["agent_hold"] + A] = 0xFF
        s[L["item_loc"]:L["item_loc"] + K] = 0xFF
        held = []  # canonical rows -> slots; each holder takes the held item at its cell with its mask
        for j in range(len(it)):
            m, x, y, h = (int(v) for v in it[j])
            if m == 255:
                continue
            s[L["item_loc"] + j], s[L["item_mask"] + j] = y * lv.width + x, m
            if h:
                held.append((j, x, y, m))
        for q in range(A):
            x, y, hm = (int(v) for v in ag[q])
            if hm not in (0, 255):
                i = next(i for i, (_, ix, iy, m) in enumerate(held) if (ix, iy, m) == (x, y, hm))
                s[L["agent_hold"] + q] = held.pop(i)[0]
        env = PlanEnv(lv, A, s, [g for g in c["groups"] if g not in static], device=dev)
        planner = E2E_BRTDP(**fx["params"], rng=np.random.RandomState(c["np_seed"]), **planner_kw)
        d = BayesianDelegator(c["self"], env.get_agent_names(), "bd", planner, fx["none_action_prob"],
                              rng=_random.Random(c["random_seed"]))
        allocs = [tuple(SubtaskAllocation(None if st is None else subtask(st), tuple(a)) for st, a in rec)
                  for rec, _ in c["before"]]
        d.probs = SubtaskAllocDistribution(allocs)
        for k, (_, p) in zip(allocs, c["before"]):
            d.probs.probs[k] = p
        return d, env, {n: tuple(a) for n, a in c["actions"].items()}

    return make, calls, fx


def measure_planner(dev, world) -> dict:
    """Secondary line: the engine-backed navigation planner (gym_cooking_amd.planner.E2E_BRTDP,
    Level 0, main.py's default hyper-parameters) on C1's level: one get_next_action call from
    the reset state for Chop(Tomato) by agent-1 alone and by both agents jointly (np.random
    seeded 1).  The reference planner takes 0.31 s and 13.2 s for these two calls on the
    survey container's CPU."""
    import numpy as np
    from gym_cooking_amd import envs, recipes
    from gym_cooking_amd.planner import E2E_BRTDP
    env = envs.OvercookedEnvironment(level="open-divider_salad", num_agents=2, device=dev)
    env.reset()
    out = {}
    for tag, agn in (("single", ("agent-1",)), ("joint", ("agent-1", "agent-2"))):
        best = None
        for rep in range(3):
            p = E2E_BRTDP(alpha=0.01, tau=2, cap=75, main_cap=100, device=dev)
            np.random.seed(1)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a = p.get_next_action(env, recipes.Chop("Tomato"), agn, {})
            dt = time.perf_counter() - t0
            if best is None or dt < best[0]:
                best = (dt, a, len(p.v_l), p._exp.launches)
        out[tag] = {"ms_per_call": best[0] * 1e3, "action": list(best[1]), "states": best[2],
                    "rollout_launches": best[3]}
    # Level 1 (a Bayesian-delegation agent's call): agent-1 plans Chop(Tomato) while agent-2's
    # planner (a shallow copy, as the delegator makes it) is believed to do Chop(Lettuce).
    import copy as _copy
    best = None
    for rep in range(3):
        p = E2E_BRTDP(alpha=0.01, tau=2, cap=75, main_cap=100, device=dev)
        op = _copy.copy(p)
        op.set_settings(env, recipes.Chop("Lettuce"), ("agent-2",))
        np.random.seed(1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a = p.get_next_action(env, recipes.Chop("Tomato"), ("agent-1",), {"agent-2": op})
        dt = time.perf_counter() - t0
        if best is None or dt < best[0]:
            best = (dt, a, len(p.v_l), p._exp.launches)
    out["level1"] = {"ms_per_call": best[0] * 1e3, "action": list(best[1]), "states": best[2],
                     "rollout_launches": best[3], "other_planners": {"agent-2": "Chop(Lettuce)"}}
    out["reference_seconds_survey_container"] = {"single": 0.31, "joint": 13.2, "level1": 0.58}
    out["workload"] = "C1 level open-divider_salad, reset state, Chop(Tomato), alpha 0.01 tau 2 cap 75 main_cap 100"
    out["batch"] = measure_plan_batch(dev)
    return out


def measure_plan_batch(dev, B: int = 1024, steps: int = 12) -> dict:
    """plan_batch: B independent Level-0 searches (Chop(Tomato) by agent-1 on C1's level) from
    the states of B random-play envs after `steps` steps, each with its own RandomState; the
    searches share oc_rollout launches."""
    import numpy as np
    from gym_cooking_amd.engine import OvercookedBatch
    from gym_cooking_amd import recipes
    from gym_cooking_amd.planner import E2E_BRTDP, PlanEnv, plan_batch
    eb = OvercookedBatch("open-divider_salad", 2, B, max_T=0, device=dev)
    s, s2, a = eb.new_state(), eb.new_state(), eb.new_actions()
    eb.reset(s)
    for t in range(steps):
        eb.gen_actions(a, t, 21)
        eb.step(s, s2, a)
        s, s2 = s2, s
    NP, P, tp = eb.layout.num_planes, eb.pitch, eb.layout.plane_t
    host = s.view(NP, P).cpu().numpy()
    tv = host[tp:tp + 2].reshape(-1).view(np.uint16)
    names = ["Tomato", "Lettuce", "Plate"]
    envs_, planners = [], []
    for b in range(B):
        by = host[:, b].copy()
        by[tp], by[tp + 1] = tv[b] & 0xFF, tv[b] >> 8
        envs_.append(PlanEnv(eb.level, 2, by, names, device=dev))
        planners.append(E2E_BRTDP(alpha=0.01, tau=2, cap=75, main_cap=100, device=dev, rng=np.random.RandomState(b)))
    sub = recipes.Chop("Tomato")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    acts = plan_batch(planners, envs_, [sub] * B, [("agent-1",)] * B)
    dt = time.perf_counter() - t0
    exp = planners[0]._exp
    return {"searches": B, "seconds": dt, "plans_per_s": B / dt, "launches": exp.launches, "rows": exp.rows_done,
            "states_initialised": int(sum(len(p.v_l) for p in planners)), "none_actions": sum(x is None for x in acts),
            "workload": "B random-play states of open-divider_salad after %d steps, Chop(Tomato) by agent-1" % steps}


def measure_c3(dev, world, B: int = 1 << 20, n: int = 100, reps: int = 6, replay_reps: int = 20) -> dict:
    """Secondary line, config C3: 3-agent full-divider_tl (the collision-heavy path), 2^20 envs
    per GPU, oc_step_n launches of n steps with every step's outputs written.

    Measured the headline's way: the envs first run ten episodes and more in untimed launches
    (each on its own action stream), so the timed launches start mid-run with timeouts and
    auto-resets inside them; each timed launch continues from the previous one's last state
    and reads actions written by gen_actions just before it (fresh, never replayed).  Its
    duration is HIP events on the launch stream around it; the action generation queued just
    ahead keeps the GPU busy, so the first event does not time the host's launch call.  The
    round-4 figure (one launch replayed back to back from a reset) is kept beside it as
    `replay_from_reset`."""
    from gym_cooking_amd.engine import OvercookedBatch
    eb = OvercookedBatch("full-divider_tl", 3, B, max_T=100, device=dev)
    P, A, S = eb.pitch, eb.A, eb.layout.state_bytes
    acts = torch.empty((n, A * P), dtype=torch.uint8, device=dev)
    trajs = [torch.empty(n * S, dtype=torch.uint8, device=dev) for _ in range(2)]
    ex, coll = torch.empty(n * A * P, dtype=torch.uint8, device=dev), torch.empty(n * P, dtype=torch.uint8, device=dev)
    s, stats = eb.new_state(), eb.new_stats()
    tot = torch.zeros(5, dtype=torch.int64, device=dev)
    eb.reset(s)
    # as the headline launches it: state_out is the trajectory's last state, statistics folded
    # in-launch; consecutive launches alternate between two trajectory buffers
    fs = []
    for k in range(2):
        src = s if k == 0 else trajs[0][(n - 1) * S:]
        fs.append(eb.step_n_launcher(src, trajs[k][(n - 1) * S:], acts.reshape(-1), n, trajs[k], ex, coll, stats, tot))
    f_loop = eb.step_n_launcher(trajs[1][(n - 1) * S:], trajs[0][(n - 1) * S:], acts.reshape(-1), n, trajs[0], ex,
                                coll, stats, tot)
    stream_step = 0

    def fresh():
        nonlocal stream_step
        for i in range(n):
            eb.gen_actions(acts[i], step=stream_step + i, seed=3)
        stream_step += n

    warm = -(-(10 * 101 + 50) // n)  # ten episodes and more: the envs' phases spread over max_T + 1
    # launch i reads the state launch i-1 wrote: fs[0], fs[1], f_loop, fs[1], f_loop, ...
    order = [fs[0]] + [fs[1] if i % 2 == 1 else f_loop for i in range(1, warm + reps)]
    for f in order[:warm]:
        fresh()
        f()
    ms_l, colls = [], 0
    for f in order[warm:]:
        fresh()
        stats.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ms_l.append(e0.elapsed_time(e1))
        colls += int(tot[3])
    ms = ocdist.max_over_ranks(sum(ms_l) / len(ms_l) * 1e-3, dev) * 1e3
    # round 4's measurement: one launch from a reset, replayed back to back
    eb.reset(s)
    fresh()
    ms_rep = time_launches(fs[0], replay_reps, dev)
    nS = eb.layout.num_planes
    bytes_step = (nS + n * (nS + 2 * A + 1)) / n
    gbs = bytes_step * B * n / (ms * 1e-3) / 1e9
    return {"value": world * B * n / (ms * 1e-3), "unit": "env-steps/s", "envs_per_gpu": B, "steps": n,
            "ms_per_step": ms / n, "kernel": "oc_step_n_kernel<3,4>", "algorithmic_bytes_per_env_step": bytes_step,
            "achieved_GBs": gbs, "frac_hbm": gbs / HBM_PEAK_GBS, "timed_launches": len(ms_l),
            "ms_per_launch_each": ms_l, "collision_pairs_per_launch": colls / len(ms_l),
            "window": "mid-run after %d untimed launches, fresh actions per launch, HIP events per launch" % warm,
            "replay_from_reset": {"ms_per_step": ms_rep / n,
                                  "frac_hbm": bytes_step * B * n / (ms_rep * 1e-3) / 1e9 / HBM_PEAK_GBS},
            "workload": "C3: full-divider_tl, 3 agents, random actions"}


WIDE_LEVEL = os.path.join(ROOT, "tests", "golden", "levels", "widegraph-24x24_salad.txt")


def measure_wide(dev, world, B: int = 1 << 20, n: int = 20, reps: int = 20) -> dict:
    """Secondary line, SURVEY 8(f) #3: a wide level (more than 255 cells: u16 cell ids, the
    scalar step kernel oc_step_wide_kernel), the 24x24 Salad kitchen of tests/golden/levels,
    2 agents, 2^20 envs, one n-step oc_step_n launch with every step's outputs written (the
    headline's launch shape), replayed back to back from a mid-run state.  Algorithmic bytes
    per env-step: S/n + S + 2A + 1 with the wide layout's S = 3A + 3K + 3."""
    from gym_cooking_amd.engine import OvercookedBatch
    eb = OvercookedBatch(WIDE_LEVEL, 2, B, max_T=100, device=dev)
    P, A, S = eb.pitch, eb.A, eb.layout.state_bytes
    acts = torch.empty((n, A * P), dtype=torch.uint8, device=dev)
    for i in range(n):
        eb.gen_actions(acts[i], step=i, seed=7)
    traj = torch.empty(n * S, dtype=torch.uint8, device=dev)
    ex, coll = torch.empty(n * A * P, dtype=torch.uint8, device=dev), torch.empty(n * P, dtype=torch.uint8, device=dev)
    s, stats = eb.new_state(), eb.new_stats()
    tot = torch.zeros(5, dtype=torch.int64, device=dev)
    eb.reset(s)
    for _ in range(3):  # mid-run: 60 steps from the reset
        eb.step_n(s, traj[(n - 1) * S:], acts.reshape(-1), n, traj, ex, coll, stats)
        s.copy_(traj[(n - 1) * S:])
    f = eb.step_n_launcher(s, traj[(n - 1) * S:], acts.reshape(-1), n, traj, ex, coll, stats, tot)
    ms = time_launches(f, reps, dev)
    nS = eb.layout.num_planes
    bytes_step = (nS + n * (nS + 2 * A + 1)) / n
    gbs = bytes_step * B * n / (ms * 1e-3) / 1e9
    return {"value": world * B * n / (ms * 1e-3), "unit": "env-steps/s", "envs_per_gpu": B, "steps": n,
            "ms_per_launch": ms, "ms_per_step": ms / n, "kernel": "oc_step_wide_kernel<2,%d>" % eb.K,
            "state_bytes": nS, "algorithmic_bytes_per_env_step": bytes_step, "achieved_GBs": gbs,
            "frac_hbm": gbs / HBM_PEAK_GBS,
            "workload": "widegraph-24x24_salad (576 cells, u16 cell ids), 2 agents, random actions"}


def per_step_launch(eb, acts, n_act, W, dev, world, use_graph=True) -> dict:
    """Secondary line: one oc_step launch per step, K steps replayed from a hipGraph (or eager),
    ping-pong state buffers; kernel duration = event window / K on the launch stream."""
    s_a, s_b = eb.new_state(), eb.new_state()
    eb.reset(s_a)
    exe, coll, stats = eb.new_exec(), eb.new_coll(), eb.new_stats()

    def run_steps(n):
        for i in range(n):
            src, dst = (s_a, s_b) if i % 2 == 0 else (s_b, s_a)
            eb.step(src, dst, acts[i % n_act], exe, coll, stats)

    run_steps(W + (W % 2))
    torch.cuda.synchronize()
    graph = None
    if use_graph:
        graph = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(device=dev)
        cap.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.graph(graph, stream=cap):
            run_steps(n_act)
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
    ocdist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    if graph is not None:
        graph.replay()
    else:
        run_steps(n_act)
    e1.record()
    torch.cuda.synchronize()
    ms = ocdist.max_over_ranks(e0.elapsed_time(e1) * 1e-3, dev) * 1e3
    bytes_step = algorithmic_bytes_per_env_step(eb.A, eb.K)
    gbs = bytes_step * eb.B / (ms / n_act * 1e-3) / 1e9
    return {"value": world * eb.B * n_act / (ms * 1e-3), "unit": "env-steps/s", "steps": n_act,
            "ms_per_step": ms / n_act, "launch": "hipGraph of %d oc_step launches" % n_act if graph else "eager",
            "kernel": "oc_step_kernel<%d,%d>" % (eb.A, eb.K), "algorithmic_bytes_per_env_step": bytes_step,
            "achieved_GBs": gbs, "frac": gbs / HBM_PEAK_GBS}


def host_cores() -> dict:
    """The host cores this job may use: the CPU affinity set, capped by the cgroup CPU quota
    and by OMP_NUM_THREADS when the box sets it (the GPU pool gives each GPU's job a share of
    the machine: nproc there shows every core of the host, not the share)."""
    nproc = os.cpu_count() or 1
    share, limits = nproc, {"nproc": nproc}
    try:
        share = len(os.sched_getaffinity(0))
        limits["affinity"] = share
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
            limits["cgroup_quota"] = quota
            share = min(share, quota)
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if omp > 0:
        limits["OMP_NUM_THREADS"] = omp
        share = min(share, omp)
    return {"threads": share, "limits": limits}


def timed_window(launches, gather, sync, barrier, clock=time.perf_counter):
    """The timed region, shared by the headline window, the cold-actions window and the gloo
    self-test that pins its contents (tests/test_bench_launcher.py).

    Entry: barrier + synchronize (every rank starts from an idle GPU at the same moment).
    Inside: the window's launches, the summary all-gather (RCCL, on the launch stream), and the
    rank's closing synchronize -- nothing else.  Each rank's window ends at its own synchronize;
    the closing barrier comes after the clock is read, so it brackets the region without being
    timed (`value` takes the max over ranks of the windows, ocdist.max_over_ranks, so a barrier
    inside would only add a collective round trip to every rank's window).  Returns (seconds,
    gather's result)."""
    barrier()
    sync()
    t0 = clock()
    for f in launches:
        f()
    g = gather()
    sync()
    t1 = clock()
    barrier()
    return t1 - t0, g


class WindowLog:
    """--window-log PATH: host timestamps of the timed windows, to lay them beside a rocprofv3
    kernel trace of the same run (tools/window_split.py itemises the window's fixed cost:
    launch to kernel start, kernel, all-gather, completion seen by the host).  Each event is
    (tag, CLOCK_MONOTONIC ns, CLOCK_BOOTTIME ns): the window's start and end (the timed_window
    clock), and the moment each launch call and the all-gather call returned.  Without a path
    nothing is wrapped or recorded."""

    def __init__(self, path):
        self.path, self.events, self.win = path, [], ""

    def _mark(self, tag):
        self.events.append((self.win + ":" + tag, time.clock_gettime_ns(time.CLOCK_MONOTONIC),
                            time.clock_gettime_ns(time.CLOCK_BOOTTIME)))

    def clock(self, win):
        if self.path is None:
            return time.perf_counter
        self.win = win
        n = [0]

        def f():
            self._mark("t0" if n[0] == 0 else "t1")
            n[0] += 1
            return time.perf_counter()
        return f

    def wrap(self, launches):
        if self.path is None:
            return launches

        def w(i, fn):
            def g():
                fn()
                self._mark("launch%d_returned" % i)
            return g
        return [w(i, fn) for i, fn in enumerate(launches)]

    def dump(self, rank):
        if self.path is not None:
            with open("%s.rank%d.json" % (self.path, rank), "w") as f:
                json.dump({"events": self.events}, f)


def cpu_baseline_line(args, world: int, batch: int):
    """the C restatement timed beside the GPU line, on rank 0, at every world size.
    Its threads are the host cores this rank may use: the job's share (the CPU affinity set
    capped by the cgroup quota; the GPU pool gives each GPU's job a share of the machine, and
    nproc there counts every core of the host) divided among the job's ranks.  At N = 1 the same
    sample on nproc threads is reported beside it, labelled oversubscribed when nproc exceeds
    the share.  The sample is one rank's shard (`batch` envs), the workload one GPU runs."""
    if args.no_cpu_baseline:
        return None
    hc = host_cores()
    nproc, share = hc["limits"]["nproc"], max(1, hc["threads"] // max(1, world))
    out = cpu_baseline(args.level, args.agents, batch, args.max_T, args.cpu_budget, share)
    out["host_cpu_limits"] = hc["limits"]
    out["nproc"] = nproc
    out["ranks_sharing_the_job_cores"] = world
    if world == 1 and share != nproc:
        o = cpu_baseline(args.level, args.agents, batch, args.max_T, args.cpu_budget / 2, nproc)
        out["nproc_threads_oversubscribed"] = dict(
            {k: o[k] for k in ("value", "cores", "sample")},
            note="%d threads (nproc) on a job granted %d CPUs" % (nproc, hc["threads"]))
    out["reference_python_container"] = {
        "full_step": 695, "logic_only": 9076, "unit": "env-steps/s", "cores": 1,
        "host": "survey container (Intel Xeon, 8 cores, Python 3.10.12), not the GPU box; BASELINE.md section 2",
        "sample": "reference OvercookedEnvironment.step() on one partial-divider_salad 2-agent env; logic_only = "
                  "check_collisions + execute_navigation + done + reward without the copies"}
    return out


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` outside torchrun: start the N ranks (one process per GPU) as child
    processes and exit with their status.  The rendezvous store is a TCPStore this parent hosts
    on 127.0.0.1, bound to port 0: the kernel picks a free port at bind time and the store keeps
    it for the job, so no probe-then-bind race; the ranks join it as clients
    (TORCHELASTIC_USE_AGENT_STORE, the way torchrun's agent hands its store to workers).  The
    parent never touches the GPU, and nothing is exec'd: the ranks are fresh processes, rank 0
    prints the JSON line.  If a rank fails, the others are terminated (by their PIDs)."""
    import subprocess
    from torch.distributed import TCPStore
    store = TCPStore("127.0.0.1", 0, n, is_master=True, wait_for_workers=False)
    base = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(store.port), TORCHELASTIC_USE_AGENT_STORE="True")
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                              env=dict(base, RANK=str(r), LOCAL_RANK=str(r))) for r in range(n)]
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    del store
    return rc


def selftest_ranks(args) -> int:
    """--selftest-ranks: the launcher, shard and all-gather plumbing on gloo without any GPU
    work (tests/test_bench_launcher.py).  Every rank reports its shard, and runs timed_window
    with recording stand-ins (the launches, a real gloo all-gather of the summary row, the
    synchronize, the barrier, the clock) so the test can check what the timed region holds;
    rank 0 prints both."""
    rank, world, local = ocdist.world_from_env()
    ocdist.init("gloo")
    sh = ocdist.shard(args.batch, rank, world, local)
    g = ocdist.gather_summaries(torch.tensor([rank, world, sh.env_offset, sh.batch, os.getpid()]))
    trace = []

    def rec(tag, ret=None):
        def f():
            trace.append(tag)
            return ret() if ret is not None else None
        return f

    row = torch.tensor([rank, 1, 2, 3, 4], dtype=torch.int64)
    _, gathered = timed_window([rec("launch"), rec("launch")],
                               rec("all_gather", lambda: ocdist.gather_summaries(row)),
                               rec("synchronize"), rec("barrier", ocdist.barrier),
                               clock=lambda: trace.append("clock") or time.perf_counter())
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks": g.tolist(), "window_trace": trace,
                          "window_gathered": gathered.tolist(),
                          "cpu_baseline": cpu_baseline_line(args, world, sh.batch)}), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    return 0


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
    ap.add_argument("--steps-per-launch", type=int, default=100, help="oc_step_n launch length (headline)")
    ap.add_argument("--min-warmup-ms", type=float, default=50.0, help="repeat the untimed warmup for at least this long")
    ap.add_argument("--kernel-replay-ms", type=float, default=20.0,
                    help="after the timed region, replay its launches back to back for about this long between "
                         "two HIP events to measure the dominant kernel's mean launch duration")
    ap.add_argument("--window-actions", choices=("fresh", "replay"), default="fresh",
                    help="fresh: the window's actions are written by gen_actions just before it; replay: the "
                         "window's launches run once, untimed, just before it (both leave them cache-resident)")
    ap.add_argument("--no-graph", action="store_true", help="per-step line: eager launches instead of a hipGraph")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of CPU-baseline sampling")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-per-step", action="store_true", help="skip the secondary one-launch-per-step line")
    ap.add_argument("--no-rollout", action="store_true", help="skip the secondary oc_rollout (C5) measurement")
    ap.add_argument("--no-render", action="store_true", help="skip the secondary oc_render measurement")
    ap.add_argument("--no-c3", action="store_true", help="skip the secondary C3 (3-agent full-divider_tl) line")
    ap.add_argument("--no-planner", action="store_true", help="skip the secondary navigation-planner line")
    ap.add_argument("--no-wide", action="store_true", help="skip the secondary wide-level (24x24) step line")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--host-wait", choices=("auto", "spin"), default="spin",
                    help="spin (default): hipSetDeviceFlags(hipDeviceScheduleSpin) before the device comes up, so "
                         "the window's closing synchronize spins on the completion signal; auto: the runtime's default "
                         "wait, which let the host see a ~90 us kernel's completion 20-40 us late in some windows "
                         "(profiles/r04/window_wait/)")
    ap.add_argument("--window-launch", choices=("call", "graph"), default="call",
                    help="call (default): one launch call per launch, then the all-gather call; graph: the "
                         "window's oc_step_n launches and its all-gather replayed from one hipGraph captured before "
                         "the window (round 6, measured no faster: 117.9-128.5 us windows either way over three "
                         "alternating runs each, profiles/r06/pass_b/)")
    ap.add_argument("--window-log", default=None,
                    help="write the timed windows' host timestamps to PATH.rankR.json (tools/window_split.py)")
    ap.add_argument("--selftest-ranks", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])
    rank, world, local = ocdist.world_from_env()
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    if args.selftest_ranks:
        return selftest_ranks(args)
    # stdout carries exactly one JSON line: RCCL prints its version banner to file descriptor 1
    # when the communicator comes up, so fd 1 goes to stderr and the line to a copy of stdout.
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if args.host_wait == "spin":  # torch's own HIP runtime, before anything initialises the device
        hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        if hip.hipSetDevice(ctypes.c_int(local)) != 0 or hip.hipSetDeviceFlags(ctypes.c_uint(1)) != 0:
            raise SystemExit("hipSetDeviceFlags(hipDeviceScheduleSpin) failed")
    ocdist.init("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from gym_cooking_amd.engine import OvercookedBatch  # raises without liboc_engine.so

    sh = ocdist.shard(args.batch, rank, world, local)
    eb = OvercookedBatch(args.level, args.agents, sh.batch, max_T=args.max_T, device=dev)
    K, W = args.steps, args.warmup
    P, A, S = eb.pitch, eb.A, eb.layout.state_bytes
    # pre-materialised synthetic actions, one buffer per step (untimed)
    acts = torch.empty((K, A * P), dtype=torch.uint8, device=dev)
    for i in range(K):
        eb.gen_actions(acts[i], step=i, seed=args.seed, env_offset=sh.env_offset)
    # launch plan: equal launches of <= steps_per_launch steps
    n_launch = -(-K // max(1, args.steps_per_launch))
    n_per = -(-K // n_launch)
    segs = [(i, min(n_per, K - i)) for i in range(0, K, n_per)]
    # outputs of one launch (every step's state, executed actions, collision mask), reused per launch
    # two output sets, alternated between consecutive launches (a launch starts from the previous
    # launch's last trajectory state, so the set it writes must be the other one)
    n_sets = 2
    outs = [(torch.empty(n_per * S, dtype=torch.uint8, device=dev),
             torch.empty(n_per * A * P, dtype=torch.uint8, device=dev),
             torch.empty(n_per * P, dtype=torch.uint8, device=dev)) for _ in range(n_sets)]
    s_a = eb.new_state()
    stats = eb.new_stats()
    # the rank's summary row: the OC_NSTATS totals the last launch folds in, then the GPU's PCI
    # (domain, bus, device), all-gathered through RCCL inside the window (at N=1 as well)
    # (in place: the row is this rank's slice of the gathered [world, 8] buffer)
    summary_all, summary_row = ocdist.summary_rows(5 + 3, dev)
    summary_row[5:] = ocdist.device_ident(dev).to(dev)
    totals = summary_row[:5]

    def plan(n_steps_total, act_buf):
        """The launches of a window, bound once (engine.step_n_launcher: buffers validated
        here, each launch is then one ctypes call).  A launch's state_out is its trajectory's
        last state (oc_step_n then writes the final state once), and the next launch starts
        from there.  The last launch also folds the episode statistics into `totals`
        (in-launch, no separate reduce kernel)."""
        out, src, done, li = [], s_a, 0, 0
        while done < n_steps_total:
            n = min(n_per, n_steps_total - done)
            i0 = done % K
            n = min(n, K - i0)
            traj, ex_all, coll_all = outs[li % n_sets]
            dst = traj[(n - 1) * S:n * S]
            last = done + n >= n_steps_total
            out.append(eb.step_n_launcher(src, dst, act_buf[i0:i0 + n].reshape(-1), n, traj[:n * S], ex_all,
                                          coll_all, stats, totals if last else None))
            src = dst
            done += n
            li += 1
        return out, src

    timed, _ = plan(K, acts)
    window_graph = None
    if args.window_launch == "graph":
        # The window's launches and its summary all-gather captured once as one hipGraph, so the
        # timed region holds one host call (graph launch) instead of a launch call per launch
        # plus the all-gather call.  Captured (and replayed once, untimed) here, well before the
        # window: torch's capture collects Python's garbage first, and the warmup below rewrites
        # everything the replay touched (s_a, the outputs, stats, the summary rows).
        window_graph = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(device=dev)
        cap.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.graph(window_graph, stream=cap):
            for f in plan(K, acts)[0]:  # launchers bound to the capture stream
                f()
            ocdist.gather_summaries(summary_row, summary_all)
        torch.cuda.synchronize()
        window_graph.replay()
        torch.cuda.synchronize()
    # The warmup steps its own action stream (another seed): the window never replays a launch
    # the warmup ran.  The window's actions are written just before it (untimed), as a policy
    # writes them before a step: at the driver's shape (K = 20, 42 MB) they are then
    # Infinity-Cache resident.  The same window is timed again with the actions evicted
    # (window_cold_actions).
    acts_w = torch.empty_like(acts)
    for i in range(K):
        eb.gen_actions(acts_w[i], step=i, seed=args.seed + 1, env_offset=sh.env_offset)
    # warmup 1: at least W untimed steps, rounded up to whole launches of the timed length
    # (every oc_step_n launch a profiler sees has the timed shape, summary path included), and
    # repeated for at least --min-warmup-ms so that the clocks have left their idle state
    warm, _ = plan(-(-max(W, 1) // n_per) * n_per, acts_w)
    warm_steps, t_w = 0, time.perf_counter()
    while True:
        eb.reset(s_a)
        for f in warm:
            f()
        ocdist.gather_summaries(summary_row, summary_all)
        torch.cuda.synchronize()
        warm_steps += len(warm) * n_per
        if warm_steps >= W and (time.perf_counter() - t_w) * 1e3 >= args.min_warmup_ms:
            break
    # warmup 2: the window starts where a long run is, not at a reset.  From a reset, W_run
    # steps (ten episodes and more) desynchronise the envs that finish early; W_run is chosen
    # so that the window's middle falls on the step where the timed-out episodes end (t =
    # max_T) and the one after, where they auto-reset: the window runs the rare
    # path (reset, timeout, episode statistics), at 1 step in max_T + 1 otherwise.
    period = args.max_T + 1
    w_run = max(n_per, 10 * period + (args.max_T - K // 2 if args.max_T > 0 else 0))
    eb.reset(s_a)
    chain, end = plan(w_run, acts_w)
    for f in chain:
        f()
    s_a.copy_(end)
    warm_steps += w_run
    if args.window_actions == "fresh":
        for i in range(K):  # the window's actions, written now (same values as generated above)
            eb.gen_actions(acts[i], step=i, seed=args.seed, env_offset=sh.env_offset)
    else:  # "replay": the window's own launches once, untimed (they read s_a and write outs only)
        for f in timed:
            f()
    stats.zero_()
    torch.cuda.synchronize()

    # ---------------- timed region (timed_window: launches + all-gather + synchronize) ----------
    sync = torch.cuda.synchronize
    wlog = WindowLog(args.window_log)
    if window_graph is not None:
        win_launches, win_gather = [window_graph.replay], (lambda: summary_all)
    else:
        win_launches, win_gather = timed, (lambda: ocdist.gather_summaries(summary_row, summary_all))
    elapsed, gathered = timed_window(wlog.wrap(win_launches), win_gather, sync, ocdist.barrier,
                                     clock=wlog.clock("warm"))
    # -------------------------------------------------------------------------------------------
    elapsed_max = ocdist.max_over_ranks(elapsed, dev)
    summary = ocdist.summarize(gathered)

    # Dominant kernel: oc_step_n_kernel.  Its mean launch duration is measured right after the
    # timed region with HIP events on its launch stream around replays of the timed launches
    # (same shapes, buffers and in-launch statistics fold), so the GPU queue never drains
    # between launches and the events bracket kernel time only.  Events inside the timed region
    # itself would add their own record cost (~4 us, tools/window_probe.py) to a window of one
    # ~90 us launch, and the first event would also time the host's launch call.  A one-launch
    # window is replayed back to back (each replay follows an identical launch, as the window
    # follows its warmup).  A window of several launches is replayed each time after the warmup's
    # launches, as in the timed region: back to back, its launches would alternate and stream
    # every launch's actions from HBM, while in the window the first launch reads the actions
    # the warmup left in the Infinity Cache (0.57 vs 0.44 ms per 100-step launch,
    # profiles/r02/outalias_ab.log).
    reps = max(1, int(math.ceil(args.kernel_replay_ms / max(1e-3, elapsed * 1e3))))
    if len(timed) == 1:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(reps):
            timed[0]()
        ev1.record()
        torch.cuda.synchronize()
        kern_total_ms = ev0.elapsed_time(ev1)
    else:
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for e0, e1 in evs:
            for f in warm:
                f()
            e0.record()
            for f in timed:
                f()
            e1.record()
        torch.cuda.synchronize()
        kern_total_ms = sum(e0.elapsed_time(e1) for e0, e1 in evs)
    kern_ms = ocdist.max_over_ranks(kern_total_ms / (reps * len(segs)) * 1e-3, dev) * 1e3
    # the same window with its actions evicted from the Infinity Cache (1 GiB written between)
    flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    flush.fill_(1)
    stats.zero_()
    del flush
    cold, _ = timed_window(wlog.wrap(win_launches), win_gather, sync, ocdist.barrier, clock=wlog.clock("cold"))
    cold_max = ocdist.max_over_ranks(cold, dev)
    wlog.dump(rank)
    nS = eb.layout.num_planes  # state bytes per env (the u16 t counts 2)
    bytes_launch = (nS + n_per * (nS + 2 * A + 1)) * sh.batch
    bytes_env_step = bytes_launch / (n_per * sh.batch)
    achieved_gbs = bytes_launch / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = load_traffic(args.traffic_json, "oc_step_n_kernel", n_per, bytes_launch)
    value = world * sh.batch * K / elapsed_max
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "rccl_ranks": ocdist.rccl_ranks(),
        "steps": K,
        "warmup": W,
        "ms_per_step": elapsed_max * 1e3 / K,
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
            "launch": "oc_step_n: %d launches x %d steps; every step's state, executed actions and collision "
                      "mask written to HBM" % (len(segs), n_per),
            "warmup_steps_run": warm_steps,
            "window_starts_after_steps": w_run,
            "window_actions": ("written by gen_actions just before the window (untimed)" if args.window_actions == "fresh"
                               else "read by an untimed run of the window's launches just before it") +
                              "; the warmup steps another stream",
            "host_wait": args.host_wait,
            "window_launch": ("one hipGraph (the launches + the RCCL all-gather), captured before the window"
                              if window_graph is not None else "a launch call per launch, then the all-gather call"),
        },
        "open_loop": True,
        "window_cold_actions": {
            "value": world * sh.batch * K / cold_max, "ms_per_step": cold_max * 1e3 / K,
            "note": "the same window from the same state, its actions evicted from the Infinity Cache first"},
        "roofline": {
            "bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
            "frac_wall": bytes_env_step * sh.batch * K / elapsed_max / 1e9 / HBM_PEAK_GBS,
            "frac_wall_cold": bytes_env_step * sh.batch * K / cold_max / 1e9 / HBM_PEAK_GBS,
            "kernel": "oc_step_n_kernel<%d,%d>" % (A, eb.K), "steps_per_launch": n_per,
            "algorithmic_bytes_per_launch": bytes_launch, "algorithmic_bytes_per_env_step": bytes_env_step,
            "kernel_ms_mean": kern_ms, "kernel_ms_source": ("HIP events around %d back-to-back replays of the timed "
                                                             "launch on its stream (max over ranks)" % reps
                                                             if len(timed) == 1 else
                                                             "HIP events around %d replays of the timed launches on "
                                                             "their stream, each after the warmup's launches (max "
                                                             "over ranks)" % reps), "traffic_source": traffic_src,
        },
        "episodes": summary,
    }
    if not args.no_per_step:
        n_ps = K if K % 2 == 0 or K == 1 else K - 1  # even: the replayed graph ends on its start buffer
        line["per_step_launch"] = per_step_launch(eb, acts, n_ps, W, dev, world, use_graph=not args.no_graph)
        line["per_step_launch"]["traffic"] = load_traffic(args.traffic_json, "oc_step_kernel")[0]
    if not args.no_rollout:
        line["rollout"] = measure_rollout(dev, world)
    if not args.no_render:
        line["render"] = measure_render(dev, world, args.level, args.agents)
    if not args.no_c3:
        line["c3"] = measure_c3(dev, world)
    if not args.no_wide:
        line["wide"] = measure_wide(dev, world)
    if not args.no_planner:
        line["planner"] = measure_planner(dev, world)
        line["bayes"] = measure_bayes(dev, world)
    if rank == 0:
        line["cpu_baseline"] = cpu_baseline_line(args, world, sh.batch)
    if rank == 0:
        print(json.dumps(line), file=json_out, flush=True)
    ocdist.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
