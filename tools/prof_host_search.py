#!/usr/bin/env python3
"""cProfile of the planner's and the belief update's host side on the CPU (no GPU): bench.py's
plan_batch workload (B Level-0 searches, Chop(Tomato) by agent-1, from random-play states of
open-divider_salad) and its bayes workload (the recorded 4-agent Level-1 updates, replicated),
with the CPU oracle's rollout rows standing in for the oc_rollout launches (test
infrastructure, tests/test_planner_host.py's OracleExpander, batched per round).  Tells where
the host time goes; the oracle rows themselves show up as OracleExpander.* and are excluded.
  python tools/prof_host_search.py plan|bayes [B]"""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cooking_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

from gym_cooking_amd import capi, levels, recipes  # noqa: E402
from oracle import oracle  # noqa: E402


class BatchOracleExpander:
    """Evaluates a round's requests with one oracle rollout call over all their rows."""
    ROWS = 1 << 16

    def __init__(self, level, num_agents, device):
        self.level = levels.load_level(level) if isinstance(level, str) else level
        self.A, self.enc, self.wide = num_agents, self.level.encoding, capi.is_wide(self.level)
        self.ob = oracle.OracleBatch(self.level, num_agents, 0, 4096)
        self.K = self.ob.K
        P = capi.layout_planes(num_agents, self.K, self.wide)
        self.NP, self.t_plane = P["num_planes"], P["t"]
        self.launches = self.rows_done = 0
        self._obs = {}

    def _batch(self, n):
        pitch = capi.pitch_for(n)
        if pitch not in self._obs:
            self._obs[pitch] = oracle.OracleBatch(self.level, self.A, 0, pitch)
        return self._obs[pitch]

    busy = 0.0  # seconds inside run() over all instances: the stand-in for the GPU's share

    def run(self, requests):
        t0 = time.perf_counter()
        try:
            return self._run(requests)
        finally:
            BatchOracleExpander.busy += time.perf_counter() - t0

    def _run(self, requests):
        subs, sub_id, rows = [], {}, []
        for state, codes, sub in requests:
            key = bytes(sub)
            if key not in sub_id:
                sub_id[key] = len(subs)
                subs.append(sub)
            rows.append((state, codes, sub_id[key], sub))
        n = sum(len(r[1]) for r in rows)
        ob = self._batch(n)
        P = ob.pitch
        sin = np.zeros((self.NP, P), np.uint8)
        act = np.full((self.A, P), 4, np.uint8)
        alloc = np.zeros(P, np.uint8)
        r0 = 0
        for state, codes, si, sub in rows:
            m = len(codes)
            sin[:, r0:r0 + m] = state[:, None]
            c = np.asarray(codes, np.uint8).reshape(m, -1)
            for q in range(sub.num_agents):
                act[sub.agent[q], r0:r0 + m] = c[:, q]
            alloc[r0:r0 + m] = si
            r0 += m
        sin[self.t_plane:, :] = 0
        sout = np.zeros_like(sin)
        fl, lb = ob.rollout(sin.reshape(-1), sout.reshape(-1), act.reshape(-1), subs[:64], alloc, nthreads=4)
        assert len(subs) <= 64
        self.launches += 1
        self.rows_done += n
        out, r0 = [], 0
        for state, codes, si, sub in rows:
            m = len(codes)
            nxt = sout[:, r0:r0 + m].T.copy()
            nxt[:, self.t_plane:] = 0
            out.append((nxt, fl[r0:r0 + m], lb[r0:r0 + m]))
            r0 += m
        return out

    def bounds_many(self, states, subs):
        ob = self._batch(len(states))
        sin = np.zeros((self.NP, ob.pitch), np.uint8)
        for b, st in enumerate(states):
            sin[:, b] = st
        sin[self.t_plane:, :] = 0
        lb, ok = ob.subtask_bounds(sin.reshape(-1), subs, nthreads=4)
        return lb[:, :len(states)], ok[:, :len(states)]

    def bounds(self, state, subs):
        lb, ok = self.bounds_many([state], subs)
        return lb[:, 0], ok[:, 0]


def plan_workload(B=256, steps=12):
    from gym_cooking_amd.planner import E2E_BRTDP, PlanEnv, plan_batch
    lv = levels.load_level("open-divider_salad")
    ob = oracle.OracleBatch(lv, 2, 0, B)
    s, s2, a = ob.new_state(), ob.new_state(), ob.new_actions()
    ob.reset(s)
    for t in range(steps):
        ob.gen_actions(a, 0, t, 21)
        ob.step(s, s2, a)
        s, s2 = s2, s
    NP, P, tp = capi.layout_planes(2, ob.K)["num_planes"], ob.pitch, capi.layout_planes(2, ob.K)["t"]
    host = s.reshape(NP, P)
    tv = host[tp:tp + 2].reshape(-1).view(np.uint16)
    envs_, planners = [], []
    for b in range(B):
        by = host[:, b].copy()
        by[tp], by[tp + 1] = tv[b] & 0xFF, tv[b] >> 8
        envs_.append(PlanEnv(lv, 2, by, ["Tomato", "Lettuce", "Plate"], device="cpu"))
        planners.append(E2E_BRTDP(alpha=0.01, tau=2, cap=75, main_cap=100, device="cpu",
                                  expander=BatchOracleExpander, rng=np.random.RandomState(b)))
    return lambda: plan_batch(planners, envs_, [recipes.Chop("Tomato")] * B, [("agent-1",)] * B), planners


def bayes_workload(B=128):
    import bench
    from gym_cooking_amd.delegation import bayes_update_batch
    make, calls, fx = bench.bayes_jobs("cpu", expander=BatchOracleExpander)
    warm = [make(c) for c in calls]
    bayes_update_batch([w[0] for w in warm], [w[1] for w in warm], [w[2] for w in warm], fx["beta"])
    jobs = [make(calls[i % len(calls)]) for i in range(B)]
    return (lambda: bayes_update_batch([j[0] for j in jobs], [j[1] for j in jobs], [j[2] for j in jobs],
                                       fx["beta"])), [j[0].planner for j in jobs]


def main():
    what = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    if what == "plan":
        run, planners = plan_workload(B)
    elif what == "bayes":
        run, planners = bayes_workload(B)
    else:
        raise SystemExit("unknown workload")
    if len(sys.argv) > 3 and sys.argv[3] == "time":  # no profiler: host seconds outside the expander
        t0 = time.perf_counter()
        run()
        dt = time.perf_counter() - t0
        exp = planners[0]._exp
        print("%s: %d in %.2f s, host %.2f s (%.1f per s), %d rounds, %d rows" % (
            what, B, dt, dt - BatchOracleExpander.busy, B / (dt - BatchOracleExpander.busy), exp.launches,
            exp.rows_done))
        return
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    run()
    pr.disable()
    dt = time.perf_counter() - t0
    exp = planners[0]._exp
    print("%s: %d in %.2f s (%d rounds, %d rows)" % (what, B, dt, exp.launches, exp.rows_done))
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_stats(40)
    print(s.getvalue())


if __name__ == "__main__":
    main()
