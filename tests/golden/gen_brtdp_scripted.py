#!/usr/bin/env python3
"""Generate tests/golden/brtdp_scripted.json: reference navigation-planner decisions
(E2E_BRTDP.get_next_action, Level 0) along the scripted salad episodes of SURVEY App. A.9
(open-divider_salad) and A.10 (open-divider_tl), where chopped food and plated dishes exist,
so the Merge and Deliver subtasks are doable (gen_brtdp.py's goal-directed states mostly allow
Chop).  At every SAMPLE_EVERY-th step, every doable (Merge / Deliver subtask, 1-agent set) is
planned by a fresh planner, and by one planner per (subtask, agents) kept across the episode.
Same record format as gen_brtdp.py.

Usage:  PYTHONHASHSEED=0 python tests/golden/gen_brtdp_scripted.py
"""
from __future__ import annotations

import contextlib
import io
import itertools
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_brtdp as gb  # noqa: E402
import gen_golden as gg  # noqa: E402

CONFIGS = [  # (level, A, agent-1 script, agent-2 script)
    ("open-divider_salad", 2, gg.A9_AGENT1, gg.A9_AGENT2),
    ("open-divider_tl", 2, gg.TL_AGENT1, "D D" + " N" * 60),
]
SAMPLE_EVERY = 3


def main():
    ref = gg.load_reference()
    _, nav_utils, _ = ref
    from navigation_planner.planners.e2e_brtdp import E2E_BRTDP  # noqa: E402
    from delegation_planner.bayesian_delegator import BayesianDelegator  # noqa: E402

    calls = []
    t0 = time.time()
    for ci, (level, A, s1, s2) in enumerate(CONFIGS):
        env = gg.RefEnv(ref, level, A, 100)
        seqs = [[gg.LETTER[c] for c in s.split()] for s in (s1, s2)]
        rng = np.random.default_rng(4000 + ci)
        chain = {}
        for T in range(len(seqs[0])):
            if T % SAMPLE_EVERY == 0:
                names = [a.name for a in env.env.sim_agents]
                for sub in env.env.all_subtasks:
                    if type(sub).__name__ not in ("Merge", "Deliver"):
                        continue
                    for ags in itertools.combinations(range(A), 1):
                        agn = tuple(names[i] for i in ags)
                        with contextlib.redirect_stdout(io.StringIO()):
                            ok = BayesianDelegator.subtask_alloc_is_doable(None, env.env, sub, agn)
                        if not ok:
                            continue
                        for mode in ("fresh", "chain"):
                            p = (E2E_BRTDP(**gb.PARAMS) if mode == "fresh"
                                 else chain.setdefault((str(sub), agn), E2E_BRTDP(**gb.PARAMS)))
                            seed = int(rng.integers(0, 2**31 - 1))
                            rec = gb.record_call(p, env, sub, ags, agn, nav_utils, seed, ci, 0, T, mode)
                            calls.append(rec)
                            print("  call %d: cfg %d t %d %s %s %s -> %s (%.1f s, %d states)" % (
                                len(calls), ci, T, mode, sub, agn, rec["action"], rec["ref_seconds"],
                                rec["n_states"]), flush=True)
            codes = [seqs[0][T], seqs[1][T] if T < len(seqs[1]) else 4]
            st, _, _ = env.step(codes)
            if env.err or st["flags"] & 1:
                break
    out = {"configs": [{"level": c[0], "A": c[1]} for c in CONFIGS], "params": gb.PARAMS, "calls": calls}
    with open(os.path.join(HERE, "brtdp_scripted.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote %d planner calls in %.0f s" % (len(calls), time.time() - t0))


if __name__ == "__main__":
    main()
