#!/usr/bin/env python3
"""Record config C1 (BASELINE.json configs[0]): the reference's own ``main.py`` loop with
greedy agents, one env on the CPU, and its full trace as a golden fixture.

Runs ONLY in the build container, where the read-only reference is mounted at
/root/reference (never on the GPU box; only ``greedy.npz`` travels).  It replays
gym_cooking/main.py:85-117 step for step -- ``fix_seed`` (:138-140), env ``reset``,
``initialize_agents`` (:52-82, RealAgent per level-file spawn line), then
``while not env.done()``: every agent's ``select_action(obs)``, ``env.step``, every agent's
``refresh_subtasks(world)`` -- with the same stubs as gen_golden.py (gym / termcolor /
pygame; ``Bag`` is skipped because it writes to a hard-coded Windows path,
misc/metrics/metrics_bag.py:9).

Recorded per step (same canonical encoding as streams.npz): the action
dict the agents chose, the executed actions, the collision-pair mask, t / done / reward
flags, agents and items; plus ``env.get_repr()`` as text after reset and after every step
(pins the shim's repr surface), ``env.all_subtasks`` and the episode's termination_info.
The greedy planners' decisions depend on the hash seed (set iteration), so the generator
pins PYTHONHASHSEED=0; the recorded actions are what the engine replays.

Usage:  PYTHONHASHSEED=0 python tests/golden/gen_greedy.py
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import random
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as gg  # noqa: E402

# (level, num_agents, seed): C1 first, then the other two recipe families on 2 agents.
EPISODES = [("open-divider_salad", 2, 1), ("open-divider_salad", 2, 2),
            ("partial-divider_tomato", 2, 1), ("open-divider_tl", 2, 1)]


def arglist_for(level, A, seed, max_T=100):
    """main.py parse_arguments() defaults (main.py:15-40) with model1..A = greedy."""
    a = argparse.Namespace(level=level, num_agents=A, max_num_timesteps=max_T, max_num_subtasks=14,
                           seed=seed, with_image_obs=False, beta=1.3, alpha=0.01, tau=2, cap=75,
                           main_cap=100, play=False, record=False,
                           model1=None, model2=None, model3=None, model4=None)
    for i in range(A):
        setattr(a, "model%d" % (i + 1), "greedy")
    return a


def initialize_agents(arglist):
    """main.py:52-82: a RealAgent per spawn line (up to num_agents), recipes from phase 2."""
    from utils.agent import RealAgent, COLORS
    import recipe_planner.recipe as rmod
    agents, recipes, phase = [], [], 1
    with open("utils/levels/{}.txt".format(arglist.level)) as f:
        for line in f:
            line = line.strip("\n")
            if line == "":
                phase += 1
            elif phase == 2:
                recipes.append(getattr(rmod, line)())
            elif phase == 3 and len(agents) < arglist.num_agents:
                agents.append(RealAgent(arglist=arglist, name="agent-" + str(len(agents) + 1),
                                        id_color=COLORS[len(agents)], recipes=recipes))
    return agents


def run_episode(ref, level, A, seed):
    arglist = arglist_for(level, A, seed)
    np.random.seed(seed)          # fix_seed, main.py:138-140
    random.seed(seed)
    OE = ref[0]
    re = gg.RefEnv.__new__(gg.RefEnv)
    re.OE, re.nav_utils, re.recipe = ref
    re.A, re.args, re.err = A, arglist, False
    quiet = contextlib.redirect_stdout(io.StringIO())
    with quiet:
        re.env = env = OE(arglist)
        obs = env.reset()
    env.game = gg._NoImage()
    with contextlib.redirect_stdout(io.StringIO()):
        agents = initialize_agents(arglist)
    states = [re.canon(0)]
    reprs = [repr(env.get_repr())]
    acts, exes, colls = [], [], []
    t0 = time.perf_counter()
    while True:
        with contextlib.redirect_stdout(io.StringIO()):
            if env.done():
                break
            action_dict = {ag.name: ag.select_action(obs=obs) for ag in agents}
        codes = [gg.CODE[tuple(action_dict["agent-%d" % (i + 1)])] for i in range(A)]
        with contextlib.redirect_stdout(io.StringIO()):
            st, ex, coll = re.step(codes)
        assert not re.err, "greedy episode hit the co-location crash"
        obs = _OBS[id(env)]  # new_obs returned by env.step (main.py:104)
        with contextlib.redirect_stdout(io.StringIO()):
            for ag in agents:
                ag.refresh_subtasks(world=env.world)
        row = np.full(gg.MAXA, gg.PAD, np.uint8)
        row[:A] = codes
        acts.append(row)
        exes.append(ex)
        colls.append(coll)
        states.append(st)
        reprs.append(repr(env.get_repr()))
    wall = time.perf_counter() - t0
    return dict(level=level, A=A, seed=seed, states=states, reprs=reprs, act=acts, exe=exes, coll=colls,
                termination_info=env.termination_info, successful=bool(env.successful),
                all_subtasks=[str(s) for s in env.all_subtasks], wall_s=wall, T=len(acts))


_OBS = {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", type=int, default=None, help="index into EPISODES")
    args = ap.parse_args()
    if os.environ.get("PYTHONHASHSEED") != "0":
        raise SystemExit("run with PYTHONHASHSEED=0 (the greedy planners iterate over sets)")
    ref = gg.load_reference()
    # env.step returns new_obs = copy.copy(env); main.py feeds that to select_action.
    OE = ref[0]
    step0 = OE.step

    def step(self, action_dict):
        out = step0(self, action_dict)
        _OBS[id(self)] = out[0]
        return out
    OE.step = step
    eps = [run_episode(ref, *EPISODES[i]) for i in ([args.only] if args.only is not None else range(len(EPISODES)))]
    # same layout as streams.npz (gen_golden.Recorder), kind "greedy"
    rec = gg.Recorder()
    meta, reprs = [], []
    for k, e in enumerate(eps):
        s0, a0 = len(rec.S["t"]), len(rec.act)
        for st in e["states"]:
            rec.add_state(st)
        rec.act += e["act"]
        rec.exe += e["exe"]
        rec.coll += e["coll"]
        rec.eps.append(dict(level=gg.LEVEL_NAMES.index(e["level"]), A=e["A"], max_T=100, kind="greedy",
                            seed=e["seed"], state_off=s0, act_off=a0, T=e["T"],
                            start=np.full((gg.MAXA, 2), gg.PAD, np.uint8)))
        meta.append(dict(level=e["level"], A=e["A"], seed=e["seed"], T=e["T"],
                         termination_info=e["termination_info"], successful=e["successful"],
                         all_subtasks=sorted(e["all_subtasks"]), reference_wall_s=round(e["wall_s"], 1)))
        reprs.append(e["reprs"])
        print("%s A=%d seed=%d: %d steps, %s (%.1f s)" % (e["level"], e["A"], e["seed"], e["T"],
                                                        e["termination_info"], e["wall_s"]))
    rec.save(os.path.join(HERE, "greedy.npz"), ["greedy"])
    with open(os.path.join(HERE, "greedy.json"), "w") as f:
        json.dump(dict(episodes=meta, reprs=reprs), f, indent=0)


if __name__ == "__main__":
    main()
