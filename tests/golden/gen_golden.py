#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the reference itself.

Runs ONLY in the build container, where the read-only reference checkout is mounted at
/root/reference (it never travels to the GPU box; the committed .npz/.json fixtures do).
The reference is pure Python; its few missing third-party imports are replaced by inert
in-process stubs (gym 0.17.2 -> a bare ``Env`` base and a no-op ``register``; termcolor
1.1.0 -> identity ``colored``; pygame 1.9.6 -> the four key constants read at import,
gym_cooking/misc/game/utils.py:11-16), exactly as SURVEY.md 8(c) prescribes.  Nothing on
the step path uses them.

What is recorded, per episode, is the *canonical* state of SURVEY App. A.7 after reset and
after every ``OvercookedEnvironment.step`` (overcooked_environment.py:255-306):
  t, flags (done / reward / ERR), agents (x, y, held-content mask), items as a sorted
  multiset of (content mask, x, y, is_held), executed actions (``env.agent_actions``,
  :770) and the collision pair mask (``env.collisions`` entries of this t, :747-752).
ERR = the step raised (two co-located agents both holding).

Usage:  python tests/golden/gen_golden.py [--quick]
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import random
import sys
import types
from collections import deque

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
LEVEL_NAMES = [
    "open-divider_salad", "open-divider_tomato", "open-divider_tl",
    "partial-divider_salad", "partial-divider_tomato", "partial-divider_tl",
    "full-divider_salad", "full-divider_tomato", "full-divider_tl",
]
NAV = [(0, 1), (0, -1), (-1, 0), (1, 0), (0, 0)]
CODE = {a: i for i, a in enumerate(NAV)}
LETTER = {"D": 0, "U": 1, "L": 2, "R": 3, "N": 4}
MAXA, MAXK = 4, 4
PAD = 255
FOODS = (("Tomato", 0x01), ("Lettuce", 0x02), ("Onion", 0x04))


# ----------------------------------------------------------------------------- reference

def load_reference():
    def mod(name):
        m = types.ModuleType(name)
        sys.modules[name] = m
        return m

    gym = mod("gym")
    gym.Env = type("Env", (), {})
    for sub in ("error", "spaces", "utils", "envs"):
        setattr(gym, sub, mod("gym." + sub))
    gym.utils.seeding = mod("gym.utils.seeding")
    gym.envs.registration = mod("gym.envs.registration")
    gym.envs.registration.register = lambda **kw: None
    mod("termcolor").colored = lambda s, *a, **k: s
    pg = mod("pygame")
    for i, k in enumerate(("K_UP", "K_DOWN", "K_RIGHT", "K_LEFT")):
        setattr(pg, k, 273 + i)
    sys.path[:0] = [REF, REF + "/gym_cooking"]
    os.chdir(REF + "/gym_cooking")  # load_level opens utils/levels/<level>.txt relative
    from envs.overcooked_environment import OvercookedEnvironment  # noqa: E402
    import navigation_planner.utils as nav_utils  # noqa: E402
    import recipe_planner.utils as recipe  # noqa: E402
    return OvercookedEnvironment, nav_utils, recipe


class _NoImage:
    def get_image_obs(self):
        return None


def content_mask(obj) -> int:
    m = 0
    for c in obj.contents:
        if c.name == "Plate":
            m |= 0x08
            continue
        for name, bit in FOODS:
            if c.name == name:
                m |= bit
                if c.get_state() == "Chopped":
                    m |= bit << 4
    return m


class RefEnv:
    """One reference OvercookedEnvironment driven by integer action codes."""

    def __init__(self, ref, level, num_agents, max_T):
        self.OE, self.nav_utils, self.recipe = ref
        import argparse as ap
        self.args = ap.Namespace(level=level, num_agents=num_agents, max_num_timesteps=max_T,
                                 max_num_subtasks=14, seed=1, with_image_obs=False, record=False,
                                 play=False, model1=None, model2=None, model3=None, model4=None)
        self.A = num_agents
        self.env = self.OE(self.args)
        with contextlib.redirect_stdout(io.StringIO()):
            self.env.reset()
        self.env.game = _NoImage()
        self.err = False

    def relocate(self, xys):
        for ag, (x, y) in zip(self.env.sim_agents, xys):
            ag.location = (x, y)

    def canon(self, flags):
        env = self.env
        agents = np.full((MAXA, 3), PAD, np.uint8)
        for i, ag in enumerate(env.sim_agents):
            agents[i] = (ag.location[0], ag.location[1], 0 if ag.holding is None else content_mask(ag.holding))
        items = []
        for key, objs in env.world.objects.items():
            for o in objs:
                if isinstance(o, self._Object):
                    items.append((content_mask(o), o.location[0], o.location[1], int(bool(o.is_held))))
        items.sort()
        assert len(items) <= MAXK
        it = np.full((MAXK, 4), PAD, np.uint8)
        for i, row in enumerate(items):
            it[i] = row
        return dict(t=env.t, flags=flags, agents=agents, items=it)

    @property
    def _Object(self):
        from utils.core import Object
        return Object

    def step(self, codes):
        env = self.env
        t_before = env.t
        action_dict = {ag.name: NAV[c] for ag, c in zip(env.sim_agents, codes)}
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                _, reward, done, _ = env.step(action_dict)
        except Exception:
            # Must be the new_obs copy crash: two co-located agents both holding.
            locs = [ag.location for ag in env.sim_agents if ag.holding is not None]
            assert len(locs) != len(set(locs)), "unexpected reference exception"
            self.err = True
            flags = 0x05
            ex = np.full(MAXA, PAD, np.uint8)
            return self.canon(flags), ex, 0
        assert env.t == t_before + 1
        flags = (1 if done else 0) | (2 if reward == 1 else 0)
        ex = np.full(MAXA, PAD, np.uint8)
        for i, ag in enumerate(env.sim_agents):
            ex[i] = CODE[tuple(env.agent_actions[ag.name])]
        names = [ag.name for ag in env.sim_agents]
        pairs = [(i, j) for i in range(self.A) for j in range(i + 1, self.A)]
        coll = 0
        for c in env.collisions:
            if c.time == env.t:
                i, j = names.index(c.agent_names[0]), names.index(c.agent_names[1])
                coll |= 1 << pairs.index((i, j))
        return self.canon(flags), ex, coll

    # ---- level export (what load_level/run_recipes built) ----
    def level_info(self):
        env = self.env
        w = env.world
        cls = {"Floor": 0, "Counter": 1, "Cutboard": 2, "Delivery": 3}
        tiles = [[None] * w.width for _ in range(w.height)]
        for key, objs in w.objects.items():
            for o in objs:
                if type(o).__name__ in cls:
                    x, y = o.location
                    assert tiles[y][x] is None
                    tiles[y][x] = cls[type(o).__name__]
        items = []
        for key, objs in w.objects.items():
            for o in objs:
                if isinstance(o, self._Object):
                    items.append((o.location[1] * w.width + o.location[0], content_mask(o)))
        items.sort()
        goals = []
        for st in env.all_subtasks:
            if isinstance(st, self.recipe.Deliver):
                _, g = self.nav_utils.get_subtask_obj(st)
                m = content_mask(g)
                if m not in goals:
                    goals.append(m)
        return dict(width=w.width, height=w.height, tiles=[t for row in tiles for t in row],
                    items=items, spawns=[list(a.location) for a in env.sim_agents],
                    goals=sorted(goals), perimeter=w.perimeter)


# ----------------------------------------------------------------------------- policies

def splitmix64(x):
    M = (1 << 64) - 1
    z = (x + 0x9E3779B97F4A7C15) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def rng_action(seed, gid, step, agent):
    """Counter RNG of include/oc_engine.h oc_gen_actions."""
    M = (1 << 64) - 1
    x = seed ^ ((gid * 0x9E3779B97F4A7C15) & M) ^ ((step * 0xC2B2AE3D27D4EB4F) & M) ^ agent
    return splitmix64(x) % 5


class GoalPolicy:
    """State-aware random policy that walks to useful counters and interacts, so that
    pick-up / put-down / chop / merge / deliver branches are exercised (uniform random
    streams almost never reach them)."""

    def __init__(self, info, A, seed, eps=0.15):
        self.W, self.H = info["width"], info["height"]
        self.tiles = info["tiles"]
        self.goals = info["goals"]
        self.A = A
        self.rng = random.Random(seed)
        self.eps = eps
        self.target = [None] * A
        self.ttl = [0] * A

    def floor(self, x, y):
        return 0 <= x < self.W and 0 <= y < self.H and self.tiles[y * self.W + x] == 0

    def path_action(self, start, goal_cell):
        gx, gy = goal_cell % self.W, goal_cell // self.W
        # adjacent: face the target
        for c, (dx, dy) in enumerate(NAV[:4]):
            if (start[0] + dx, start[1] + dy) == (gx, gy):
                return c
        goals = {(gx - dx, gy - dy) for dx, dy in NAV[:4] if self.floor(gx - dx, gy - dy)}
        prev = {start: None}
        q = deque([start])
        while q:
            cur = q.popleft()
            if cur in goals:
                while prev[cur] is not None and prev[cur][0] != start:
                    cur = prev[cur][0]
                return prev[cur][1] if prev[cur] is not None else 4
            for c, (dx, dy) in enumerate(NAV[:4]):
                n = (cur[0] + dx, cur[1] + dy)
                if n not in prev and self.floor(*n):
                    prev[n] = (cur, c)
                    q.append(n)
        return self.rng.randrange(5)

    def pick_target(self, i, st):
        ag = st["agents"][i]
        held = int(ag[2])
        items = [tuple(r) for r in st["items"] if r[0] != PAD and not r[3]]
        deliv = [c for c, t in enumerate(self.tiles) if t == 3]
        cuts = [c for c, t in enumerate(self.tiles) if t == 2]
        counters = [c for c, t in enumerate(self.tiles) if t != 0]
        cell_of = lambda r: int(r[2]) * self.W + int(r[1])
        r = self.rng.random()
        if held:
            n = bin(held & 0x0F).count("1")
            if n == 1 and held in (1, 2, 4) and r < 0.8:
                return self.rng.choice(cuts)
            if n >= 2 and (held & 0x07) & ~(held >> 4) == 0 and (held in self.goals or r < 0.3):
                if r < 0.85:
                    return self.rng.choice(deliv)
            merge_ok = [cell_of(it) for it in items if cell_of(it) not in deliv
                        and not (held & 0x08 and it[0] & 0x08)
                        and (held & 0x07) & ~(held >> 4) == 0 and (it[0] & 0x07) & ~(it[0] >> 4) == 0]
            if merge_ok and r < 0.7:
                return self.rng.choice(merge_ok)
            return self.rng.choice(counters)
        cand = [cell_of(it) for it in items if cell_of(it) not in deliv]
        if cand and r < 0.85:
            return self.rng.choice(cand)
        return self.rng.choice(counters)

    def act(self, st):
        codes = []
        for i in range(self.A):
            if self.rng.random() < self.eps:
                codes.append(self.rng.randrange(5))
                continue
            if self.target[i] is None or self.ttl[i] <= 0:
                self.target[i] = self.pick_target(i, st)
                self.ttl[i] = 20
            self.ttl[i] -= 1
            ag = st["agents"][i]
            c = self.path_action((int(ag[0]), int(ag[1])), self.target[i])
            tx, ty = int(ag[0]) + NAV[c][0], int(ag[1]) + NAV[c][1]
            if c != 4 and tx + ty * self.W == self.target[i]:
                self.target[i] = None  # interacting now; choose a new target next step
            codes.append(c)
        return codes


# ----------------------------------------------------------------------------- episodes

class Recorder:
    def __init__(self):
        self.eps = []
        self.S = {k: [] for k in ("t", "flags", "agents", "items")}
        self.act, self.exe, self.coll = [], [], []

    def add_state(self, st):
        for k in self.S:
            self.S[k].append(st[k])

    def run(self, ref, level, A, max_T, kind, seed, actions_fn, relocate=None, max_steps=None):
        env = RefEnv(ref, level, A, max_T)
        if relocate:
            env.relocate(relocate)
        s0 = len(self.S["t"])
        a0 = len(self.act)
        st = env.canon(0)
        self.add_state(st)
        T = 0
        limit = max_steps if max_steps is not None else max(max_T, 1) + 5
        while T < limit:
            codes = actions_fn(T, st)
            if codes is None:
                break
            st, ex, coll = env.step(codes)
            row = np.full(MAXA, PAD, np.uint8)
            row[:A] = codes
            self.act.append(row)
            self.exe.append(ex)
            self.coll.append(coll)
            self.add_state(st)
            T += 1
            if st["flags"] & 1:
                break
        start = np.full((MAXA, 2), PAD, np.uint8)
        if relocate:
            start[:len(relocate)] = relocate
        self.eps.append(dict(level=LEVEL_NAMES.index(level), A=A, max_T=max_T, kind=kind, seed=seed,
                             state_off=s0, act_off=a0, T=T, start=start))
        return st

    def save(self, path, kinds):
        E = self.eps
        np.savez_compressed(
            path,
            ep_level=np.array([e["level"] for e in E], np.int32),
            ep_A=np.array([e["A"] for e in E], np.int32),
            ep_maxT=np.array([e["max_T"] for e in E], np.int32),
            ep_kind=np.array([kinds.index(e["kind"]) for e in E], np.int32),
            ep_seed=np.array([e["seed"] for e in E], np.int64),
            ep_state_off=np.array([e["state_off"] for e in E], np.int64),
            ep_act_off=np.array([e["act_off"] for e in E], np.int64),
            ep_T=np.array([e["T"] for e in E], np.int32),
            ep_start=np.stack([e["start"] for e in E]).astype(np.uint8),
            t=np.array(self.S["t"], np.uint16),
            flags=np.array(self.S["flags"], np.uint8),
            agents=np.stack(self.S["agents"]).astype(np.uint8),
            items=np.stack(self.S["items"]).astype(np.uint8),
            act=np.stack(self.act).astype(np.uint8) if self.act else np.zeros((0, MAXA), np.uint8),
            exe=np.stack(self.exe).astype(np.uint8) if self.exe else np.zeros((0, MAXA), np.uint8),
            coll=np.array(self.coll, np.uint8),
            level_names=np.array(LEVEL_NAMES),
            kinds=np.array(kinds),
        )


def scripted(seq_by_agent, A):
    seqs = [[LETTER[c] for c in s.split()] for s in seq_by_agent]

    def fn(T, st):
        if T >= max(len(s) for s in seqs):
            return None
        return [(seqs[i][T] if i < len(seqs) and T < len(seqs[i]) else 4) for i in range(A)]
    return fn


A9_AGENT1 = "N N R R R U L L L L L L R R R R R L L L L D L U L D D D D R R R R R L L L L U U L"
A9_AGENT2 = "D D" + " N" * 39
TL_AGENT1 = ("N N R R R U L L L L L D D D D R R R R R L L L L U U L U U R R R R R L L L L D L D D D "
             "R R R R D L L L L U U L")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    args = ap.parse_args()
    ref = load_reference()
    kinds = ["kat", "collision", "uniform", "goal", "prefix"]

    # --- level descriptions as the reference builds them
    levels = {}
    for name in LEVEL_NAMES:
        levels[name] = RefEnv(ref, name, 4, 100).level_info()
    with open(os.path.join(HERE, "levels.json"), "w") as f:
        json.dump(levels, f, indent=1, sort_keys=True)

    # --- known-answer episodes
    kat = Recorder()
    kat.run(ref, "open-divider_salad", 2, 100, "kat", 0, scripted([A9_AGENT1, A9_AGENT2], 2))
    kat.run(ref, "open-divider_salad", 2, 41, "kat", 1, scripted([A9_AGENT1, A9_AGENT2], 2))
    a1 = A9_AGENT1.split()
    kat.run(ref, "open-divider_salad", 2, 100, "kat", 2,
            scripted([" ".join(a1[:25] + ["D", "D", "L"]), A9_AGENT2], 2))
    kat.run(ref, "open-divider_salad", 2, 100, "kat", 3,
            scripted([" ".join(a1[:6] + ["D", "D", "D", "D", "R"]), A9_AGENT2], 2))
    kat.run(ref, "open-divider_tl", 2, 100, "kat", 4, scripted([TL_AGENT1, "D D" + " N" * 60], 2))
    # collision table, agents relocated on the open level
    R, L_, U, N = 3, 2, 1, 4
    table = [
        ([(2, 2), (3, 2)], [R, L_]),   # swap
        ([(2, 2), (4, 2)], [R, L_]),   # same target
        ([(2, 2), (3, 2)], [N, L_]),   # stay vs enter
        ([(1, 2), (2, 2)], [L_, L_]),  # A bumps counter, B enters A
        ([(2, 2), (3, 2)], [L_, L_]),  # follow
        ([(2, 2), (3, 2)], [N, N]),    # both stay
        ([(2, 2), (3, 3)], [R, U]),    # perpendicular same target
    ]
    for i, (locs, acts) in enumerate(table):
        kat.run(ref, "open-divider_salad", 2, 100, "collision", i,
                lambda T, st, a=acts: a if T == 0 else None, relocate=locs)
    # 3- and 4-agent collision chains (co-location is reachable with A >= 3)
    rng = random.Random(7)
    for i in range(60):
        A = 3 + (i % 2)
        floor = [(x, y) for x in range(1, 6) for y in range(1, 6)]
        locs = rng.sample(floor, A)
        acts = [rng.randrange(5) for _ in range(A)]
        kat.run(ref, "open-divider_salad", A, 100, "collision", 100 + i,
                lambda T, st, a=acts: a if T == 0 else None, relocate=locs)
    kat.save(os.path.join(HERE, "kat.npz"), kinds)

    # --- random / goal-directed / scripted-prefix streams on every level and agent count
    n_uni, n_goal = (1, 1) if args.quick else (4, 6)
    rec = Recorder()
    gid = 0
    for name in LEVEL_NAMES:
        info = levels[name]
        for A in (2, 3, 4):
            for e in range(n_uni):
                seed = 1000 + e
                g = gid
                rec.run(ref, name, A, 100, "uniform", seed,
                        lambda T, st, s=seed, g=g, A=A: [rng_action(s, g, T, a) for a in range(A)])
                gid += 1
            for e in range(n_goal):
                pol = GoalPolicy(info, A, seed=31 * gid + e)
                rec.run(ref, name, A, 100, "goal", gid, lambda T, st, p=pol: p.act(st))
                gid += 1
    # scripted prefix of the A.9 success episode, then goal-directed suffix (2 agents)
    for cut in ([] if args.quick else (10, 18, 24, 30, 34, 38)):
        pre = [[LETTER[c] for c in a1[:cut]], [LETTER[c] for c in A9_AGENT2.split()[:cut]]]
        pol = GoalPolicy(levels["open-divider_salad"], 2, seed=cut)

        def fn(T, st, pre=pre, pol=pol):
            if T < len(pre[0]):
                return [pre[0][T], pre[1][T]]
            return pol.act(st)
        rec.run(ref, "open-divider_salad", 2, 100, "prefix", cut, fn)
    rec.save(os.path.join(HERE, "streams.npz"), kinds)
    n_steps = len(rec.act) + len(kat.act)
    print("wrote %d episodes / %d steps" % (len(rec.eps) + len(kat.eps), n_steps))
    fl = np.array(rec.S["flags"])
    print("done-success", int(((fl & 3) == 3).sum()), "err", int((fl & 4).sum()))


if __name__ == "__main__":
    main()
