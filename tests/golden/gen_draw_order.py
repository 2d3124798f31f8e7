#!/usr/bin/env python3
"""Record the reference's object draw order: ``Game.on_render`` draws the
objects that are not held in ``world.objects`` order (misc/game/game.py:62-74) -- the dict's
groups in the order their names were first inserted, each group's list in insertion order
(``World.insert``: ``objects.setdefault(obj.name, []).append(obj)``, utils/world.py:304-305).
A merge removes both objects and re-inserts the merged one under its new name
(utils/interact.py:46-52), so the order is history, not state.  It matters where objects
share a square: dishes delivered to one Delivery cell stay there (``gs.acquire``,
interact.py:35-40) and the later-drawn one covers the earlier.

Runs ONLY in the build container (the reference is imported with gen_golden.py's stubs).
Goal-directed episodes that deliver every deliverable dish they hold (so dishes pile up on
the Delivery squares), on Salad / Tomato+Lettuce kitchens and a repeated-food one.  Per
state: the canonical items (gen_golden.RefEnv.canon, sorted) and the same rows in the
reference's world.objects order.  Output: tests/golden/draw_order.npz.

Usage:  PYTHONHASHSEED=0 python tests/golden/gen_draw_order.py
"""
from __future__ import annotations

import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_duplevels as gd  # noqa: E402
import gen_golden as gg  # noqa: E402

# (level, agents, episodes, seed, counts encoding)
CONFIGS = [("open-divider_salad", 2, 10, 8100, False), ("partial-divider_tl", 3, 10, 8200, False),
           ("open-divider_tl", 2, 10, 8300, False), ("dup-12x12_salad3t", 3, 8, 8400, True)]
MAXK = 8


def world_order(env):
    from utils.core import Object
    rows = [(gg.content_mask(o), o.location[0], o.location[1], int(bool(o.is_held)))
            for objs in env.world.objects.values() for o in objs if isinstance(o, Object)]
    out = np.full((MAXK, 4), gg.PAD, np.uint8)
    for i, r in enumerate(rows):
        out[i] = r
    return out


def main():
    ref = gg.load_reference()
    presence = gg.content_mask
    gg.MAXK = MAXK
    scratch = tempfile.mkdtemp(prefix="oc_draw_")
    os.makedirs(os.path.join(scratch, "utils", "levels"))
    shutil.copy(os.path.join(HERE, "levels", "dup-12x12_salad3t.txt"), os.path.join(scratch, "utils", "levels"))
    for name, *_ in CONFIGS[:3]:  # builtin kitchens, read from the reference checkout
        shutil.copy(os.path.join(gg.REF, "gym_cooking", "utils", "levels", name + ".txt"), os.path.join(scratch, "utils", "levels"))
    cwd = os.getcwd()
    os.chdir(scratch)
    names = [c[0] for c in CONFIGS]
    ep = {k: [] for k in ("level", "A", "T", "state_off", "act_off")}
    acts, canon, order, flags = [], [], [], []
    for li, (name, A, n_eps, seed0, counts) in enumerate(CONFIGS):
        gg.content_mask = gd.content_mask_counts if counts else presence
        info = gg.RefEnv(ref, name, A, 100).level_info()
        for e in range(n_eps):
            env = gg.RefEnv(ref, name, A, 100)
            cls = gd.CountsGoalPolicy if counts else gg.GoalPolicy
            pol = cls(info, A, seed=seed0 + e, eps=0.1)
            pol.goals = list(range(256))  # deliver whatever deliverable dish is held
            ep["level"].append(li)
            ep["A"].append(A)
            ep["state_off"].append(len(canon))
            ep["act_off"].append(len(acts))
            st = env.canon(0)
            canon.append(st["items"])
            order.append(world_order(env.env))
            flags.append(0)
            T = 0
            while T < 100:
                codes = pol.act(st)
                st, _, _ = env.step(codes)
                row = np.full(4, gg.PAD, np.uint8)
                row[:A] = codes
                acts.append(row)
                canon.append(st["items"])
                order.append(world_order(env.env) if not env.err else np.full((MAXK, 4), gg.PAD, np.uint8))
                flags.append(int(st["flags"]))
                T += 1
                if env.err or st["flags"] & 1:
                    break
            ep["T"].append(T)
    os.chdir(cwd)
    shutil.rmtree(scratch)
    order = np.array(order, np.uint8)
    stacked = 0
    for o in order:
        live = o[o[:, 0] != gg.PAD]
        cells = [(int(r[1]), int(r[2])) for r in live if not r[3]]
        stacked += len(cells) != len(set(cells))
    np.savez_compressed(os.path.join(HERE, "draw_order.npz"), level_names=np.array(names),
                        ep_level=np.array(ep["level"], np.int32), ep_A=np.array(ep["A"], np.int32),
                        ep_T=np.array(ep["T"], np.int32), ep_state_off=np.array(ep["state_off"], np.int32),
                        ep_act_off=np.array(ep["act_off"], np.int32), act=np.array(acts, np.uint8),
                        items=np.array(canon, np.uint8), order=order, flags=np.array(flags, np.uint8))
    print("wrote %d episodes / %d steps; states with two objects on one square: %d" % (
        len(ep["T"]), len(acts), stacked))


if __name__ == "__main__":
    main()
