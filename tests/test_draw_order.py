"""Draw order of objects that share a square, on the CPU.

``Game.on_render`` draws the objects that are not held in ``world.objects`` order
(misc/game/game.py:62-74): name groups in first-insertion order, each group in insertion order;
a merge re-inserts the merged object under its new name (utils/interact.py:46-52).  Dishes
delivered to one Delivery square stay there, so the later one covers the earlier.
tests/golden/gen_draw_order.py recorded the reference's world.objects order along 38
goal-directed episodes that deliver every dish they make (372 states with two or more objects
on one square).  render.DrawOrder, replayed over the CPU oracle's states of the same
episodes, must give that order at every state, held objects included; and the numpy render
restatement drawn in that order must differ from slot order where the order shows."""
import os

import numpy as np
import pytest

import oc_testlib as tl
from gym_cooking_amd import levels
from gym_cooking_amd.render import DrawOrder

from oracle import oracle


def _level(name):
    path = os.path.join(tl.GOLDEN, "levels", name + ".txt")
    return levels.load_level(path if os.path.exists(path) else name)


def _rows(ev, A, K, W):
    """(mask, x, y, held) per live slot of one env's state bytes, by slot."""
    ax, ay, ah = ev[0:A], ev[A:2 * A], ev[2 * A:3 * A]
    loc, mask = ev[3 * A:3 * A + K], ev[3 * A + K:3 * A + 2 * K]
    out = {}
    for j in range(K):
        if loc[j] == 0xFF:
            continue
        holder = [a for a in range(A) if ah[a] == j]
        x, y = (ax[holder[0]], ay[holder[0]]) if holder else (loc[j] % W, loc[j] // W)
        out[j] = (int(mask[j]), int(x), int(y), int(bool(holder)))
    return out


def replay(fx, e):
    """Yield (state index, env bytes, DrawOrder) along fixture episode e on the CPU oracle."""
    name = str(fx["level_names"][fx["ep_level"][e]])
    A, T = int(fx["ep_A"][e]), int(fx["ep_T"][e])
    lv = _level(name)
    ob = oracle.OracleBatch(lv, A, 100, 1)
    s, s2 = ob.new_state(), ob.new_state()
    ob.reset(s)
    act = ob.new_actions()
    d = DrawOrder(lv, ob.K)
    off, aoff = int(fx["ep_state_off"][e]), int(fx["ep_act_off"][e])
    ev = tl.env_view(s, A, ob.K, ob.pitch, 1)[:, 0]
    yield off, lv, A, ob.K, ev, d
    for step in range(T):
        for a in range(A):
            act[a * ob.pitch] = fx["act"][aoff + step][a]
        ob.step(s, s2, act)
        s, s2 = s2, s
        nv = tl.env_view(s, A, ob.K, ob.pitch, 1)[:, 0]
        pl = lambda v: {"ah": v[2 * A:3 * A], "loc": v[3 * A:3 * A + ob.K], "mask": v[3 * A + ob.K:3 * A + 2 * ob.K]}  # noqa: E731
        d.update(pl(ev), pl(nv))
        ev = nv
        yield off + step + 1, lv, A, ob.K, ev, d


def test_draw_order_matches_reference_world_objects_order():
    fx = tl.load_fixture("draw_order.npz")
    checked = stacked = 0
    for e in range(len(fx["ep_T"])):
        for i, lv, A, K, ev, d in replay(fx, e):
            ref = [tuple(int(v) for v in r) for r in fx["order"][i] if r[0] != tl.PAD]
            if not ref:  # the reference raised (copy crash) at this step
                continue
            rows = _rows(ev, A, K, lv.width)
            assert sorted(rows.values()) == sorted(ref), (e, i)
            r = d.ranks()
            ours = [rows[j] for j in sorted(rows, key=lambda j: (r[j], j))]
            assert ours == ref, (e, i, ours, ref)
            checked += 1
            cells = [(x, y) for (_, x, y, h) in ref if not h]
            stacked += len(cells) != len(set(cells))
    assert checked > 3000 and stacked > 300


def test_slot_order_differs_where_the_order_shows():
    """Without the replayed order, some stacked states would draw wrongly: the reference's
    order of the objects on one square is not their slot order."""
    fx = tl.load_fixture("draw_order.npz")
    differs = 0
    for e in range(len(fx["ep_T"])):
        for i, lv, A, K, ev, d in replay(fx, e):
            rows = _rows(ev, A, K, lv.width)
            r = d.ranks()
            by_cell = {}
            for j in sorted(rows, key=lambda j: (r[j], j)):
                m, x, y, h = rows[j]
                if not h:
                    by_cell.setdefault((x, y), []).append(j)
            differs += any(len(v) > 1 and v != sorted(v) and len({rows[j][0] for j in v}) > 1 for v in by_cell.values())
    assert differs > 20


def test_sync_takes_slot_order_of_live_objects():
    lv = _level("open-divider_salad")
    d = DrawOrder(lv, 4)
    d.sync({"ah": np.array([0xFF, 0xFF], np.uint8), "loc": np.array([10, 0xFF, 12, 20], np.uint8),
            "mask": np.array([0x19, 0, 0x02, 0x19], np.uint8)})
    assert d.ranks().tolist() == [0, 0xFF, 2, 1]
