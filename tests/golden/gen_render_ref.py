#!/usr/bin/env python3
"""Pin the image-observation restatement to the reference's own pixels.

Runs ONLY in the build container (reads the read-only reference checkout at /root/reference;
only the small derived fixture travels).  Two kinds of reference pixels exist there:

* images/{2,3,4}_{open,partial,full}.png -- 560x560 RGB screenshots of the initial states of
  the Salad kitchens with 2, 3 and 4 agents (drawn by Game.on_render, misc/game/game.py:56-186).
  They are exact: the fixture keeps each image's SHA-256 and the image itself (zlib).
* images/{2_open_salad,2_full_salad,2_partial_tl}.gif -- whole episodes (one frame per step,
  the first frame the reset state), palette-quantised by the GIF writer.  The episodes' action
  sequences are not recorded anywhere, so they are recovered here: from each frame's state,
  every one of the 25 joint actions is stepped with the CPU oracle and rendered with
  oracle/render_oracle.py, and the successors whose image quantises to the next frame are
  kept (a breadth-first search over the frames).  "Quantises to" is exact: every pixel's GIF
  colour must be a nearest colour, among the frame's colours, to the rendered colour (the
  writer maps each pixel to its nearest palette colour; a few pixels sit at equal distance from
  two palette colours).  The fixture keeps, per frame, its colours, the recovered state's
  joint action, the frame's SHA-256, and the pixels where the nearest colour is tied (their
  GIF colour), so a test can rebuild the exact GIF frame from a render with no reference file.

Usage:  python tests/golden/gen_render_ref.py   ->  tests/golden/render_ref.npz
"""
from __future__ import annotations

import hashlib
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from gym_cooking_amd import capi, levels  # noqa: E402
from oracle import oracle, render_oracle  # noqa: E402

import oc_testlib as tl  # noqa: E402

IMAGES = "/root/reference/images"
HOLD = 255  # "no step": a repeated final frame after the episode ended
PNGS = [("%d_%s" % (A, kind), "%s-divider_salad" % kind, A) for A in (2, 3, 4) for kind in ("open", "partial", "full")]
GIFS = [("2_open_salad", "open-divider_salad", 2), ("2_full_salad", "full-divider_salad", 2),
        ("2_partial_tl", "partial-divider_tl", 2)]


def quantise(render: np.ndarray, colours: np.ndarray):
    """(index of the first nearest colour per pixel, bool mask of pixels with a tie)."""
    flat = render.reshape(-1, 3).astype(np.int64)
    cols, inv = np.unique(flat, axis=0, return_inverse=True)
    d = ((cols[:, None, :] - colours[None, :, :].astype(np.int64)) ** 2).sum(-1)
    near = d.argmin(1)
    ties = (d == d.min(1, keepdims=True)).sum(1) > 1
    inv = inv.reshape(-1)
    return near[inv].reshape(render.shape[:2]), ties[inv].reshape(render.shape[:2]), d[inv].reshape(
        render.shape[:2] + (len(colours),))


def frame_matches(render: np.ndarray, frame_idx: np.ndarray, colours: np.ndarray) -> bool:
    near, ties, d = quantise(render, colours)
    if np.array_equal(near, frame_idx):
        return True
    bad = near != frame_idx
    gd = np.take_along_axis(d[bad], frame_idx[bad][:, None], 1)[:, 0]
    return bool((gd == d[bad].min(1)).all())


def gif_frames(path):
    from PIL import Image
    im = Image.open(path)
    out = []
    for f in range(im.n_frames):
        im.seek(f)
        rgb = np.asarray(im.convert("RGB"))
        colours, idx = np.unique(rgb.reshape(-1, 3), axis=0, return_inverse=True)
        out.append((rgb, colours.astype(np.uint8), idx.reshape(rgb.shape[:2]).astype(np.uint8)))
    return out


def env_bytes(ob, s):
    return tl.env_view(s, ob.A, ob.K, ob.pitch, ob.B)


def recover(name, level_name, A):
    lv = levels.load_level(level_name)
    spr = render_oracle._sprites()
    frames = gif_frames(os.path.join(IMAGES, name + ".gif"))
    one = oracle.OracleBatch(lv, A, 0, 1)
    s0 = one.new_state()
    one.reset(s0)
    K = one.K
    cur = [(env_bytes(one, s0)[:, 0], [])]  # (state bytes, joint actions so far)
    rgb0, cols0, idx0 = frames[0]
    assert frame_matches(render_oracle.render_env(lv, cur[0][0], A, K, spr, "rgb"), idx0, cols0), name
    joint = [(a, b) for a in range(5) for b in range(5)]
    nJ = len(joint)
    ob = oracle.OracleBatch(lv, A, 0, nJ)
    per_frame_states = [cur[0][0]]
    for f in range(1, len(frames)):
        rgb, cols, idx = frames[f]
        nxt = {}
        P = capi.layout_planes(A, K)
        done = [(st, path) for st, path in cur if st[P["flags"]] & 1]
        if done:  # the recording holds the last frame after the episode ended: no step
            assert len(done) == len(cur)
            for st, path in done:
                assert frame_matches(render_oracle.render_env(lv, st, A, K, spr, "rgb"), idx, cols), (name, f)
            cur = [(st, path + [(HOLD, HOLD)]) for st, path in done]
            per_frame_states.append(cur[0][0])
            print("%s frame %d: final frame held" % (name, f), flush=True)
            continue
        for st, path in cur:
            s = ob.new_state()
            v = s.reshape(-1, ob.pitch)
            # every row: the same state bytes (t as two byte planes), one joint action each
            for p in range(P["num_planes"]):
                if p == P["t"]:
                    tt = np.full(ob.pitch, int(st[p]) | (int(st[p + 1]) << 8), np.uint16)
                    s[P["t"] * ob.pitch:(P["t"] + 2) * ob.pitch] = tt.view(np.uint8)
                elif p == P["t"] + 1:
                    continue
                else:
                    v[p, :] = st[p]
            act = ob.new_actions().reshape(A, ob.pitch)
            for j, ja in enumerate(joint):
                act[0, j], act[1, j] = ja
            s2 = ob.new_state()
            ob.step(s, s2, act.reshape(-1))
            ev = env_bytes(ob, s2)
            for j in range(nJ):
                key = bytes(ev[:, j])
                if key in nxt:
                    continue
                img = render_oracle.render_env(lv, ev[:, j], A, K, spr, "rgb")
                if frame_matches(img, idx, cols):
                    nxt[key] = (ev[:, j].copy(), path + [joint[j]])
        if not nxt:
            raise SystemExit("%s: no successor of frame %d matches frame %d" % (name, f - 1, f))
        cur = list(nxt.values())
        per_frame_states.append(cur[0][0])
        print("%s frame %d: %d matching state(s)" % (name, f, len(cur)), flush=True)
    assert len(cur) == 1, "%s: %d distinct states match the last frame" % (name, len(cur))
    return lv, frames, per_frame_states, cur[0][1], [len(cur)]


def frame_record(render, rgb, cols, idx):
    near, ties, _ = quantise(render, cols)
    tpos = np.flatnonzero(ties.reshape(-1) & (near.reshape(-1) != idx.reshape(-1)))
    return hashlib.sha256(rgb.tobytes()).hexdigest(), tpos.astype(np.int32), idx.reshape(-1)[tpos].astype(np.uint8)


def main():
    out = {}
    spr = render_oracle._sprites()
    from PIL import Image
    for name, level_name, A in PNGS:
        rgb = np.asarray(Image.open(os.path.join(IMAGES, name + ".png")).convert("RGB"))
        lv = levels.load_level(level_name)
        ob = oracle.OracleBatch(lv, A, 0, 1)
        s = ob.new_state()
        ob.reset(s)
        img = render_oracle.render_env(lv, env_bytes(ob, s)[:, 0], A, ob.K, spr, "rgb")
        nd = int((img != rgb).any(-1).sum())
        print("%s: %d differing pixels against render_oracle" % (name, nd))
        out["png_%s" % name] = np.frombuffer(zlib.compress(rgb.tobytes(), 9), np.uint8)
        out["png_%s_sha256" % name] = np.array(hashlib.sha256(rgb.tobytes()).hexdigest())
        out["png_%s_meta" % name] = np.array([level_name, str(A)])
    for name, level_name, A in GIFS:
        lv, frames, states, actions, _ = recover(name, level_name, A)
        shas, tie_pos, tie_idx, tie_off, cols_all, col_off = [], [], [], [0], [], [0]
        for f, (rgb, cols, idx) in enumerate(frames):
            img = render_oracle.render_env(lv, states[f], A, capi.item_slots(lv), spr, "rgb")
            sha, tp, ti = frame_record(img, rgb, cols, idx)
            shas.append(sha)
            tie_pos.append(tp)
            tie_idx.append(ti)
            tie_off.append(tie_off[-1] + len(tp))
            cols_all.append(cols)
            col_off.append(col_off[-1] + len(cols))
        out["gif_%s_meta" % name] = np.array([level_name, str(A)])
        out["gif_%s_actions" % name] = np.array(actions, np.uint8).reshape(-1, A)
        out["gif_%s_states" % name] = np.stack(states).astype(np.uint8)
        out["gif_%s_sha256" % name] = np.array(shas)
        out["gif_%s_colours" % name] = np.concatenate(cols_all)
        out["gif_%s_colour_off" % name] = np.array(col_off, np.int64)
        out["gif_%s_tie_pos" % name] = np.concatenate(tie_pos)
        out["gif_%s_tie_idx" % name] = np.concatenate(tie_idx)
        out["gif_%s_tie_off" % name] = np.array(tie_off, np.int64)
    path = os.path.join(HERE, "render_ref.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
