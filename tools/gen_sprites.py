#!/usr/bin/env python3
"""Build the renderer's sprite atlas from the reference's art (build container only).

Reads gym_cooking/misc/game/graphics/*.png from the read-only reference checkout with PIL
(PNG is lossless: the same RGBA bytes pygame.image.load gets) and scales each sprite to the
sizes gym_cooking/misc/game/game.py draws it at, with pygame 1.9.6's nearest-neighbour
``transform.scale`` (transform.c ``stretch``: per axis, copy the current source pixel, then
advance while the error term 2*src - 2*dst stays >= 0), restated in ``stretch_index``:

  tile 80 x 80            agents, delivery, cutboard, plate and food on a counter (game.py:26-33)
  container 56 x 56       food on a plate on a counter        (container_scale 0.7)
  holding 40 x 40         held plate / held unplated food     (holding_scale 0.5)
  holding container 28    food on a held plate                (0.7 x 0.5)

Only these scaled RGBA arrays are stored (gym_cooking_amd/assets/sprites.npz, derived data);
the reference PNGs themselves are not copied.  Note: game.py asks for 'Plate.png' while the
file is 'plate.png' (it only loads on a case-insensitive file system); 'plate.png' is used.

Usage:  python tools/gen_sprites.py
"""
from __future__ import annotations

import os

import numpy as np
from PIL import Image

SRC = "/root/reference/gym_cooking/misc/game/graphics"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "gym-cooking_amd", "gym_cooking_amd", "assets", "sprites.npz")
TILE = 80
SIZES = (80, 56, 40, 28)  # tile, container, holding, holding container (game.py:26-33)
FOODS = ["FreshTomato", "FreshLettuce", "FreshOnion", "ChoppedTomato", "ChoppedLettuce", "ChoppedOnion",
         "ChoppedLettuce-ChoppedTomato", "ChoppedLettuce-ChoppedOnion", "ChoppedOnion-ChoppedTomato",
         "ChoppedLettuce-ChoppedOnion-ChoppedTomato"]


def stretch_index(src: int, dst: int) -> np.ndarray:
    """Source index of every destination index (pygame transform.c stretch, one axis)."""
    idx, s, err = [], 0, 2 * src - 2 * dst
    for _ in range(dst):
        idx.append(s)
        while err >= 0:
            s += 1
            err -= 2 * dst
        err += 2 * src
    return np.array(idx, np.int64)


def scaled(name: str, size: int) -> np.ndarray:
    im = np.asarray(Image.open(os.path.join(SRC, name + ".png")).convert("RGBA"), np.uint8)  # [h, w, 4]
    h, w = im.shape[:2]
    return np.ascontiguousarray(im[stretch_index(h, size)][:, stretch_index(w, size)])


def main():
    out = {}
    for f in FOODS:
        for n in SIZES:
            out["%s@%d" % (f, n)] = scaled(f, n)
    for n in (80, 40):
        out["Plate@%d" % n] = scaled("plate", n)
    for c in ("blue", "magenta", "yellow", "green"):
        out["agent-%s@80" % c] = scaled("agent-" + c, 80)
    out["delivery@80"] = scaled("delivery", 80)
    out["cutboard@80"] = scaled("cutboard", 80)
    np.savez_compressed(OUT, **out)
    print("wrote %d sprites to %s (%d bytes)" % (len(out), OUT, os.path.getsize(OUT)))


if __name__ == "__main__":
    main()
