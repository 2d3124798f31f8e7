"""Batched image observations: the host side of ``oc_render`` (include/oc_engine.h).

This is ``GameImage.get_image_obs`` (gym_cooking/misc/game/gameimage.py:31-51) for a whole
batch.  ``Game.on_render`` (gym_cooking/misc/game/game.py:56-186) draws, in order:

* the floor colour over the whole screen;
* every grid square: Counter = counter colour and a 1-px border, Delivery = grey and the
  delivery sprite, Cutboard = counter, border and the cutboard sprite;
* every object that is not held, at tile size (a plate first, then its contents at the
  container size, inset 12 px);
* every agent in order, then what it holds at the holding size in the cell's lower-right
  quarter (a plate first, then its contents at the holding-container size, inset 46 px).

The first two steps never change in an episode, so this module renders them once per level
on the host (``static_background``).  The kernel then composes the dynamic sprites for every
env.  Sprites come from ``assets/sprites.npz``, which tools/gen_sprites.py scales from the
reference art with pygame's nearest-neighbour ``transform.scale``.  Blending follows SDL 1.2's
per-pixel-alpha blit (``sdl_blend``).

Channel order.  The reference reads ``0x00RRGGBB`` pixel ints through ``pygame.Color(int)``,
which parses ``0xRRGGBBAA``, and stores ``(color.g, color.b, color.r)``.  That yields
``(R, G, 0)``, which ``channels="reference"`` reproduces.  ``channels="rgb"`` gives the drawn
RGB image instead.

Draw order of objects that share a square.  ``on_render`` draws the objects that are not held
in ``world.objects`` order (game.py:62-74): the groups in the order their names were first
inserted, each group's list in insertion order (``World.insert``, utils/world.py:304-305).  A
merge re-inserts the merged object under its new name (utils/interact.py:46-52), so the order
is episode history the state does not hold.  Only dishes delivered to one Delivery square
share a square (they stay there, interact.py:35-40).  ``DrawOrder`` replays that history from
consecutive states and gives ``oc_render_ordered`` a per-slot draw rank; without ranks the
kernel draws a square's objects in slot order.

Parity: the kernel and an independent numpy restatement (oracle/render_oracle.py) reproduce
the reference's screenshots and recorded GIF frames (tests/test_render.py); the draw order is
pinned to the reference's world.objects order along recorded episodes
(tests/golden/gen_draw_order.py, tests/test_draw_order.py).
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional, Tuple

import numpy as np

from . import capi
from . import levels as _levels

ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "sprites.npz")

# game.py:26-33 and holding/container locations :166-186, evaluated as the reference does
TILE = 80
_HOLD, _CONT = 0.5, 0.7
SIZES = (TILE, int(_CONT * TILE), int(_HOLD * TILE), int(_CONT * int(_HOLD * TILE)))      # 80, 56, 40, 28
OFFSETS = (0, int(TILE * (1 - _CONT) / 2), int(TILE * (1 - _HOLD)),
           int(TILE * ((1 - _HOLD) + (1 - _CONT) / 2 * _HOLD)))                             # 0, 12, 40, 46
FLOOR, COUNTER, COUNTER_BORDER, DELIVERY = (245, 230, 210), (220, 170, 110), (114, 93, 51), (96, 96, 96)  # misc/game/utils.py
AGENT_COLORS = ("blue", "magenta", "yellow", "green")  # utils/agent.py:25
FOOD_SPRITES = ("FreshTomato", "FreshLettuce", "FreshOnion", "ChoppedTomato", "ChoppedLettuce", "ChoppedOnion",
                "ChoppedLettuce-ChoppedTomato", "ChoppedLettuce-ChoppedOnion", "ChoppedOnion-ChoppedTomato",
                "ChoppedLettuce-ChoppedOnion-ChoppedTomato")
CHANNELS = {"reference": capi.OC_CHAN_REFERENCE, "rgb": capi.OC_CHAN_RGB}


def food_sprite_name(mask: int) -> Optional[str]:
    """Sprite file of a plate-less content mask: ``Object.full_name`` (core.py:161-171).
    Returns None for a mask no sprite exists for."""
    name = _levels.mask_full_name(mask & ~_levels.M_PLATE) if mask & _levels.M_FOODS else None
    return name if name in FOOD_SPRITES else None


def load_sprites(path: str = ASSETS) -> Dict[str, np.ndarray]:
    with np.load(path) as z:
        return {k: z[k] for k in z.files}


def pack_rgba(img: np.ndarray) -> np.ndarray:
    """[h, w, 3|4] uint8 -> [h, w] uint32 R | G<<8 | B<<16 | A<<24."""
    img = img.astype(np.uint32)
    a = img[..., 3] if img.shape[-1] == 4 else 0
    return img[..., 0] | (img[..., 1] << 8) | (img[..., 2] << 16) | (a << 24)


def sdl_blend(dst: np.ndarray, src: np.ndarray) -> np.ndarray:
    """SDL 1.2 per-pixel alpha blit (BlitNtoNPixelAlpha, ALPHA_BLEND): per channel
    d = (((s - d) * a + 255) >> 8) + d where a != 0.  dst [.., 3] uint8, src [.., 4] uint8."""
    d = dst.astype(np.int32)
    s = src[..., :3].astype(np.int32)
    a = src[..., 3:4].astype(np.int32)
    out = (((s - d) * a + 255) >> 8) + d
    return np.where(a > 0, out, d).astype(np.uint8)


def static_background(level: "_levels.Level", sprites: Dict[str, np.ndarray]) -> np.ndarray:
    """The level image before any object or agent: ``screen.fill(FLOOR)`` then
    ``draw_gridsquare`` for every square (game.py:56-96).  [H*80, W*80, 3] uint8."""
    img = np.empty((level.height * TILE, level.width * TILE, 3), np.uint8)
    img[...] = FLOOR
    for c, kind in enumerate(level.tiles):
        x, y = level.xy(c)
        tile = img[y * TILE:(y + 1) * TILE, x * TILE:(x + 1) * TILE]
        if kind == _levels.TILE_FLOOR:
            continue
        tile[...] = DELIVERY if kind == _levels.TILE_DELIVERY else COUNTER
        if kind in (_levels.TILE_COUNTER, _levels.TILE_CUTBOARD):  # pygame.draw.rect(..., 1): 1-px outline
            tile[0, :] = tile[-1, :] = tile[:, 0] = tile[:, -1] = COUNTER_BORDER
        if kind == _levels.TILE_DELIVERY:
            tile[...] = sdl_blend(tile, sprites["delivery@80"])
        elif kind == _levels.TILE_CUTBOARD:
            tile[...] = sdl_blend(tile, sprites["cutboard@80"])
    return img


class RenderTables:
    """Host-built device inputs of ``oc_render`` for one level: the sprite atlas, the static
    background and the ``oc_render_desc``."""

    def __init__(self, level: "_levels.Level", sprites: Optional[Dict[str, np.ndarray]] = None):
        sprites = load_sprites() if sprites is None else sprites
        self.level = level
        chunks, off = [], 0
        desc = capi.OcRenderDesc()
        desc.tile = TILE
        for c in range(capi.OC_RENDER_SIZES):
            desc.size[c], desc.offset[c] = SIZES[c], OFFSETS[c]
            desc.food_base[c] = off
            for name in FOOD_SPRITES:
                a = pack_rgba(sprites["%s@%d" % (name, SIZES[c])])
                chunks.append(a.ravel())
                off += a.size
        for i, n in enumerate((SIZES[0], SIZES[2])):
            desc.plate_off[i] = off
            a = pack_rgba(sprites["Plate@%d" % n])
            chunks.append(a.ravel())
            off += a.size
        for i, col in enumerate(AGENT_COLORS):
            desc.agent_off[i] = off
            a = pack_rgba(sprites["agent-%s@80" % col])
            chunks.append(a.ravel())
            off += a.size
        for m in range(128):
            name = food_sprite_name(m)
            desc.food_sprite[m] = 0xFF if name is None else FOOD_SPRITES.index(name)
        self.desc = desc
        self.atlas = np.concatenate(chunks).astype(np.uint32)
        self.background_rgb = static_background(level, sprites)
        self.background = pack_rgba(self.background_rgb)
        self.height_px, self.width_px = self.background.shape

    def desc_with(self, channels: str) -> capi.OcRenderDesc:
        if channels not in CHANNELS:
            raise ValueError("channels must be one of %s" % sorted(CHANNELS))
        d = capi.OcRenderDesc()
        ctypes.memmove(ctypes.byref(d), ctypes.byref(self.desc), ctypes.sizeof(d))
        d.chan_map = CHANNELS[channels]
        return d


def _group_name(mask: int, enc: int) -> str:
    """``Object.name``: the contents' names, sorted, without their states (core.py:161-171)."""
    return "-".join(n for n, _ in _levels.mask_contents(mask, enc))


class DrawOrder:
    """The reference's ``world.objects`` order of one env's objects, replayed from its
    consecutive states.  ``load_level`` inserts the objects in map scan order
    (overcooked_environment.py:158-165), which is slot order; a merge removes the object it
    absorbed and the holder's object, and re-inserts the holder's (the engine keeps the
    holder's slot) at the end of its new name's group, creating the group if the name is new
    (utils/interact.py:46-52, world.py:304-315).  Groups stay when emptied, as dict keys do."""

    def __init__(self, level: "_levels.Level", K: int):
        self.level, self.K = level, K
        self.reset()

    def reset(self) -> None:
        enc = self.level.encoding
        self.groups: Dict[str, list] = {}
        for j, (_cell, m) in enumerate(self.level.items):
            self.groups.setdefault(_group_name(m, enc), []).append(j)

    def update(self, prev: Dict[str, np.ndarray], nxt: Dict[str, np.ndarray]) -> None:
        """Advance over one step.  `prev` / `nxt` hold one env's planes: ``ah`` [A], ``loc``
        [K], ``mask`` [K], ``t`` (and ``fl``); a state with DONE set is followed by a reset."""
        if int(prev.get("fl", 0)) & 1:  # auto-reset: the next state is the template
            self.reset()
            return
        enc = self.level.encoding
        gone = {j for j in range(self.K) if prev["loc"][j] != 0xFF and nxt["loc"][j] == 0xFF}
        if gone:
            for g in self.groups.values():
                g[:] = [j for j in g if j not in gone]
        for a, h in enumerate(nxt["ah"]):
            h = int(h)
            if h >= self.K or int(prev["ah"][a]) != h:
                continue
            old, new = _group_name(int(prev["mask"][h]), enc), _group_name(int(nxt["mask"][h]), enc)
            if old != new:  # a merge into the object this agent holds
                self.groups[old].remove(h)
                self.groups.setdefault(new, []).append(h)

    def sync(self, planes: Dict[str, np.ndarray]) -> None:
        """Start from a state of unknown history (a loaded state): each live object in the
        group of its current name, groups and objects in slot order."""
        enc = self.level.encoding
        self.groups = {}
        for j in range(self.K):
            if planes["loc"][j] != 0xFF:
                self.groups.setdefault(_group_name(int(planes["mask"][j]), enc), []).append(j)

    def ranks(self) -> np.ndarray:
        """u8 [K]: each slot's position in world.objects order (0xFF: merged away)."""
        r = np.full(self.K, 0xFF, np.uint8)
        i = 0
        for g in self.groups.values():
            for j in g:
                r[j] = i
                i += 1
        return r


class Renderer:
    """Image observations of an :class:`engine.OvercookedBatch`'s states on its GPU."""

    def __init__(self, batch, sprites: Optional[Dict[str, np.ndarray]] = None):
        import torch
        self.batch = batch
        self.tables = RenderTables(batch.level, sprites)
        dev = batch.device
        self.atlas = torch.from_numpy(self.tables.atlas.view(np.int32)).to(dev)
        self.background = torch.from_numpy(np.ascontiguousarray(self.tables.background).view(np.int32)).to(dev)
        self.shape = (self.tables.height_px, self.tables.width_px, 3)

    def new_images(self):
        import torch
        return torch.empty((self.batch.B,) + self.shape, dtype=torch.uint8, device=self.batch.device)

    def render(self, state, out=None, channels: str = "reference", draw_rank=None):
        """u8 [B, H*80, W*80, 3] images of all B envs of `state`.  `draw_rank` (optional u8
        [K, pitch] device tensor, e.g. stacked ``DrawOrder.ranks()``): the objects of one
        square are drawn in ascending rank, ties in slot order; without it, in slot order."""
        self.batch._check(state, self.batch.layout.state_bytes)
        shape = (self.batch.B,) + self.shape
        out = self.new_images() if out is None else out
        if tuple(out.shape) != shape or not out.is_contiguous() or out.device != self.batch.device:
            raise ValueError("out must be a contiguous u8 %s tensor on %s" % (shape, self.batch.device))
        rank_ptr = None
        if draw_rank is not None:
            self.batch._check(draw_rank, self.batch.K * self.batch.pitch)
            rank_ptr = ctypes.c_void_p(draw_rank.data_ptr())
        desc = self.tables.desc_with(channels)
        capi.check(self.batch.lib.oc_render_ordered(self.batch._h, ctypes.c_void_p(state.data_ptr()), rank_ptr,
                                                    ctypes.c_void_p(self.atlas.data_ptr()),
                                                    ctypes.c_void_p(self.background.data_ptr()), ctypes.byref(desc),
                                                    ctypes.c_void_p(out.data_ptr()), self.batch.B,
                                                    self.batch._stream()))
        return out


def image_shape(level: "_levels.Level") -> Tuple[int, int, int]:
    return level.height * TILE, level.width * TILE, 3
