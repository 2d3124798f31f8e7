"""Kitchen levels for the batched Overcooked step engine (host side).

This module turns a kitchen level into the static tables the engine needs:
a tile-class grid, the initial item slots, the agent spawns and the recipe
goal masks.  It restates the parsing rules of the reference loader
``OvercookedEnvironment.load_level`` (gym_cooking/envs/overcooked_environment.py:130-198):

* map characters go through ``RepToClass`` (gym_cooking/utils/core.py:372-381):
  ``' '`` Floor, ``-`` Counter, ``/`` Cutboard, ``*`` Delivery, ``t l o p`` a Counter
  holding a fresh Tomato / Lettuce / Onion / a Plate (overcooked_environment.py:158-165);
  any other character becomes Floor (overcooked_environment.py:170-173);
* only Floor is non-collidable (core.py:34, 64);
* width is the last map row's length, height the number of map rows
  (overcooked_environment.py:196-197).  Ragged maps follow from that: a row longer than
  the last one puts squares past the world width: ``reset`` works, but every ``step``
  raises ``IndexError`` after executing the actions, when ``display`` writes those squares
  into a width-wide character grid (overcooked_environment.py:283 -> world.py:50, :302);
  a row shorter than the last one leaves squares of the grid without a GridSquare, and
  ``reset`` raises ``KeyError`` in ``make_reachability_graph`` (overcooked_environment.py:235
  -> world.py:79-86).  The batched engine refuses both (IndexError / KeyError at creation);
  the single-env shim mirrors the reference call by call;
* agents ``agent-1..A`` take the first A spawn lines (overcooked_environment.py:186-193);
* recipe lines name recipe classes (recipe_planner/recipe.py:199-228); each recipe
  contributes one ``Deliver(full_plate_name)`` subtask (recipe.py:39-47) whose goal
  object has every food in its last state (navigation_planner/utils.py:231-238).

Item contents are encoded as a byte mask in one of two encodings (include/oc_engine.h):
* ENC_PRESENCE, for levels with at most one of each food type
  (every shipped level): bit0 Tomato, bit1 Lettuce, bit2 Onion, bit3 Plate, bit4/5/6
  Tomato/Lettuce/Onion chopped;
* ENC_COUNTS, chosen when the map holds a food type more than once (load_level makes one
  Object per map character with no uniqueness check, overcooked_environment.py:158-165, and
  merges may then stack two of one food, core.py:194-202): 2-bit counts of Tomato (bits 0-1),
  Lettuce (2-3) and Onion (4-5), bit6 Plate, bit7 Fresh.  An object's identity is its
  full_name, a sorted multiset of content names (core.py:143-171); a merged object holds only
  foods in their last state and at most one plate (mergeable, core.py:222-241), so the Fresh
  bit only ever marks a single fresh food and the mask is exact for up to 3 of each food.
Grids of up to 1,024 cells (width and height up to 255) are supported: cell ids are bytes
(0xFF = dead) up to 255 cells, u16 (0xFFFF = dead) past that (the engine's wide layout).
"""
from __future__ import annotations

import dataclasses
import os
from typing import Dict, List, Sequence, Tuple

TILE_FLOOR = 0
TILE_COUNTER = 1
TILE_CUTBOARD = 2
TILE_DELIVERY = 3

M_TOMATO = 0x01
M_LETTUCE = 0x02
M_ONION = 0x04
M_PLATE = 0x08
M_TOMATO_CHOPPED = 0x10
M_LETTUCE_CHOPPED = 0x20
M_ONION_CHOPPED = 0x40
M_FOODS = M_TOMATO | M_LETTUCE | M_ONION

ENC_PRESENCE = 0
ENC_COUNTS = 1
MC_TOMATO = 0x01   # count fields: Tomato bits 0-1, Lettuce 2-3, Onion 4-5
MC_LETTUCE = 0x04
MC_ONION = 0x10
MC_PLATE = 0x40
MC_FRESH = 0x80
MAX_PER_FOOD = 3   # ENC_COUNTS: 2-bit counts

# Engine limits (include/oc_engine.h).
MAX_AGENTS = 4
MAX_ITEMS = 16
MAX_CELLS = 1024          # OC_MAX_CELLS
MAX_NARROW_CELLS = 255    # OC_MAX_NARROW_CELLS: byte cell ids up to here
MAX_GOALS = 4
LOC_DEAD = 0xFF
HOLD_NONE = 0xFF

# Action codes: World.NAV_ACTIONS order (gym_cooking/utils/world.py:16) + no-op.
ACTIONS: Tuple[Tuple[int, int], ...] = ((0, 1), (0, -1), (-1, 0), (1, 0), (0, 0))
NOOP = 4
ACTION_CODE = {a: i for i, a in enumerate(ACTIONS)}

_CHAR_TILE = {" ": TILE_FLOOR, "-": TILE_COUNTER, "/": TILE_CUTBOARD, "*": TILE_DELIVERY}
_CHAR_ITEM = {"t": "FreshTomato", "l": "FreshLettuce", "o": "FreshOnion", "p": "Plate"}  # content full names
_FOOD_NAMES = (("Tomato", M_TOMATO), ("Lettuce", M_LETTUCE), ("Onion", M_ONION))
_FOOD_COUNT = {"Tomato": MC_TOMATO, "Lettuce": MC_LETTUCE, "Onion": MC_ONION}


def chopped(mask_bit: int) -> int:
    """Chopped-state bit of a food presence bit."""
    return mask_bit << 4


# Recipe -> Deliver goal object full name (recipe.py:199-228; foods in last state, plated).
RECIPE_GOAL_NAMES: Dict[str, str] = {
    "SimpleTomato": "ChoppedTomato-Plate",
    "SimpleLettuce": "ChoppedLettuce-Plate",
    "Salad": "ChoppedLettuce-ChoppedTomato-Plate",
    "OnionSalad": "ChoppedLettuce-ChoppedOnion-ChoppedTomato-Plate",
}


def mask_contents(mask: int, enc: int = ENC_PRESENCE) -> List[Tuple[str, str]]:
    """The (name, full_name) of every content of an item mask, sorted by name as
    Object.update_names sorts them (core.py:161-171)."""
    parts = []
    if enc == ENC_COUNTS:
        for name, bit in _FOOD_COUNT.items():
            n = (mask // bit) & 3
            state = "Fresh" if mask & MC_FRESH else "Chopped"
            parts += [(name, state + name)] * n
        if mask & MC_PLATE:
            parts.append(("Plate", "Plate"))
    else:
        for name, bit in _FOOD_NAMES:
            if mask & bit:
                parts.append((name, ("Chopped" if mask & chopped(bit) else "Fresh") + name))
        if mask & M_PLATE:
            parts.append(("Plate", "Plate"))
    parts.sort(key=lambda p: p[0])
    return parts


def contents_mask(full_names: Sequence[str], enc: int = ENC_PRESENCE) -> int:
    """The item mask of an object whose contents have these full names ("FreshTomato",
    "ChoppedLettuce", "Plate", ...).  Raises ValueError for contents the encoding cannot hold
    (two of one food under ENC_PRESENCE, a fresh food inside a merge or more than 3 of one
    food under ENC_COUNTS, two plates)."""
    mask = 0
    plates = 0
    foods = []
    for part in full_names:
        if part == "Plate":
            plates += 1
            continue
        for name, bit in _FOOD_NAMES:
            if part in ("Fresh" + name, "Chopped" + name):
                foods.append((name, part.startswith("Chopped")))
                break
        else:
            raise ValueError("unknown content %r" % part)
    if plates > 1:
        raise ValueError("two plates in one object")
    if enc == ENC_COUNTS:
        mask = MC_PLATE if plates else 0
        for name, ch in foods:
            if (mask // _FOOD_COUNT[name]) & 3 == MAX_PER_FOOD:
                raise ValueError("more than %d %s in one object" % (MAX_PER_FOOD, name))
            mask += _FOOD_COUNT[name]
        fresh = [not ch for _, ch in foods]
        if any(fresh):
            if len(foods) + plates != 1:
                raise ValueError("a fresh food inside a merged object")
            mask |= MC_FRESH
        return mask
    mask = M_PLATE if plates else 0
    for name, ch in foods:
        bit = dict(_FOOD_NAMES)[name]
        if mask & bit:
            raise ValueError("two %s in one object: use ENC_COUNTS" % name)
        mask |= bit | (chopped(bit) if ch else 0)
    return mask


def mask_full_name(mask: int, enc: int = ENC_PRESENCE) -> str:
    """Reference ``Object.full_name`` of an item mask (core.py:161-171): contents sorted by
    base name, foods prefixed by their state, joined by '-'."""
    return "-".join(p[1] for p in mask_contents(mask, enc))


def full_name_mask(full_name: str, enc: int = ENC_PRESENCE) -> int:
    """Inverse of :func:`mask_full_name`."""
    return contents_mask(full_name.split("-"), enc)


def goal_mask(recipe: str, enc: int = ENC_PRESENCE) -> int:
    """The Deliver goal mask of a recipe class in an encoding."""
    return full_name_mask(RECIPE_GOAL_NAMES[recipe], enc)


# Recipe -> Deliver goal mask in the presence encoding (every shipped level).
RECIPE_GOALS: Dict[str, int] = {r: goal_mask(r) for r in RECIPE_GOAL_NAMES}


def needs_chopped(mask: int, enc: int = ENC_PRESENCE) -> bool:
    """Object.needs_chopped (core.py:176-178): one content, a fresh food."""
    if enc == ENC_COUNTS:
        return bool(mask & MC_FRESH)
    foods = mask & M_FOODS
    return len(mask_contents(mask)) == 1 and foods != 0 and not (mask >> 4) & foods


def is_deliverable(mask: int, enc: int = ENC_PRESENCE) -> bool:
    """Object.is_deliverable (core.py:214-219): merged, every food in its last state."""
    parts = mask_contents(mask, enc)
    return len(parts) >= 2 and all(fn == "Plate" or fn.startswith("Chopped") for _, fn in parts)


@dataclasses.dataclass
class Level:
    """Static description of one kitchen (what ``load_level`` builds)."""

    name: str
    width: int
    height: int
    tiles: List[int]                      # row-major, cell = y * width + x
    items: List[Tuple[int, int]]          # (cell, mask) in map scan order
    spawns: List[Tuple[int, int]]         # (x, y) spawn lines
    recipes: List[str]
    encoding: int = ENC_PRESENCE  # item / goal mask encoding (ENC_COUNTS when a food type repeats)
    # ragged maps: grid squares with no map character (a row shorter than the last one) and
    # map characters past the world width (a row longer than the last one), as (x, y, char)
    missing: List[Tuple[int, int]] = dataclasses.field(default_factory=list)
    overflow: List[Tuple[int, int, str]] = dataclasses.field(default_factory=list)

    @property
    def ncells(self) -> int:
        return self.width * self.height

    @property
    def goals(self) -> List[int]:
        """Unique Deliver goal masks, in recipe order."""
        out: List[int] = []
        for r in self.recipes:
            g = goal_mask(r, self.encoding)
            if g not in out:
                out.append(g)
        return out

    @property
    def delivery_cell(self) -> int:
        """First Delivery in scan order: ``done()`` reads only that one
        (overcooked_environment.py:349)."""
        for c, t in enumerate(self.tiles):
            if t == TILE_DELIVERY:
                return c
        raise ValueError("level %s has no Delivery" % self.name)

    def food_counts(self) -> Dict[str, int]:
        """Items of each food type on the map."""
        out = {name: 0 for name, _ in _FOOD_NAMES}
        for _, m in self.items:
            for name, _fn in mask_contents(m, self.encoding):
                if name != "Plate":
                    out[name] += 1
        return out

    @property
    def edge(self) -> bool:
        """Some Floor square lies on the grid's border (an action there can point off it)."""
        W, H = self.width, self.height
        return any(t == TILE_FLOOR and (c % W in (0, W - 1) or c // W in (0, H - 1)) for c, t in enumerate(self.tiles))

    def off_grid(self, x: int, y: int, code: int) -> bool:
        """Action `code` from (x, y) points outside the grid (World.NAV_ACTIONS order + no-op)."""
        dx, dy = ((0, 1), (0, -1), (-1, 0), (1, 0), (0, 0))[min(code, 4)]
        return not (0 <= x + dx < self.width and 0 <= y + dy < self.height)

    def tile_at(self, x: int, y: int) -> int:
        return self.tiles[y * self.width + x]

    def cell(self, x: int, y: int) -> int:
        return y * self.width + x

    def xy(self, cell: int) -> Tuple[int, int]:
        return cell % self.width, cell // self.width

    def within_width(self) -> "Level":
        """The same level without the squares past the world width (what a step sees before
        the reference's display raises)."""
        return dataclasses.replace(self, overflow=[])

    def reset_key_error(self) -> Tuple[int, int]:
        """The location whose lookup raises KeyError when the reference's reset builds the
        reachability graph of a map with missing squares: make_reachability_graph visits x
        then y and reads each square, then its four inbounds neighbours (world.py:79-86)."""
        miss = set(self.missing)
        W, H = self.width, self.height
        for x in range(W):
            for y in range(H):
                if (x, y) in miss:
                    return (x, y)
                for dx, dy in ACTIONS[:4]:
                    n = (min(max(x + dx, 0), W - 1), min(max(y + dy, 0), H - 1))
                    if n in miss:
                        return n
        raise AssertionError("no missing square")

    def validate(self, num_agents: int) -> None:
        """Reject levels outside the engine's exact-semantics envelope (raises ValueError)."""
        if not 1 <= num_agents <= MAX_AGENTS:
            raise ValueError("num_agents must be in 1..%d" % MAX_AGENTS)
        if self.missing:  # the reference cannot reset this level
            raise KeyError(self.reset_key_error())
        if self.overflow:  # the reference raises in every step
            x, y, _ = self.overflow[0]
            raise IndexError("level %s: square (%d,%d) lies past the world width %d; the reference's step "
                             "raises IndexError in World.add_object (world.py:302)" % (self.name, x, y, self.width))
        if len(self.spawns) < num_agents:
            raise ValueError("level %s has %d spawns < %d agents" % (self.name, len(self.spawns), num_agents))
        if self.ncells > MAX_CELLS or self.width > 255 or self.height > 255:
            raise ValueError("level %s: %dx%d = %d cells (at most %d, sides <= 255)"
                             % (self.name, self.width, self.height, self.ncells, MAX_CELLS))
        if len(self.items) > MAX_ITEMS:
            raise ValueError("level %s has %d items > %d" % (self.name, len(self.items), MAX_ITEMS))
        per_food = self.food_counts()
        if self.encoding == ENC_PRESENCE and max(per_food.values()) > 1:
            raise ValueError("level %s holds a food type twice: it needs ENC_COUNTS" % self.name)
        if max(per_food.values()) > MAX_PER_FOOD:
            raise ValueError("level %s holds %d of one food type > %d (2-bit content counts)"
                             % (self.name, max(per_food.values()), MAX_PER_FOOD))
        if not self.recipes:
            raise ValueError("level %s has no recipe (done() asserts a Deliver subtask)" % self.name)
        if len(self.goals) > MAX_GOALS:
            raise ValueError("too many goals")
        self.delivery_cell  # noqa: B018 -- raises if absent
        # A Floor on the border is allowed: is_collision looks the unclamped next square up
        # (overcooked_environment.py:692-700), so with 2+ agents an action off the grid makes
        # step raise (the engine's ERR, include/oc_engine.h), and interact clamps it for one.
        W, H = self.width, self.height
        for (x, y) in self.spawns[:num_agents]:
            if not (0 <= x < W and 0 <= y < H) or self.tile_at(x, y) != TILE_FLOOR:
                raise ValueError("level %s: spawn (%d,%d) is not a Floor" % (self.name, x, y))


def parse_level_text(text: str, name: str = "custom") -> Level:
    """Parse the reference's level file format (overcooked_environment.py:144-193):
    map rows, blank line, recipe class names, blank line, ``x y`` spawn lines."""
    phase = 1
    rows: List[str] = []
    recipes: List[str] = []
    spawns: List[Tuple[int, int]] = []
    for line in text.split("\n"):
        line = line.rstrip("\r")
        if line == "":
            phase += 1
        elif phase == 1:
            rows.append(line)
        elif phase == 2:
            if line not in RECIPE_GOAL_NAMES:
                raise ValueError("unknown recipe %r" % line)
            recipes.append(line)
        elif phase == 3:
            xs = line.split(" ")
            spawns.append((int(xs[0]), int(xs[1])))
    if not rows:
        raise ValueError("empty map")
    width = len(rows[-1])  # world.width = x + 1 of the last map row (:196)
    tiles: List[int] = []
    items: List[Tuple[int, str]] = []
    missing: List[Tuple[int, int]] = []
    overflow: List[Tuple[int, int, str]] = []
    for y, row in enumerate(rows):
        for x in range(width):
            if x >= len(row):  # no GridSquare here: the reference's reset raises KeyError
                missing.append((x, y))
                tiles.append(TILE_COUNTER)
                continue
            ch = row[x]
            if ch in _CHAR_ITEM:
                tiles.append(TILE_COUNTER)
                items.append((y * width + x, _CHAR_ITEM[ch]))
            else:
                tiles.append(_CHAR_TILE.get(ch, TILE_FLOOR))
        overflow.extend((x, y, row[x]) for x in range(width, len(row)))
    foods = [fn for _, fn in items if fn != "Plate"]
    enc = ENC_COUNTS if len(foods) != len(set(foods)) else ENC_PRESENCE
    return Level(name=name, width=width, height=len(rows), tiles=tiles,
                 items=[(c, contents_mask([fn], enc)) for c, fn in items], spawns=spawns, recipes=recipes,
                 encoding=enc, missing=missing, overflow=overflow)


def _builtin(divider: str, recipes: Sequence[str], name: str) -> Level:
    """The nine shipped kitchens share one 7x7 frame: tomato (5,0), lettuce (6,1),
    plates (6,5) and (5,6), delivery (0,3), cutboards (0,1) and (0,2); they differ
    only in the x=3 divider (open: none, partial: y=1..4, full: y=1..5) and the recipes."""
    div_rows = {"open": (), "partial": (1, 2, 3, 4), "full": (1, 2, 3, 4, 5)}[divider]
    left = {1: "/", 2: "/", 3: "*", 4: "-", 5: "-"}
    right = {1: "l", 2: "-", 3: "-", 4: "-", 5: "p"}
    rows = ["-----t-"]
    for y in range(1, 6):
        mid = "  " + ("-" if y in div_rows else " ") + "  "
        rows.append(left[y] + mid + right[y])
    rows.append("-----p-")
    text = "\n".join(rows) + "\n\n" + "\n".join(recipes) + "\n\n" + "2 1\n4 1\n4 4\n2 4\n"
    return parse_level_text(text, name)


_RECIPE_SETS = {"salad": ("Salad",), "tomato": ("SimpleTomato",), "tl": ("SimpleTomato", "SimpleLettuce")}

BUILTIN_LEVELS: Dict[str, Level] = {
    "%s-divider_%s" % (d, r): _builtin(d, rs, "%s-divider_%s" % (d, r))
    for d in ("open", "partial", "full") for r, rs in _RECIPE_SETS.items()
}


def load_level(name_or_path: str) -> Level:
    """A builtin level by name, or a level file in the reference's text format."""
    if name_or_path in BUILTIN_LEVELS:
        return BUILTIN_LEVELS[name_or_path]
    if os.path.isfile(name_or_path):
        with open(name_or_path) as f:
            return parse_level_text(f.read(), os.path.splitext(os.path.basename(name_or_path))[0])
    raise KeyError("unknown level %r" % name_or_path)
