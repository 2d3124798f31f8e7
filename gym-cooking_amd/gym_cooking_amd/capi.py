"""ctypes binding of the engine's C-ABI (include/oc_engine.h).

The product path loads ``liboc_engine.so`` (built in-tree by ``csrc/Makefile``) and fails
loudly when it is missing: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

from . import levels as _lv

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "liboc_engine.so")

OC_MAX_AGENTS = 4
OC_MAX_ITEMS = 16
OC_MAX_CELLS = 1024         # grid cells (width and height <= 255)
OC_MAX_NARROW_CELLS = 255   # up to this many cells: byte cell ids; more ("wide"): u16 ids
OC_MAX_GOALS = 4
OC_PITCH_ALIGN = 4096
OC_NSTATS = 5
OC_ABI_VERSION = 10  # include/oc_engine.h
OC_DEVICE_HOST = -1  # oc_create: a host-only handle (no HIP call)
OC_LIK_FORM_AUTO, OC_LIK_FORM_GROUPED = 0, 1
OC_EINVAL, OC_EHIP, OC_ELEVEL = -1, -2, -3

OC_FLAG_DONE = 0x01
OC_FLAG_SUCCESS = 0x02
OC_FLAG_ERR = 0x04

OC_STAT_NAMES = ("episodes", "successes", "steps", "collisions", "errors")

# Every symbol include/oc_engine.h declares (tests check the library exports them all).
EXPORTED_SYMBOLS = (
    "oc_abi_version", "oc_last_error", "oc_create", "oc_destroy", "oc_get_layout", "oc_reset",
    "oc_step", "oc_step_n", "oc_cpu_step", "oc_rollout", "oc_nav_likelihood", "oc_subtask_bounds", "oc_reachability", "oc_reachability16", "oc_render", "oc_render_ordered",
    "oc_gen_actions", "oc_state_checksum", "oc_stats_size", "oc_stats_reduce", "oc_get_last_error",
    "oc_set_likelihood_form",
)


class OcLevelDesc(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32), ("num_items", ctypes.c_int32),
        ("num_spawns", ctypes.c_int32), ("num_goals", ctypes.c_int32),
        ("tiles", ctypes.c_uint8 * OC_MAX_CELLS),
        ("item_cell", ctypes.c_uint16 * OC_MAX_ITEMS), ("item_mask", ctypes.c_uint8 * OC_MAX_ITEMS),
        ("spawn_x", ctypes.c_uint8 * OC_MAX_AGENTS), ("spawn_y", ctypes.c_uint8 * OC_MAX_AGENTS),
        ("goal_mask", ctypes.c_uint8 * OC_MAX_GOALS),
        ("encoding", ctypes.c_int32),
    ]


class OcLayout(ctypes.Structure):
    _fields_ = [
        ("pitch", ctypes.c_int64), ("state_bytes", ctypes.c_int64),
        ("num_agents", ctypes.c_int32), ("num_items", ctypes.c_int32),
        ("plane_agent_x", ctypes.c_int32), ("plane_agent_y", ctypes.c_int32),
        ("plane_agent_hold", ctypes.c_int32), ("plane_item_loc", ctypes.c_int32),
        ("plane_item_mask", ctypes.c_int32), ("plane_t", ctypes.c_int32),
        ("plane_flags", ctypes.c_int32), ("num_planes", ctypes.c_int32),
        ("plane_item_loc_hi", ctypes.c_int32), ("cell_bytes", ctypes.c_int32),
    ]


SUB_NONE, SUB_CHOP, SUB_MERGE, SUB_DELIVER = 0, 1, 2, 3
ROLL_LEGAL, ROLL_GOAL, ROLL_ASSERT, ROLL_BADALLOC = 0x01, 0x02, 0x04, 0x80
MAX_SUBTASKS = 64
LIK_OK, LIK_RAISES, LIK_ZERODIV, LIK_BADALLOC = 0x01, 0x04, 0x08, 0x80
ROLL_RAISES = 0x08


class OcSubtask(ctypes.Structure):
    """oc_subtask (include/oc_engine.h): one navigation-planner configuration."""
    _fields_ = [("kind", ctypes.c_int32), ("num_agents", ctypes.c_int32), ("agent", ctypes.c_uint8 * 2),
                ("start_mask", ctypes.c_uint8 * 2), ("goal_mask", ctypes.c_uint8),
                ("goal_count", ctypes.c_uint8), ("level", ctypes.c_uint8), ("reserved", ctypes.c_uint8)]


OC_RENDER_SIZES = 4
OC_CHAN_RGB = 0x00020100
OC_CHAN_REFERENCE = 0x00030100


class OcRenderDesc(ctypes.Structure):
    """oc_render_desc (include/oc_engine.h): sprite atlas layout and output channel map."""
    _fields_ = [("tile", ctypes.c_int32), ("size", ctypes.c_int32 * OC_RENDER_SIZES),
                ("offset", ctypes.c_int32 * OC_RENDER_SIZES), ("food_base", ctypes.c_int32 * OC_RENDER_SIZES),
                ("plate_off", ctypes.c_int32 * 2), ("agent_off", ctypes.c_int32 * OC_MAX_AGENTS),
                ("food_sprite", ctypes.c_uint8 * 128), ("chan_map", ctypes.c_uint32)]


def subtask(kind: int, agents, start_masks, goal_mask: int, goal_count: int = 0, level: int = 0) -> OcSubtask:
    s = OcSubtask()
    s.level = level
    s.kind = kind
    s.num_agents = len(agents)
    for i, a in enumerate(agents):
        s.agent[i] = a
    for i, m in enumerate(start_masks):
        s.start_mask[i] = m
    s.goal_mask = goal_mask
    s.goal_count = goal_count
    return s


def subtask_array(subtasks):
    arr = (OcSubtask * len(subtasks))()
    for i, s in enumerate(subtasks):
        arr[i] = s
    return arr


def level_desc(level: "_lv.Level", num_agents: int) -> OcLevelDesc:
    """Pack a :class:`levels.Level` into the C struct (validates it first)."""
    level.validate(num_agents)
    d = OcLevelDesc()
    d.width, d.height = level.width, level.height
    d.num_items = len(level.items)
    d.num_spawns = min(len(level.spawns), OC_MAX_AGENTS)
    goals = level.goals
    d.num_goals = len(goals)
    for c, t in enumerate(level.tiles):
        d.tiles[c] = t
    for i, (cell, mask) in enumerate(level.items):
        d.item_cell[i] = cell
        d.item_mask[i] = mask
    for i, (x, y) in enumerate(level.spawns[:OC_MAX_AGENTS]):
        d.spawn_x[i] = x
        d.spawn_y[i] = y
    for i, g in enumerate(goals):
        d.goal_mask[i] = g
    d.encoding = level.encoding
    return d


def item_slots(level: "_lv.Level") -> int:
    """K: item slots of the state layout (level items rounded up to 4, 8 or 16)."""
    n = len(level.items)
    return 4 if n <= 4 else (8 if n <= 8 else 16)


def is_wide(level: "_lv.Level") -> bool:
    """More than 255 cells: u16 cell ids (the wide layout, include/oc_engine.h oc_layout)."""
    return level.width * level.height > OC_MAX_NARROW_CELLS


def layout_planes(A: int, K: int, wide: bool = False) -> dict:
    """Plane indices of oc_layout for (A, K) -- mirrors oc_get_layout (pure arithmetic).  A wide
    level has its item cells' high bytes in K planes after the low ones (item_loc_hi)."""
    LK = 2 * K if wide else K
    return dict(agent_x=0, agent_y=A, agent_hold=2 * A, item_loc=3 * A, item_loc_hi=3 * A + K if wide else -1,
                item_mask=3 * A + LK, t=3 * A + LK + K, flags=3 * A + LK + K + 2, num_planes=3 * A + LK + K + 3,
                cell_bytes=2 if wide else 1)


def pitch_for(B: int) -> int:
    return max(OC_PITCH_ALIGN, (B + OC_PITCH_ALIGN - 1) // OC_PITCH_ALIGN * OC_PITCH_ALIGN)


_lib: Optional[ctypes.CDLL] = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load liboc_engine.so; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.isfile(path):
        raise RuntimeError("liboc_engine.so not built at %s (run __graft_entry__.build() or "
                           "make -C gym-cooking_amd/csrc)" % path)
    lib = ctypes.CDLL(path)
    vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    lib.oc_abi_version.restype = ctypes.c_int
    lib.oc_abi_version.argtypes = []
    lib.oc_last_error.restype = ctypes.c_char_p
    lib.oc_last_error.argtypes = []
    lib.oc_create.restype = ctypes.c_int
    lib.oc_create.argtypes = [ctypes.POINTER(OcLevelDesc), i32, i32, i32, ctypes.POINTER(vp)]
    lib.oc_destroy.restype = ctypes.c_int
    lib.oc_destroy.argtypes = [vp]
    lib.oc_get_layout.restype = ctypes.c_int
    lib.oc_get_layout.argtypes = [vp, i64, ctypes.POINTER(OcLayout)]
    lib.oc_reset.restype = ctypes.c_int
    lib.oc_reset.argtypes = [vp, vp, i64, vp]
    lib.oc_step.restype = ctypes.c_int
    lib.oc_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, i64, vp]
    lib.oc_rollout.restype = ctypes.c_int
    lib.oc_rollout.argtypes = [vp, vp, vp, vp, vp, ctypes.POINTER(OcSubtask), i32, vp, vp, i64, vp]
    lib.oc_nav_likelihood.restype = ctypes.c_int
    lib.oc_nav_likelihood.argtypes = [vp, vp, vp, vp, ctypes.POINTER(OcSubtask), i32, i32, ctypes.c_double,
                                      ctypes.c_double, vp, vp, i64, vp]
    lib.oc_render.restype = ctypes.c_int
    lib.oc_subtask_bounds.restype = ctypes.c_int
    lib.oc_subtask_bounds.argtypes = [vp, vp, ctypes.POINTER(OcSubtask), i32, vp, vp, i64, vp]
    lib.oc_reachability.restype = ctypes.c_int
    lib.oc_reachability.argtypes = [vp, ctypes.POINTER(i32), vp, i64, vp, i64]
    lib.oc_reachability16.restype = ctypes.c_int
    lib.oc_reachability16.argtypes = [vp, ctypes.POINTER(i32), vp, i64, vp, i64]
    lib.oc_render.argtypes = [vp, vp, vp, vp, ctypes.POINTER(OcRenderDesc), vp, i64, vp]
    lib.oc_render_ordered.restype = ctypes.c_int
    lib.oc_render_ordered.argtypes = [vp, vp, vp, vp, vp, ctypes.POINTER(OcRenderDesc), vp, i64, vp]
    lib.oc_get_last_error.restype = ctypes.c_int
    lib.oc_get_last_error.argtypes = [vp, ctypes.c_char_p, i64]
    lib.oc_set_likelihood_form.restype = ctypes.c_int
    lib.oc_set_likelihood_form.argtypes = [vp, i32]
    lib.oc_cpu_step.restype = ctypes.c_int
    lib.oc_cpu_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, i64, i32]
    lib.oc_step_n.restype = ctypes.c_int
    lib.oc_step_n.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, vp]
    lib.oc_gen_actions.restype = ctypes.c_int
    lib.oc_gen_actions.argtypes = [vp, vp, i64, i64, i64, u64, vp]
    lib.oc_state_checksum.restype = ctypes.c_int
    lib.oc_state_checksum.argtypes = [vp, vp, i64, vp, vp]
    lib.oc_stats_size.restype = ctypes.c_int
    lib.oc_stats_size.argtypes = [vp, i64, ctypes.POINTER(i64)]
    lib.oc_stats_reduce.restype = ctypes.c_int
    lib.oc_stats_reduce.argtypes = [vp, vp, i64, vp, vp]
    if lib.oc_abi_version() != OC_ABI_VERSION:
        raise RuntimeError("liboc_engine ABI %d, binding expects %d (rebuild)" % (lib.oc_abi_version(), OC_ABI_VERSION))
    _lib = lib
    return lib


class LevelError(RuntimeError):
    """OC_ELEVEL: the level is outside an entry point's envelope (oc_create's validation: more
    than 1,024 cells, a 17th object or a 4th of one food; oc_reachability's u8 table: a
    reachability graph with a BFS distance of 255 or more, which oc_reachability16 exports)."""


def check(rc: int) -> None:
    if rc != 0:
        msg = _lib.oc_last_error().decode() if _lib is not None else "?"
        cls = LevelError if rc == OC_ELEVEL else RuntimeError
        raise cls("oc_engine error %d: %s" % (rc, msg))
