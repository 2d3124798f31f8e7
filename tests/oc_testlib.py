"""Shared test helpers: canonical state views, golden-fixture replay."""
from __future__ import annotations

import os
import sys
from typing import Dict, List

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))
sys.path.insert(0, ROOT)

from gym_cooking_amd import capi, levels  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
PAD = 255


def _layout(state: np.ndarray, A: int, K: int, pitch: int) -> dict:
    """oc_layout planes of a flat buffer: narrow (3A + 2K + 3 planes) or wide (3A + 3K + 3,
    u16 item cells), told apart by the buffer's size."""
    wide = state.size // pitch >= 3 * A + 3 * K + 3
    return capi.layout_planes(A, K, wide)


def planes_view(state: np.ndarray, A: int, K: int, pitch: int) -> Dict[str, np.ndarray]:
    """Split a flat layout buffer (host numpy) into named plane views.  `il` is the item cells:
    a view of the byte planes (narrow) or a u16 copy (wide: low | high << 8)."""
    P = _layout(state, A, K, pitch)
    s = state.reshape(-1, pitch)[:P["num_planes"]]
    il = s[P["item_loc"]:P["item_loc"] + K]
    if P["cell_bytes"] == 2:
        il = il.astype(np.uint16) | (s[P["item_loc_hi"]:P["item_loc_hi"] + K].astype(np.uint16) << 8)
    return dict(
        ax=s[P["agent_x"]:P["agent_x"] + A], ay=s[P["agent_y"]:P["agent_y"] + A],
        ah=s[P["agent_hold"]:P["agent_hold"] + A], il=il,
        im=s[P["item_mask"]:P["item_mask"] + K],
        t=s[P["t"]:P["t"] + 2].reshape(-1).view(np.uint16)[:pitch], fl=s[P["flags"]],
    )


def env_view(state: np.ndarray, A: int, K: int, pitch: int, B: int) -> np.ndarray:
    """All state bytes of envs [0, B) as a [num_planes, B] array (the u16 t plane split into
    its low/high bytes), independent of the pitch."""
    P = _layout(state, A, K, pitch)
    s = state.reshape(P["num_planes"], pitch)
    t = s[P["t"]:P["t"] + 2].reshape(-1).view(np.uint16)[:B]
    rows = [s[:P["t"], :B], (t & 0xFF).astype(np.uint8)[None], (t >> 8).astype(np.uint8)[None],
            s[P["flags"]:P["flags"] + 1, :B]]
    return np.concatenate(rows, 0)


def checksum(state: np.ndarray, A: int, K: int, pitch: int, B: int) -> int:
    """Host twin of oc_state_checksum (include/oc_engine.h)."""
    ev = env_view(state, A, K, pitch, B).astype(np.uint64)           # [planes, B]
    p = np.arange(ev.shape[0], dtype=np.uint64)
    M = np.uint64(0x9E3779B97F4A7C15) * (np.uint64(2) * p + np.uint64(1))
    with np.errstate(over="ignore"):
        h = ((ev + np.uint64(1)) * M[:, None]).sum(axis=0, dtype=np.uint64)
        w = np.uint64(2) * np.arange(B, dtype=np.uint64) + np.uint64(1)
        return int((h * w).sum(dtype=np.uint64))


def canonical(state: np.ndarray, A: int, K: int, pitch: int, width: int, B: int):
    """SURVEY App. A.7 canonical form of the first B envs: t, flags, agents [B,4,3]
    (x, y, held mask), items [B,K,4] sorted (mask, x, y, held), PAD rows last."""
    v = planes_view(state, A, K, pitch)
    ax, ay, ah = v["ax"][:, :B].T, v["ay"][:, :B].T, v["ah"][:, :B].T      # [B, A]
    il, im = v["il"][:, :B].T.astype(np.int64), v["im"][:, :B].T.astype(np.int64)  # [B, K]
    agents = np.full((B, 4, 3), PAD, np.uint8)
    agents[:, :A, 0] = ax
    agents[:, :A, 1] = ay
    hold = ah.astype(np.int64)
    hm = np.where(hold < K, np.take_along_axis(im, np.minimum(hold, K - 1), axis=1), 0)
    agents[:, :A, 2] = hm
    held = np.zeros((B, K), bool)
    for a in range(A):
        held |= hold[:, a:a + 1] == np.arange(K)[None, :]
    alive = il != (0xFFFF if v["il"].dtype == np.uint16 else 0xFF)
    x, y = il % width, il // width
    key = (im << 24) | (x << 16) | (y << 8) | held.astype(np.int64)
    key = np.where(alive, key, 0xFFFFFFFF)
    key.sort(axis=1)
    items = np.stack([(key >> 24) & 0xFF, (key >> 16) & 0xFF, (key >> 8) & 0xFF, key & 0xFF], -1)
    items = np.where((key == 0xFFFFFFFF)[..., None], PAD, items).astype(np.uint8)
    if K < 4:
        items = np.concatenate([items, np.full((B, 4 - K, 4), PAD, np.uint8)], 1)
    # 4 item rows (the 7x7 fixtures' width), 8 for levels with 8 item slots
    return dict(t=v["t"][:B].copy(), flags=v["fl"][:B].copy(), agents=agents, items=items[:, :max(4, K)])


def load_level(name: str) -> levels.Level:
    """A builtin level by name, or a committed level file (tests/golden/levels/*.txt, stored
    in fixtures as a path relative to tests/golden)."""
    if name.endswith(".txt") and not os.path.isabs(name):
        name = os.path.join(GOLDEN, name)
    return levels.load_level(name)


def load_fixture(name: str) -> Dict[str, np.ndarray]:
    """All arrays of a golden .npz, materialised (NpzFile re-reads an array on every index)."""
    with np.load(os.path.join(GOLDEN, name)) as z:
        return {k: z[k] for k in z.files}


class EpisodeGroup:
    """Fixture episodes sharing (level, A, max_T), replayed in lockstep as one batch."""

    def __init__(self, fx, idx: List[int]):
        self.fx = fx
        self.idx = idx
        e0 = idx[0]
        self.level = load_level(str(fx["level_names"][fx["ep_level"][e0]]))
        self.A = int(fx["ep_A"][e0])
        self.max_T = int(fx["ep_maxT"][e0])
        self.B = len(idx)
        self.T = np.array([fx["ep_T"][e] for e in idx])
        self.K = capi.item_slots(self.level)

    def actions_at(self, step: int) -> np.ndarray:
        """[A, B] action codes at `step` (noop past an episode's end)."""
        out = np.full((self.A, self.B), 4, np.uint8)
        for b, e in enumerate(self.idx):
            if step < self.fx["ep_T"][e]:
                out[:, b] = self.fx["act"][self.fx["ep_act_off"][e] + step][:self.A]
        return out

    def relocate(self, state: np.ndarray, pitch: int) -> None:
        v = planes_view(state, self.A, self.K, pitch)
        for b, e in enumerate(self.idx):
            st = self.fx["ep_start"][e]
            for a in range(self.A):
                if st[a, 0] != PAD:
                    v["ax"][a, b], v["ay"][a, b] = st[a, 0], st[a, 1]

    def expected(self, step_state: int, b: int):
        """Expected canonical record after `step_state` steps for batch env b (None past end)."""
        e = self.idx[b]
        if step_state > self.fx["ep_T"][e]:
            return None
        o = self.fx["ep_state_off"][e] + step_state
        return dict(t=self.fx["t"][o], flags=self.fx["flags"][o], agents=self.fx["agents"][o],
                    items=self.fx["items"][o])

    def expected_step(self, step: int, b: int):
        e = self.idx[b]
        if step >= self.fx["ep_T"][e]:
            return None
        o = self.fx["ep_act_off"][e] + step
        return self.fx["exe"][o], self.fx["coll"][o]


def episode_groups(fx) -> List[EpisodeGroup]:
    keys = {}
    for e in range(len(fx["ep_T"])):
        k = (int(fx["ep_level"][e]), int(fx["ep_A"][e]), int(fx["ep_maxT"][e]))
        keys.setdefault(k, []).append(e)
    return [EpisodeGroup(fx, v) for _, v in sorted(keys.items())]


def compare_group(group: EpisodeGroup, step_fn, init_state: np.ndarray, pitch: int, width: int):
    """Replay `group` through step_fn(state_in, actions[A,B]) -> (state_out, exec[A,B], coll[B]),
    comparing against the fixtures; returns the list of mismatch descriptions."""
    errs = []
    state = init_state
    alive = np.ones(group.B, bool)
    c = canonical(state, group.A, group.K, pitch, width, group.B)
    for b in range(group.B):
        exp = group.expected(0, b)
        if not _eq(c, b, exp):
            errs.append("env %d: initial state mismatch" % group.idx[b])
    for step in range(int(group.T.max())):
        acts = group.actions_at(step)
        state, ex, coll = step_fn(state, acts)
        c = canonical(state, group.A, group.K, pitch, width, group.B)
        for b in range(group.B):
            if not alive[b]:
                continue
            exp = group.expected(step + 1, b)
            if exp is None:
                alive[b] = False
                continue
            if exp["flags"] & 0x04:  # ERR: the reference raised; only the flag is defined
                if c["flags"][b] != exp["flags"]:
                    errs.append("env %d step %d: ERR flag %d vs %d" % (group.idx[b], step + 1,
                                                                       c["flags"][b], exp["flags"]))
                alive[b] = False
                continue
            if not _eq(c, b, exp):
                errs.append("env %d step %d: state mismatch got t=%d fl=%d ag=%s it=%s | exp t=%d fl=%d ag=%s it=%s" % (
                    group.idx[b], step + 1, c["t"][b], c["flags"][b], c["agents"][b].tolist(),
                    c["items"][b].tolist(), exp["t"], exp["flags"], exp["agents"].tolist(),
                    exp["items"].tolist()))
                alive[b] = False
                continue
            eex, ecoll = group.expected_step(step, b)
            if not (np.array_equal(ex[:, b], eex[:group.A]) and coll[b] == ecoll):
                errs.append("env %d step %d: exec %s coll %d vs %s %d" % (
                    group.idx[b], step + 1, ex[:, b].tolist(), coll[b], eex[:group.A].tolist(), ecoll))
                alive[b] = False
        if len(errs) > 20:
            break
    return errs


def _eq(c, b, exp) -> bool:
    # a fixture may carry more (PAD) item rows than the level's slots (8-row records of 4-slot levels)
    ci, ei = c["items"][b], exp["items"]
    items_ok = np.array_equal(ci, ei[:len(ci)]) and bool((ei[len(ci):] == PAD).all())
    return (int(c["t"][b]) == int(exp["t"]) and int(c["flags"][b]) == int(exp["flags"])
            and np.array_equal(c["agents"][b], exp["agents"]) and items_ok)


def state_from_canonical(level, A: int, K: int, pitch: int, agents: np.ndarray, items: np.ndarray,
                         t: np.ndarray) -> np.ndarray:
    """Engine-layout state buffer whose env b has the canonical state (agents [B,4,3], items
    [B,4,4], t [B]): items take slots in canonical order, and each holding agent holds the
    held item at its location with its held mask."""
    B = len(agents)
    wide = capi.is_wide(level)
    P = capi.layout_planes(A, K, wide)
    s = np.zeros(P["num_planes"] * pitch, np.uint8)
    v = planes_view(s, A, K, pitch)
    il = np.full((K, pitch), 0xFFFF if wide else 0xFF, np.uint16)  # item cells, written back below
    v["ah"][:] = 0xFF
    W = level.width
    for b in range(B):
        held_slots = []
        for j in range(items.shape[1]):
            m, x, y, h = (int(c) for c in items[b, j])
            if m == PAD:
                continue
            il[j, b], v["im"][j, b] = y * W + x, m
            if h:
                held_slots.append((j, x, y, m))
        for a in range(A):
            x, y, hm = (int(c) for c in agents[b, a])
            v["ax"][a, b], v["ay"][a, b] = x, y
            if hm not in (0, PAD):
                for i, (j, ix, iy, m) in enumerate(held_slots):
                    if (ix, iy, m) == (x, y, hm):
                        v["ah"][a, b] = j
                        held_slots.pop(i)
                        break
                else:
                    raise AssertionError("no held item for agent %d of env %d" % (a, b))
        v["t"][b] = t[b]
    sp = s.reshape(P["num_planes"], pitch)
    sp[P["item_loc"]:P["item_loc"] + K] = il & 0xFF
    if wide:
        sp[P["item_loc_hi"]:P["item_loc_hi"] + K] = il >> 8
    return s


class RolloutRows:
    """Rows of tests/golden/rollout.npz (planner Level 0) or rollout_level1.npz (Level 1) for
    one (level, A) config, with their subtask table."""

    def __init__(self, fx, cfg: int, limit=None, planner_level: int = 0):
        sel = np.nonzero(fx["cfg"] == cfg)[0]
        if limit is not None and len(sel) > limit:
            sel = sel[np.linspace(0, len(sel) - 1, limit).astype(int)]
        self.idx = sel
        self.level = load_level(str(fx["cfg_level"][cfg]))
        self.A = int(fx["cfg_A"][cfg])
        self.K = capi.item_slots(self.level)
        st = fx["state"][sel]
        self.agents, self.items, self.t = fx["st_agents"][st], fx["st_items"][st], fx["st_t"][st]
        self.B = len(sel)
        keys, self.alloc = {}, np.zeros(self.B, np.uint8)
        self.subtasks = []
        for r, i in enumerate(sel):
            n = int((fx["agents"][i] != PAD).sum())
            key = (int(fx["kind"][i]), tuple(int(a) for a in fx["agents"][i][:n]),
                   tuple(int(m) for m in fx["start"][i]), int(fx["goal_mask"][i]), int(fx["goal_count"][i]))
            if key not in keys:
                keys[key] = len(self.subtasks)
                self.subtasks.append(capi.subtask(key[0], key[1], key[2], key[3], key[4], planner_level))
            self.alloc[r] = keys[key]
        self.sub_agents = [tuple(int(a) for a in fx["agents"][i] if a != PAD) for i in sel]
        self.codes = fx["action"][sel]
        self.exp_flags = (fx["legal"][sel] * capi.ROLL_LEGAL | fx["goal"][sel] * capi.ROLL_GOAL
                          | fx["assert_"][sel] * capi.ROLL_ASSERT).astype(np.uint8)
        self.exp_lb = fx["lb"][sel]
        # rows where the reference's T raised copying a state with two co-located holders
        # (Level 1, actions outside get_actions only): only get_actions membership is compared
        self.copy_raise = fx["copy_raise"][sel] if "copy_raise" in fx else np.zeros(len(sel), np.int64)
        self.exp_next = fx["next"][sel]
        self.exp_vl, self.exp_vu = fx["v_l"][sel], fx["v_u"][sel]

    def split(self, max_sub: int = 64) -> List["RolloutRows"]:
        """The rows as chunks of at most `max_sub` subtask configurations (one oc_rollout call each)."""
        out = []
        for c0 in range(0, len(self.subtasks), max_sub):
            sel = np.nonzero((self.alloc >= c0) & (self.alloc < c0 + max_sub))[0]
            part = object.__new__(RolloutRows)
            part.__dict__ = dict(self.__dict__)
            for k in ("idx", "agents", "items", "t", "codes", "exp_flags", "exp_lb", "exp_next", "exp_vl", "exp_vu",
                      "copy_raise"):
                setattr(part, k, getattr(self, k)[sel])
            part.sub_agents = [self.sub_agents[i] for i in sel]
            part.alloc = (self.alloc[sel] - c0).astype(np.uint8)
            part.subtasks = self.subtasks[c0:c0 + max_sub]
            part.B = len(sel)
            out.append(part)
        return out

    def actions(self, pitch: int) -> np.ndarray:
        a = np.full((self.A, pitch), 4, np.uint8)
        for r in range(self.B):
            for q, ag in enumerate(self.sub_agents[r]):
                a[ag, r] = self.codes[r, q]
        return a.reshape(-1)

    def compare(self, sout: np.ndarray, flags: np.ndarray, lb: np.ndarray, pitch: int):
        """Mismatch descriptions of a rollout output against the reference rows."""
        errs = []
        c = canonical(sout, self.A, self.K, pitch, self.level.width, self.B)
        for r in range(self.B):
            if self.copy_raise[r]:
                if (flags[r] ^ self.exp_flags[r]) & capi.ROLL_LEGAL or self.exp_flags[r] & capi.ROLL_LEGAL:
                    errs.append("row %d: legal flag on a raising row" % self.idx[r])
                continue
            if flags[r] != self.exp_flags[r]:
                errs.append("row %d: flags %d vs %d" % (self.idx[r], flags[r], self.exp_flags[r]))
                continue
            if self.exp_flags[r] & capi.ROLL_ASSERT:
                continue
            if float(lb[r]) != float(self.exp_lb[r]):
                errs.append("row %d: lb %r vs %r" % (self.idx[r], float(lb[r]), float(self.exp_lb[r])))
            exp_ag = self.exp_next[r][:12].reshape(4, 3)
            exp_it = self.exp_next[r][12:].reshape(-1, 4)  # 4 item rows, or 8 (8-slot levels)
            for a in self.sub_agents[r]:
                if not np.array_equal(c["agents"][r, a], exp_ag[a]):
                    errs.append("row %d: agent %d %s vs %s" % (self.idx[r], a, c["agents"][r, a].tolist(),
                                                               exp_ag[a].tolist()))
            ci = c["items"][r]
            # a fixture may carry more (PAD) item rows than the level's slots (MAXK = 8 records of
            # 4-slot levels, as in _eq)
            if not (np.array_equal(ci, exp_it[:len(ci)]) and bool((exp_it[len(ci):] == PAD).all())):
                errs.append("row %d: items %s vs %s" % (self.idx[r], c["items"][r].tolist(), exp_it.tolist()))
            if len(errs) > 20:
                break
        return errs


class LikelihoodRows:
    """Rows of tests/golden/likelihood.npz for one (config, self agent), with subtask tables
    split into chunks of <= 64 configurations."""

    def __init__(self, fx, cfg: int, self_agent: int):
        st_cfg = fx["st_cfg"][fx["state"]]
        sel = np.nonzero((st_cfg == cfg) & (fx["self_agent"] == self_agent))[0]
        self.idx = sel
        self.self_agent = self_agent
        self.level = load_level(str(fx["cfg_level"][cfg]))
        self.A = int(fx["cfg_A"][cfg])
        self.K = capi.item_slots(self.level)
        st = fx["state"][sel]
        self.agents, self.items, self.t = fx["st_agents"][st], fx["st_items"][st], fx["st_t"][st]
        self.taken = fx["st_taken"][st]
        self.beta, self.nap = float(fx["beta"]), float(fx["none_action_prob"])
        self.B = len(sel)
        keys, self.alloc, self.subtasks = {}, np.zeros(self.B, np.int64), []
        for r, i in enumerate(sel):
            n = int((fx["agents"][i] != PAD).sum())
            key = (int(fx["kind"][i]), tuple(int(a) for a in fx["agents"][i][:n]),
                   tuple(int(m) for m in fx["start"][i]), int(fx["goal_mask"][i]), int(fx["goal_count"][i]))
            if key not in keys:
                keys[key] = len(self.subtasks)
                self.subtasks.append(capi.subtask(*key))
            self.alloc[r] = keys[key]
        self.exp_value, self.exp_raised = fx["value"][sel], fx["raised"][sel]

    def chunks(self, max_sub: int = 64):
        for c0 in range(0, len(self.subtasks), max_sub):
            sel = np.nonzero((self.alloc >= c0) & (self.alloc < c0 + max_sub))[0]
            yield sel, (self.alloc[sel] - c0).astype(np.uint8), self.subtasks[c0:c0 + max_sub]

    def inputs(self, sel, pitch):
        s = state_from_canonical(self.level, self.A, self.K, pitch, self.agents[sel], self.items[sel], self.t[sel])
        taken = np.full((self.A, pitch), 4, np.uint8)
        taken[:, :len(sel)] = self.taken[sel][:, :self.A].T
        return s, taken.reshape(-1)

    def compare(self, sel, value, flags, rtol=1e-12):
        errs = []
        for k, r in enumerate(sel):
            raised = self.exp_raised[r]
            if raised:
                if not (flags[k] & (capi.LIK_RAISES | capi.LIK_ZERODIV)):
                    errs.append("row %d: reference raised (%d), got flags %d value %r" % (self.idx[r], raised, flags[k],
                                                                                      value[k]))
                continue
            if flags[k] != capi.LIK_OK or abs(value[k] - self.exp_value[r]) > rtol * abs(self.exp_value[r]):
                errs.append("row %d: %r (flags %d) vs %r" % (self.idx[r], value[k], flags[k], self.exp_value[r]))
            if len(errs) > 20:
                break
        return errs


class BoundRows:
    """Rows of tests/golden/bounds.npz for one (level, A) config: the config's states (one env
    each) and its subtask table; every row is one (state, subtask) cell of the
    oc_subtask_bounds output."""

    def __init__(self, fx, cfg: int):
        st_sel = np.nonzero(fx["st_cfg"] == cfg)[0]
        self.level = load_level(str(fx["cfg_level"][cfg]))
        self.A = int(fx["cfg_A"][cfg])
        self.K = capi.item_slots(self.level)
        self.agents, self.items, self.t = fx["st_agents"][st_sel], fx["st_items"][st_sel], fx["st_t"][st_sel]
        self.B = len(st_sel)
        env_of = {int(s): b for b, s in enumerate(st_sel)}
        sel = np.nonzero(np.isin(fx["state"], st_sel))[0]
        keys, self.subtasks = {}, []
        self.row_env = np.zeros(len(sel), np.int64)
        self.row_sub = np.zeros(len(sel), np.int64)
        for r, i in enumerate(sel):
            n = int((fx["agents"][i] != PAD).sum())
            key = (int(fx["kind"][i]), tuple(int(a) for a in fx["agents"][i][:n]),
                   tuple(int(m) for m in fx["start"][i]), int(fx["goal_mask"][i]))
            if key not in keys:
                keys[key] = len(self.subtasks)
                self.subtasks.append(capi.subtask(key[0], key[1], key[2], key[3], 0))
            self.row_env[r] = env_of[int(fx["state"][i])]
            self.row_sub[r] = keys[key]
        self.idx = sel
        self.exp_lb = fx["lb"][sel]
        # rows where the reference's T raised copying a state with two co-located holders
        # (Level 1, actions outside get_actions only): only get_actions membership is compared
        self.copy_raise = fx["copy_raise"][sel] if "copy_raise" in fx else np.zeros(len(sel), np.int64)
        self.exp_doable = fx["doable"][sel].astype(np.uint8)

    def state(self, pitch: int) -> np.ndarray:
        return state_from_canonical(self.level, self.A, self.K, pitch, self.agents, self.items, self.t)

    def compare(self, lb: np.ndarray, doable: np.ndarray, sub0: int = 0):
        """Mismatches of [S][B] outputs covering subtasks [sub0, sub0 + S) against the rows."""
        errs = []
        S = lb.shape[0]
        for r in np.nonzero((self.row_sub >= sub0) & (self.row_sub < sub0 + S))[0]:
            s, b = self.row_sub[r] - sub0, self.row_env[r]
            if float(lb[s, b]) != float(self.exp_lb[r]) or int(doable[s, b]) != int(self.exp_doable[r]):
                errs.append("row %d (env %d, subtask %d): lb %r doable %d vs %r %d" % (
                    self.idx[r], b, self.row_sub[r], float(lb[s, b]), int(doable[s, b]), float(self.exp_lb[r]),
                    int(self.exp_doable[r])))
            if len(errs) > 20:
                break
        return errs


def window_totals(fl_in: np.ndarray, state_out: np.ndarray, coll: np.ndarray, A: int, K: int, pitch: int,
                  B: int) -> np.ndarray:
    """Host restatement of one step's contribution to the OC_STAT_* counters
    (include/oc_engine.h): episodes whose DONE bit was newly set, their successes, their
    lengths t, colliding pairs (popcount of the collision mask) and ERR ends."""
    v = planes_view(state_out, A, K, pitch)
    fl = v["fl"][:B]
    ended = ((fl_in[:B] & 1) == 0) & ((fl & 1) == 1)
    return np.array([ended.sum(), (ended & ((fl & 2) > 0)).sum(), v["t"][:B][ended].astype(np.int64).sum(),
                     np.unpackbits(coll[:B]).sum(), (ended & ((fl & 4) > 0)).sum()], dtype=np.int64)
