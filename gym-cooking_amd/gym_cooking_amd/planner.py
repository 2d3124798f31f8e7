"""Engine-backed navigation planner: a drop-in for
gym_cooking/navigation_planner/planners/e2e_brtdp.py ``E2E_BRTDP`` (Level 0 and Level 1).

The reference planner's time goes into its environment rollouts: every ``T(state, action)``
deep-copies a whole ``OvercookedEnvironment`` and runs ``interact`` on it, and every new
state's ``value_init`` walks the reachability graph for a lower bound.
Here a state is expanded ONCE, for all its candidate actions together, by one ``oc_rollout``
launch: each row of the launch is (Level-0 state, subtask configuration, joint action) and
returns the next state, the ``get_actions`` membership, the goal test and the next state's
lower bound.  The bounded-RTDP search itself -- ``get_next_action``, ``main``,
``runSampleTrial``, the Bellman backups, the numpy tie-breaking ``argmin`` -- is restated on
the host line by line (e2e_brtdp.py:27-36, 257-331, 736-878), so a call makes exactly the
reference's decisions and draws exactly the reference's random numbers
(tests/golden/brtdp.json, recorded from the reference).

State identity.  The reference keys its value tables by ``env.get_repr()``: the subtask
agents, every dynamic object group in name order with its objects in insertion order
(``World.objects`` keeps emptied groups, world.py:304-337) and the frozen agents'
``Agent-Counter`` squares.  Here a state is (its engine state bytes without ``t`` / flags, with
the item slots ordered by (group name, slot); the set of object-group names; the subtask
agents), which identifies the same states: frozen agents keep their cells in the bytes, an
item is known by its group and its rank there, and which slot a merged dish occupies is not
part of it (see ``_canon``).

Level 1 (``other_agent_planners`` non-empty, the Bayesian-delegation agents' call): every
agent stays in the planner's states (the rollout rows run with ``OC_LEVEL1``), and at every
state the search visits, each other agent's planner -- a shallow copy of this one, sharing
its value tables, as ``BayesianDelegator.get_other_agent_planners`` makes them -- is set up
there and picks its greedy action (``_get_modified_state_with_other_agent_actions``,
e2e_brtdp.py:842-878), drawing the same random numbers as the reference.
"""
from __future__ import annotations

import contextlib
import functools
import gc
import itertools
import types
from typing import Dict, FrozenSet, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import capi
from . import envs as _envs
from . import levels as _levels
from .engine import _ptr
from . import recipes as _recipes

try:  # the sample trial's loop in C (csrc/brtdp_host.c, built in-tree by csrc/Makefile)
    from . import _brtdp as _native
except ImportError:  # not built: the same loop in Python (tests/test_planner_host.py compares the two)
    _native = None

_NAV = [(0, 1), (0, -1), (-1, 0), (1, 0), (0, 0)]  # action codes 0..4 (World.NAV_ACTIONS + no-op)


@contextlib.contextmanager
def searching():
    """The cyclic garbage collector paused for a search call.  A search allocates millions of
    small tuples (its table keys and successor lists) that form no reference cycles; CPython's
    collector would walk them over and over as they accumulate -- 40 % of plan_batch's host
    time (tools/prof_host_search.py).  Nothing is collected late but cycles, and collection
    resumes, in its previous state, when the call returns."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()
_NOOP = 4


_NAMES: Dict[tuple, str] = {}


def _group_name(mask: int, enc: int = 0) -> str:
    """World.objects group name of an item mask in encoding `enc` (its base contents,
    core.py:161-171)."""
    n = _NAMES.get((mask, enc))
    if n is None:
        n = _NAMES[(mask, enc)] = _envs.item_name(mask, enc)
    return n


def _encoding(level) -> int:
    """The item-mask encoding of a level (a levels.Level or a builtin name / level file)."""
    if isinstance(level, str):
        level = _levels.load_level(level)
    return level.encoding


_CAND = {n: list(itertools.product(range(5), repeat=n)) for n in (1, 2)}


def _lay(A: int, K: int, wide: bool = False):
    """(first item-cell plane, first high-byte plane or -1, first mask plane) of a state's bytes:
    the narrow layout (byte cells) or the wide one (u16 cells: high bytes in K planes after the
    low ones, include/oc_engine.h oc_layout)."""
    return (3 * A, 3 * A + K, 3 * A + 2 * K) if wide else (3 * A, -1, 3 * A + K)


def _live(b, A: int, K: int, wide: bool = False) -> List[bool]:
    """Per slot: the item is in the world (its cell is not OC_LOC_DEAD / OC_LOC_DEAD16)."""
    l0, lh, _ = _lay(A, K, wide)
    if lh < 0:
        return [b[l0 + j] != 0xFF for j in range(K)]
    return [b[l0 + j] != 0xFF or b[lh + j] != 0xFF for j in range(K)]


def _canon(sb: bytes, A: int, K: int, enc: int = 0, wide: bool = False) -> bytes:
    """The planner's form of a state: live item slots ordered by (object-group name, slot).
    The reference's repr lists each group's objects in insertion order and nothing else, so
    an item's identity is its group name plus its rank in that group; which slot a merged
    dish happens to occupy is not part of it (the engine keeps the holder's slot, world.py
    re-inserts the merged object).  Plates, the only name with two members, keep their
    relative slot order, as they keep their order in World.objects."""
    b = bytearray(sb)
    l0, lh, m0 = _lay(A, K, wide)
    alive = _live(b, A, K, wide)
    live = sorted((_group_name(b[m0 + j], enc), j) for j in range(K) if alive[j])
    order = [j for _, j in live]
    if order == list(range(len(order))):
        return bytes(b)
    new_of = {j: i for i, j in enumerate(order)}
    locs = [b[l0 + j] for j in order] + [0xFF] * (K - len(order))
    masks = [b[m0 + j] for j in order] + [0] * (K - len(order))
    b[l0:l0 + K], b[m0:m0 + K] = bytes(locs), bytes(masks)
    if lh >= 0:
        b[lh:lh + K] = bytes([b[lh + j] for j in order] + [0xFF] * (K - len(order)))
    for a in range(A):
        h = b[2 * A + a]
        if h != 0xFF:
            b[2 * A + a] = new_of[h]
    return bytes(b)


_CODES: Dict[int, np.ndarray] = {}


def _codes_array(codes) -> np.ndarray:
    """u8 [len, agents] of a candidate list; kept for the fixed get_actions lists (_CAND)."""
    c = _CODES.get(id(codes))
    if c is not None and c.shape[0] == len(codes):
        return c
    c = np.array(codes, np.uint8).reshape(len(codes), -1)
    if any(codes is v for v in _CAND.values()):
        _CODES[id(codes)] = c
    return c


def _cost(action) -> float:  # E2E_BRTDP.cost (e2e_brtdp.py:816-826): 1.0, + 0.1 per moving agent, in order
    cost = 1.0
    for a in action:
        if a != _NOOP:
            cost += 0.1
    return cost


_COST = {c: _cost(c) for n in (1, 2) for c in _CAND[n]}


def argmin(vector, rng=np.random):
    """e2e_brtdp.py:27-30: the index of a minimum, ties broken by numpy's global generator
    (one ``multinomial`` draw per call, ties or not).  `rng` is the module ``np.random`` (the
    reference's generator) or a ``np.random.RandomState`` of a batched search.

    A unique minimum is answered without the multinomial, consuming what it would: the legacy
    multinomial(1, one-hot at i) draws binomial(1, 0) -> 0 with no variate for every entry
    before i, then binomial(1, 1.0) = 1 - binomial-inversion(1, 0.0), which reads one uniform
    double; at the last index it draws nothing (numpy's legacy distributions, mtrand
    multinomial; checked against multinomial itself in tests/test_planner_host.py)."""
    m = min(vector)
    i = vector.index(m) if isinstance(vector, list) else int(np.argmin(vector))
    if vector.count(m) == 1 if isinstance(vector, list) else (np.asarray(vector) == m).sum() == 1:
        if i != len(vector) - 1:
            rng.random_sample()
        return i
    if _native is not None:  # the same draw, restated over rng's uniforms (csrc/brtdp_host.c tie_pick)
        return _native.tie_pick([v == m for v in vector], rng.random_sample)
    e_x = np.array(vector) == m
    return np.where(rng.multinomial(1, e_x / e_x.sum()))[0][0]


def _sampler(rng):
    """What the native loop draws its uniforms with: for a legacy RandomState over MT19937 (the
    reference's np.random, or a batched search's RandomState(seed)) its bit generator's capsule
    -- brtdp_host.c calls the capsule's next_double, the function random_sample() itself calls,
    so the stream is the same -- else the bound random_sample."""
    rs = np.random.mtrand._rand if rng is np.random else rng
    if type(rs) is np.random.RandomState:
        cap = getattr(getattr(rs, "_bit_generator", None), "capsule", None)
        if cap is not None:
            return cap
    return rng.random_sample


def _argmin_plan(vector: list):
    """What argmin(vector, rng) draws and returns, as data: (index, None) for a unique minimum,
    (None, tie mask) for ties.  Lets a caller that meets the same Q vector again replay the
    draw (_argmin_apply) without recomputing it."""
    m = min(vector)
    if vector.count(m) == 1:
        return (vector.index(m), len(vector))
    return (None, [v == m for v in vector])


def _argmin_apply(plan, rng) -> int:
    """argmin's draw and result from its _argmin_plan (the same consumption of rng)."""
    i, n = plan
    if i is not None:
        if i != n - 1:
            rng.random_sample()
        return i
    if _native is not None:
        return _native.tie_pick(n, rng.random_sample)
    e_x = np.array(n, dtype=float)
    return np.where(rng.multinomial(1, e_x / e_x.sum()))[0][0]


class _Expander:
    """An engine batch of up to ROWS rollout rows for a level.  ``run(requests)`` evaluates
    any number of expansion requests -- (state bytes, joint actions, subtask configuration) --
    in as few oc_rollout launches as the row and configuration limits allow (one, for up to
    ROWS rows and 64 distinct configurations)."""

    ROWS = 4096

    def __init__(self, level, num_agents: int, device):
        from .engine import OvercookedBatch  # raises without liboc_engine.so / a GPU
        self.eb = OvercookedBatch(level, num_agents, self.ROWS, max_T=0, device=device)
        self.wide = self.eb.layout.cell_bytes == 2  # u16 item cells (a level of more than 255 cells)
        self.A, self.K, self.P = self.eb.A, self.eb.K, self.eb.pitch
        self.enc = self.eb.level.encoding
        self.NP = self.eb.layout.num_planes
        self.t_plane = self.eb.layout.plane_t
        dev = self.eb.device
        NP, A, P = self.NP, self.A, self.P
        # One contiguous input block (state planes | actions | allocation ids) and one output
        # block (next-state planes | flags | f32 bounds), each moved by ONE pinned copy per
        # launch: every buffer is a full-pitch slice (P = ROWS), so no strided per-plane copies.
        n_in, n_out = (NP + A + 1) * P, (NP + 1 + 4) * P
        self._d_in = torch.empty(n_in, dtype=torch.uint8, device=dev)
        self._d_out = torch.empty(n_out, dtype=torch.uint8, device=dev)
        self._h_in_all = torch.empty(n_in, dtype=torch.uint8).pin_memory()
        self._h_out_all = torch.empty(n_out, dtype=torch.uint8).pin_memory()
        self.s_in, self.act, self.alloc = (self._d_in[:NP * P], self._d_in[NP * P:(NP + A) * P],
                                           self._d_in[(NP + A) * P:])
        self.s_out, self.flags = self._d_out[:NP * P], self._d_out[NP * P:(NP + 1) * P]
        self.lb = self._d_out[(NP + 1) * P:].view(torch.float32)
        hin, hout = self._h_in_all.numpy(), self._h_out_all.numpy()
        self._hi, self._ha, self._hal = (hin[:NP * P].reshape(NP, P), hin[NP * P:(NP + A) * P].reshape(A, P),
                                         hin[(NP + A) * P:])
        self._ho, self._hf = hout[:NP * P].reshape(NP, P), hout[NP * P:(NP + 1) * P]
        self._hl = hout[(NP + 1) * P:].view(np.float32)
        self.launches = 0
        self.rows_done = 0

    def rows(self, state: np.ndarray, codes: Sequence[Tuple[int, ...]], sub: capi.OcSubtask):
        """One request: (next states [n, NP], flags [n], lower bounds [n])."""
        return self.run([(state, codes, sub)])[0]

    def bounds(self, state: np.ndarray, subs):
        """oc_subtask_bounds of one state (env_view bytes) under each configuration:
        (lower bounds [S], doable [S])."""
        hi = self._hi
        hi[:, 0] = state
        hi[self.t_plane:, 0] = 0
        self._d_in.copy_(self._h_in_all, non_blocking=True)
        S = len(subs)
        lbt = torch.empty((S, self.P), dtype=torch.float32, device=self.eb.device)
        okt = torch.empty((S, self.P), dtype=torch.uint8, device=self.eb.device)
        capi.check(self.eb.lib.oc_subtask_bounds(self.eb._h, _ptr(self.s_in), capi.subtask_array(subs), S, _ptr(lbt),
                                                 _ptr(okt), 1, self.eb._stream()))
        return lbt[:, 0].cpu().numpy(), okt[:, 0].cpu().numpy()

    def bounds_many(self, states: np.ndarray, subs):
        """oc_subtask_bounds of up to ROWS states (env_view bytes, [B, NP]) under each of up to
        64 configurations in one launch: (lower bounds [S][B], doable [S][B])."""
        B, S = len(states), len(subs)
        hi = self._hi
        hi[:, :B] = np.asarray(states).T
        hi[self.t_plane:, :B] = 0
        self._d_in.copy_(self._h_in_all, non_blocking=True)
        lbt = torch.empty((S, self.P), dtype=torch.float32, device=self.eb.device)
        okt = torch.empty((S, self.P), dtype=torch.uint8, device=self.eb.device)
        capi.check(self.eb.lib.oc_subtask_bounds(self.eb._h, _ptr(self.s_in), capi.subtask_array(subs), S, _ptr(lbt),
                                                 _ptr(okt), B, self.eb._stream()))
        return lbt[:, :B].cpu().numpy(), okt[:, :B].cpu().numpy()

    def run(self, requests):
        out, chunk, nrows, subs = [], [], 0, {}
        key_of = {}  # id(sub) -> its bytes: the requests hold their subtask rows alive for this call
        for req in requests:
            n = len(req[1])
            sub = req[2]
            key = key_of.get(id(sub))
            if key is None:
                key = key_of[id(sub)] = bytes(sub)
            if chunk and (nrows + n > self.ROWS or (key not in subs and len(subs) == capi.MAX_SUBTASKS)):
                out += self._launch(chunk, subs)
                chunk, nrows, subs = [], 0, {}
            if key not in subs:
                subs[key] = (len(subs), sub)
            chunk.append((req, subs[key][0]))
            nrows += n
        if chunk:
            out += self._launch(chunk, subs)
        return out

    def _launch(self, chunk, subs):
        """One oc_rollout launch over the chunk's requests, packed with whole-array copies: the
        states repeated per candidate row, each (candidate list, agents) group's action codes
        scattered at once.  A chunk whose requests share one candidate list (a round of
        expansions: every request is _CAND[1] or _CAND[2]) is packed and split with fixed-stride
        reshapes instead of per-request offsets."""
        hi, ha, hal = self._hi, self._ha, self._hal
        m = len(chunk)
        codes0 = chunk[0][0][1]
        # the request states (byte arrays or bytes) joined into one [m, NP] array: one join and
        # one frombuffer instead of np.stack's per-array work (10x faster at 100 requests)
        states = np.frombuffer(b"".join([req[0] for req, _ in chunk]), np.uint8).reshape(m, self.NP)
        sids = np.fromiter((si for _, si in chunk), np.uint8, m)
        uniform = all(req[1] is codes0 for req, _ in chunk)
        if uniform:
            c = len(codes0)
            n = c * m
            counts = starts = None
            hi[:, :n] = np.repeat(states, c, axis=0).T
            hal[:n] = np.repeat(sids, c)
        else:
            counts = np.fromiter((len(req[1]) for req, _ in chunk), np.int64, m)
            starts = np.zeros(m, np.int64)
            np.cumsum(counts[:-1], out=starts[1:])
            n = int(counts.sum())
            hi[:, :n] = np.repeat(states, counts, axis=0).T
            hal[:n] = np.repeat(sids, counts)
        hi[self.t_plane:, :n] = 0  # t and flags: copied through by the kernel, not part of a planner state
        ha[:, :n] = _NOOP
        groups, agents_of = {}, {}
        for i, (req, _) in enumerate(chunk):
            codes, sub = req[1], req[2]
            ag = agents_of.get(id(sub))
            if ag is None:
                ag = agents_of[id(sub)] = tuple(sub.agent[:sub.num_agents])
            g = groups.get((id(codes), ag))
            if g is None:
                g = groups[(id(codes), ag)] = (codes, ag, [])
            g[2].append(i)
        for codes, ag, idx in groups.values():
            cA = _codes_array(codes)
            k = len(codes)
            if uniform and len(idx) == m:  # every request: the whole row range
                for q, a in enumerate(ag):
                    ha[a, :n] = np.tile(cA[:, q], m)
                continue
            s0 = np.asarray(idx) * k if uniform else starts[idx]
            rows = (s0[:, None] + np.arange(k)[None, :]).ravel()
            for q, a in enumerate(ag):
                ha[a, rows] = np.tile(cA[:, q], len(idx))
        table = [sub for _, sub in sorted(subs.values(), key=lambda v: v[0])]
        self._d_in.copy_(self._h_in_all, non_blocking=True)  # one H2D
        lib, eb = self.eb.lib, self.eb
        capi.check(lib.oc_rollout(eb._h, _ptr(self.s_in), _ptr(self.s_out), _ptr(self.act), _ptr(self.alloc),
                                  capi.subtask_array(table), len(table), _ptr(self.flags), _ptr(self.lb), n,
                                  eb._stream()))
        self.launches += 1
        self.rows_done += n
        self._h_out_all.copy_(self._d_out, non_blocking=True)  # one D2H
        torch.cuda.current_stream(eb.device).synchronize()
        nxt = self._ho[:, :n].T.copy()  # [n, NP]: each request's rows are a contiguous slice
        nxt[:, self.t_plane:] = 0
        fl, lb = self._hf[:n].copy(), self._hl[:n].copy()
        if uniform:  # m views of c rows each
            c = n // m
            return list(zip(nxt.reshape(m, c, self.NP), fl.reshape(m, c), lb.reshape(m, c)))
        return [(nxt[s0:s0 + c], fl[s0:s0 + c], lb[s0:s0 + c]) for s0, c in zip(starts.tolist(), counts.tolist())]


def _changed_row(A: int, K: int, enc: int, wide: bool, m0: int, ns: bytes, groups: FrozenSet[str]):
    """A successor row whose item masks changed (a chop or a merge): its canonical bytes and
    its group names, plus a merge's new object group (world.py:304-306)."""
    ns = _canon(ns, A, K, enc, wide)
    return ns, groups | frozenset(_group_name(m, enc) for m, l in zip(ns[m0:m0 + K], _live(ns, A, K, wide)) if l)


def _copy_crashes(sb: bytes, A: int) -> bool:
    """Two agents on one square that both hold an item: the reference's copy of such a state
    raises (overcooked_environment.py:108-113 -> world.py:417).  At Level 1 every agent is in the
    planner's env, so T's repr_init copy of a successor like that raises (e2e_brtdp.py:147)."""
    for i in range(A):
        if sb[2 * A + i] == 0xFF:
            continue
        for j in range(i + 1, A):
            if sb[2 * A + j] != 0xFF and sb[i] == sb[j] and sb[A + i] == sb[A + j]:
                return True
    return False


def _raise_copy_crash(action):
    raise AttributeError("T{}: the next state has two co-located agents holding items; the reference's "
                         "copy of it raises (world.py:417)".format(action))


class E2E_BRTDP:
    """Bounded RTDP navigation planner (e2e_brtdp.py:38-878), Levels 0 and 1, over the HIP engine.

    Same constructor, same ``get_next_action(env, subtask, subtask_agent_names,
    other_agent_planners)``, same value tables ``v_l`` / ``v_u`` (keyed by (state, subtask)),
    ``cur_state``, ``cur_obj_count``, ``is_joint``.  ``env`` is the engine-backed
    :class:`gym_cooking_amd.envs.OvercookedEnvironment`.

    The search is written as a generator that yields an expansion request whenever it meets a
    state it has not expanded; :meth:`get_next_action` serves each request with its own launch,
    :func:`plan_batch` serves the requests of many searches with shared launches.
    """

    def __init__(self, alpha, tau, cap, main_cap, device: Optional[str] = None, expander=None, rng=None):
        """`expander(level, num_agents, device)` builds the row evaluator; the default is the
        HIP engine (``oc_rollout``).  Tests pass the CPU oracle's rollout here to check the
        host search without a GPU.  `rng`: the tie-breaking generator (default numpy's global
        one, as the reference)."""
        self.alpha, self.tau, self.cap, self.main_cap = alpha, tau, cap, main_cap
        self.use_native = True  # the C sample-trial loop when built (False: the Python loop)
        self._make_expander = expander or _Expander
        self._rng = rng if rng is not None else np.random
        self.v_l: Dict = {}
        self.v_u: Dict = {}
        self.time_cost = 1.0
        self.action_cost = 0.1
        self.is_joint = False
        self.subtask = None
        self.device = device
        self._exp = None
        self._exp_key = None
        self._succ: Dict = {}  # (state key, subtask key) -> [actions, successors, costs, value keys, goal flags, lower bounds, initialised]
        self._tmemo: Dict = {}  # this object's T memo: (repr, action) -> successor (bytes, groups)
        self._illegal: Dict = {}  # (state key, subtask key) -> {action outside get_actions: (next bytes, flags)}
        self._vkeys: Dict = {}  # value key -> the one object of it the native expansions use (identity lookups)

    # ---- configuration (set_settings, e2e_brtdp.py:582-652) --------------------------------
    def __copy__(self):  # e2e_brtdp.py:97-101: a shallow copy shares the value tables (and here the caches)
        new = object.__new__(E2E_BRTDP)
        new.__dict__ = self.__dict__.copy()
        new._tmemo = {}  # T's lru_cache is keyed by the planner object
        # a belief update's memo belongs to the delegator's own planner and that update only
        # (delegation.py drops it when the update ends): a copy made during an update must not
        # keep it alive or read it later
        if "_bayes_memo" in new.__dict__:
            new._bayes_memo = None
        return new

    def _configure(self, env, subtask, subtask_agent_names, other_agent_planners=None):
        # _configure_planner_level (e2e_brtdp.py:383-406): Level 1 when other agents' planners
        # are given -- every agent stays -- else Level 0
        self.other_agent_planners = dict(other_agent_planners or {})
        self._level = 1 if self.other_agent_planners else 0
        if subtask is None:
            raise NotImplementedError("the reference agents do not plan the None subtask")
        assert len(subtask_agent_names) <= 2, "Cannot have more than 2 agents! Hm... {}".format(subtask_agent_names)
        names = env.get_agent_names()
        level, A = env.level, len(names)
        key = expander_key(env, self.device)
        if self._exp is None or self._exp_key != key:
            self._exp = self._make_expander(level, A, self.device or env._device)
            self._exp_key = key
        fast = getattr(env, "planner_bytes", None)
        if fast is not None:
            full = fast(self._exp.t_plane)
        else:
            b = env.state_bytes()
            b[self._exp.t_plane:] = 0
            full = b.tobytes()
        return self._configure_raw(level, A, self.device or env._device, full, _groups(env), subtask,
                                   subtask_agent_names)

    def _configure_raw(self, level, A, dev, full: bytes, groups, subtask, subtask_agent_names):
        """The set-up of _configure from a state's bytes (t and flags zeroed) and group names,
        once the expander is chosen.  What it derives from (state, Level, agents, subtask) --
        the planner's start bytes, cur_obj_count, the subtask row -- is a pure function of
        those, kept per expander (many planners set up on the same states: the delegators'
        other-agent planners at every state a Level-1 search visits)."""
        exp = self._exp
        self.subtask = subtask
        san = self.subtask_agent_names = tuple(subtask_agent_names)
        self.is_joint = len(san) == 2
        agents = _AGENT_IX.get((A, san))
        if agents is None:
            names = _agent_names(A)
            agents = tuple(names.index(n) for n in san)
            assert list(agents) == sorted(agents), "subtask agent names are not in order"
            _AGENT_IX[(A, san)] = agents
        self._agents = list(agents)
        sk = str(subtask)
        self._sub_key = sk
        ck = (full, self._level, agents, sk)
        cache = exp.__dict__.get("_conf_cache")
        if cache is None:
            cache = exp.__dict__["_conf_cache"] = {}
        hit = cache.get(ck)
        if hit is None:
            kind, starts, goal = _recipes.subtask_masks(subtask, exp.enc)
            self._kind, self._goal_mask = kind, goal  # _obj_count reads them
            start = np.frombuffer(full, np.uint8).copy()
            if not self._level:
                start = self._level0(start, exp)
            start = np.frombuffer(_canon(start.tobytes(), exp.A, exp.K, exp.enc, exp.wide), np.uint8).copy()
            count = self._obj_count(start, exp, level)  # _define_goal_state on the Level-0 env
            # [start, kind, goal mask, cur_obj_count, subtask row, (goal, bound) of the no-op row]
            hit = [start, kind, goal, count, capi.subtask(kind, list(agents), list(starts), goal, count, self._level),
                   None]
            if len(exp._conf_cache) > 1 << 18:
                exp._conf_cache.clear()
            exp._conf_cache[ck] = hit
        start, self._kind, self._goal_mask, self.cur_obj_count, self._sub, _ = hit
        self._conf = hit
        self._level_name = level
        self._A = A
        self._dev = dev
        self.start = self._key(start, groups)
        # the start state: a no-op row gives its goal flag and lower bound
        return (start, _NOOP_ROW[len(agents)], self._sub)

    def _configured(self, res) -> None:
        _, fl, lb = res
        self._start_goal = bool(fl[0] & capi.ROLL_GOAL)  # is_goal_state with this call's cur_obj_count
        self._value_init(self.start, self._start_goal, float(lb[0]))

    def _configure_gen(self, req):
        """Finish a set-up whose request `req` _configure / _configure_raw made: the start's goal
        flag and lower bound come from one no-op row, a pure function of the set-up, so a set-up
        seen before (its cache entry) needs no row."""
        hit = self._conf
        if hit[5] is None:
            _, fl, lb = yield req
            hit[5] = (bool(fl[0] & capi.ROLL_GOAL), float(lb[0]))
        self._start_goal = hit[5][0]
        self._value_init(self.start, hit[5][0], hit[5][1])

    def set_settings(self, env, subtask, subtask_agent_names, other_agent_planners=None):
        self._drive(self._set_settings_gen(env, subtask, subtask_agent_names, other_agent_planners))

    def _set_settings_gen(self, env, subtask, subtask_agent_names, other_agent_planners=None):
        yield from self._configure_gen(self._configure(env, subtask, subtask_agent_names, other_agent_planners))

    def _exp_run(self, req):
        return self._exp.run([req])[0]

    def _level0(self, full: np.ndarray, exp) -> np.ndarray:
        """E2E_BRTDP._configure_planner_level, Level 0 (e2e_brtdp.py:383-406): the items held by
        agents outside the subtask leave the world (their frozen cells stay in the bytes; the
        kernel treats them as AgentCounters)."""
        s = full.copy()
        A, K = exp.A, exp.K
        l0, lh, m0 = _lay(A, K, exp.wide)
        for a in range(A):
            if a in self._agents:
                continue
            h = int(s[2 * A + a])
            if h != 0xFF:
                s[l0 + h], s[m0 + h] = 0xFF, 0
                if lh >= 0:
                    s[lh + h] = 0xFF
                s[2 * A + a] = 0xFF
        return s

    def _obj_count(self, s: np.ndarray, exp, level) -> int:
        """cur_obj_count of _define_goal_state (e2e_brtdp.py:435-566) on a Level-0 state."""
        A, K = exp.A, exp.K
        l0, lh, m0 = _lay(A, K, exp.wide)
        held = {int(s[2 * A + a]) for a in range(A)} - {0xFF}
        deliv = _level_tables(level)[1]
        locs = []
        alive = _live(s, A, K, exp.wide)
        for j in range(K):
            c, m = int(s[l0 + j]) | (int(s[lh + j]) << 8 if lh >= 0 else 0), int(s[m0 + j])
            if not alive[j] or m != self._goal_mask:
                continue
            if self._kind == 3:
                if j not in held and c in deliv:
                    locs.append(c)
            else:
                if j in held:  # a held item sits at its holder's cell
                    a = [a for a in range(A) if int(s[2 * A + a]) == j][0]
                    c = int(s[A + a]) * level.width + int(s[a])
                locs.append(c)
        return len(locs) if self._kind == 3 else len(set(locs))

    def _key(self, s: np.ndarray, groups: FrozenSet[str]):
        """A planner state: its bytes, its object-group names and which agents are the subtask
        agents (the reference's Level-0 repr lists those as agents and the others as
        Agent-Counter squares)."""
        return (s.tobytes(), groups, tuple(self._agents), self._level)

    def _repr(self, key):
        """The reference's ``env.get_repr()`` of a planner state (overcooked_environment.py:50-62):
        the dynamic objects -- at Level 0 including the Agent-Counter squares that stand for the
        agents outside the subtask (utils/core.py:79-87) -- and the agents present in the
        planner's env: all of them at Level 1, the subtask agents at Level 0.  So a Level-0
        state of every agent and the Level-1 state of the same bytes share one repr.  The value
        tables are keyed by (repr, subtask) as the reference's are, so that planners of
        different agent sets or levels meet in them exactly where the reference's do (the
        delegator's planner and its copies share one table pair)."""
        sb, groups, agents, lvl = key
        return (sb, groups, None if lvl or len(agents) == self._exp.A else agents)

    # ---- values (value_init, e2e_brtdp.py:678-729) --------------------------------------------
    def _value_init(self, key, goal: bool, lb: float) -> None:
        vk = (self._repr(key), self._sub_key)
        if vk in self.v_l and vk in self.v_u:
            return
        if goal:
            self.v_l[vk] = 0.0
            self.v_u[vk] = 0.0
            return
        lower = lb * (self.time_cost + self.action_cost)
        assert lower > 0, "lower: {}".format(lower)
        self.v_l[vk] = lower - 1.09
        self.v_u[vk] = lower * 5 * (self.time_cost + self.action_cost)

    # ---- transitions: one request per new state --------------------------------------------
    def _need(self, key):
        """Generator: make sure `key` is expanded (yields one request if it is not)."""
        if (key, self._sub_key) not in self._succ:
            cand = _CAND[len(self._agents)]  # product order of get_actions
            res = yield (np.frombuffer(key[0], np.uint8), cand, self._sub)
            self._expanded(key, cand, res)

    def _expanded(self, key, cand, res) -> None:
        nxt, fl, lb = res
        sb, groups, agents, lvl = key
        if _native is not None and self.use_native and fl.dtype == np.uint8 and lb.dtype == np.float32:
            return self._expanded_native(key, cand, nxt, fl, lb)
        NP, K, A, enc, wide = len(sb), self._exp.K, self._exp.A, self._exp.enc, self._exp.wide
        l0, lh, m0 = _lay(A, K, wide)
        raw = nxt.tobytes()
        pmask = sb[m0:m0 + K]
        sk = self._sub_key
        actions, succ, goals, lbs = [], [], [], []
        illegal = {}
        crash = None
        fl, lb = fl.tolist(), lb.tolist()  # Python ints / floats (the f32 bounds exactly)
        LEGAL, ASSERT, GOAL = capi.ROLL_LEGAL, capi.ROLL_ASSERT, capi.ROLL_GOAL
        for r, c in enumerate(cand):
            f = fl[r]
            if not f & LEGAL:
                illegal[c] = r
                continue
            if f & ASSERT:  # T raises (e2e_brtdp.py:143)
                raise AssertionError("action {} led to co-located subtask agents".format(c))
            ns = raw[r * NP:(r + 1) * NP]
            ng = groups
            if ns[m0:m0 + K] != pmask:  # a chop or a merge: a merge makes a new object group (world.py:304-306)
                ns = _canon(ns, A, K, enc, wide)
                ng = groups | frozenset(_group_name(m, enc) for m, l in zip(ns[m0:m0 + K], _live(ns, A, K, wide)) if l)
            nk = (ns, ng, agents, lvl)
            if lvl and _copy_crashes(ns, A):
                crash = crash or set()
                crash.add(len(actions))
            actions.append(c)
            succ.append(nk)
            goals.append(bool(f & GOAL))
            lbs.append(lb[r])
        # T's value_init of a successor runs when T is first asked for it (e2e_brtdp.py:145-148):
        # all of them by _init_succ on the first full Q pass, one by T / _expected_diff before
        # that, so that value tables shared between planners fill in the reference's order.
        # [actions, successor keys, costs, successor value keys, goal flags, bounds,
        #  successors initialised, copy-crash action indices, this state's value key]
        ra = None if lvl or len(agents) == A else agents  # _repr's agents entry, the same for every successor
        self._succ[(key, sk)] = [actions, succ, [_COST[c] for c in actions], [((nk[0], nk[1], ra), sk) for nk in succ],
                                 goals, lbs, False, crash, ((sb, groups, ra), sk)]
        if illegal:  # what T would do with them (only asked for by taken_action_error): decoded there
            self._illegal[(key, sk)] = (illegal, raw, NP, fl)

    def _native_expander(self):
        """(m0, changed) of _brtdp.expand for this planner's expander: the item-mask plane
        offset and the callback for a row whose masks changed (a chop or a merge: canonical slot
        order, a merge's new object group), kept per expander."""
        exp = self._exp
        got = exp.__dict__.get("_native_x")
        if got is None:
            A, K, enc, wide = exp.A, exp.K, exp.enc, exp.wide
            m0 = _lay(A, K, wide)[2]
            got = exp.__dict__["_native_x"] = (m0, functools.partial(_changed_row, A, K, enc, wide, m0))
        return got

    def _expanded_native(self, key, cand, nxt, fl, lb) -> None:
        """_expanded with the row loop in C (_brtdp.expand, which also stores the entry and the
        illegal candidates): the same entry, field for field."""
        m0, changed = self._native_expander()
        _native.expand(np.ascontiguousarray(nxt), np.ascontiguousarray(fl), np.ascontiguousarray(lb), cand, key,
                       self._sub_key, m0, self._exp.K, self._exp.A, _COST, changed, self.__dict__.get("_vkeys"),
                       self._succ, self._illegal)

    def _drive(self, gen):
        """Run a search generator to completion, one launch per request."""
        try:
            req = next(gen)
            while True:
                req = gen.send(self._exp_run(req))
        except StopIteration as stop:
            return stop.value

    def _expand(self, key):
        self._drive(self._need(key))
        return self._succ[(key, self._sub_key)]

    def get_actions(self, key) -> List[tuple]:  # e2e_brtdp.py:151-206
        return self._expand(key)[0]

    def _init_succ(self, got) -> None:
        """value_init of every successor of an expanded state, in action order (what a pass of
        Q over get_actions does through T)."""
        if got[7]:
            _raise_copy_crash(got[0][min(got[7])])
        v_l, v_u = self.v_l, self.v_u
        tc = self.time_cost + self.action_cost
        if _native is not None and self.use_native:  # the same loop in C (brtdp_host.c init_entry)
            return _native.init_succ(got, v_l, v_u, tc)
        for vk, g, lb in zip(got[3], got[4], got[5]):  # _value_init of each, inlined (same arithmetic)
            if vk in v_l and vk in v_u:
                continue
            if g:
                v_l[vk] = 0.0
                v_u[vk] = 0.0
                continue
            lower = lb * tc
            assert lower > 0, "lower: {}".format(lower)
            v_l[vk] = lower - 1.09
            v_u[vk] = lower * 5 * tc
        got[6] = True

    def T(self, key, action):  # e2e_brtdp.py:103-149
        """The successor of a legal action.  The reference memoises T per planner object by
        (state repr, action) only (``@lru_cache`` on the method), whatever subtask, agents or
        level the object is configured for at the time: a planner reconfigured on the same
        state -- the delegator's planner across prob_nav_actions calls -- gets the successor
        its first configuration computed.  This T keeps that memo (per object, as the
        reference's); such a successor is value-initialised under the current configuration
        (Q's value_init, e2e_brtdp.py:768-770) from one no-op row of it."""
        return self._drive(self._T_gen(key, action))

    def _T_gen(self, key, action):
        """T as a generator (yields the rollout request it may need)."""
        memo = (self._repr(key), action)
        hit = self._tmemo.get(memo)
        if hit is not None:
            if self._level and _copy_crashes(hit[0], self._exp.A):
                _raise_copy_crash(action)
            nk = (hit[0], hit[1], tuple(self._agents), self._level)
            vk = (self._repr(nk), self._sub_key)
            if vk not in self.v_l or vk not in self.v_u:
                _, fl, lb = yield (np.frombuffer(hit[0], np.uint8), [(_NOOP,) * len(self._agents)], self._sub)
                self._value_init(nk, bool(fl[0] & capi.ROLL_GOAL), float(lb[0]))
            return nk
        yield from self._need(key)
        got = self._succ[(key, self._sub_key)]
        i = got[0].index(action)
        if got[7] and i in got[7]:
            _raise_copy_crash(action)
        if not got[6]:
            self._value_init(got[1][i], got[4][i], got[5][i])
        nk = got[1][i]
        if len(self._tmemo) < 10000:  # lru_cache(maxsize=10000)
            self._tmemo[memo] = (nk[0], nk[1])
        return nk

    def cost(self, action) -> float:  # e2e_brtdp.py:816-826
        cost = self.time_cost
        for c in action:
            if c != _NOOP:
                cost += self.action_cost
        return cost

    def Q(self, key, action, value_f) -> float:  # e2e_brtdp.py:736-760
        return self._drive(self._Q_gen(key, action, value_f))

    def _Q_gen(self, key, action, value_f):
        cost = self.cost(action)
        nk = yield from self._T_gen(key, action)
        expected_value = 1.0 * value_f[(self._repr(nk), self._sub_key)]
        return float(cost + expected_value)

    def _Q_seq_gen(self, key, actions, value_f):
        """[Q(key, a, value_f) for a in actions], evaluated in order with the side effects of
        as many _Q_gen calls (T's memo, value_init, the copy-crash raise), as one generator:
        the belief update's Q passes (bayesian_delegator.py:657-689) without a generator pair
        per action."""
        out = []
        sk = self._sub_key
        rk = self._repr(key)
        tmemo, v_l, v_u, succ = self._tmemo, self.v_l, self.v_u, self._succ
        agents, lvl = tuple(self._agents), self._level
        for action in actions:
            cost = self.cost(action)
            hit = tmemo.get((rk, action))
            if hit is not None:  # _T_gen's memo path
                if lvl and _copy_crashes(hit[0], self._exp.A):
                    _raise_copy_crash(action)
                nk = (hit[0], hit[1], agents, lvl)
                vk = (self._repr(nk), sk)
                if vk not in v_l or vk not in v_u:
                    _, fl, lb = yield (np.frombuffer(hit[0], np.uint8), [(_NOOP,) * len(agents)], self._sub)
                    self._value_init(nk, bool(fl[0] & capi.ROLL_GOAL), float(lb[0]))
            else:
                if (key, sk) not in succ:
                    yield from self._need(key)
                got = succ[(key, sk)]
                i = got[0].index(action)
                if got[7] and i in got[7]:
                    _raise_copy_crash(action)
                if not got[6]:
                    self._value_init(got[1][i], got[4][i], got[5][i])
                nk = got[1][i]
                if len(tmemo) < 10000:  # lru_cache(maxsize=10000)
                    tmemo[(rk, action)] = (nk[0], nk[1])
            out.append(float(cost + 1.0 * value_f[(self._repr(nk), sk)]))
        return out

    def _q_all(self, key, value_f) -> List[float]:
        """[Q(key, a, value_f) for a in get_actions(key)] in one pass (same float64 ops);
        `key` must be expanded."""
        got = self._succ[(key, self._sub_key)]
        if not got[6]:
            self._init_succ(got)
        return [c + value_f[vk] for c, vk in zip(got[2], got[3])]  # floats: c + 1.0 * v, exactly

    def _expected_diff(self, key, action):  # get_expected_diff, e2e_brtdp.py:828-840
        got = self._succ[(key, self._sub_key)]
        i = got[0].index(action)
        if got[7] and i in got[7]:
            _raise_copy_crash(action)
        if not got[6]:
            self._value_init(got[1][i], got[4][i], got[5][i])
        vk = got[3][i]
        return {got[1][i]: 1.0 * (self.v_u[vk] - self.v_l[vk])}

    # ---- search (e2e_brtdp.py:208-331, 842-878), as generators --------------------------------
    def _sample_trial(self):  # runSampleTrial
        """runSampleTrial; _q_all / _expected_diff / _need inlined (the same float64 operations
        in the same order).  At Level 0 the loop runs in C (_brtdp.forward / backprop) and comes
        back here only to expand a state or initialise its successors."""
        if _native is not None and not self._level and self.use_native:
            return (yield from self._sample_trial_native())
        x = self.start
        traj = []
        counter = 0
        sk = self._sub_key
        succ, v_u, v_l, rng, lvl = self._succ, self.v_u, self.v_l, self._rng, self._level
        rs = (self._repr(self.start), sk)
        while True:
            counter += 1
            if counter > self.cap:
                break
            traj.append(x)
            if lvl:
                yield from self._modified_state(x)
            if (x, sk) not in succ:
                yield from self._need(x)
            got = succ[(x, sk)]
            if not got[6]:
                self._init_succ(got)
            costs, vks, rx = got[2], got[3], got[8]
            v_u[rx] = min([c + v_u[vk] for c, vk in zip(costs, vks)])
            ql = [c + v_l[vk] for c, vk in zip(costs, vks)]
            i = argmin(ql, rng)
            v_l[rx] = ql[i]  # = Q(x, a, v_l): that table did not change since
            if got[7] and i in got[7]:  # get_expected_diff's T raises
                _raise_copy_crash(got[0][i])
            vk = vks[i]
            B = v_u[vk] - v_l[vk]
            diff = (v_u[rs] - v_l[rs]) / self.tau
            if B <= diff:
                break
            x = got[1][i]
        while traj:
            x = traj.pop()
            got = succ[(x, sk)]
            costs, vks, rx = got[2], got[3], got[8]
            v_u[rx] = min([c + v_u[vk] for c, vk in zip(costs, vks)])
            v_l[rx] = min([c + v_l[vk] for c, vk in zip(costs, vks)])

    def _sample_trial_native(self):
        """The trial in C: forward runs until a state needs expanding (it initialises
        successors itself), this generator yields that state's request (what _need yields),
        and backprop walks the trajectory's entries."""
        sk = self._sub_key
        succ, v_u, v_l, rng = self._succ, self.v_u, self.v_l, self._rng
        rs = (self._repr(self.start), sk)
        traj, ents = [], []
        tc = self.time_cost + self.action_cost
        cand = _CAND[len(self._agents)]
        x, counter, resume = self.start, 0, False
        while True:
            st, x, counter, i = _native.forward(succ, v_u, v_l, x, sk, rs, self.cap, counter, self.tau, traj,
                                                rng.random_sample, resume, ents, tc)
            if st == 0:
                break
            if st == 2:  # get_expected_diff's T raises (or _init_succ's, on the first crashing successor)
                _raise_copy_crash(succ[(x, sk)][0][i])
            res = yield (np.frombuffer(x[0], np.uint8), cand, self._sub)  # st == 1: _need(x)
            self._expanded(x, cand, res)
            resume = True
        _native.backprop(v_u, v_l, traj, ents)

    def _main(self):  # main
        if _native is not None and not self._level and self.use_native:
            return (yield from self._main_native())
        main_counter = 0
        sk = (self._repr(self.start), self._sub_key)
        diff = self.v_u[sk] - self.v_l[sk]
        while diff > self.alpha and main_counter < self.main_cap:
            diff = self.v_u[sk] - self.v_l[sk]
            main_counter += 1
            yield from self._sample_trial()

    def _main_native(self):
        """main() at Level 0 with _sample_trial_native inlined: one generator for all of a
        search's trials, the loop's constants bound once (none of them changes while it runs)."""
        sk = self._sub_key
        succ, v_u, v_l = self._succ, self.v_u, self.v_l
        rs = (self._repr(self.start), sk)
        sample = _sampler(self._rng)
        tc = self.time_cost + self.action_cost
        cand = _CAND[len(self._agents)]
        fwd, backprop, expanded = _native.forward, _native.backprop, self._expanded
        m0, changed = self._native_expander()
        K, A, expand, vkeys, ill_tbl = self._exp.K, self._exp.A, _native.expand, self.__dict__.get("_vkeys"), self._illegal
        u8, f32 = np.dtype(np.uint8), np.dtype(np.float32)
        cap, tau, alpha, main_cap, start, sub = self.cap, self.tau, self.alpha, self.main_cap, self.start, self._sub
        main_counter = 0
        diff = v_u[rs] - v_l[rs]
        while diff > alpha and main_counter < main_cap:
            diff = v_u[rs] - v_l[rs]
            main_counter += 1
            traj, ents = [], []
            x, counter, resume = start, 0, False
            while True:
                st, x, counter, i = fwd(succ, v_u, v_l, x, sk, rs, cap, counter, tau, traj, sample, resume, ents, tc)
                if st == 0:
                    break
                if st == 2:  # get_expected_diff's T raises (or _init_succ's, on the first crashing successor)
                    _raise_copy_crash(succ[(x, sk)][0][i])
                res = yield (np.frombuffer(x[0], np.uint8), cand, sub)  # st == 1: _need(x)
                nxt, fl, lb = res
                if fl.dtype == u8 and lb.dtype == f32:  # _expanded_native, inlined
                    expand(np.ascontiguousarray(nxt), np.ascontiguousarray(fl), np.ascontiguousarray(lb), cand, x, sk,
                           m0, K, A, _COST, changed, vkeys, succ, ill_tbl)
                else:
                    expanded(x, cand, res)
                resume = True
            backprop(v_u, v_l, traj, ents)

    def _next_action(self, env, subtask, subtask_agent_names, other_agent_planners):
        yield from self._configure_gen(self._configure(env, subtask, subtask_agent_names, other_agent_planners))
        cur = self.start
        self.cur_state = cur
        yield from self._modified_state(cur)
        yield from self._need(cur)
        actions = self._succ[(cur, self._sub_key)][0]
        action_index = argmin(self._q_all(cur, self.v_l), self._rng)
        a = actions[action_index]
        B = sum(self._expected_diff(cur, a).values())
        sk = (self._repr(cur), self._sub_key)
        diff = (self.v_u[sk] - self.v_l[sk]) / self.tau
        if B > diff:
            yield from self._main()
        if self._start_goal:  # is_goal_state(cur_state)
            return None
        qvals = self._q_all(cur, self.v_l)
        a = actions[argmin(np.array(qvals), self._rng)]
        return _NAV[a[0]] if len(a) == 1 else tuple(_NAV[c] for c in a)

    def runSampleTrial(self) -> None:
        self._drive(self._sample_trial())

    def main(self) -> None:
        self._drive(self._main())

    def get_next_action(self, env, subtask, subtask_agent_names, other_agent_planners=None):
        """The next (joint) action for the subtask agents, as the reference's
        ``get_next_action`` returns it: a (dx, dy) tuple for one agent, a pair of them for two,
        ``None`` when the start state already satisfies the subtask."""
        with searching():
            return self._drive(self._next_action(env, subtask, subtask_agent_names, other_agent_planners))

    def taken_action_error(self, key, action) -> Optional[type]:
        """For an action outside get_actions(key): the exception the reference raises on
        Q(state, action) followed by ``assert action in valid_nav_actions``
        (bayesian_delegator.py:657-673) -- AttributeError when T's copy of the next state
        meets two co-located agents that both hold (world.py:417), else AssertionError (T's
        joint co-location assert, or the membership assert).  None for a legal action."""
        return self._drive(self._taken_action_error_gen(key, action))

    def _taken_action_error_gen(self, key, action):
        yield from self._need(key)
        ill = self._illegal.get((key, self._sub_key))
        if ill is None or action not in ill[0]:
            return None
        r, raw, NP, fl = ill[0][action], ill[1], ill[2], ill[3]
        if isinstance(raw, np.ndarray):  # the rows array the native expansion kept, [n, NP]
            raw = raw.reshape(-1)
        got = {action: (bytes(raw[r * NP:(r + 1) * NP]), int(fl[r]))}
        if (self._repr(key), action) in self._tmemo:  # T answers from its memo; the assert raises
            return AssertionError
        ns, f = got[action]
        A = self._exp.A
        held = [(ns[a], ns[A + a]) for a in range(A) if ns[2 * A + a] != 0xFF]
        if len(held) != len(set(held)):
            return AttributeError
        return AssertionError

    def modified_state(self, env) -> None:
        """_get_modified_state_with_other_agent_actions(state=env) under the planner's current
        configuration (what BayesianDelegator.prob_nav_actions calls first, :435-459): at Level
        1 the other agents' planners are set up on env's state and pick their actions."""
        self._drive(self._modified_state_env(env))

    def _modified_state_env(self, env):
        if not getattr(self, "_level", 0):
            return
        memo = self.__dict__.get("_bayes_memo")
        got = memo.get(("env", self._exp_key, tuple(self._agents), self._level)) if memo is not None else None
        if got is not None and got[0] is env:  # the update's one state, keyed once
            key = got[1]
        else:
            exp = self._exp
            full = env.state_bytes()
            full[exp.t_plane:] = 0
            groups = _groups(env)
            key = (_canon(full.tobytes(), exp.A, exp.K, exp.enc, exp.wide), groups, tuple(self._agents), self._level)
            if memo is not None:
                memo[("env", self._exp_key, key[2], key[3])] = (env, key)
        yield from self._modified_state(key)

    def _modified_state(self, key):
        """_get_modified_state_with_other_agent_actions (e2e_brtdp.py:842-878) as a generator.
        Level 0: nothing.  Level 1: every other agent's planner is set up on the state (a Level-0
        planner of its own subtask) and picks its greedy action by argmin over its Q values --
        drawing from the same generator as the reference.  The chosen actions only mark the
        agents (agent.action is not part of T or of a repr), so the state itself is unchanged
        and already initialised."""
        if not self._level:
            return
        groups = key[1]
        memo = self.__dict__.get("_bayes_memo")  # set during a belief update (delegation.py)
        for name, op in self.other_agent_planners.items():
            op._exp, op._exp_key, op._rng = self._exp, self._exp_key, self._rng
            op.other_agent_planners, op._level = {}, 0  # _configure without other planners: Level 0
            mk = None
            if memo is not None:
                # Within one belief update no value is overwritten (value_init only inserts), so
                # an other-agent set-up met again -- same state, subtask and agents -- has its
                # start initialised and expanded and the same Q vector: only the draw remains.
                mk = ("ms", key[0], groups, str(op.subtask), tuple(op.subtask_agent_names))
                plan = memo.get(mk)
                if plan is not None:
                    _argmin_apply(plan, op._rng)
                    continue
            yield from op._configure_gen(op._configure_raw(self._level_name, self._A, self._dev, key[0], groups,
                                                           op.subtask, op.subtask_agent_names))
            yield from op._need(op.start)
            plan = _argmin_plan(op._q_all(op.start, op.v_l))
            if mk is not None:
                memo[mk] = plan
            _argmin_apply(plan, op._rng)

    def start_values(self) -> Tuple[float, float]:
        """(v_l, v_u) of the current start state."""
        sk = (self._repr(self.start), self._sub_key)
        return self.v_l[sk], self.v_u[sk]


class PlanEnv:
    """A planning start state without a live env (what :meth:`E2E_BRTDP.get_next_action` reads
    from one): the level, the agent count, the env's state bytes (``ax[A] ay[A] ah[A] loc[K]
    mask[K] t_lo t_hi flags``) and the object-group names the env has had since reset."""

    def __init__(self, level, num_agents: int, state_bytes, group_names=(), device="cuda:0"):
        self.level = level
        self._device = device
        self._A = num_agents
        self._bytes = np.asarray(state_bytes, dtype=np.uint8).copy()
        wide = capi.is_wide(level if not isinstance(level, str) else _levels.load_level(level))
        K = (len(self._bytes) - 3 * num_agents - 3) // (3 if wide else 2)
        _, _, m0 = _lay(num_agents, K, wide)
        mask = self._bytes[m0:m0 + K]
        self._live = [(j, int(m)) for j, (l, m) in enumerate(zip(_live(self._bytes, num_agents, K, wide), mask)) if l]
        self._world = None
        self._group_names = frozenset(group_names)
        self._enc = _encoding(level)
        self._names = None
        self._zero = None

    @property
    def world(self):
        if self._world is None:  # built on first use: the planner itself only needs item_names()
            self._world = types.SimpleNamespace(items=[_envs.ItemView(j, m, None, False, self._enc)
                                                       for j, m in self._live])
        return self._world

    def item_names(self) -> FrozenSet[str]:
        """The current items' object-group names (ItemView.name of every item not merged away)."""
        if self._names is None:
            self._names = frozenset(_envs.item_name(m, self._enc) for _, m in self._live)
        return self._names

    def get_agent_names(self) -> List[str]:
        return list(_agent_names(self._A))

    def planner_bytes(self, t_plane: int) -> bytes:
        """The state bytes with t and flags zeroed (what a planner set-up reads), kept."""
        if self._zero is None or self._zero[0] != t_plane:
            b = self._bytes.copy()
            b[t_plane:] = 0
            self._zero = (t_plane, b.tobytes())
        return self._zero[1]

    def state_bytes(self) -> np.ndarray:
        return self._bytes.copy()


_AGENT_NAMES: Dict[int, List[str]] = {}


# what a set-up (_configure, _configure_raw, _configure_gen) assigns on the planner, besides
# other_agent_planners (the belief update's memo replays them)
CONF_FIELDS = ("_level", "subtask", "subtask_agent_names", "is_joint", "_agents", "_sub_key", "_kind", "_goal_mask",
               "cur_obj_count", "_sub", "_conf", "_level_name", "_A", "_dev", "start", "_start_goal", "_exp",
               "_exp_key")
_AGENT_IX: Dict[tuple, tuple] = {}  # (A, subtask agent names) -> their indices
_NOOP_ROW = {1: [(_NOOP,)], 2: [(_NOOP, _NOOP)]}  # the one candidate of a set-up's no-op row


def _agent_names(A: int) -> List[str]:
    n = _AGENT_NAMES.get(A)
    if n is None:
        n = _AGENT_NAMES[A] = ["agent-%d" % (a + 1) for a in range(A)]
    return n


def _level_tables(level):
    """Per-level values the planner reads at every set-up, computed once per Level object (a
    level is not edited once planners use it): (tiles as a tuple, the Delivery cells)."""
    t = level.__dict__.get("_planner_tables")
    if t is None:
        tiles = tuple(level.tiles)
        t = (tiles, frozenset(c for c, k in enumerate(tiles) if k == 3))
        level.__dict__["_planner_tables"] = t
    return t


def _groups(env) -> FrozenSet[str]:
    """The env's object-group names since reset plus its current items' names."""
    fast = getattr(env, "item_names", None)
    names = fast() if fast is not None else frozenset(it.name for it in env.world.items)
    return frozenset(env._group_names) | names


def expander_key(env, device=None):
    """What an expander is built for: the level's grid and tiles, the agent count, the device.
    Planners may share an expander only when their keys are equal."""
    level = env.level
    return (level.width, _level_tables(level)[0], len(env.get_agent_names()), str(device or env._device))


def plan_batch(planners: Sequence[E2E_BRTDP], envs_, subtasks, agent_names, other_agent_planners=None) -> list:
    """get_next_action of many independent searches at once: planner i plans `subtasks[i]` for
    `agent_names[i]` in `envs_[i]`, at Level 0, or at Level 1 with `other_agent_planners[i]`
    (a dict of the other agents' planners, as get_next_action takes; None or {} for Level 0).
    The searches run in lockstep; every round, the states all of them need expanded -- their
    own and, at Level 1, their other agents' planners' -- go to the GPU in shared oc_rollout
    launches (up to 4,096 rows and 64 subtask configurations each), so the number of launches
    is about that of the longest single search.  Each search gives exactly its sequential
    result when its planner has its own generator (``rng=np.random.RandomState(seed)``; its
    other agents' planners draw from the same one).  All planners must share one level and
    agent count; they share the first planner's expander."""
    assert len(planners) == len(envs_) == len(subtasks) == len(agent_names)
    if not planners:
        return []
    others = other_agent_planners or [None] * len(planners)
    assert len(others) == len(planners)
    keys = {expander_key(e, p.device) for p, e in zip(planners, envs_)}
    if len(keys) != 1:
        raise ValueError("plan_batch: the searches must share one level, agent count and device "
                         "(they share one expander); got %d different ones" % len(keys))
    with searching():
        return _plan_batch(planners, envs_, subtasks, agent_names, others)


def _plan_batch(planners, envs_, subtasks, agent_names, others) -> list:
    gens = [p._next_action(e, st, an, o) for p, e, st, an, o in zip(planners, envs_, subtasks, agent_names, others)]
    out = [None] * len(gens)
    pending = {}
    exp = None
    for i, g in enumerate(gens):  # the first request of each search builds (or shares) its expander
        if exp is not None:
            planners[i]._exp, planners[i]._exp_key = exp, planners[0]._exp_key
        try:
            pending[i] = next(g)
        except StopIteration as stop:
            out[i] = stop.value
        exp = exp or planners[i]._exp
    while pending:
        idx = list(pending)
        results = exp.run([pending[i] for i in idx])
        nxt = {}
        for i, res in zip(idx, results):
            try:
                nxt[i] = gens[i].send(res)
            except StopIteration as stop:
                out[i] = stop.value
        pending = nxt
    return out
