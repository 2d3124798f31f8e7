"""Engine-backed navigation planner: a drop-in for
gym_cooking/navigation_planner/planners/e2e_brtdp.py ``E2E_BRTDP`` at Level 0.

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
agents, every dynamic object group (``World.objects`` keeps emptied groups, world.py:304-337)
and the frozen agents' ``Agent-Counter`` squares.  Here a state is (its engine state bytes
without ``t`` / flags, the set of object-group names), which identifies the same states:
frozen agents keep their cells in the bytes, and a group name set plus per-slot items fixes
every group's list.

Level 1 (``other_agent_planners`` non-empty, the BD agents' call) predicts the other agents'
moves with their own planners; it is not restated here and raises ``NotImplementedError``.
"""
from __future__ import annotations

import itertools
from typing import Dict, FrozenSet, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import capi
from . import envs as _envs
from . import recipes as _recipes

_NAV = [(0, 1), (0, -1), (-1, 0), (1, 0), (0, 0)]  # action codes 0..4 (World.NAV_ACTIONS + no-op)
_NOOP = 4


_NAMES: Dict[int, str] = {}


def _group_name(mask: int) -> str:
    """World.objects group name of an item mask (its base contents, core.py:161-171)."""
    n = _NAMES.get(mask)
    if n is None:
        n = _NAMES[mask] = _envs.ItemView(-1, mask, None, False).name
    return n


def argmin(vector):
    """e2e_brtdp.py:27-30: the index of a minimum, ties broken by numpy's global generator
    (one ``np.random.multinomial`` draw per call, ties or not)."""
    e_x = np.array(vector) == min(vector)
    return np.where(np.random.multinomial(1, e_x / e_x.sum()))[0][0]


class _Expander:
    """One engine batch of ROWS rows for a level: expands a state for all its joint actions in
    one oc_rollout launch."""

    ROWS = 32  # >= 25 joint actions

    def __init__(self, level, num_agents: int, device):
        from .engine import OvercookedBatch  # raises without liboc_engine.so / a GPU
        self.eb = OvercookedBatch(level, num_agents, self.ROWS, max_T=0, device=device)
        self.A, self.K, self.P = self.eb.A, self.eb.K, self.eb.pitch
        self.NP = self.eb.layout.num_planes
        self.t_plane = self.eb.layout.plane_t
        dev = self.eb.device
        self.s_in = self.eb.new_state()
        self.s_out = self.eb.new_state()
        self.act = self.eb.new_actions()
        self.flags = torch.empty(self.P, dtype=torch.uint8, device=dev)
        self.lb = torch.empty(self.P, dtype=torch.float32, device=dev)
        self._host_in = torch.empty((self.NP, self.ROWS), dtype=torch.uint8).pin_memory()
        self._host_act = torch.empty((self.A, self.ROWS), dtype=torch.uint8).pin_memory()
        self._host_out = torch.empty((self.NP, self.ROWS), dtype=torch.uint8).pin_memory()
        self._host_fl = torch.empty(self.ROWS, dtype=torch.uint8).pin_memory()
        self._host_lb = torch.empty(self.ROWS, dtype=torch.float32).pin_memory()
        self.launches = 0

    def rows(self, state: np.ndarray, codes: Sequence[Tuple[int, ...]], sub: capi.OcSubtask):
        """Rollout rows of `state` (engine bytes, env_view order) under `sub` for each joint
        action in `codes` (tuples of the subtask agents' codes).  Returns (next states
        [n, NP] u8, flags [n], lower bounds [n])."""
        n = len(codes)
        assert 0 < n <= self.ROWS
        hi = self._host_in.numpy()
        hi[:, :] = state[:, None]
        hi[self.t_plane:, :] = 0  # t and flags: copied through by the kernel, not part of a planner state
        ha = self._host_act.numpy()
        ha[:, :] = _NOOP
        for r, c in enumerate(codes):
            for q, a in enumerate(sub.agent[:sub.num_agents]):
                ha[a, r] = c[q]
        self.s_in.view(self.NP, self.P)[:, :self.ROWS].copy_(self._host_in, non_blocking=True)
        self.act.view(self.A, self.P)[:, :self.ROWS].copy_(self._host_act, non_blocking=True)
        self.eb.rollout(self.s_in, self.s_out, self.act, [sub], None, self.flags, self.lb)
        self.launches += 1
        # three async copies into pinned memory, one wait
        self._host_out.copy_(self.s_out.view(self.NP, self.P)[:, :self.ROWS], non_blocking=True)
        self._host_fl.copy_(self.flags[:self.ROWS], non_blocking=True)
        self._host_lb.copy_(self.lb[:self.ROWS], non_blocking=True)
        torch.cuda.current_stream(self.eb.device).synchronize()
        nxt = self._host_out.numpy()[:, :n].T.copy()
        nxt[:, self.t_plane:] = 0
        return nxt, self._host_fl.numpy()[:n].copy(), self._host_lb.numpy()[:n].copy()


class E2E_BRTDP:
    """Bounded RTDP navigation planner (e2e_brtdp.py:38-878), Level 0, over the HIP engine.

    Same constructor, same ``get_next_action(env, subtask, subtask_agent_names,
    other_agent_planners)``, same value tables ``v_l`` / ``v_u`` (keyed by (state, subtask)),
    ``cur_state``, ``cur_obj_count``, ``is_joint``.  ``env`` is the engine-backed
    :class:`gym_cooking_amd.envs.OvercookedEnvironment`.
    """

    def __init__(self, alpha, tau, cap, main_cap, device: Optional[str] = None, expander=None):
        """`expander(level, num_agents, device)` builds the row evaluator; the default is the
        HIP engine (``oc_rollout``).  Tests pass the CPU oracle's rollout here to check the
        host search without a GPU."""
        self.alpha, self.tau, self.cap, self.main_cap = alpha, tau, cap, main_cap
        self._make_expander = expander or _Expander
        self.v_l: Dict = {}
        self.v_u: Dict = {}
        self.time_cost = 1.0
        self.action_cost = 0.1
        self.is_joint = False
        self.subtask = None
        self.device = device
        self._exp: Optional[_Expander] = None
        self._exp_key = None
        self._succ: Dict = {}  # (state key, subtask key) -> (actions, [(next key, next state)])
        self._states: Dict = {}  # state key -> (bytes, groups)

    # ---- configuration (set_settings, e2e_brtdp.py:582-652) --------------------------------
    def set_settings(self, env, subtask, subtask_agent_names, other_agent_planners=None):
        if other_agent_planners:
            raise NotImplementedError("Level-1 planning (other_agent_planners) is not restated")
        if subtask is None:
            raise NotImplementedError("the reference agents do not plan the None subtask")
        assert len(subtask_agent_names) <= 2, "Cannot have more than 2 agents! Hm... {}".format(subtask_agent_names)
        names = env.get_agent_names()
        self.subtask = subtask
        self.subtask_agent_names = tuple(subtask_agent_names)
        self.is_joint = len(subtask_agent_names) == 2
        agents = [names.index(n) for n in subtask_agent_names]
        assert agents == sorted(agents), "subtask agent names are not in order"
        self._agents = agents
        level, A = env.level, len(names)
        key = (id(level), A, str(self.device or env._device))
        if self._exp is None or self._exp_key != key:
            self._exp = self._make_expander(level, A, self.device or env._device)
            self._exp_key = key
        exp = self._exp
        kind, starts, goal = _recipes.subtask_masks(subtask)
        self._sub_key = str(subtask)
        self._kind, self._goal_mask = kind, goal
        full = env.state_bytes()
        groups = frozenset(env._group_names) | frozenset(it.name for it in env.world.items)
        start = self._level0(full, exp)
        start[exp.t_plane:] = 0
        self.cur_obj_count = self._obj_count(start, exp, env.level)  # _define_goal_state on the Level-0 env
        self._sub = capi.subtask(kind, agents, list(starts), goal, self.cur_obj_count)
        # the start state: a no-op row gives its goal flag and lower bound
        nxt, fl, lb = exp.rows(start, [(_NOOP,) * len(agents)], self._sub)
        self.start = self._key(start, groups)
        self._states.setdefault(self.start, (start, groups))
        self._start_goal = bool(fl[0] & capi.ROLL_GOAL)  # is_goal_state with this call's cur_obj_count
        self._value_init(self.start, self._start_goal, float(lb[0]))

    def _level0(self, full: np.ndarray, exp: _Expander) -> np.ndarray:
        """E2E_BRTDP._configure_planner_level, Level 0 (e2e_brtdp.py:383-406): the items held by
        agents outside the subtask leave the world (their frozen cells stay in the bytes; the
        kernel treats them as AgentCounters)."""
        s = full.copy()
        A, K = exp.A, exp.K
        for a in range(A):
            if a in self._agents:
                continue
            h = int(s[2 * A + a])
            if h != 0xFF:
                s[3 * A + h], s[3 * A + K + h] = 0xFF, 0
                s[2 * A + a] = 0xFF
        return s

    def _obj_count(self, s: np.ndarray, exp: _Expander, level) -> int:
        """cur_obj_count of _define_goal_state (e2e_brtdp.py:435-566) on a Level-0 state."""
        A, K = exp.A, exp.K
        held = {int(s[2 * A + a]) for a in range(A)} - {0xFF}
        deliv = {c for c, t in enumerate(level.tiles) if t == 3}
        locs = []
        for j in range(K):
            c, m = int(s[3 * A + j]), int(s[3 * A + K + j])
            if c == 0xFF or m != self._goal_mask:
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
        return (s.tobytes(), groups, tuple(self._agents))

    # ---- values (value_init, e2e_brtdp.py:678-729) --------------------------------------------
    def _value_init(self, key, goal: bool, lb: float) -> None:
        vk = (key, self._sub_key)
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


    # ---- transitions: one launch per state -------------------------------------------------
    def _expand(self, key):
        ek = (key, self._sub_key)
        got = self._succ.get(ek)
        if got is not None:
            return got
        s, groups = self._states[key]
        n = len(self._agents)
        cand = list(itertools.product(range(5), repeat=n))  # product order of get_actions
        nxt, fl, lb = self._exp.rows(s, cand, self._sub)
        K = self._exp.K
        l0, m0 = 3 * self._exp.A, 3 * self._exp.A + K
        actions, succ = [], []
        for r, c in enumerate(cand):
            if not fl[r] & capi.ROLL_LEGAL:
                continue
            if fl[r] & capi.ROLL_ASSERT:  # T raises (e2e_brtdp.py:143)
                raise AssertionError("action {} led to co-located subtask agents".format(c))
            ns = nxt[r]
            ng = groups | frozenset(_group_name(int(m)) for m, l in zip(ns[m0:m0 + K], ns[l0:l0 + K]) if l != 0xFF)
            nk = self._key(ns, ng)
            self._states.setdefault(nk, (ns, ng))
            self._value_init(nk, bool(fl[r] & capi.ROLL_GOAL), float(lb[r]))
            actions.append(c)
            succ.append(nk)
        got = (actions, succ)
        self._succ[ek] = got
        return got

    def get_actions(self, key) -> List[tuple]:  # e2e_brtdp.py:151-206
        return self._expand(key)[0]

    def T(self, key, action):  # e2e_brtdp.py:103-149
        actions, succ = self._expand(key)
        return succ[actions.index(action)]

    def cost(self, action) -> float:  # e2e_brtdp.py:816-826
        cost = self.time_cost
        for c in action:
            if c != _NOOP:
                cost += self.action_cost
        return cost

    def Q(self, key, action, value_f) -> float:  # e2e_brtdp.py:736-760
        cost = self.cost(action)
        nk = self.T(key, action)
        expected_value = 1.0 * value_f[(nk, self._sub_key)]
        return float(cost + expected_value)

    def get_expected_diff(self, key, action):  # e2e_brtdp.py:828-840
        nk = self.T(key, action)
        return {nk: 1.0 * (self.v_u[(nk, self._sub_key)] - self.v_l[(nk, self._sub_key)])}

    # ---- search (e2e_brtdp.py:208-331, 842-878) ----------------------------------------------
    def runSampleTrial(self) -> None:
        x = self.start
        traj = []
        counter = 0
        sk = self._sub_key
        while True:
            counter += 1
            if counter > self.cap:
                break
            traj.append(x)
            actions = self.get_actions(x)
            new_upper = min([self.Q(x, a, self.v_u) for a in actions])
            self.v_u[(x, sk)] = new_upper
            action_index = argmin([self.Q(x, a, self.v_l) for a in actions])
            a = actions[action_index]
            new_lower = self.Q(x, a, self.v_l)
            self.v_l[(x, sk)] = new_lower
            b = self.get_expected_diff(x, a)
            B = sum(b.values())
            diff = (self.v_u[(self.start, sk)] - self.v_l[(self.start, sk)]) / self.tau
            if B <= diff:
                break
            x = list(b.keys())[0]
        while traj:
            x = traj.pop()
            actions = self.get_actions(x)
            self.v_u[(x, sk)] = min([self.Q(x, a, self.v_u) for a in actions])
            self.v_l[(x, sk)] = min([self.Q(x, a, self.v_l) for a in actions])

    def main(self) -> None:
        main_counter = 0
        sk = (self.start, self._sub_key)
        diff = self.v_u[sk] - self.v_l[sk]
        while diff > self.alpha and main_counter < self.main_cap:
            diff = self.v_u[sk] - self.v_l[sk]
            main_counter += 1
            self.runSampleTrial()

    def get_next_action(self, env, subtask, subtask_agent_names, other_agent_planners=None):
        """The next (joint) action for the subtask agents, as the reference's
        ``get_next_action`` returns it: a (dx, dy) tuple for one agent, a pair of them for two,
        ``None`` when the start state already satisfies the subtask."""
        self.set_settings(env, subtask, subtask_agent_names, other_agent_planners)
        cur = self.start
        self.cur_state = cur
        actions = self.get_actions(cur)
        action_index = argmin([self.Q(cur, a, self.v_l) for a in actions])
        a = actions[action_index]
        B = sum(self.get_expected_diff(cur, a).values())
        sk = (cur, self._sub_key)
        diff = (self.v_u[sk] - self.v_l[sk]) / self.tau
        if B > diff:
            self.main()
        if self._start_goal:  # is_goal_state(cur_state)
            return None
        actions = self.get_actions(cur)
        qvals = [self.Q(cur, a, self.v_l) for a in actions]
        a = actions[argmin(np.array(qvals))]
        return _NAV[a[0]] if len(a) == 1 else tuple(_NAV[c] for c in a)

    def start_values(self) -> Tuple[float, float]:
        """(v_l, v_u) of the current start state."""
        sk = (self.start, self._sub_key)
        return self.v_l[sk], self.v_u[sk]
