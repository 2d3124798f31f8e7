"""Bayesian delegation's belief update over the engine: the part of
gym_cooking/delegation_planner/bayesian_delegator.py that runs every step of a
Bayesian-delegation agent (``bayes_update``, utils/agent.py:200-203).

``bayes_update`` (bayesian_delegator.py:1026-1072) drops the allocations that are no longer
doable, then multiplies each allocation by Σ len(agents) · prob_nav_actions(...) over its
(subtask, agents) pairs and normalises.  ``prob_nav_actions`` (:461-689) is inverse planning:
the softmax of β·(Q(s, taken) − Q(s, a')) over the planner's actions at Level 1, with the other
agents' planners built from the delegator's own beliefs (``get_other_agent_planners``,
:375-433).  Every Q, ``get_actions`` and ``subtask_alloc_is_doable`` here is answered by the HIP
engine: the navigation planner's rollout rows (gym_cooking_amd.planner) and the
``oc_subtask_bounds`` kernel.  The bookkeeping -- the allocation distribution, the
``random.choice`` tie-break of ``get_max`` (delegation_planner/utils.py:41), the scipy softmax --
is restated so that an update gives the reference's posterior bit for bit
(tests/golden/bayes.json).

Allocation enumeration and the spatial priors (``set_priors``) stay with the reference; a
distribution is built here from its allocations (``SubtaskAllocDistribution``).
"""
from __future__ import annotations

import copy
import random
from collections import namedtuple
from typing import Dict, List, Optional

import numpy as np
import scipy.special

from . import capi
from . import recipes as _recipes
from . import levels as _levels
from . import planner as _planner

SubtaskAllocation = namedtuple("SubtaskAllocation", "subtask subtask_agent_names")  # bayesian_delegator.py:14


class SubtaskAllocDistribution:
    """delegation_planner/utils.py:8-193: allocation -> probability, in insertion order."""

    def __init__(self, subtask_allocs):
        self.probs: Dict[tuple, float] = {}
        if len(subtask_allocs) == 0:
            return
        prior = 1. / (len(subtask_allocs))
        for subtask_alloc in subtask_allocs:
            self.probs[tuple(subtask_alloc)] = prior

    def enumerate_subtask_allocs(self) -> list:
        return list(self.probs.keys())

    def get_list(self) -> list:
        return list(self.probs.items())

    def get(self, subtask_alloc) -> float:
        return self.probs[tuple(subtask_alloc)]

    def get_max(self):
        if len(self.probs) > 0:
            max_prob = max(self.probs.values())
            max_subtask_allocs = [subtask_alloc for subtask_alloc, p in self.probs.items() if p == max_prob]
            return random.choice(max_subtask_allocs)
        return None

    def update(self, subtask_alloc, factor) -> None:
        self.probs[tuple(subtask_alloc)] *= factor

    def delete(self, subtask_alloc) -> None:
        self.probs.pop(tuple(subtask_alloc), None)

    def normalize(self) -> dict:
        total = sum(self.probs.values())
        for subtask_alloc in self.probs.keys():
            if total == 0:
                self.probs[subtask_alloc] = 1. / len(self.probs)
            else:
                self.probs[subtask_alloc] *= 1. / total
        return self.probs


_CODE = {a: i for i, a in enumerate(_levels.ACTIONS)}


class BayesianDelegator:
    """The belief update of the reference's ``BayesianDelegator`` (constructor and the methods
    ``bayes_update`` calls), over an engine-backed ``planner`` (gym_cooking_amd.planner.E2E_BRTDP).
    ``probs`` is a :class:`SubtaskAllocDistribution` of tuples of :data:`SubtaskAllocation`."""

    def __init__(self, agent_name, all_agent_names, model_type, planner, none_action_prob):
        self.name = "Bayesian Delegator"
        self.agent_name = agent_name
        self.all_agent_names = all_agent_names
        self.probs: Optional[SubtaskAllocDistribution] = None
        self.model_type = model_type
        self.priors = "uniform" if model_type == "up" else "spatial"
        self.planner = planner
        self.none_action_prob = none_action_prob

    # ---- beliefs ------------------------------------------------------------------------
    def select_subtask(self, agent_name):  # :1009-1017
        max_subtask_alloc = self.probs.get_max()
        if max_subtask_alloc is not None:
            for t in max_subtask_alloc:
                if agent_name in t.subtask_agent_names:
                    return t.subtask, t.subtask_agent_names
        return None, agent_name

    def ensure_at_least_one_subtask(self) -> None:  # :1019-1024
        if self.model_type == "greedy" or self.model_type == "dc":
            if not self.probs.probs:
                subtask_allocs = [[SubtaskAllocation(subtask=None, subtask_agent_names=(self.agent_name,))]]
                self.probs = SubtaskAllocDistribution(subtask_allocs)

    def subtask_alloc_is_doable(self, env, subtask, subtask_agent_names) -> bool:  # :98-156
        if subtask is None:
            return True
        names = env.get_agent_names()
        agents = [names.index(n) for n in subtask_agent_names]
        kind, starts, goal = _recipes.subtask_masks(subtask)
        _, ok = self._expander(env).bounds(env.state_bytes(), [capi.subtask(kind, agents, list(starts), goal, 0)])
        return bool(ok[0])

    def _expander(self, env):
        p = self.planner
        key = _planner.expander_key(env, p.device)
        if p._exp is None or p._exp_key != key:  # a planner last used on another level: rebuild
            p._exp = p._make_expander(env.level, len(env.get_agent_names()), p.device or env._device)
            p._exp_key = key
        return p._exp

    # ---- inverse planning ---------------------------------------------------------------
    def get_other_agent_planners(self, obs, backup_subtask):  # :375-433
        planners = {}
        for other_agent_name in self.all_agent_names:
            if other_agent_name != self.agent_name:
                subtask, subtask_agent_names = self.select_subtask(agent_name=other_agent_name)
                if subtask is None:
                    subtask = backup_subtask
                    subtask_agent_names = tuple(sorted([other_agent_name, self.agent_name]))
                planner = copy.copy(self.planner)
                planner.set_settings(obs, subtask, subtask_agent_names)
                planners[other_agent_name] = planner
        return planners

    def get_appropriate_state_and_other_agent_planners(self, obs_tm1, backup_subtask, no_level_1):  # :435-459
        if no_level_1:
            return obs_tm1, {}
        self.planner.modified_state(obs_tm1)
        return obs_tm1, self.get_other_agent_planners(obs=obs_tm1, backup_subtask=backup_subtask)

    def prob_nav_actions(self, obs_tm1, actions_tm1, subtask, subtask_agent_names, beta, no_level_1) -> float:
        """:461-689.  Q values, legal actions and the None branch's action count come from
        engine rollout rows; the softmax is scipy's, as the reference's."""
        assert len(subtask_agent_names) == 1 or len(subtask_agent_names) == 2
        names = obs_tm1.get_agent_names()
        if subtask is None:
            assert len(subtask_agent_names) != 2, "Two agents are doing None."
            me = names.index(self.agent_name)
            # get_single_actions(obs_tm1, self agent) - 1: its legal moves with every agent in place
            probe = capi.subtask(1, [me], [0, 0], 0, 0, 1)
            _, fl, _ = self._expander(obs_tm1).rows(obs_tm1.state_bytes(), [(c,) for c in range(4)], probe)
            num_actions = int(sum(1 for f in fl if f & capi.ROLL_LEGAL))
            action_prob = (1.0 - self.none_action_prob) / (num_actions)
            diffs = [self.none_action_prob] + [action_prob] * num_actions
            softmax_diffs = scipy.special.softmax(beta * np.asarray(diffs))
            if tuple(actions_tm1[subtask_agent_names[0]]) == (0, 0):
                return softmax_diffs[0]
            return softmax_diffs[1]
        action = tuple(_CODE[tuple(actions_tm1[a_name])] for a_name in subtask_agent_names)
        state, other_planners = self.get_appropriate_state_and_other_agent_planners(
            obs_tm1=obs_tm1, backup_subtask=subtask, no_level_1=no_level_1)
        if not other_planners:
            raise NotImplementedError("prob_nav_actions without other agents (a 1-agent env or no_level_1)")
        p = self.planner
        p.set_settings(obs_tm1, subtask, subtask_agent_names, other_planners)
        err = p.taken_action_error(p.start, action)  # Q(state, taken) and the assert below raise
        if err is not None:
            raise err("valid_nav_actions do not hold the taken action {}".format(action))
        old_q = p.Q(p.start, action, p.v_l)
        valid_nav_actions = p.get_actions(p.start)
        assert action in valid_nav_actions, "valid_nav_actions: {}\naction: {}".format(valid_nav_actions, action)
        if len(subtask_agent_names) == 2 and self.agent_name in subtask_agent_names:
            other_index = 1 - subtask_agent_names.index(self.agent_name)
            valid_nav_actions = list(filter(lambda x: x[other_index] == action[other_index], valid_nav_actions))
        qdiffs = [old_q - p.Q(p.start, nav_action, p.v_l) for nav_action in valid_nav_actions]
        softmax_diffs = scipy.special.softmax(beta * np.asarray(qdiffs))
        return softmax_diffs[valid_nav_actions.index(action)]

    def bayes_update(self, obs_tm1, actions_tm1, beta) -> None:  # :1026-1072
        for subtask_alloc in self.probs.enumerate_subtask_allocs():
            for t in subtask_alloc:
                if not self.subtask_alloc_is_doable(env=obs_tm1, subtask=t.subtask,
                                                    subtask_agent_names=t.subtask_agent_names):
                    self.probs.delete(subtask_alloc)
                    break
        self.ensure_at_least_one_subtask()
        if self.model_type == "fb":
            return
        for subtask_alloc in self.probs.enumerate_subtask_allocs():
            update = 0.0
            for t in subtask_alloc:
                if self.model_type == "greedy":
                    if self.agent_name in t.subtask_agent_names:
                        update += self.prob_nav_actions(obs_tm1=obs_tm1, actions_tm1=actions_tm1, subtask=t.subtask,
                                                        subtask_agent_names=t.subtask_agent_names, beta=beta,
                                                        no_level_1=False)
                else:
                    p = self.prob_nav_actions(obs_tm1=obs_tm1, actions_tm1=actions_tm1, subtask=t.subtask,
                                              subtask_agent_names=t.subtask_agent_names, beta=beta, no_level_1=False)
                    update += len(t.subtask_agent_names) * p
            self.probs.update(subtask_alloc=subtask_alloc, factor=update)
        self.probs.normalize()
