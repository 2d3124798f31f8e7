"""TEST INFRASTRUCTURE: ctypes wrapper of the CPU oracle (oracle/oc_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module;
the product path never does.  See oc_oracle.c for what the oracle restates and how it is
pinned to the reference (tests/golden/).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboc_oracle.so")
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "gym-cooking_amd"))
from gym_cooking_amd import capi  # noqa: E402

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.isfile(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64
        L.oco_step.restype = ctypes.c_int
        L.oco_step.argtypes = [ctypes.POINTER(capi.OcLevelDesc), i32, i32, i32, vp, vp, vp, vp, vp,
                               i64, i64, i32]
        L.oco_reset.restype = ctypes.c_int
        L.oco_reset.argtypes = [ctypes.POINTER(capi.OcLevelDesc), i32, i32, vp, i64, i64]
        L.oco_gen_actions.restype = ctypes.c_int
        L.oco_gen_actions.argtypes = [i32, vp, i64, i64, i64, i64, u64]
        L.oco_rollout.restype = ctypes.c_int
        L.oco_rollout.argtypes = [ctypes.POINTER(capi.OcLevelDesc), i32, i32, vp, vp, vp, vp,
                                  ctypes.POINTER(capi.OcSubtask), i32, vp, vp, i64, i64, i32]
        L.oco_nav_likelihood.restype = ctypes.c_int
        L.oco_nav_likelihood.argtypes = [ctypes.POINTER(capi.OcLevelDesc), i32, i32, vp, vp, vp,
                                         ctypes.POINTER(capi.OcSubtask), i32, i32, ctypes.c_double, ctypes.c_double,
                                         vp, vp, i64, i64, i32]
        L.oco_subtask_bounds.restype = ctypes.c_int
        L.oco_subtask_bounds.argtypes = [ctypes.POINTER(capi.OcLevelDesc), i32, i32, vp,
                                         ctypes.POINTER(capi.OcSubtask), i32, vp, vp, i64, i64, i32]
        L.oco_action_code.restype = ctypes.c_uint8
        L.oco_action_code.argtypes = [u64, u64, u64, u64]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


class OracleBatch:
    """B envs of one level in the engine's byte-plane layout, stepped by the oracle."""

    def __init__(self, level, num_agents: int, max_T: int, B: int):
        self.level = level
        self.A = num_agents
        self.K = capi.item_slots(level)
        self.max_T = max_T
        self.B = B
        self.pitch = capi.pitch_for(B)
        self.wide = capi.is_wide(level)
        self.planes = capi.layout_planes(self.A, self.K, self.wide)
        self.desc = capi.level_desc(level, num_agents)

    def new_state(self) -> np.ndarray:
        return np.zeros(self.planes["num_planes"] * self.pitch, np.uint8)

    def new_actions(self) -> np.ndarray:
        return np.full(self.A * self.pitch, 4, np.uint8)

    def reset(self, state: np.ndarray) -> None:
        rc = lib().oco_reset(ctypes.byref(self.desc), self.A, self.K, _p(state), self.B, self.pitch)
        assert rc == 0

    def step(self, sin, sout, actions, exec_out=None, coll=None, nthreads=1) -> None:
        rc = lib().oco_step(ctypes.byref(self.desc), self.A, self.K, self.max_T, _p(sin), _p(sout),
                            _p(actions), _p(exec_out), _p(coll), self.B, self.pitch, nthreads)
        assert rc == 0

    def rollout(self, sin, sout, actions, subtasks, alloc=None, nthreads=8):
        """Planner rollout rows (oco_rollout): returns (flags u8 [B], lower bound f32 [B])."""
        subs = capi.subtask_array(subtasks)
        flags = np.zeros(self.pitch, np.uint8)
        lb = np.zeros(self.pitch, np.float32)
        rc = lib().oco_rollout(ctypes.byref(self.desc), self.A, self.K, _p(sin), _p(sout), _p(actions),
                               _p(alloc), subs, len(subtasks), _p(flags), _p(lb), self.B, self.pitch, nthreads)
        assert rc == 0, rc
        return flags[:self.B], lb[:self.B]

    def nav_likelihood(self, state, taken, subtasks, alloc, self_agent, beta, none_action_prob, nthreads=8):
        """prob_nav_actions rows (oco_nav_likelihood): returns (f64 [B], flags u8 [B])."""
        out = np.zeros(self.pitch, np.float64)
        flags = np.zeros(self.pitch, np.uint8)
        rc = lib().oco_nav_likelihood(ctypes.byref(self.desc), self.A, self.K, _p(state), _p(taken), _p(alloc),
                                      capi.subtask_array(subtasks), len(subtasks), self_agent, beta,
                                      none_action_prob, _p(out), _p(flags), self.B, self.pitch, nthreads)
        assert rc == 0, rc
        return out[:self.B], flags[:self.B]

    def subtask_bounds(self, state, subtasks, nthreads=8):
        """Full-state subtask bounds (oco_subtask_bounds): returns (lb f32 [S][B], doable u8 [S][B])."""
        S = len(subtasks)
        lb = np.zeros(S * self.pitch, np.float32)
        doable = np.zeros(S * self.pitch, np.uint8)
        rc = lib().oco_subtask_bounds(ctypes.byref(self.desc), self.A, self.K, _p(state), capi.subtask_array(subtasks),
                                      S, _p(lb), _p(doable), self.B, self.pitch, nthreads)
        assert rc == 0, rc
        return lb.reshape(S, self.pitch)[:, :self.B], doable.reshape(S, self.pitch)[:, :self.B]

    def gen_actions(self, actions, env_offset, step, seed) -> None:
        rc = lib().oco_gen_actions(self.A, _p(actions), self.B, self.pitch, env_offset, step, seed)
        assert rc == 0


def action_code(seed: int, gid: int, step: int, agent: int) -> int:
    return int(lib().oco_action_code(seed, gid, step, agent))
