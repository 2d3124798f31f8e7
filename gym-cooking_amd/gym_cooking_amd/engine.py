"""OvercookedBatch: B independent kitchens stepped by the HIP engine (torch ROCm buffers).

This is the batched counterpart of ``OvercookedEnvironment.reset/step``
(gym_cooking/envs/overcooked_environment.py:201-306).  All buffers are torch uint8/uint64
tensors on one GPU in the structure-of-arrays layout of include/oc_engine.h; every call is
enqueued on torch's current stream through the C-ABI (liboc_engine.so).  There is no CPU
fallback: without the built library or a GPU the constructor raises.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import numpy as np
import torch

from . import capi
from . import levels as _levels


_U64 = (torch.uint64, torch.int64)


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _bound(fn, args):
    """A zero-argument callable issuing fn(*args) and raising on its status: one ctypes call
    per launch (the arguments were validated and converted when it was made)."""
    check = capi.check

    def launch():
        check(fn(*args))
    return launch


class OvercookedBatch:
    """B envs of one level on one GPU.

    Args:
        level: builtin level name, level-file path, or :class:`levels.Level`.
        num_agents: A (1..4).
        B: batch size (envs on this device).
        max_T: ``--max-num-timesteps`` (main.py:24; 0 = unlimited).
        device: torch device (``cuda:N``).
    """

    def __init__(self, level, num_agents: int, B: int, max_T: int = 100, device="cuda:0"):
        if isinstance(level, str):
            level = _levels.load_level(level)
        self.level = level
        self.A = num_agents
        self.B = int(B)
        self.max_T = max_T
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("OvercookedBatch runs on the GPU only (no CPU fallback)")
        self.lib = capi.load_library()
        self._desc = capi.level_desc(level, num_agents)
        h = ctypes.c_void_p()
        capi.check(self.lib.oc_create(ctypes.byref(self._desc), num_agents, max_T,
                                      self.device.index or 0, ctypes.byref(h)))
        self._h = h
        lay = capi.OcLayout()
        capi.check(self.lib.oc_get_layout(self._h, self.B, ctypes.byref(lay)))
        self.layout = lay
        self.K = lay.num_items
        self.pitch = lay.pitch
        n = ctypes.c_int64()
        capi.check(self.lib.oc_stats_size(self._h, self.B, ctypes.byref(n)))
        self.stats_bytes = n.value

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and getattr(self, "lib", None) is not None:
            self.lib.oc_destroy(h)
            self._h = None

    # ---- buffers ---------------------------------------------------------------------
    def new_state(self) -> torch.Tensor:
        return torch.empty(self.layout.state_bytes, dtype=torch.uint8, device=self.device)

    def new_actions(self, steps: int = 1) -> torch.Tensor:
        return torch.full((steps, self.A * self.pitch), 4, dtype=torch.uint8, device=self.device).squeeze(0)

    def new_exec(self) -> torch.Tensor:
        return torch.empty(self.A * self.pitch, dtype=torch.uint8, device=self.device)

    def new_coll(self) -> torch.Tensor:
        return torch.empty(self.pitch, dtype=torch.uint8, device=self.device)

    def new_stats(self) -> torch.Tensor:
        """A zeroed statistics buffer.  Besides the partial rows it holds step_n's completion
        counters, which must be zero when a launch with `totals` starts (every completed launch
        leaves them zero): zero it again after a faulted launch, and do not share one buffer
        between concurrent step_n calls on different streams."""
        return torch.zeros(self.stats_bytes // 8, dtype=torch.uint64, device=self.device)

    def planes(self, state: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Named views of a state buffer ([A|K, pitch] u8 planes; t is [pitch] u16)."""
        L, P, A, K = self.layout, self.pitch, self.A, self.K
        s = state.view(L.num_planes, P)
        return dict(
            agent_x=s[L.plane_agent_x:L.plane_agent_x + A], agent_y=s[L.plane_agent_y:L.plane_agent_y + A],
            agent_hold=s[L.plane_agent_hold:L.plane_agent_hold + A],
            item_loc=s[L.plane_item_loc:L.plane_item_loc + K], item_mask=s[L.plane_item_mask:L.plane_item_mask + K],
            t=s[L.plane_t:L.plane_t + 2].reshape(-1).view(torch.int16)[:P], flags=s[L.plane_flags],
        )

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # ---- hot path ----------------------------------------------------------------------
    def reset(self, state: torch.Tensor) -> torch.Tensor:
        """Broadcast the level template (reset(), overcooked_environment.py:201-250)."""
        self._check(state, self.layout.state_bytes)
        capi.check(self.lib.oc_reset(self._h, _ptr(state), self.B, self._stream()))
        return state

    def step(self, state_in: torch.Tensor, state_out: torch.Tensor, actions: torch.Tensor,
             exec_out: Optional[torch.Tensor] = None, coll: Optional[torch.Tensor] = None,
             stats: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One step of every env (step(), overcooked_environment.py:255-306)."""
        self._check(state_in, self.layout.state_bytes)
        self._check(state_out, self.layout.state_bytes)
        self._check(actions, self.A * self.pitch)
        if exec_out is not None:
            self._check(exec_out, self.A * self.pitch)
        if coll is not None:
            self._check(coll, self.pitch)
        if stats is not None:
            self._check(stats, self.stats_bytes, _U64)
        capi.check(self.lib.oc_step(self._h, _ptr(state_in), _ptr(state_out), _ptr(actions), _ptr(exec_out),
                                    _ptr(coll), _ptr(stats), self.B, self._stream()))
        return state_out

    def step_n(self, state_in: torch.Tensor, state_out: torch.Tensor, actions: torch.Tensor, n: int,
               traj: Optional[torch.Tensor] = None, exec_out: Optional[torch.Tensor] = None,
               coll: Optional[torch.Tensor] = None, stats: Optional[torch.Tensor] = None,
               totals: Optional[torch.Tensor] = None) -> torch.Tensor:
        """n consecutive steps in one launch (oc_step_n): identical outputs to n step() calls.
        With `totals` (int64 [OC_NSTATS], needs `stats`) the launch also folds the statistics
        into it, as reduce_stats() after it would."""
        self.step_n_launcher(state_in, state_out, actions, n, traj, exec_out, coll, stats, totals)()
        return state_out

    def step_n_launcher(self, state_in: torch.Tensor, state_out: torch.Tensor, actions: torch.Tensor, n: int,
                        traj: Optional[torch.Tensor] = None, exec_out: Optional[torch.Tensor] = None,
                        coll: Optional[torch.Tensor] = None, stats: Optional[torch.Tensor] = None,
                        totals: Optional[torch.Tensor] = None):
        """Validate the buffers of an oc_step_n call once and return a zero-argument callable
        that issues it (the buffers must stay alive and unchanged in shape): a repeated launch
        then costs one ctypes call, no per-call checks.  The stream is bound here: the callable
        launches on the stream that was current when it was made, whichever is current later."""
        self._check(state_in, self.layout.state_bytes)
        self._check(state_out, self.layout.state_bytes)
        self._check(actions, n * self.A * self.pitch)
        if traj is not None:
            self._check(traj, n * self.layout.state_bytes)
        if exec_out is not None:
            self._check(exec_out, n * self.A * self.pitch)
        if coll is not None:
            self._check(coll, n * self.pitch)
        if stats is not None:
            self._check(stats, self.stats_bytes, _U64)
        if totals is not None:
            if stats is None:
                raise ValueError("totals need the stats buffer")
            self._check(totals, 8 * capi.OC_NSTATS, _U64)
        args = (self._h, _ptr(state_in), _ptr(state_out), _ptr(actions), _ptr(traj), _ptr(exec_out), _ptr(coll),
                _ptr(stats), _ptr(totals), self.B, int(n), self._stream())
        return _bound(self.lib.oc_step_n, args)

    def rollout(self, state_in: torch.Tensor, state_out: torch.Tensor, actions: torch.Tensor, subtasks,
                alloc: Optional[torch.Tensor] = None, flags: Optional[torch.Tensor] = None,
                lower_bound: Optional[torch.Tensor] = None):
        """Navigation-planner rollout rows (oc_rollout): the Level-0 next state of every row
        under its subtask configuration, and (flags u8 [pitch], lower bound f32 [pitch])."""
        flags = torch.empty(self.pitch, dtype=torch.uint8, device=self.device) if flags is None else flags
        lower_bound = (torch.empty(self.pitch, dtype=torch.float32, device=self.device)
                       if lower_bound is None else lower_bound)
        self.rollout_launcher(state_in, state_out, actions, subtasks, alloc, flags, lower_bound)()
        return flags, lower_bound

    def rollout_launcher(self, state_in: torch.Tensor, state_out: torch.Tensor, actions: torch.Tensor, subtasks,
                         alloc: Optional[torch.Tensor], flags: torch.Tensor, lower_bound: torch.Tensor):
        """An oc_rollout call bound once (buffers validated, the subtask table packed): the
        returned callable issues it on the stream current now with one ctypes call."""
        self._check(state_in, self.layout.state_bytes)
        self._check(state_out, self.layout.state_bytes)
        self._check(actions, self.A * self.pitch)
        if alloc is not None:
            self._check(alloc, self.pitch)
        self._check(flags, self.pitch)
        self._check(lower_bound, 4 * self.pitch, (torch.float32,))
        subs = capi.subtask_array(subtasks)
        args = (self._h, _ptr(state_in), _ptr(state_out), _ptr(actions), _ptr(alloc), subs, len(subtasks),
                _ptr(flags), _ptr(lower_bound), self.B, self._stream())
        return _bound(self.lib.oc_rollout, args)

    def nav_likelihood(self, state: torch.Tensor, taken: torch.Tensor, subtasks, self_agent: int,
                       beta: float = 1.3, none_action_prob: float = 0.5, alloc: Optional[torch.Tensor] = None):
        """Bayesian-delegation likelihoods (oc_nav_likelihood): prob_nav_actions of every row's
        allocation given the executed actions `taken` (u8 [A][pitch]); returns
        (likelihood f64 [pitch], flags u8 [pitch])."""
        out = torch.empty(self.pitch, dtype=torch.float64, device=self.device)
        flags = torch.empty(self.pitch, dtype=torch.uint8, device=self.device)
        self.nav_likelihood_launcher(state, taken, subtasks, self_agent, beta, none_action_prob, alloc, out, flags)()
        return out, flags

    def nav_likelihood_launcher(self, state: torch.Tensor, taken: torch.Tensor, subtasks, self_agent: int,
                                beta: float, none_action_prob: float, alloc: Optional[torch.Tensor],
                                out: torch.Tensor, flags: torch.Tensor):
        """An oc_nav_likelihood call bound once (see rollout_launcher)."""
        self._check(state, self.layout.state_bytes)
        self._check(taken, self.A * self.pitch)
        if alloc is not None:
            self._check(alloc, self.pitch)
        self._check(out, 8 * self.pitch, (torch.float64,))
        self._check(flags, self.pitch)
        args = (self._h, _ptr(state), _ptr(taken), _ptr(alloc), capi.subtask_array(subtasks), len(subtasks),
                self_agent, beta, none_action_prob, _ptr(out), _ptr(flags), self.B, self._stream())
        return _bound(self.lib.oc_nav_likelihood, args)

    def subtask_bounds(self, state: torch.Tensor, subtasks, lower_bound: Optional[torch.Tensor] = None,
                       doable: Optional[torch.Tensor] = None):
        """Full-state subtask bounds (oc_subtask_bounds): for every env and configuration,
        get_lower_bound_for_subtask_given_objs and subtask_alloc_is_doable; returns
        (lower bound f32 [S][pitch], doable u8 [S][pitch])."""
        S = len(subtasks)
        if lower_bound is None:
            lower_bound = torch.empty((S, self.pitch), dtype=torch.float32, device=self.device)
        if doable is None:
            doable = torch.empty((S, self.pitch), dtype=torch.uint8, device=self.device)
        self.subtask_bounds_launcher(state, subtasks, lower_bound, doable)()
        return lower_bound, doable

    def subtask_bounds_launcher(self, state: torch.Tensor, subtasks, lower_bound: torch.Tensor,
                                doable: torch.Tensor):
        """An oc_subtask_bounds call bound once (see rollout_launcher)."""
        S = len(subtasks)
        self._check(state, self.layout.state_bytes)
        self._check(lower_bound, 4 * S * self.pitch, (torch.float32,))
        self._check(doable, S * self.pitch)
        args = (self._h, _ptr(state), capi.subtask_array(subtasks), S, _ptr(lower_bound), _ptr(doable), self.B,
                self._stream())
        return _bound(self.lib.oc_subtask_bounds, args)

    def set_likelihood_form(self, form: int) -> None:
        """oc_set_likelihood_form: capi.OC_LIK_FORM_AUTO (default) or OC_LIK_FORM_GROUPED (the
        grouped likelihood kernel on any level; the same outputs, for its parity test)."""
        capi.check(self.lib.oc_set_likelihood_form(self._h, int(form)))

    def last_error(self) -> str:
        """oc_get_last_error: the message of the last failed call on this handle."""
        buf = ctypes.create_string_buffer(512)
        self.lib.oc_get_last_error(self._h, buf, len(buf))
        return buf.value.decode()

    def reachability(self):
        """The level's static reachability graph (oc_reachability16): (node_of u16 [W*H*5] with
        0xFFFF = not a node, dist u16 [n][n] with 0xFFFF = no path; any level, a maze's BFS
        distances of 255 and more included)."""
        import ctypes
        n = ctypes.c_int32()
        capi.check(self.lib.oc_reachability16(self._h, ctypes.byref(n), None, 0, None, 0))
        cells = self.level.width * self.level.height
        node_of = np.zeros(cells * 5, np.uint16)
        dist = np.zeros((n.value, n.value), np.uint16)
        capi.check(self.lib.oc_reachability16(self._h, ctypes.byref(n), node_of.ctypes.data, node_of.size,
                                              dist.ctypes.data, dist.size))
        return node_of, dist

    def gen_actions(self, actions: torch.Tensor, step: int, seed: int = 0, env_offset: int = 0) -> torch.Tensor:
        self._check(actions, self.A * self.pitch)
        capi.check(self.lib.oc_gen_actions(self._h, _ptr(actions), self.B, env_offset, step, seed, self._stream()))
        return actions

    def checksum(self, state: torch.Tensor) -> torch.Tensor:
        """[1] int64 device checksum of envs [0, B) (include/oc_engine.h oc_state_checksum)."""
        self._check(state, self.layout.state_bytes)
        out = torch.empty(1, dtype=torch.int64, device=self.device)
        capi.check(self.lib.oc_state_checksum(self._h, _ptr(state), self.B, _ptr(out), self._stream()))
        return out

    def reduce_stats(self, stats: torch.Tensor) -> torch.Tensor:
        """[OC_NSTATS] uint64 device totals of a partial-stats buffer."""
        out = torch.empty(capi.OC_NSTATS, dtype=torch.int64, device=self.device)  # u64 sums < 2^63
        capi.check(self.lib.oc_stats_reduce(self._h, _ptr(stats), self.B, _ptr(out), self._stream()))
        return out

    def _check(self, t: torch.Tensor, nbytes: int, dtypes=(torch.uint8,)) -> None:
        """Device, contiguity, size, alignment and element type of a buffer handed to the
        C-ABI (the kernels read raw bytes: an int64 action tensor would pass a size check
        and be read as 8 bytes per code)."""
        if t.dtype not in dtypes:
            raise TypeError("buffer dtype %s, expected %s" % (t.dtype, " or ".join(str(d) for d in dtypes)))
        if t.device != self.device or not t.is_contiguous():
            raise ValueError("buffer must be contiguous on %s" % self.device)
        if t.numel() * t.element_size() < nbytes:
            raise ValueError("buffer too small: %d < %d bytes" % (t.numel() * t.element_size(), nbytes))
        if t.data_ptr() % 16:
            raise ValueError("buffer must be 16-byte aligned")


class CpuStepper:
    """oc_cpu_step: the engine's step on the host, for a caller without a GPU (numpy buffers in
    the oc_step layout).  The same SWAR step as the kernels (its host pass); the GPU path never
    calls it.  `step` mirrors OvercookedBatch.step (overcooked_environment.py:255-306)."""

    def __init__(self, level, num_agents: int, B: int, max_T: int = 100, nthreads: int = 0):
        if isinstance(level, str):
            level = _levels.load_level(level)
        self.level, self.A, self.B, self.max_T, self.nthreads = level, num_agents, int(B), max_T, nthreads
        self.lib = capi.load_library()
        self._desc = capi.level_desc(level, num_agents)
        h = ctypes.c_void_p()
        # a host-only handle: oc_create makes no HIP call (no device query, no device tables)
        capi.check(self.lib.oc_create(ctypes.byref(self._desc), num_agents, max_T, capi.OC_DEVICE_HOST,
                                      ctypes.byref(h)))
        self._h = h
        lay = capi.OcLayout()
        capi.check(self.lib.oc_get_layout(self._h, self.B, ctypes.byref(lay)))
        self.layout, self.K, self.pitch = lay, lay.num_items, lay.pitch

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and getattr(self, "lib", None) is not None:
            self.lib.oc_destroy(h)
            self._h = None

    def new_state(self) -> np.ndarray:
        """The level template in every env (reset(), overcooked_environment.py:201-250), built
        on the host from the level description."""
        A, K, P, L = self.A, self.K, self.pitch, self.layout
        s = np.zeros((L.num_planes, P), np.uint8)
        lv = self.level
        for a in range(A):
            s[a], s[A + a], s[2 * A + a] = lv.spawns[a][0], lv.spawns[a][1], 0xFF
        dead = 0xFFFF if L.cell_bytes == 2 else 0xFF
        for j in range(K):
            c, m = (lv.items[j] if j < len(lv.items) else (dead, 0))
            s[L.plane_item_loc + j], s[L.plane_item_mask + j] = c & 0xFF, m
            if L.cell_bytes == 2:
                s[L.plane_item_loc_hi + j] = c >> 8
        return s.reshape(-1)

    def step(self, state_in: np.ndarray, state_out: np.ndarray, actions: np.ndarray,
             exec_out: Optional[np.ndarray] = None, coll: Optional[np.ndarray] = None,
             totals: Optional[np.ndarray] = None) -> np.ndarray:
        for a, n in ((state_in, self.layout.state_bytes), (state_out, self.layout.state_bytes),
                     (actions, self.A * self.pitch), (exec_out, self.A * self.pitch), (coll, self.pitch)):
            if a is not None and (a.dtype != np.uint8 or not a.flags.c_contiguous or a.nbytes < n):
                raise ValueError("host buffers: contiguous uint8 of at least %d bytes" % n)
        if totals is not None and (totals.dtype not in (np.uint64, np.int64) or totals.size < capi.OC_NSTATS):
            raise ValueError("totals: %d uint64" % capi.OC_NSTATS)
        p = lambda a: None if a is None else a.ctypes.data  # noqa: E731
        capi.check(self.lib.oc_cpu_step(self._h, p(state_in), p(state_out), p(actions), p(exec_out), p(coll),
                                        p(totals), self.B, self.nthreads))
        return state_out
