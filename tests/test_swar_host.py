"""CPU check of the device SWAR step logic (gym-cooking_amd/csrc/oc_swar.h), compiled for the
host by tests/swar_host/ with the two AMDGCN intrinsics emulated bit-exactly: replays the
reference fixtures and random streams against the CPU oracle.  Catches logic errors in the
kernel's step without a GPU; the GPU tests then check the real device build."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oc_testlib as tl
from gym_cooking_amd import capi, levels

from oracle import oracle

HERE = os.path.join(tl.ROOT, "tests", "swar_host")
LIB = os.path.join(HERE, "_build", "libswar_host.so")
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists("/opt/rocm/llvm/bin/clang++"):
            pytest.skip("no clang++ for the host SWAR harness")
        subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        L.swar_host_step.restype = ctypes.c_int
        L.swar_host_step.argtypes = [ctypes.POINTER(capi.OcLevelDesc), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     vp, vp, vp, vp, vp, ctypes.c_int64, ctypes.c_int64]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


class SwarHostBatch(oracle.OracleBatch):
    def step(self, sin, sout, actions, exec_out=None, coll=None, nthreads=1):
        rc = _load().swar_host_step(ctypes.byref(self.desc), self.A, self.K, self.max_T, _p(sin), _p(sout),
                                    _p(actions), _p(exec_out), _p(coll), self.B, self.pitch)
        assert rc == 0


def _step_fn(sb):
    def fn(state, acts):
        a = sb.new_actions()
        a.reshape(sb.A, sb.pitch)[:, :sb.B] = acts
        out = sb.new_state()
        ex = np.zeros(sb.A * sb.pitch, np.uint8)
        coll = np.zeros(sb.pitch, np.uint8)
        sb.step(state, out, a, ex, coll)
        return out, ex.reshape(sb.A, sb.pitch)[:, :sb.B], coll[:sb.B]
    return fn


@pytest.mark.parametrize("fixture", ["kat.npz", "streams.npz", "greedy.npz"])
def test_swar_step_matches_reference_fixtures(fixture):
    _load()
    fx = tl.load_fixture(fixture)
    for g in tl.episode_groups(fx):
        sb = SwarHostBatch(g.level, g.A, g.max_T, g.B)
        s = sb.new_state()
        sb.reset(s)
        g.relocate(s, sb.pitch)
        errs = tl.compare_group(g, _step_fn(sb), s, sb.pitch, g.level.width)
        assert not errs, "\n".join(errs[:10])


@pytest.mark.parametrize("level", sorted(levels.BUILTIN_LEVELS))
@pytest.mark.parametrize("A", [1, 2, 3, 4])
def test_swar_step_matches_oracle_random(level, A):
    _load()
    B, steps, max_T = 1003, 130, 60
    lv = levels.load_level(level)
    ob = oracle.OracleBatch(lv, A, max_T, B)
    sb = SwarHostBatch(lv, A, max_T, B)
    s1, s2, n1, n2 = ob.new_state(), sb.new_state(), ob.new_state(), sb.new_state()
    ob.reset(s1)
    sb.reset(s2)
    act = ob.new_actions()
    e1, e2 = np.zeros(A * ob.pitch, np.uint8), np.zeros(A * ob.pitch, np.uint8)
    c1, c2 = np.zeros(ob.pitch, np.uint8), np.zeros(ob.pitch, np.uint8)
    for t in range(steps):
        ob.gen_actions(act, 0, t, A * 131 + t % 3)
        ob.step(s1, n1, act, e1, c1)
        sb.step(s2, n2, act, e2, c2)
        s1, n1, s2, n2 = n1, s1, n2, s2
        v1, v2 = tl.env_view(s1, A, ob.K, ob.pitch, B), tl.env_view(s2, A, ob.K, ob.pitch, B)
        if not np.array_equal(v1, v2):
            bad = np.argwhere(v1 != v2)
            raise AssertionError("step %d: %d bytes differ, first (plane, env) %s" % (t, len(bad), bad[:5].tolist()))
        assert np.array_equal(e1.reshape(A, -1)[:, :B], e2.reshape(A, -1)[:, :B]), t
        assert np.array_equal(c1[:B], c2[:B]), t


def test_swar_invalid_action_codes():
    _load()
    lv = levels.load_level("open-divider_salad")
    B = 512
    ob = oracle.OracleBatch(lv, 2, 100, B)
    sb = SwarHostBatch(lv, 2, 100, B)
    s = ob.new_state()
    ob.reset(s)
    rng = np.random.default_rng(0)
    for t in range(20):
        act = rng.integers(0, 256, 2 * ob.pitch).astype(np.uint8)
        o1, o2 = ob.new_state(), sb.new_state()
        ob.step(s, o1, act)
        sb.step(s, o2, act)
        assert np.array_equal(tl.env_view(o1, 2, 4, ob.pitch, B), tl.env_view(o2, 2, 4, ob.pitch, B))
        s = o1


def _step_n_host(sb, s, acts, n):
    """swar_host_step_n: n steps per lane with the state kept between steps (oc_step_n's lane
    loop: the loaded state takes the full path once, then the rare-event split decides)."""
    L = _load()
    if not hasattr(L, "_sn"):
        vp = ctypes.c_void_p
        L.swar_host_step_n.restype = ctypes.c_int
        L.swar_host_step_n.argtypes = [ctypes.POINTER(capi.OcLevelDesc), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       vp, vp, vp, vp, vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
        L._sn = True
    S = s.size
    traj = np.zeros(n * S, np.uint8)
    ex = np.zeros(n * sb.A * sb.pitch, np.uint8)
    coll = np.zeros(n * sb.pitch, np.uint8)
    rc = L.swar_host_step_n(ctypes.byref(sb.desc), sb.A, sb.K, sb.max_T, _p(s), _p(traj), _p(acts), _p(ex), _p(coll),
                            sb.B, sb.pitch, n)
    assert rc == 0
    return traj.reshape(n, S), ex.reshape(n, sb.A, sb.pitch), coll.reshape(n, sb.pitch)


@pytest.mark.parametrize("level,A,max_T", [("partial-divider_salad", 2, 30), ("full-divider_tl", 3, 45),
                                           ("open-divider_salad", 4, 25), ("open-divider_tl", 2, 0),
                                           ("levels/dup-12x12_salad3t.txt", 3, 40)])
def test_swar_step_n_rare_event_split_matches_oracle(level, A, max_T):
    """The rare-event split over long multi-step runs (resets at max_T, goal-directed-ish play
    from the reference fixtures' states, deliveries), every step against the oracle."""
    _load()
    B, n = 2003, 120
    lv = tl.load_level(level)
    ob = oracle.OracleBatch(lv, A, max_T, B)
    sb = SwarHostBatch(lv, A, max_T, B)
    s = ob.new_state()
    ob.reset(s)
    acts = np.zeros(n * A * ob.pitch, np.uint8)
    a1 = ob.new_actions()
    for t in range(n):
        ob.gen_actions(a1, 0, t, 5 + A)
        acts[t * A * ob.pitch:(t + 1) * A * ob.pitch] = a1
    traj, ex, coll = _step_n_host(sb, s, acts, n)
    c, c2 = s.copy(), ob.new_state()
    e1, c1 = np.zeros(A * ob.pitch, np.uint8), np.zeros(ob.pitch, np.uint8)
    for t in range(n):
        ob.step(c, c2, acts[t * A * ob.pitch:(t + 1) * A * ob.pitch], e1, c1)
        c, c2 = c2, c
        assert np.array_equal(tl.env_view(traj[t], A, ob.K, ob.pitch, B), tl.env_view(c, A, ob.K, ob.pitch, B)), t
        assert np.array_equal(ex[t][:, :B], e1.reshape(A, -1)[:, :B]), t
        assert np.array_equal(coll[t][:B], c1[:B]), t


def test_swar_step_n_pending_state_with_items_on_delivery():
    """A loaded state that already has the goal dish on the Delivery square but DONE cleared
    (the gym shim keeps stepping a finished env, as the reference does): the first step of the
    launch must report success again, with no delivery in that step."""
    _load()
    fx = tl.load_fixture("kat.npz")
    g = next(g for g in tl.episode_groups(fx) if any(fx["flags"][fx["ep_state_off"][e] + fx["ep_T"][e]] & 2
                                                      for e in g.idx))
    b = next(i for i, e in enumerate(g.idx) if fx["flags"][fx["ep_state_off"][e] + fx["ep_T"][e]] & 2)
    e = g.idx[b]
    o = fx["ep_state_off"][e] + fx["ep_T"][e]
    ob = oracle.OracleBatch(g.level, g.A, 0, 1)
    sb = SwarHostBatch(g.level, g.A, 0, 1)
    s = tl.state_from_canonical(g.level, g.A, ob.K, ob.pitch, fx["agents"][o][None], fx["items"][o][None],
                                fx["t"][o][None])
    acts = np.full(3 * g.A * ob.pitch, 4, np.uint8)
    traj, _, _ = _step_n_host(sb, s, acts, 3)
    c, c2 = s.copy(), ob.new_state()
    for t in range(3):
        ob.step(c, c2, acts[:g.A * ob.pitch])
        c, c2 = c2, c
        assert np.array_equal(tl.env_view(traj[t], g.A, ob.K, ob.pitch, 1), tl.env_view(c, g.A, ob.K, ob.pitch, 1)), t
    fl = tl.planes_view(traj[0], g.A, ob.K, ob.pitch)["fl"][0]
    assert (fl & 3) == 3  # done and successful again after a no-op step
