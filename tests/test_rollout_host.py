"""CPU check of the device rollout row (gym-cooking_amd/csrc/oc_rollout.h, compiled for the
host by tests/swar_host/roll_host.cpp): against the rows recorded from the reference planner
and against the CPU oracle on random states x random planner configurations."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oc_testlib as tl
from gym_cooking_amd import capi, levels

from oracle import oracle

HERE = os.path.join(tl.ROOT, "tests", "swar_host")
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists("/opt/rocm/llvm/bin/clang++"):
            pytest.skip("no clang++ for the host harness")
        subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(os.path.join(HERE, "_build", "libroll_host.so"))
        vp = ctypes.c_void_p
        L.roll_host.restype = ctypes.c_int
        L.roll_host.argtypes = [ctypes.POINTER(capi.OcLevelDesc), ctypes.c_int, ctypes.c_int, vp, vp, vp, vp,
                                ctypes.POINTER(capi.OcSubtask), ctypes.c_int, vp, vp, ctypes.c_int64, ctypes.c_int64]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def host_rollout(ob, sin, act, subtasks, alloc):
    sout = ob.new_state()
    flags = np.zeros(ob.pitch, np.uint8)
    lb = np.zeros(ob.pitch, np.float32)
    rc = _load().roll_host(ctypes.byref(ob.desc), ob.A, ob.K, _p(sin), _p(sout), _p(act), _p(alloc),
                           capi.subtask_array(subtasks), len(subtasks), _p(flags), _p(lb), ob.B, ob.pitch)
    assert rc == 0
    return sout, flags[:ob.B], lb[:ob.B]


@pytest.mark.parametrize("name,level", [("rollout.npz", 0), ("rollout_level1.npz", 1)])
@pytest.mark.parametrize("cfg", range(5))
def test_host_rollout_matches_reference_rows(name, level, cfg):
    if not os.path.exists(os.path.join(tl.GOLDEN, name)):
        pytest.skip("%s not generated" % name)
    fx = tl.load_fixture(name)
    rows = tl.RolloutRows(fx, cfg, planner_level=level)
    ob = oracle.OracleBatch(rows.level, rows.A, 100, rows.B)
    sin = tl.state_from_canonical(rows.level, rows.A, ob.K, ob.pitch, rows.agents, rows.items, rows.t)
    alloc = np.zeros(ob.pitch, np.uint8)
    alloc[:rows.B] = rows.alloc
    sout, flags, lb = host_rollout(ob, sin, rows.actions(ob.pitch), rows.subtasks, alloc)
    errs = rows.compare(sout, flags, lb, ob.pitch)
    assert not errs, "\n".join(errs[:20])


def random_rollout_case(level_name, A, B, seed, steps=40, planner_levels=(0,)):
    """Random mid-episode states (oracle goal-free random streams) x random subtask tables."""
    rng = np.random.default_rng(seed)
    lv = levels.load_level(level_name)
    ob = oracle.OracleBatch(lv, A, 1000, B)
    s, s2 = ob.new_state(), ob.new_state()
    ob.reset(s)
    act = ob.new_actions()
    for t in range(int(rng.integers(1, steps))):
        ob.gen_actions(act, 0, t, seed)
        ob.step(s, s2, act)
        s, s2 = s2, s
    # masks that can occur: every subset-merge of the level's items, fresh or chopped
    foods = [m for _, m in lv.items]
    cand = sorted({0x01, 0x02, 0x04, 0x08, 0x11, 0x22, 0x44, 0x19, 0x2A, 0x3B, 0x18, 0x28, 0x33, 0x0B, 0x09}
                  | set(foods) | set(lv.goals))
    subs = []
    for i in range(int(rng.integers(1, capi.MAX_SUBTASKS + 1))):
        n = int(rng.integers(1, 3)) if A >= 2 else 1
        ags = sorted(rng.choice(A, n, replace=False).tolist())
        kind = int(rng.integers(0, 4))
        subs.append(capi.subtask(kind, ags, [int(rng.choice(cand)), int(rng.choice(cand))], int(rng.choice(cand)),
                                 int(rng.integers(0, 3)), int(rng.choice(planner_levels))))
    alloc = rng.integers(0, len(subs), ob.pitch).astype(np.uint8)
    acts = rng.integers(0, 7, A * ob.pitch).astype(np.uint8)  # codes > 4 act as no-ops
    return ob, s, acts, subs, alloc


@pytest.mark.parametrize("level", ["open-divider_salad", "partial-divider_tl", "full-divider_salad"])
@pytest.mark.parametrize("A", [1, 2, 3, 4])
def test_host_rollout_matches_oracle_random(level, A):
    _load()
    ob, s, acts, subs, alloc = random_rollout_case(level, A, 3000, seed=A * 17 + len(level), planner_levels=(0, 1))
    o_out = ob.new_state()
    o_fl, o_lb = ob.rollout(s, o_out, acts, subs, alloc)
    h_out, h_fl, h_lb = host_rollout(ob, s, acts, subs, alloc)
    assert np.array_equal(o_fl, h_fl), np.argwhere(o_fl != h_fl)[:5]
    assert np.array_equal(o_lb, h_lb), np.argwhere(o_lb != h_lb)[:5]
    v1 = tl.env_view(o_out, A, ob.K, ob.pitch, ob.B)
    v2 = tl.env_view(h_out, A, ob.K, ob.pitch, ob.B)
    assert np.array_equal(v1, v2), np.argwhere(v1 != v2)[:5]


def test_host_rollout_bad_alloc_rows_are_flagged():
    _load()
    ob, s, acts, subs, alloc = random_rollout_case("open-divider_salad", 2, 512, seed=3)
    alloc[:ob.B:3] = len(subs) + 1
    h_out, h_fl, h_lb = host_rollout(ob, s, acts, subs, alloc)
    bad = alloc[:ob.B] >= len(subs)
    assert np.all(h_fl[bad] == capi.ROLL_BADALLOC) and np.all(h_lb[bad] == 0)
    v_in, v_out = tl.env_view(s, 2, ob.K, ob.pitch, ob.B), tl.env_view(h_out, 2, ob.K, ob.pitch, ob.B)
    assert np.array_equal(v_in[:, bad], v_out[:, bad])


def host_likelihood(ob, s, taken, subs, alloc, self_agent, beta, nap):
    L = _load()
    if not hasattr(L, "_lik"):
        vp = ctypes.c_void_p
        L.lik_host.restype = ctypes.c_int
        L.lik_host.argtypes = [ctypes.POINTER(capi.OcLevelDesc), ctypes.c_int, ctypes.c_int, vp, vp, vp,
                               ctypes.POINTER(capi.OcSubtask), ctypes.c_int, ctypes.c_int, ctypes.c_double,
                               ctypes.c_double, vp, vp, ctypes.c_int64, ctypes.c_int64]
        L._lik = True
    out = np.zeros(ob.pitch, np.float64)
    flags = np.zeros(ob.pitch, np.uint8)
    rc = L.lik_host(ctypes.byref(ob.desc), ob.A, ob.K, _p(s), _p(taken), _p(alloc), capi.subtask_array(subs),
                    len(subs), self_agent, beta, nap, _p(out), _p(flags), ob.B, ob.pitch)
    assert rc == 0
    return out[:ob.B], flags[:ob.B]


@pytest.mark.parametrize("cfg", range(4))
@pytest.mark.parametrize("self_agent", [0, 1])
def test_host_likelihood_matches_reference(cfg, self_agent):
    fx = tl.load_fixture("likelihood.npz")
    rows = tl.LikelihoodRows(fx, cfg, self_agent)
    for sel, alloc, subs in rows.chunks(capi.MAX_SUBTASKS):
        ob = oracle.OracleBatch(rows.level, rows.A, 100, len(sel))
        s, taken = rows.inputs(sel, ob.pitch)
        a = np.zeros(ob.pitch, np.uint8)
        a[:len(sel)] = alloc
        v, f = host_likelihood(ob, s, taken, subs, a, self_agent, rows.beta, rows.nap)
        errs = rows.compare(sel, v, f, 1e-12)
        assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("level,A", [("open-divider_salad", 2), ("full-divider_salad", 4), ("partial-divider_tl", 3)])
def test_host_likelihood_matches_oracle_random(level, A):
    ob, s, acts, subs, alloc = random_rollout_case(level, A, 2000, seed=7 * A)
    for self_agent in range(min(A, 2)):
        o_v, o_f = ob.nav_likelihood(s, acts, subs, alloc, self_agent, 1.3, 0.5)
        h_v, h_f = host_likelihood(ob, s, acts, subs, alloc, self_agent, 1.3, 0.5)
        assert np.array_equal(o_f, h_f), np.argwhere(o_f != h_f)[:5]
        ok = o_f == capi.LIK_OK
        assert ok.sum() > 100
        np.testing.assert_allclose(h_v[ok], o_v[ok], rtol=1e-13)


def test_host_rollout_flags_level0_double_removal():
    """Two agents outside the subtask on one square: the reference raises in set_settings."""
    _load()
    lv = levels.load_level("open-divider_salad")
    ob = oracle.OracleBatch(lv, 3, 100, 4)
    s = ob.new_state()
    ob.reset(s)
    v = tl.planes_view(s, 3, ob.K, ob.pitch)
    v["ax"][2, :4], v["ay"][2, :4] = v["ax"][0, :4], v["ay"][0, :4]  # agents 1 and 3 co-located
    subs = [capi.subtask(capi.SUB_CHOP, (1,), (0x01, 0), 0x11)]
    acts = np.full(3 * ob.pitch, 3, np.uint8)
    o_out = ob.new_state()
    o_fl, o_lb = ob.rollout(s, o_out, acts, subs, None)
    h_out, h_fl, h_lb = host_rollout(ob, s, acts, subs, None)
    assert np.all(o_fl == capi.ROLL_RAISES) and np.all(h_fl == capi.ROLL_RAISES)
    assert np.array_equal(tl.env_view(h_out, 3, ob.K, ob.pitch, 4), tl.env_view(s, 3, ob.K, ob.pitch, 4))
