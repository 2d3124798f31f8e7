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


@pytest.mark.parametrize("cfg", range(5))
def test_host_rollout_matches_reference_rows(cfg):
    fx = tl.load_fixture("rollout.npz")
    rows = tl.RolloutRows(fx, cfg)
    ob = oracle.OracleBatch(rows.level, rows.A, 100, rows.B)
    sin = tl.state_from_canonical(rows.level, rows.A, ob.K, ob.pitch, rows.agents, rows.items, rows.t)
    alloc = np.zeros(ob.pitch, np.uint8)
    alloc[:rows.B] = rows.alloc
    sout, flags, lb = host_rollout(ob, sin, rows.actions(ob.pitch), rows.subtasks, alloc)
    errs = rows.compare(sout, flags, lb, ob.pitch)
    assert not errs, "\n".join(errs[:20])


def random_rollout_case(level_name, A, B, seed, steps=40):
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
                                 int(rng.integers(0, 3))))
    alloc = rng.integers(0, len(subs), ob.pitch).astype(np.uint8)
    acts = rng.integers(0, 7, A * ob.pitch).astype(np.uint8)  # codes > 4 act as no-ops
    return ob, s, acts, subs, alloc


@pytest.mark.parametrize("level", ["open-divider_salad", "partial-divider_tl", "full-divider_salad"])
@pytest.mark.parametrize("A", [1, 2, 3, 4])
def test_host_rollout_matches_oracle_random(level, A):
    _load()
    ob, s, acts, subs, alloc = random_rollout_case(level, A, 3000, seed=A * 17 + len(level))
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
