"""CPU check of the device full-state bound row (ocro::RowOps::full_bound in
gym-cooking_amd/csrc/oc_rollout.h, compiled for the host by tests/swar_host/roll_host.cpp):
against the reference rows (tests/golden/bounds.npz) and against the CPU oracle on random
states x random configuration tables."""
import ctypes

import numpy as np
import pytest

import oc_testlib as tl
import test_rollout_host as th
from gym_cooking_amd import capi


def host_bounds(ob, sin, subtasks):
    L = th._load()
    if not hasattr(L, "_bounds_bound"):
        vp = ctypes.c_void_p
        L.bounds_host.restype = ctypes.c_int
        L.bounds_host.argtypes = [ctypes.POINTER(capi.OcLevelDesc), ctypes.c_int, ctypes.c_int, vp,
                                  ctypes.POINTER(capi.OcSubtask), ctypes.c_int, vp, vp, ctypes.c_int64, ctypes.c_int64]
        L._bounds_bound = True
    S = len(subtasks)
    lb = np.zeros(S * ob.pitch, np.float32)
    doable = np.zeros(S * ob.pitch, np.uint8)
    rc = L.bounds_host(ctypes.byref(ob.desc), ob.A, ob.K, th._p(sin), capi.subtask_array(subtasks), S, th._p(lb),
                       th._p(doable), ob.B, ob.pitch)
    assert rc == 0
    return lb.reshape(S, ob.pitch)[:, :ob.B], doable.reshape(S, ob.pitch)[:, :ob.B]


@pytest.mark.parametrize("cfg", range(5))
def test_host_bounds_match_reference_rows(cfg):
    from oracle import oracle
    rows = tl.BoundRows(tl.load_fixture("bounds.npz"), cfg)
    ob = oracle.OracleBatch(rows.level, rows.A, 100, rows.B)
    lb, doable = host_bounds(ob, rows.state(ob.pitch), rows.subtasks)
    errs = rows.compare(lb, doable)
    assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("level", ["open-divider_salad", "partial-divider_tl", "full-divider_salad"])
@pytest.mark.parametrize("A", [1, 2, 4])
def test_host_bounds_match_oracle_random(level, A):
    ob, s, _, subs, _ = th.random_rollout_case(level, A, 2000, seed=A * 31 + len(level))
    o_lb, o_ok = ob.subtask_bounds(s, subs)
    h_lb, h_ok = host_bounds(ob, s, subs)
    assert np.array_equal(o_lb, h_lb), np.argwhere(o_lb != h_lb)[:5]
    assert np.array_equal(o_ok, h_ok), np.argwhere(o_ok != h_ok)[:5]
