"""The CPU oracle's planner-rollout restatement (oracle/oc_oracle.c, oco_rollout) against
the rows recorded from the reference planner (tests/golden/rollout.npz, gen_rollout.py):
legality, co-location assert, goal test, next state and lower bound, bit-exact; and the
planner's value_init arithmetic on top of the lower bound."""
import os

import numpy as np
import pytest

import oc_testlib as tl
from gym_cooking_amd import capi

from oracle import oracle


@pytest.fixture(scope="module")
def fx():
    return tl.load_fixture("rollout.npz")


FIXTURES = [("rollout.npz", 0), ("rollout_level1.npz", 1)]  # (file, planner level)


@pytest.mark.parametrize("name,level", FIXTURES)
@pytest.mark.parametrize("cfg", range(5))
def test_oracle_rollout_matches_reference_rows(name, level, cfg):
    if not os.path.exists(os.path.join(tl.GOLDEN, name)):
        pytest.skip("%s not generated" % name)
    rows = tl.RolloutRows(tl.load_fixture(name), cfg, planner_level=level)
    ob = oracle.OracleBatch(rows.level, rows.A, 100, rows.B)
    sin = tl.state_from_canonical(rows.level, rows.A, ob.K, ob.pitch, rows.agents, rows.items, rows.t)
    sout = ob.new_state()
    flags, lb = ob.rollout(sin, sout, rows.actions(ob.pitch), rows.subtasks, rows.alloc)
    errs = rows.compare(sout, flags, lb, ob.pitch)
    assert not errs, "\n".join(errs[:20])


def test_value_init_arithmetic(fx):
    """v_l / v_u of the reference rows follow from lb exactly (e2e_brtdp.py:716-729)."""
    ok = (fx["assert_"] == 0) & (fx["goal"] == 0)
    lower = fx["lb"][ok] * (1.0 + 0.1)
    assert np.array_equal(fx["v_l"][ok], lower - 1.09)
    assert np.array_equal(fx["v_u"][ok], lower * 5 * (1.0 + 0.1))
    g = (fx["assert_"] == 0) & (fx["goal"] == 1)
    assert np.all(fx["v_l"][g] == 0) and np.all(fx["v_u"][g] == 0)
