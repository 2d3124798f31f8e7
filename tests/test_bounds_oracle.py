"""The CPU oracle's full-state subtask bounds (oracle/oc_oracle.c, oco_subtask_bounds) against
the reference's get_lower_bound_for_subtask_given_objs and BayesianDelegator.subtask_alloc_is_doable
recorded on full environment states (tests/golden/bounds.npz, gen_bounds.py), bit-exact."""
import numpy as np
import pytest

import oc_testlib as tl

from oracle import oracle


@pytest.fixture(scope="module")
def fx():
    return tl.load_fixture("bounds.npz")


@pytest.mark.parametrize("cfg", range(5))
def test_oracle_bounds_match_reference_rows(fx, cfg):
    rows = tl.BoundRows(fx, cfg)
    ob = oracle.OracleBatch(rows.level, rows.A, 100, rows.B)
    lb, doable = ob.subtask_bounds(rows.state(ob.pitch), rows.subtasks)
    errs = rows.compare(lb, doable)
    assert not errs, "\n".join(errs[:20])
    assert len(rows.idx) == int(np.isin(fx["state"], np.nonzero(fx["st_cfg"] == cfg)[0]).sum())


def test_fixture_covers_every_kind(fx):
    for k in range(4):
        assert (fx["kind"] == k).any()
    assert fx["doable"].any() and not fx["doable"].all()
    assert (fx["doable"][fx["kind"] == 0] == 1).all()  # None is always doable (bayesian_delegator.py:127-128)
