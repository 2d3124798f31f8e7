"""The CPU oracle's Bayesian-delegation likelihood (oco_nav_likelihood) against
prob_nav_actions values recorded from the reference (tests/golden/likelihood.npz,
gen_likelihood.py): float64, relative tolerance 1e-12 (numpy's summation order)."""
import numpy as np
import pytest

import oc_testlib as tl
from gym_cooking_amd import capi

from oracle import oracle

RTOL = 1e-12


@pytest.fixture(scope="module")
def fx():
    return tl.load_fixture("likelihood.npz")


@pytest.mark.parametrize("cfg", range(4))
@pytest.mark.parametrize("self_agent", [0, 1])
def test_oracle_likelihood_matches_reference(fx, cfg, self_agent):
    rows = tl.LikelihoodRows(fx, cfg, self_agent)
    assert rows.B > 0
    for sel, alloc, subs in rows.chunks(capi.MAX_SUBTASKS):
        ob = oracle.OracleBatch(rows.level, rows.A, 100, len(sel))
        s, taken = rows.inputs(sel, ob.pitch)
        a = np.zeros(ob.pitch, np.uint8)
        a[:len(sel)] = alloc
        v, f = ob.nav_likelihood(s, taken, subs, a, self_agent, rows.beta, rows.nap)
        errs = rows.compare(sel, v, f, RTOL)
        assert not errs, "\n".join(errs[:20])
