"""GPU parity of the Bayesian-delegation likelihood (oc_nav_likelihood through the C-ABI):
the prob_nav_actions values recorded from the reference (float64, rtol 1e-12), and random
states x random planner tables against the CPU oracle, including the C5 shape."""
import numpy as np
import pytest

import oc_testlib as tl
from gym_cooking_amd import capi

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _gpu_lik(level, A, B, s, taken, subs, alloc, self_agent, beta, nap, form=None):
    from gym_cooking_amd.engine import OvercookedBatch
    eb = OvercookedBatch(level, A, B, max_T=100, device="cuda:0")
    if form is not None:
        eb.set_likelihood_form(form)
    a = torch.from_numpy(alloc).cuda() if alloc is not None else None
    v, f = eb.nav_likelihood(torch.from_numpy(s).cuda(), torch.from_numpy(taken).cuda(), subs, self_agent, beta, nap, a)
    torch.cuda.synchronize()
    return v[:B].cpu().numpy(), f[:B].cpu().numpy()


@pytest.mark.parametrize("cfg", range(4))
@pytest.mark.parametrize("self_agent", [0, 1])
def test_likelihood_matches_reference(cfg, self_agent):
    fx = tl.load_fixture("likelihood.npz")
    rows = tl.LikelihoodRows(fx, cfg, self_agent)
    for sel, alloc, subs in rows.chunks(capi.MAX_SUBTASKS):
        P = capi.pitch_for(len(sel))
        s, taken = rows.inputs(sel, P)
        a = np.zeros(P, np.uint8)
        a[:len(sel)] = alloc
        v, f = _gpu_lik(rows.level, rows.A, len(sel), s, taken, subs, a, self_agent, rows.beta, rows.nap)
        errs = rows.compare(sel, v, f, 1e-12)
        assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("level,A,B", [("open-divider_salad", 2, 3000), ("full-divider_salad", 4, 1 << 16)])
def test_likelihood_matches_oracle_random(level, A, B):
    import test_rollout_host as th
    ob, s, acts, subs, alloc = th.random_rollout_case(level, A, B, seed=B % 97)
    for self_agent in range(2):
        o_v, o_f = ob.nav_likelihood(s, acts, subs, alloc, self_agent, 1.3, 0.5, nthreads=16)
        g_v, g_f = _gpu_lik(level, A, B, s, acts, subs, alloc, self_agent, 1.3, 0.5)
        assert np.array_equal(o_f, g_f), np.argwhere(o_f != g_f)[:5]
        ok = o_f == capi.LIK_OK
        assert ok.sum() > 100
        np.testing.assert_allclose(g_v[ok], o_v[ok], rtol=1e-12)
        assert np.all(g_v[~ok] == 0)


@pytest.mark.parametrize("level,A,B", [("partial-divider_salad", 2, 4000), ("full-divider_salad", 4, 20000)])
def test_likelihood_one_agent_tables_match_oracle(level, A, B):
    """Tables of one-agent configurations only take the kernel's 8-lane groups (two-agent
    tables its 32-lane groups, the tests above)."""
    import test_rollout_host as th
    ob, s, acts, subs, alloc = th.random_rollout_case(level, A, B, seed=B % 89 + 3)
    subs = [capi.subtask(x.kind, [x.agent[0]], list(x.start_mask), x.goal_mask, x.goal_count) for x in subs]
    for self_agent in range(2):
        o_v, o_f = ob.nav_likelihood(s, acts, subs, alloc, self_agent, 1.3, 0.5, nthreads=16)
        g_v, g_f = _gpu_lik(level, A, B, s, acts, subs, alloc, self_agent, 1.3, 0.5)
        assert np.array_equal(o_f, g_f), np.argwhere(o_f != g_f)[:5]
        ok = o_f == capi.LIK_OK
        assert ok.sum() > 100
        np.testing.assert_allclose(g_v[ok], o_v[ok], rtol=1e-12)


def _lik_case(kind):
    """A seeded full-divider_salad case: the two-agent table (32-lane groups) or its one-agent
    configurations (8-lane groups)."""
    import test_rollout_host as th
    ob, s, acts, subs, alloc = th.random_rollout_case("full-divider_salad", 4, 9000, seed=41)
    if kind == "single":
        subs = [capi.subtask(x.kind, [x.agent[0]], list(x.start_mask), x.goal_mask, x.goal_count) for x in subs]
    return s, acts, subs, alloc


@pytest.mark.parametrize("kind", ["joint", "single"])
def test_grouped_form_equals_compacted(kind):
    """The product runs the compacted likelihood kernel; the grouped one remains for levels whose
    tables leave too little LDS (oc_engine.hip, oc_nav_likelihood).  oc_set_likelihood_form
    (OC_LIK_FORM_GROUPED) forces the grouped form on a handle: the same rows with it, bit for bit
    (that the switch selects the grouped kernels: profiles/r04/lik_compact/
    lik_kernel_stats_grouped_env.csv, measured with the round-4 switch)."""
    s, acts, subs, alloc = _lik_case(kind)
    g = _gpu_lik("full-divider_salad", 4, 9000, s, acts, subs, alloc, 1, 1.3, 0.5, form=capi.OC_LIK_FORM_GROUPED)
    v, f = _gpu_lik("full-divider_salad", 4, 9000, s, acts, subs, alloc, 1, 1.3, 0.5)
    assert (f == capi.LIK_OK).sum() > 100
    assert np.array_equal(f, g[1])
    assert np.array_equal(v.view(np.uint64), g[0].view(np.uint64))
