"""The kitchens of tests/test_widegraph.py (more than 360 graph nodes: the 605-node wide
kitchen and the 417-node narrow one) on the GPU, through the C-ABI: their planner kernels (the
GD instantiation) stage the level's tables in LDS and read the distance table from device
memory.  oc_step replays the reference's episodes; oc_subtask_bounds and oc_rollout against
the reference's rows; rollout, bounds and likelihood rows against the oracle on random states;
the navigation planner over oc_rollout decides as the same search over the oracle's rows."""
import numpy as np
import pytest

import oc_testlib as tl
import test_rollout_host as th
import test_widegraph as twg
import test_widelevels as tw
import test_widelevels_gpu as twgpu
from gym_cooking_amd import capi, levels

from oracle import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


KIT = twg.KIT


@KIT
def test_engine_replays_widegraph_episodes(name):
    import test_gpu_parity as tg
    fx = twg._fx(name)
    n = 0
    for g in tl.episode_groups(fx):
        eb = twgpu._batch(g.level, g.A, g.B, g.max_T)
        s = eb.new_state()
        eb.reset(s)
        host = s.cpu().numpy()
        g.relocate(host, eb.pitch)
        errs = tl.compare_group(g, tg._gpu_step_fn(eb), host, eb.pitch, g.level.width)
        assert not errs, "%s A=%d: %s" % (g.level.name, g.A, "\n".join(errs[:10]))
        n += g.B
    assert n == len(fx["ep_T"])


@KIT
def test_widegraph_bounds_match_reference_rows(name):
    rows = tl.BoundRows(twg._fx(name, "bounds_"), 0)
    P = capi.pitch_for(rows.B)
    s = rows.state(P)
    eb = twgpu._batch(rows.level, rows.A, rows.B)
    for c0 in range(0, len(rows.subtasks), capi.MAX_SUBTASKS):
        subs = rows.subtasks[c0:c0 + capi.MAX_SUBTASKS]
        lb, ok = eb.subtask_bounds(torch.from_numpy(s).cuda(), subs)
        errs = rows.compare(lb[:, :rows.B].cpu().numpy(), ok[:, :rows.B].cpu().numpy(), sub0=c0)
        assert not errs, "\n".join(errs[:20])


@KIT
def test_widegraph_rollout_matches_reference_rows(name):
    fx = twg._fx(name, "rollout_")
    n = 0
    for rows in tl.RolloutRows(fx, 0).split(capi.MAX_SUBTASKS):
        P = capi.pitch_for(rows.B)
        sin = tl.state_from_canonical(rows.level, rows.A, rows.K, P, rows.agents, rows.items, rows.t)
        alloc = np.zeros(P, np.uint8)
        alloc[:rows.B] = rows.alloc
        eb = twgpu._batch(rows.level, rows.A, rows.B)
        sout = eb.new_state()
        fl, lb = eb.rollout(torch.from_numpy(sin).cuda(), sout, torch.from_numpy(rows.actions(P)).cuda(),
                            rows.subtasks, torch.from_numpy(alloc).cuda())
        errs = rows.compare(sout.cpu().numpy(), fl[:rows.B].cpu().numpy(), lb[:rows.B].cpu().numpy(), P)
        assert not errs, "\n".join(errs[:20])
        n += rows.B
    assert n == len(fx["cfg"])


@KIT
@pytest.mark.parametrize("A", [2, 4])
def test_widegraph_rows_match_oracle_random(name, A):
    B = 6000
    ob, s, acts, subs, alloc = th.random_rollout_case(tw._path(name), A, B, seed=B + A, planner_levels=(0, 1))
    eb = twgpu._batch(ob.level, A, B)
    o_out = ob.new_state()
    o_fl, o_lb = ob.rollout(s, o_out, acts, subs, alloc, nthreads=16)
    g_out = eb.new_state()
    g_fl, g_lb = eb.rollout(torch.from_numpy(s).cuda(), g_out, torch.from_numpy(acts).cuda(), subs,
                            torch.from_numpy(alloc).cuda())
    assert np.array_equal(o_fl, g_fl[:B].cpu().numpy())
    assert np.array_equal(o_lb, g_lb[:B].cpu().numpy())
    assert np.array_equal(tl.env_view(o_out, A, ob.K, ob.pitch, B),
                          tl.env_view(g_out.cpu().numpy(), A, ob.K, ob.pitch, B))
    subs0 = [capi.subtask(x.kind, list(x.agent[:x.num_agents]), list(x.start_mask), x.goal_mask, x.goal_count, 0)
             for x in subs]
    o_b, o_ok = ob.subtask_bounds(s, subs0, nthreads=16)
    g_b, g_ok = eb.subtask_bounds(torch.from_numpy(s).cuda(), subs0)
    assert np.array_equal(o_b, g_b[:, :B].cpu().numpy()) and np.array_equal(o_ok, g_ok[:, :B].cpu().numpy())
    o_v, o_f = ob.nav_likelihood(s, acts, subs0, alloc, 0, 1.3, 0.5, nthreads=16)
    g_v, g_f = eb.nav_likelihood(torch.from_numpy(s).cuda(), torch.from_numpy(acts).cuda(), subs0, 0, 1.3, 0.5,
                                 torch.from_numpy(alloc).cuda())
    g_v, g_f = g_v[:B].cpu().numpy(), g_f[:B].cpu().numpy()
    assert np.array_equal(o_f, g_f)
    ok = o_f == capi.LIK_OK
    assert ok.sum() > 50
    np.testing.assert_allclose(g_v[ok], o_v[ok], rtol=1e-12)


@KIT
@pytest.mark.parametrize("A,sub,agents", [(2, ("Chop", "Tomato"), ("agent-1",)),
                                          (3, ("Chop", "Lettuce"), ("agent-1", "agent-3"))])
def test_widegraph_planner_matches_host_search(name, A, sub, agents):
    """get_next_action over oc_rollout equals the same search over the CPU oracle's rows
    (which test_widegraph.py pins to the reference's rows on this kitchen)."""
    import test_planner_host as tp
    from gym_cooking_amd import recipes
    from gym_cooking_amd.planner import E2E_BRTDP, PlanEnv
    lv = levels.load_level(tw._path(name))
    ob = oracle.OracleBatch(lv, A, 0, 1)
    s, s2 = ob.new_state(), ob.new_state()
    ob.reset(s)
    act = ob.new_actions()
    for t in range(9):
        ob.gen_actions(act, 0, t, 5)
        ob.step(s, s2, act)
        s, s2 = s2, s
    view = tl.env_view(s, A, ob.K, ob.pitch, 1)[:, 0]
    out = []
    for exp in (None, tp.OracleExpander):
        env = PlanEnv(lv, A, view, ["Tomato", "Lettuce", "Plate"], device="cuda:0")
        kw = {} if exp is None else {"expander": exp}
        p = E2E_BRTDP(alpha=0.01, tau=2, cap=75, main_cap=100, device="cuda:0", rng=np.random.RandomState(3), **kw)
        a = p.get_next_action(env, getattr(recipes, sub[0])(sub[1]), agents, {})
        out.append((a, p.cur_obj_count, len(p.v_l), p.v_l[(p._repr(p.start), p._sub_key)]))
    assert out[0] == out[1], out
