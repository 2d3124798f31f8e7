"""Kitchens of more than 8 objects on the GPU, through the C-ABI: the 16
item-slot kernels (include/oc_engine.h OC_MAX_ITEMS; fixtures from
tests/golden/gen_manylevels.py, which runs the reference on the same level files):
  * oc_step replays the 72 recorded reference episodes bit for bit (9, 11 and 16 objects,
    presence and counts encodings, 110-156 cells);
  * oc_step_n against the CPU oracle on every step's state, executed actions and collisions;
  * oc_rollout / oc_subtask_bounds against the reference planner's rows, and oc_rollout,
    oc_subtask_bounds and oc_nav_likelihood against the oracle on random rows;
  * oc_render against the numpy restatement."""
import numpy as np
import pytest

import oc_testlib as tl
import test_manylevels as tm
from gym_cooking_amd import capi, levels

from oracle import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _batch(level, A, B, max_T=100):
    from gym_cooking_amd.engine import OvercookedBatch
    return OvercookedBatch(level, A, B, max_T=max_T, device="cuda:0")


def test_engine_replays_many_level_episodes():
    import test_gpu_parity as tg
    fx = tl.load_fixture("manylevels.npz")
    n = 0
    for g in tl.episode_groups(fx):
        eb = _batch(g.level, g.A, g.B, g.max_T)
        assert eb.K == 16
        s = eb.new_state()
        eb.reset(s)
        host = s.cpu().numpy()
        g.relocate(host, eb.pitch)
        errs = tl.compare_group(g, tg._gpu_step_fn(eb), host, eb.pitch, g.level.width)
        assert not errs, "%s A=%d: %s" % (g.level.name, g.A, "\n".join(errs[:10]))
        n += g.B
    assert n == 72


@pytest.mark.parametrize("name", tm.MANY)
@pytest.mark.parametrize("A", [2, 4])
def test_many_level_step_n_matches_oracle(name, A):
    """Two 30-step oc_step_n launches over 12,000 envs (max_T 25), every step's outputs."""
    B, n, max_T, seed = 12000, 30, 25, 57 + A
    lv = levels.load_level(tm._path(name))
    eb = _batch(lv, A, B, max_T)
    ob = oracle.OracleBatch(lv, A, max_T, B)
    P, S = eb.pitch, eb.layout.state_bytes
    s_in, s_out = eb.new_state(), eb.new_state()
    eb.reset(s_in)
    c, c2 = ob.new_state(), ob.new_state()
    ob.reset(c)
    ca, cex, ccoll = ob.new_actions(), np.zeros(A * P, np.uint8), np.zeros(P, np.uint8)
    acts = torch.empty((n, A * P), dtype=torch.uint8, device="cuda:0")
    traj = torch.empty(n * S, dtype=torch.uint8, device="cuda:0")
    ex = torch.empty(n * A * P, dtype=torch.uint8, device="cuda:0")
    coll = torch.empty(n * P, dtype=torch.uint8, device="cuda:0")
    stats, totals = eb.new_stats(), torch.zeros(5, dtype=torch.int64, device="cuda:0")
    tot = np.zeros(5, np.int64)
    for launch in range(2):
        for r in range(n):
            eb.gen_actions(acts[r], launch * n + r, seed)
        eb.step_n(s_in, s_out, acts.reshape(-1), n, traj, ex, coll, stats, totals)
        tr, exh, colh = traj.view(n, S).cpu().numpy(), ex.view(n, A, P).cpu().numpy(), coll.view(n, P).cpu().numpy()
        for r in range(n):
            ob.gen_actions(ca, 0, launch * n + r, seed)
            fl_in = tl.planes_view(c, A, ob.K, P)["fl"].copy()
            ob.step(c, c2, ca, cex, ccoll, nthreads=16)
            c, c2 = c2, c
            tot += tl.window_totals(fl_in, c, ccoll, A, ob.K, P, B)
            g, o = tl.env_view(tr[r], A, ob.K, P, B), tl.env_view(c, A, ob.K, P, B)
            assert np.array_equal(g, o), (launch, r, np.argwhere(g != o)[:5].tolist())
            assert np.array_equal(exh[r][:, :B], cex.reshape(A, P)[:, :B]), (launch, r)
            assert np.array_equal(colh[r][:B], ccoll[:B]), (launch, r)
        s_in, s_out = s_out, s_in
    assert np.array_equal(totals.cpu().numpy(), tot)


@pytest.mark.parametrize("cfg", range(3))
def test_many_level_bounds_match_reference_rows(cfg):
    rows = tl.BoundRows(tl.load_fixture("bounds_many.npz"), cfg)
    P = capi.pitch_for(rows.B)
    s = rows.state(P)
    eb = _batch(rows.level, rows.A, rows.B)
    for c0 in range(0, len(rows.subtasks), capi.MAX_SUBTASKS):
        subs = rows.subtasks[c0:c0 + capi.MAX_SUBTASKS]
        lb, ok = eb.subtask_bounds(torch.from_numpy(s).cuda(), subs)
        errs = rows.compare(lb[:, :rows.B].cpu().numpy(), ok[:, :rows.B].cpu().numpy(), sub0=c0)
        assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("cfg", range(2))
def test_many_level_rollout_matches_reference_rows(cfg):
    fx = tl.load_fixture("rollout_many.npz")
    n = 0
    for rows in tl.RolloutRows(fx, cfg).split(capi.MAX_SUBTASKS):
        P = capi.pitch_for(rows.B)
        sin = tl.state_from_canonical(rows.level, rows.A, rows.K, P, rows.agents, rows.items, rows.t)
        alloc = np.zeros(P, np.uint8)
        alloc[:rows.B] = rows.alloc
        eb = _batch(rows.level, rows.A, rows.B)
        sout = eb.new_state()
        fl, lb = eb.rollout(torch.from_numpy(sin).cuda(), sout, torch.from_numpy(rows.actions(P)).cuda(),
                            rows.subtasks, torch.from_numpy(alloc).cuda())
        errs = rows.compare(sout.cpu().numpy(), fl[:rows.B].cpu().numpy(), lb[:rows.B].cpu().numpy(), P)
        assert not errs, "\n".join(errs[:20])
        n += rows.B
    assert n == int((fx["cfg"] == cfg).sum())


@pytest.mark.parametrize("name", tm.MANY)
@pytest.mark.parametrize("A", [2, 4])
def test_many_level_rollout_bounds_likelihood_match_oracle(name, A):
    B = 6000
    ob, s, acts, subs, alloc = tm.many_rollout_case(name, A, B, seed=B + 3 * A + len(name))
    eb = _batch(ob.level, A, B)
    gs, ga, gal = torch.from_numpy(s).cuda(), torch.from_numpy(acts).cuda(), torch.from_numpy(alloc).cuda()
    o_out = ob.new_state()
    o_fl, o_lb = ob.rollout(s, o_out, acts, subs, alloc, nthreads=16)
    g_out = eb.new_state()
    g_fl, g_lb = eb.rollout(gs, g_out, ga, subs, gal)
    assert np.array_equal(o_fl, g_fl[:B].cpu().numpy())
    assert np.array_equal(o_lb, g_lb[:B].cpu().numpy())
    assert np.array_equal(tl.env_view(o_out, A, ob.K, ob.pitch, B),
                          tl.env_view(g_out.cpu().numpy(), A, ob.K, ob.pitch, B))
    subs0 = [capi.subtask(x.kind, list(x.agent[:x.num_agents]), list(x.start_mask), x.goal_mask, x.goal_count, 0)
             for x in subs]
    o_b, o_ok = ob.subtask_bounds(s, subs0)
    g_b, g_ok = eb.subtask_bounds(gs, subs0)
    assert np.array_equal(o_b[:, :B], g_b[:, :B].cpu().numpy()) and np.array_equal(o_ok[:, :B], g_ok[:, :B].cpu().numpy())
    o_v, o_f = ob.nav_likelihood(s, acts, subs0, alloc, 0, 1.3, 0.5, nthreads=16)
    g_v, g_f = eb.nav_likelihood(gs, ga, subs0, 0, 1.3, 0.5, gal)
    g_v, g_f = g_v[:B].cpu().numpy(), g_f[:B].cpu().numpy()
    assert np.array_equal(o_f, g_f)
    ok = o_f == capi.LIK_OK
    assert ok.sum() > 50
    np.testing.assert_allclose(g_v[ok], o_v[ok], rtol=1e-12)


@pytest.mark.parametrize("name", ["many-11x10_salad9", "many-13x12_full16"])
def test_render_many_level_matches_restatement(name):
    from gym_cooking_amd import render
    from oracle import render_oracle
    lv = levels.load_level(tm._path(name))
    A, B = 3, 48
    eb = _batch(lv, A, B)
    s, s2 = eb.new_state(), eb.new_state()
    eb.reset(s)
    a = eb.new_actions()
    for t in range(27):
        eb.gen_actions(a, t, 8)
        eb.step(s, s2, a)
        s, s2 = s2, s
    img = render.Renderer(eb).render(s, channels="rgb").cpu().numpy()
    ev = tl.env_view(s.cpu().numpy(), A, eb.K, eb.pitch, B)
    checked = 0
    for b in range(B):
        try:
            ref = render_oracle.render_env(lv, ev[:, b], A, eb.K, channels="rgb")
        except KeyError:  # an object of two of one food: the reference raises drawing it
            continue
        assert np.array_equal(img[b], ref), b
        checked += 1
    assert checked > B // 2
