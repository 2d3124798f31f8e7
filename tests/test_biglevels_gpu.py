"""User levels outside the shipped 7x7 kitchens on the GPU, through the C-ABI (120-, 169- and
255-cell grids from tests/golden/levels/, ragged maps):
  * the engine replays the 54 episodes recorded from the reference on those levels, and the 21
    on a 9x9 kitchen of 6 items (the 8-slot layout), bit for bit (tests/golden/biglevels*.npz),
    one oc_step launch per step;
  * oc_step_n (multi-step launches) against the CPU oracle on every step's full state;
  * oc_subtask_bounds against the reference's bound rows (bounds_big.npz, bounds_bignodes.npz:
    the 255-cell kitchen's 266-node graph), oc_rollout and
    oc_nav_likelihood against the oracle on random rows;
  * the gym shim replays recorded episodes, raises the reference's exceptions on ragged maps,
    and steps the 255-cell kitchen, whose 266-node reachability graph the planner tables hold
    with u16 node ids;
  * oc_render against the numpy restatement on the 169-cell kitchen."""
import json
import os
import types

import numpy as np
import pytest

import oc_testlib as tl
import test_rollout_host as th
from gym_cooking_amd import capi, levels

from oracle import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

BIG = ["big-10x12_salad", "big-13x13_tl", "big-15x17_salad"]
K8 = "onion-9x9_onionsalad"  # 6 items: the engine's 8 item slots


def _path(name):
    return os.path.join(tl.GOLDEN, "levels", name + ".txt")


def _batch(level, A, B, max_T=100):
    from gym_cooking_amd.engine import OvercookedBatch
    return OvercookedBatch(level, A, B, max_T=max_T, device="cuda:0")


@pytest.mark.parametrize("fixture,n_eps", [("biglevels.npz", 54), ("biglevels_k8.npz", 21)])
def test_engine_replays_big_level_episodes(fixture, n_eps):
    import test_gpu_parity as tg
    fx = tl.load_fixture(fixture)
    n = 0
    for g in tl.episode_groups(fx):
        eb = _batch(g.level, g.A, g.B, g.max_T)
        s = eb.new_state()
        eb.reset(s)
        host = s.cpu().numpy()
        g.relocate(host, eb.pitch)
        errs = tl.compare_group(g, tg._gpu_step_fn(eb), host, eb.pitch, g.level.width)
        assert not errs, "%s A=%d: %s" % (g.level.name, g.A, "\n".join(errs[:10]))
        n += g.B
    assert n == n_eps


@pytest.mark.parametrize("name", BIG + [K8])
@pytest.mark.parametrize("A", [2, 4])
def test_big_level_step_n_matches_oracle(name, A):
    """Two 30-step oc_step_n launches over 20,000 envs (max_T 25: auto-resets inside launches),
    every step's state, executed actions and collision mask against the oracle."""
    B, n, max_T, seed = 20000, 30, 25, 9 + A
    lv = levels.load_level(_path(name))
    eb = _batch(lv, A, B, max_T)
    ob = oracle.OracleBatch(lv, A, max_T, B)
    P, S = eb.pitch, eb.layout.state_bytes
    s_in, s_out = eb.new_state(), eb.new_state()
    eb.reset(s_in)
    c = ob.new_state()
    ob.reset(c)
    c2 = ob.new_state()
    ca = ob.new_actions()
    cex = np.zeros(A * P, np.uint8)
    ccoll = np.zeros(P, np.uint8)
    acts = torch.empty((n, A * P), dtype=torch.uint8, device="cuda:0")
    traj = torch.empty(n * S, dtype=torch.uint8, device="cuda:0")
    ex = torch.empty(n * A * P, dtype=torch.uint8, device="cuda:0")
    coll = torch.empty(n * P, dtype=torch.uint8, device="cuda:0")
    for launch in range(2):
        for r in range(n):
            eb.gen_actions(acts[r], launch * n + r, seed)
        eb.step_n(s_in, s_out, acts.reshape(-1), n, traj, ex, coll)
        tr = traj.view(n, S).cpu().numpy()
        exh = ex.view(n, A, P).cpu().numpy()
        colh = coll.view(n, P).cpu().numpy()
        for r in range(n):
            ob.gen_actions(ca, 0, launch * n + r, seed)
            ob.step(c, c2, ca, cex, ccoll, nthreads=16)
            c, c2 = c2, c
            g, o = tl.env_view(tr[r], A, ob.K, P, B), tl.env_view(c, A, ob.K, P, B)
            assert np.array_equal(g, o), (launch, r, np.argwhere(g != o)[:5].tolist())
            assert np.array_equal(exh[r][:, :B], cex.reshape(A, P)[:, :B]), (launch, r)
            assert np.array_equal(colh[r][:B], ccoll[:B]), (launch, r)
        s_in, s_out = s_out, s_in


@pytest.mark.parametrize("fixture,cfg", [("bounds_big.npz", 0), ("bounds_big.npz", 1), ("bounds_big.npz", 2),
                                         ("bounds_k8.npz", 0), ("bounds_bignodes.npz", 0),
                                         ("bounds_bignodes.npz", 1)])
def test_big_level_bounds_match_reference_rows(fixture, cfg):
    rows = tl.BoundRows(tl.load_fixture(fixture), cfg)
    P = capi.pitch_for(rows.B)
    s = rows.state(P)
    eb = _batch(rows.level, rows.A, rows.B)
    for c0 in range(0, len(rows.subtasks), capi.MAX_SUBTASKS):
        subs = rows.subtasks[c0:c0 + capi.MAX_SUBTASKS]
        lb, ok = eb.subtask_bounds(torch.from_numpy(s).cuda(), subs)
        errs = rows.compare(lb[:, :rows.B].cpu().numpy(), ok[:, :rows.B].cpu().numpy(), sub0=c0)
        assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("name", ["big-10x12_salad", "big-13x13_tl", "big-15x17_salad", K8])
@pytest.mark.parametrize("A", [2, 4])
def test_big_level_rollout_and_likelihood_match_oracle(name, A):
    B = 6000
    ob, s, acts, subs, alloc = th.random_rollout_case(_path(name), A, B, seed=B + A, planner_levels=(0, 1))
    eb = _batch(ob.level, A, B)
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
    o_v, o_f = ob.nav_likelihood(s, acts, subs0, alloc, 0, 1.3, 0.5, nthreads=16)
    g_v, g_f = eb.nav_likelihood(torch.from_numpy(s).cuda(), torch.from_numpy(acts).cuda(), subs0, 0, 1.3, 0.5,
                                 torch.from_numpy(alloc).cuda())
    g_v, g_f = g_v[:B].cpu().numpy(), g_f[:B].cpu().numpy()
    assert np.array_equal(o_f, g_f)
    ok = o_f == capi.LIK_OK
    assert ok.sum() > 50
    np.testing.assert_allclose(g_v[ok], o_v[ok], rtol=1e-12)


def test_planner_tables_of_a_266_node_graph():
    """The 255-cell kitchen's graph (266 nodes: u16 node ids, a 75 KB table blob staged in
    dynamic LDS past the default 64 KB) against the reference's graph (reach_big.json)."""
    eb = _batch(levels.load_level(_path("big-15x17_salad")), 2, 64)
    node_of, dist = eb.reachability()
    ref = json.load(open(os.path.join(tl.GOLDEN, "reach_big.json")))["big-15x17_salad"]
    assert dist.shape == (len(ref["nodes"]),) * 2 == (266, 266)
    assert int((node_of != 0xFFFF).sum()) == 266 and int(node_of[node_of != 0xFFFF].max()) == 265
    assert int((dist == 1).sum()) == 2 * len(ref["edges"])


def _shim(level, A, max_T=100):
    from gym_cooking_amd.envs import OvercookedEnvironment
    arg = types.SimpleNamespace(level=level, num_agents=A, max_num_timesteps=max_T, seed=1, model1=None,
                                model2=None, model3=None, model4=None, record=False, with_image_obs=False)
    return OvercookedEnvironment(arg)


def test_shim_replays_big_level_episodes():
    fx = tl.load_fixture("biglevels.npz")
    n_steps = 0
    for e in range(0, len(fx["ep_T"]), 5):
        lvname = os.path.join(tl.GOLDEN, str(fx["level_names"][fx["ep_level"][e]]))
        A = int(fx["ep_A"][e])
        env = _shim(lvname, A, int(fx["ep_maxT"][e]))
        env.reset()
        K = capi.item_slots(env.level)
        off, aoff = fx["ep_state_off"][e], fx["ep_act_off"][e]
        for step in range(int(fx["ep_T"][e])):
            codes = fx["act"][aoff + step][:A]
            ad = {"agent-%d" % (a + 1): levels.ACTIONS[min(int(codes[a]), 4)] for a in range(A)}
            if fx["flags"][off + step + 1] & 0x04:
                with pytest.raises(AttributeError):
                    env.step(ad)
                break
            obs, reward, done, info = env.step(ad)
            n_steps += 1
            c = tl.canonical(np.asarray(env.state_bytes(), np.uint8), A, K, 1, env.level.width, 1)
            assert np.array_equal(c["agents"][0], fx["agents"][off + step + 1]), (e, step)
            assert np.array_equal(c["items"][0], fx["items"][off + step + 1]), (e, step)
            assert done == bool(fx["flags"][off + step + 1] & 1)
    assert n_steps > 200


def test_shim_ragged_maps_raise_like_the_reference():
    with open(os.path.join(tl.GOLDEN, "biglevels.json")) as f:
        info = json.load(f)
    env = _shim(_path("ragged-short_salad"), 2)
    with pytest.raises(KeyError) as ei:
        env.reset()
    assert list(ei.value.args[0]) == info["ragged-short_salad"]["arg"]
    probe = info["ragged-long_salad"]["step_probe"]
    env = _shim(_path("ragged-long_salad"), 2)
    env.reset()
    assert [list(a.location) for a in env.sim_agents] == probe["before"]
    with pytest.raises(IndexError):
        env.step({"agent-1": tuple(probe["actions"][0]), "agent-2": tuple(probe["actions"][1])})
    assert env.t == probe["t"]
    assert [list(a.location) for a in env.sim_agents] == probe["after"]


def test_shim_steps_the_255_cell_kitchen():
    env = _shim(_path("big-15x17_salad"), 4)
    env.reset()
    assert len(env.world.reachability_graph) == 266  # u16 node ids
    for t in range(5):
        env.step({"agent-%d" % (a + 1): levels.ACTIONS[(t + a) % 5] for a in range(4)})
    assert env.t == 5


def test_render_big_level_matches_restatement():
    from gym_cooking_amd import render
    from oracle import render_oracle
    lv = levels.load_level(_path("big-13x13_tl"))
    A, B = 3, 40
    eb = _batch(lv, A, B)
    s, s2 = eb.new_state(), eb.new_state()
    eb.reset(s)
    a = eb.new_actions()
    for t in range(23):
        eb.gen_actions(a, t, 5)
        eb.step(s, s2, a)
        s, s2 = s2, s
    rd = render.Renderer(eb)
    img = rd.render(s, channels="rgb").cpu().numpy()
    assert img.shape[1:] == (13 * 80, 13 * 80, 3)
    ev = tl.env_view(s.cpu().numpy(), A, eb.K, eb.pitch, B)
    for b in range(0, B, 3):
        assert np.array_equal(img[b], render_oracle.render_env(lv, ev[:, b], A, eb.K, channels="rgb")), b
