"""GPU parity of the planner rollout (oc_rollout through the C-ABI): the rows recorded from
the reference planner, random states x random planner tables against the CPU oracle, the C5
shape (full-divider_salad, 4 agents, 2^18 rows), and rows with bad allocation ids."""
import numpy as np
import pytest

import oc_testlib as tl  # noqa: F401
from gym_cooking_amd import capi

from oracle import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _gpu_rollout(level, A, B, sin_host, acts_host, subs, alloc_host):
    from gym_cooking_amd.engine import OvercookedBatch
    eb = OvercookedBatch(level, A, B, max_T=100, device="cuda:0")
    sin = torch.from_numpy(sin_host).cuda()
    sout = eb.new_state()
    acts = torch.from_numpy(acts_host).cuda()
    alloc = torch.from_numpy(alloc_host).cuda() if alloc_host is not None else None
    fl, lb = eb.rollout(sin, sout, acts, subs, alloc)
    torch.cuda.synchronize()
    return sout.cpu().numpy(), fl[:B].cpu().numpy(), lb[:B].cpu().numpy()


@pytest.mark.parametrize("name,level", [("rollout.npz", 0), ("rollout_level1.npz", 1)])
@pytest.mark.parametrize("cfg", range(5))
def test_rollout_matches_reference_rows(name, level, cfg):
    fx = tl.load_fixture(name)
    n = 0
    for rows in tl.RolloutRows(fx, cfg, planner_level=level).split(capi.MAX_SUBTASKS):
        P = capi.pitch_for(rows.B)
        sin = tl.state_from_canonical(rows.level, rows.A, rows.K, P, rows.agents, rows.items, rows.t)
        alloc = np.zeros(P, np.uint8)
        alloc[:rows.B] = rows.alloc
        sout, fl, lb = _gpu_rollout(rows.level, rows.A, rows.B, sin, rows.actions(P), rows.subtasks, alloc)
        errs = rows.compare(sout, fl, lb, P)
        assert not errs, "\n".join(errs[:20])
        n += rows.B
    assert n == int((fx["cfg"] == cfg).sum())


def _random_case(level, A, B, seed):
    import test_rollout_host as th
    return th.random_rollout_case(level, A, B, seed, planner_levels=(0, 1))


# Launches of up to CUs x 256 / 4 rows (16,384 on MI355X) run a lane quad per row
# (oc_rollout_group_kernel), larger ones a row per lane: both sides of that boundary are here.
@pytest.mark.parametrize("level,A,B", [("open-divider_salad", 2, 5000), ("partial-divider_tl", 3, 4099),
                                       ("full-divider_salad", 4, 1 << 18), ("open-divider_tomato", 1, 17),
                                       ("partial-divider_tl", 3, 16384), ("open-divider_salad", 2, 16385)])
def test_rollout_matches_oracle_random(level, A, B):
    ob, s, acts, subs, alloc = _random_case(level, A, B, seed=B + A)
    o_out = ob.new_state()
    o_fl, o_lb = ob.rollout(s, o_out, acts, subs, alloc, nthreads=16)
    g_out, g_fl, g_lb = _gpu_rollout(ob.level, A, B, s, acts, subs, alloc)
    assert np.array_equal(o_fl, g_fl), np.argwhere(o_fl != g_fl)[:5]
    assert np.array_equal(o_lb, g_lb), np.argwhere(o_lb != g_lb)[:5]
    v1, v2 = tl.env_view(o_out, A, ob.K, ob.pitch, B), tl.env_view(g_out, A, ob.K, ob.pitch, B)
    assert np.array_equal(v1, v2), np.argwhere(v1 != v2)[:5]


def test_rollout_single_config_and_bad_alloc():
    ob, s, acts, subs, alloc = _random_case("full-divider_tl", 2, 3000, seed=5)
    # alloc=None: every row uses subtasks[0]
    o_out = ob.new_state()
    o_fl, o_lb = ob.rollout(s, o_out, acts, subs[:1], None)
    g_out, g_fl, g_lb = _gpu_rollout(ob.level, 2, ob.B, s, acts, subs[:1], None)
    assert np.array_equal(o_fl, g_fl) and np.array_equal(o_lb, g_lb)
    # out-of-range ids are flagged, rows copied
    alloc[:ob.B:7] = 200
    g_out, g_fl, g_lb = _gpu_rollout(ob.level, 2, ob.B, s, acts, subs, alloc)
    bad = alloc[:ob.B] >= len(subs)
    assert np.all(g_fl[bad] == capi.ROLL_BADALLOC) and np.all(g_lb[bad] == 0)
    v_in, v_out = tl.env_view(s, 2, ob.K, ob.pitch, ob.B), tl.env_view(g_out, 2, ob.K, ob.pitch, ob.B)
    assert np.array_equal(v_in[:, bad], v_out[:, bad])


def test_rollout_flags_level0_double_removal():
    import test_rollout_host as th  # noqa: F401
    from gym_cooking_amd import levels
    lv = levels.load_level("open-divider_salad")
    ob = oracle.OracleBatch(lv, 3, 100, 4)
    s = ob.new_state()
    ob.reset(s)
    v = tl.planes_view(s, 3, ob.K, ob.pitch)
    v["ax"][2, :4], v["ay"][2, :4] = v["ax"][0, :4], v["ay"][0, :4]
    subs = [capi.subtask(capi.SUB_CHOP, (1,), (0x01, 0), 0x11)]
    acts = np.full(3 * ob.pitch, 3, np.uint8)
    g_out, g_fl, g_lb = _gpu_rollout(lv, 3, 4, s, acts, subs, None)
    assert np.all(g_fl == capi.ROLL_RAISES) and np.all(g_lb == 0)
    assert np.array_equal(tl.env_view(g_out, 3, ob.K, ob.pitch, 4), tl.env_view(s, 3, ob.K, ob.pitch, 4))
