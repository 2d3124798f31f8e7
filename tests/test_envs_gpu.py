"""GPU tests of the gym shim (gym_cooking_amd/envs.py) over the HIP engine: the reference's
single-env API replays the golden fixture episodes (state, exec, collision log, reward,
done, termination_info, the ERR crash), and the vector env agrees with OvercookedBatch."""
import types

import numpy as np
import pytest

import oc_testlib as tl
from gym_cooking_amd import capi, levels

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _canon(env_bytes, A, K, width):
    return tl.canonical(np.asarray(env_bytes, np.uint8), A, K, 1, width, 1)


@pytest.mark.parametrize("fixture,limit", [("kat.npz", None), ("streams.npz", 60)])
def test_single_env_shim_replays_fixtures(fixture, limit):
    from gym_cooking_amd.envs import OvercookedEnvironment
    fx = tl.load_fixture(fixture)
    eps = range(len(fx["ep_T"])) if limit is None else np.linspace(0, len(fx["ep_T"]) - 1, limit).astype(int)
    n_steps = n_err = n_succ = 0
    for e in eps:
        lvname = str(fx["level_names"][fx["ep_level"][e]])
        A, max_T = int(fx["ep_A"][e]), int(fx["ep_maxT"][e])
        arg = types.SimpleNamespace(level=lvname, num_agents=A, max_num_timesteps=max_T, seed=1, model1=None,
                                    model2=None, model3=None, model4=None, record=False, with_image_obs=False)
        env = OvercookedEnvironment(arg)
        obs = env.reset()
        assert obs.t == 0 and not env.done()
        K = capi.item_slots(env.level)
        s = env.state_bytes()
        st = fx["ep_start"][e]
        for a in range(A):
            if st[a, 0] != tl.PAD:
                s[a], s[A + a] = st[a, 0], st[a, 1]
        env.load_state(s)
        off, aoff = fx["ep_state_off"][e], fx["ep_act_off"][e]
        for step in range(int(fx["ep_T"][e])):
            codes = fx["act"][aoff + step][:A]
            ad = {"agent-%d" % (a + 1): levels.ACTIONS[min(int(codes[a]), 4)] for a in range(A)}
            exp_fl = int(fx["flags"][off + step + 1])
            ncoll = len(env.collisions)
            if exp_fl & 0x04:
                with pytest.raises(AttributeError):
                    env.step(ad)
                n_err += 1
                break
            obs, reward, done, info = env.step(ad)
            n_steps += 1
            c = _canon(env.state_bytes(), A, K, env.level.width)
            assert int(c["t"][0]) == int(fx["t"][off + step + 1]) == env.t == info["t"]
            assert np.array_equal(c["agents"][0], fx["agents"][off + step + 1]), (e, step)
            assert np.array_equal(c["items"][0], fx["items"][off + step + 1]), (e, step)
            assert done == bool(exp_fl & 0x01) and reward == (1 if exp_fl & 0x02 else 0), (e, step)
            n_succ += reward
            if done:
                assert env.termination_info.startswith("Terminating because")
            ex = [levels.ACTION_CODE[env.agent_actions["agent-%d" % (a + 1)]] for a in range(A)]
            assert ex == [int(v) for v in fx["exe"][aoff + step][:A]], (e, step)
            assert len(env.collisions) - ncoll == bin(int(fx["coll"][aoff + step])).count("1")
            # obs_tm1: the pre-execution state with the executed actions
            assert [a.action for a in env.obs_tm1.sim_agents] == [levels.ACTIONS[v] for v in ex]
            assert obs == env and obs is not env
    assert n_steps > 50
    if fixture == "kat.npz":
        assert n_succ >= 1


def test_vec_env_matches_batch():
    from gym_cooking_amd.engine import OvercookedBatch
    from gym_cooking_amd.envs import OvercookedVecEnv
    B, A, T = 5000, 2, 150
    ve = OvercookedVecEnv("partial-divider_salad", A, B, max_num_timesteps=40)
    eb = OvercookedBatch("partial-divider_salad", A, B, max_T=40)
    s, n = eb.new_state(), eb.new_state()
    eb.reset(s)
    ve.reset()
    a = eb.new_actions()
    ends = 0
    for t in range(T):
        eb.gen_actions(a, t, 3)
        eb.step(s, n, a)
        s, n = n, s
        st, rew, done, info = ve.step(a.view(A, -1)[:, :B].contiguous())
        assert torch.equal(st.view(-1, eb.pitch)[:, :B], s.view(-1, eb.pitch)[:, :B])
        ends += int(done.sum())
        assert torch.equal(rew.bool(), done & ((st.view(-1, eb.pitch)[-1, :B] & 2) != 0))
    assert ends > 0
    tot = ve.episode_stats()
    assert int(tot[0]) == ends


def test_vec_env_int64_actions_at_pitch():
    """at B == pitch (2^k multiples of 4096) an int64 action tensor must be
    converted, not read as raw bytes; results equal the uint8 path and the batch engine."""
    from gym_cooking_amd.envs import OvercookedVecEnv
    B, A = 8192, 2
    v8 = OvercookedVecEnv("partial-divider_salad", A, B, max_num_timesteps=30)
    v64 = OvercookedVecEnv("partial-divider_salad", A, B, max_num_timesteps=30)
    assert v8.P == B
    v8.reset()
    v64.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(4)
    for t in range(45):
        a64 = torch.randint(0, 5, (A, B), device="cuda:0", generator=g)  # int64, torch's default
        s8, r8, d8, _ = v8.step(a64.to(torch.uint8))
        s64, r64, d64, _ = v64.step(a64)
        assert torch.equal(s8, s64), t
    from gym_cooking_amd.engine import OvercookedBatch
    eb = OvercookedBatch("partial-divider_salad", A, B, max_T=30)
    with pytest.raises(TypeError):
        eb.step(eb.new_state(), eb.new_state(), torch.zeros(A * B, dtype=torch.int64, device="cuda:0"))
