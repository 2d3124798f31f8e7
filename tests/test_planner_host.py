"""CPU check of the engine-backed navigation planner's host search
(gym_cooking_amd.planner.E2E_BRTDP: get_next_action / main / runSampleTrial / backups /
argmin tie-breaks) against the reference planner's recorded decisions
(tests/golden/brtdp.json), with the CPU oracle's rollout rows standing in for the oc_rollout
launches (TEST INFRASTRUCTURE: the product planner always expands on the GPU).  The same
calls run through the HIP engine in tests/test_planner_gpu.py."""
import json
import os
import types

import numpy as np
import pytest

import oc_testlib as tl
import test_planner_gpu as tg
from gym_cooking_amd import capi, envs, levels, recipes

from oracle import oracle


class OracleExpander:
    ROWS = 32

    def __init__(self, level, num_agents, device):
        self.ob = oracle.OracleBatch(level, num_agents, 0, self.ROWS)
        self.A, self.K = num_agents, self.ob.K
        lv = levels.load_level(level) if isinstance(level, str) else level
        self.enc, self.wide = lv.encoding, capi.is_wide(lv)
        P = capi.layout_planes(num_agents, self.K, self.wide)
        self.NP, self.t_plane, self.P = P["num_planes"], P["t"], self.ob.pitch
        self.launches = 0

    def run(self, requests):
        return [self.rows(*req) for req in requests]

    def bounds(self, state, subs):
        sin = np.zeros((self.NP, self.P), np.uint8)
        sin[:, 0] = state
        sin[self.t_plane:, :] = 0
        lb, ok = self.ob.subtask_bounds(sin.reshape(-1), subs, nthreads=1)
        return lb[:, 0], ok[:, 0]

    def bounds_many(self, states, subs):
        out_lb, out_ok = [], []
        for st in states:
            lb, ok = self.bounds(st, subs)
            out_lb.append(lb)
            out_ok.append(ok)
        return np.stack(out_lb, 1), np.stack(out_ok, 1)

    def rows(self, state, codes, sub):
        n = len(codes)
        sin = np.zeros((self.NP, self.P), np.uint8)
        sin[:, :n] = state[:, None]
        sin[self.t_plane:, :] = 0
        act = np.full((self.A, self.P), 4, np.uint8)
        for r, c in enumerate(codes):
            for q in range(sub.num_agents):
                act[sub.agent[q], r] = c[q]
        sout = np.zeros_like(sin)
        fl, lb = self.ob.rollout(sin.reshape(-1), sout.reshape(-1), act.reshape(-1), [sub], None, nthreads=1)
        self.launches += 1
        nxt = sout[:, :n].T.copy()
        nxt[:, self.t_plane:] = 0
        return nxt, fl[:n], lb[:n]


def _env(level_name, A, call):
    lv = levels.load_level(level_name)
    K = capi.item_slots(lv)
    P = capi.pitch_for(1)
    s = tl.state_from_canonical(lv, A, K, P, np.array([call["agents"]], np.uint8),
                                np.array([call["items"]], np.uint8), np.array([call["env_t"]]))
    b = tl.env_view(s, A, K, P, 1)[:, 0].copy()
    agents, world, _, _ = envs.build_views(lv, A, K, b)
    return types.SimpleNamespace(level=lv, _device="cpu", state_bytes=lambda: b.copy(),
                                 _group_names=frozenset(g for g in call["groups"] if g not in tg._STATIC),
                                 world=world, get_agent_names=lambda: [a.name for a in agents])


@pytest.mark.parametrize("mode", ["fresh", "chain"])
def test_host_planner_matches_reference_calls(mode):
    from gym_cooking_amd.planner import E2E_BRTDP
    fx = tg._fixture()
    params = fx["params"]
    chains, errs, n = {}, [], 0
    for i, c in enumerate(fx["calls"]):
        if c["mode"] != mode:
            continue
        cfg = fx["configs"][c["cfg"]]
        env = _env(cfg["level"], cfg["A"], c)
        names = env.get_agent_names()
        agn = tuple(names[a] for a in c["sub_agents"])
        if mode == "fresh":
            p = E2E_BRTDP(**params, expander=OracleExpander)
        else:
            p = chains.setdefault((c["cfg"], c["episode"], c["subtask"], agn), E2E_BRTDP(**params, expander=OracleExpander))
        np.random.seed(c["seed"])
        action = p.get_next_action(env=env, subtask=tg._subtask(c["subtask"]), subtask_agent_names=agn,
                                   other_agent_planners={})
        exp = None if c["action"] is None else (tg._NAV[c["action"][0]] if len(c["action"]) == 1
                                                else tuple(tg._NAV[k] for k in c["action"]))
        v_l, v_u = p.start_values()
        got = (action, p.cur_obj_count, v_l, v_u, len(p.v_l))
        want = (exp, c["goal_count"], c["v_l"], c["v_u"], c["n_states"])
        if got != want:
            errs.append("call %d (%s, %s %s, seed %d): got %s want %s" % (i, cfg["level"], c["subtask"], agn,
                                                                      c["seed"], got, want))
        n += 1
    assert n > 0
    assert not errs, "%d of %d calls differ:\n%s" % (len(errs), n, "\n".join(errs[:15]))


def test_host_plan_batch_matches_reference_calls():
    """plan_batch: every 'fresh' call of the fixture as one lockstep batch (per config), each
    search with its own RandomState(seed) -> exactly the reference's results."""
    from gym_cooking_amd.planner import E2E_BRTDP, plan_batch
    fx = tg._fixture()
    params = fx["params"]
    errs, n = [], 0
    for cfg_i, cfg in enumerate(fx["configs"]):
        calls = [c for c in fx["calls"] if c["mode"] == "fresh" and c["cfg"] == cfg_i]
        if not calls:
            continue
        envs_ = [_env(cfg["level"], cfg["A"], c) for c in calls]
        agn = [tuple(e.get_agent_names()[a] for a in c["sub_agents"]) for e, c in zip(envs_, calls)]
        planners = [E2E_BRTDP(**params, expander=OracleExpander, rng=np.random.RandomState(c["seed"])) for c in calls]
        got = plan_batch(planners, envs_, [tg._subtask(c["subtask"]) for c in calls], agn)
        for p, a, c in zip(planners, got, calls):
            exp = None if c["action"] is None else (tg._NAV[c["action"][0]] if len(c["action"]) == 1
                                                    else tuple(tg._NAV[k] for k in c["action"]))
            if (a, *p.start_values(), len(p.v_l)) != (exp, c["v_l"], c["v_u"], c["n_states"]):
                errs.append("%s %s: %s vs %s" % (cfg["level"], c["subtask"], a, exp))
            n += 1
    assert n > 0
    assert not errs, "\n".join(errs[:10])


def _level1_calls():
    path = os.path.join(tl.GOLDEN, "brtdp_level1.json")
    if not os.path.exists(path):
        pytest.skip("brtdp_level1.json not generated")
    with open(path) as f:
        return json.load(f)


def run_level1_call(fx, c, E2E_BRTDP, make_env, **kw):
    """One recorded Level-1 call: the other agents' planners are shallow copies of the main
    planner set up for their subtasks (BayesianDelegator.get_other_agent_planners)."""
    import copy
    cfg = fx["configs"][c["cfg"]]
    env = make_env(cfg["level"], cfg["A"], c)
    names = env.get_agent_names()
    p = E2E_BRTDP(**fx["params"], **kw)
    others = {}
    for j, sub, _, _, _ in c["others"]:
        op = copy.copy(p)
        op.set_settings(make_env(cfg["level"], cfg["A"], c), tg._subtask(sub), (names[j],))
        others[names[j]] = op
    np.random.seed(c["seed"])
    a = p.get_next_action(env, tg._subtask(c["subtask"]), tuple(names[i] for i in c["sub_agents"]), others)
    exp = None if c["action"] is None else (tg._NAV[c["action"][0]] if len(c["action"]) == 1
                                            else tuple(tg._NAV[k] for k in c["action"]))
    return (a, p.cur_obj_count, *p.start_values(), len(p.v_l)), (exp, c["goal_count"], c["v_l"], c["v_u"],
                                                                 c["n_states"])


def level1_batch(fx, make_env, **kw):
    """Every recorded Level-1 call as one plan_batch per config (each search with its own
    RandomState(seed), its other agents' planners copies of its planner); returns the list of
    mismatches."""
    import copy
    from gym_cooking_amd.planner import E2E_BRTDP, plan_batch
    errs = []
    for cfg_i, cfg in enumerate(fx["configs"]):
        calls = [c for c in fx["calls"] if c["cfg"] == cfg_i]
        if not calls:
            continue
        planners, envs_, subs, agn, others = [], [], [], [], []
        for c in calls:
            env = make_env(cfg["level"], cfg["A"], c)
            names = env.get_agent_names()
            p = E2E_BRTDP(**fx["params"], rng=np.random.RandomState(c["seed"]), **kw)
            o = {}
            for j, sub, _, _, _ in c["others"]:
                op = copy.copy(p)
                op.set_settings(make_env(cfg["level"], cfg["A"], c), tg._subtask(sub), (names[j],))
                o[names[j]] = op
            planners.append(p)
            envs_.append(env)
            subs.append(tg._subtask(c["subtask"]))
            agn.append(tuple(names[i] for i in c["sub_agents"]))
            others.append(o)
        got = plan_batch(planners, envs_, subs, agn, others)
        for p, a, c in zip(planners, got, calls):
            exp = None if c["action"] is None else (tg._NAV[c["action"][0]] if len(c["action"]) == 1
                                                    else tuple(tg._NAV[k] for k in c["action"]))
            if (a, p.cur_obj_count, *p.start_values(), len(p.v_l)) != (exp, c["goal_count"], c["v_l"], c["v_u"],
                                                                        c["n_states"]):
                errs.append("%s %s others %s: %s vs %s" % (cfg["level"], c["subtask"], c["others"], a, exp))
    return errs


# The oracle-row searches are slow on the CPU (a Level-1 call sets up and expands every other
# agent's planner at every visited state), so the sequential test takes the even-numbered
# recorded calls and the batched test the odd-numbered ones: every call is checked once on the
# CPU.  tests/test_planner_gpu.py runs all 32 both ways on the kernel.
def test_host_plan_batch_level1_matches_reference_calls():
    fx = dict(_level1_calls())
    fx["calls"] = fx["calls"][1::2]
    errs = level1_batch(fx, _env, expander=OracleExpander)
    assert not errs, "\n".join(errs[:10])


def test_host_planner_level1_matches_reference_calls():
    from gym_cooking_amd.planner import E2E_BRTDP
    fx = _level1_calls()
    errs = []
    for i, c in list(enumerate(fx["calls"]))[0::2]:
        got, want = run_level1_call(fx, c, E2E_BRTDP, _env, expander=OracleExpander)
        if got != want:
            errs.append("call %d (%s, others %s): got %s want %s" % (i, c["subtask"], c["others"], got, want))
    assert fx["calls"]
    assert not errs, "%d of %d calls differ:\n%s" % (len(errs), len(fx["calls"]), "\n".join(errs[:10]))


def test_argmin_matches_multinomial_draws():
    """planner.argmin answers a unique minimum without numpy's multinomial but consumes the
    generator exactly as it (one uniform double unless the minimum is the last entry): same
    index and same generator state as the reference's formula (e2e_brtdp.py:27-30), with and
    without ties, on a RandomState and on the global generator."""
    from gym_cooking_amd.planner import argmin

    def ref(vector, rng):
        e_x = np.array(vector) == min(vector)
        return np.where(rng.multinomial(1, e_x / e_x.sum()))[0][0]

    gen = np.random.default_rng(0)
    for trial in range(3000):
        n = int(gen.integers(1, 26))
        v = [float(x) for x in gen.integers(0, 4 if trial % 2 else 50, n) * 0.5]
        r1, r2 = np.random.RandomState(trial), np.random.RandomState(trial)
        r1.random_sample(int(gen.integers(0, 700)))
        r2.set_state(r1.get_state())
        assert argmin(v, r1) == ref(v, r2)
        s1, s2 = r1.get_state(), r2.get_state()
        assert s1[2] == s2[2] and np.array_equal(s1[1], s2[1])
    np.random.seed(7)
    a = [argmin([1.0, 0.5, 2.0, 0.5][:k], np.random) for k in (1, 2, 3, 4)]
    np.random.seed(7)
    b = [ref([1.0, 0.5, 2.0, 0.5][:k], np.random) for k in (1, 2, 3, 4)]
    assert a == b and np.random.random_sample() == (np.random.seed(7), [ref([1.0, 0.5, 2.0, 0.5][:k], np.random)
                                                                        for k in (1, 2, 3, 4)],
                                                    np.random.random_sample())[2]


def test_native_sample_trial_matches_python_loop():
    """The sample trial's C loop (csrc/brtdp_host.c, planner._sample_trial_native) and the Python
    loop give the same searches: the same actions, bit-identical value tables, the same
    generator state, on 40 random-play states of 2 kitchens with single and joint subtasks
    (ties included: the multinomial path runs inside the C loop)."""
    from gym_cooking_amd import planner as pl
    from gym_cooking_amd.planner import E2E_BRTDP, PlanEnv, plan_batch
    assert pl._native is not None, "the _brtdp extension is not built (make -C gym-cooking_amd/csrc)"
    for level, sub, agn, names in (("open-divider_salad", recipes.Chop("Tomato"), ("agent-1",), ["Tomato", "Lettuce", "Plate"]),
                                   ("partial-divider_salad", recipes.Chop("Lettuce"), ("agent-1", "agent-2"),
                                    ["Tomato", "Lettuce", "Plate"])):
        lv = levels.load_level(level)
        ob = oracle.OracleBatch(lv, 2, 0, 20)
        s, s2, a = ob.new_state(), ob.new_state(), ob.new_actions()
        ob.reset(s)
        for t in range(9):
            ob.gen_actions(a, 0, t, 5)
            ob.step(s, s2, a)
            s, s2 = s2, s
        ev = tl.env_view(s, 2, ob.K, ob.pitch, 20)
        runs = []
        for native in (True, False):
            envs_, ps = [], []
            for b in range(20):
                envs_.append(PlanEnv(lv, 2, ev[:, b], names, device="cpu"))
                p = E2E_BRTDP(alpha=0.01, tau=2, cap=75, main_cap=100, device="cpu", expander=OracleExpander,
                              rng=np.random.RandomState(b))
                p.use_native = native
                ps.append(p)
            acts = plan_batch(ps, envs_, [sub] * 20, [agn] * 20)
            runs.append((acts, [(p.v_l, p.v_u, p._rng.get_state()[2]) for p in ps]))
        (a1, t1), (a2, t2) = runs
        assert a1 == a2
        for (l1, u1, g1), (l2, u2, g2) in zip(t1, t2):
            assert l1 == l2 and u1 == u2 and g1 == g2


def test_native_errors_raise_python_exceptions():
    """The extension's error paths set a Python exception (no SystemError): an expanded state
    with no actions raises ValueError as Python's min() of an empty sequence does, and so does
    an empty tie pick."""
    from gym_cooking_amd import planner as pl
    nat = pl._native
    assert nat is not None, "the _brtdp extension is not built (make -C gym-cooking_amd/csrc)"
    with pytest.raises(ValueError):
        nat.tie_pick([], lambda: 0.5)
    entry = [None, [], [], [], None, None, True, None, "rx"]
    with pytest.raises(ValueError):
        nat.backprop({}, {}, ["x"], [entry])
    with pytest.raises(ValueError):  # a trajectory state without its entry
        nat.backprop({}, {}, ["x", "y"], [entry])
    with pytest.raises(ValueError):
        nat.forward({("x", "sk"): entry}, {}, {}, "x", "sk", "x", 10, 0, 2.0, [], lambda: 0.5, False, [], 1.1)
    # value_init's assert (e2e_brtdp.py:722), after the inserts before it, as _init_succ's
    got = [None, None, None, ["a", "b", "c"], [True, False, False], [2.0, 0.0, 3.0], False, None, "rx"]
    v_l, v_u = {}, {}
    with pytest.raises(AssertionError, match="lower: 0.0"):
        nat.init_succ(got, v_l, v_u, 1.1)
    assert v_l == {"a": 0.0} and v_u == {"a": 0.0} and got[6] is False
    got[5][1] = 1.0
    nat.init_succ(got, v_l, v_u, 1.1)
    assert got[6] is True and v_l["b"] == 1.0 * 1.1 - 1.09 and v_u["c"] == 3.0 * 1.1 * 5 * 1.1


def test_native_sampler_draws_the_same_stream():
    """planner._sampler hands the native loop the generator's bit-generator capsule: its draws
    (tie picks) and the generator's position afterwards equal those through random_sample, for a
    RandomState and for numpy's global generator (the reference's np.random)."""
    from gym_cooking_amd import planner as pl
    nat = pl._native
    assert nat is not None, "the _brtdp extension is not built (make -C gym-cooking_amd/csrc)"
    masks = [[True, False, True, True], [False, True], [True] * 7, [False, False, True]]
    for make in (lambda: np.random.RandomState(11), lambda: (np.random.seed(11), np.random)[1]):
        r1 = make()
        assert type(pl._sampler(r1)).__name__ == "PyCapsule"
        a = [nat.tie_pick(m, pl._sampler(r1)) for m in masks * 20]
        x1 = r1.random_sample()
        r2 = make()
        b = [nat.tie_pick(m, r2.random_sample) for m in masks * 20]
        assert a == b and x1 == r2.random_sample()
    class Other:  # anything else: its random_sample
        def random_sample(self):
            return 0.25
    o = Other()
    assert pl._sampler(o) == o.random_sample
