"""CPU check of the Bayesian-delegation belief update over the engine
(gym_cooking_amd.delegation.BayesianDelegator.bayes_update, Level-1 inverse planning through
gym_cooking_amd.planner) against the reference's own updates (tests/golden/bayes.json,
gen_bayes.py), with the CPU oracle's rollout rows and bounds standing in for the kernels
(TEST INFRASTRUCTURE).  tests/test_delegation_gpu.py runs the same updates on the GPU."""
import json
import os
import random

import numpy as np
import pytest

import oc_testlib as tl
import test_planner_gpu as tg


def load():
    path = os.path.join(tl.GOLDEN, "bayes.json")
    if not os.path.exists(path):
        pytest.skip("bayes.json not generated")
    with open(path) as f:
        return json.load(f)


def _alloc(rec):
    from gym_cooking_amd.delegation import SubtaskAllocation
    return tuple(SubtaskAllocation(None if s is None else tg._subtask(s), tuple(a)) for s, a in rec)


def run_update(fx, c, make_env, **planner_kw):
    """One recorded update: returns (posterior list or exception name, expected)."""
    from gym_cooking_amd.delegation import BayesianDelegator, SubtaskAllocDistribution
    from gym_cooking_amd.planner import E2E_BRTDP
    cfg = fx["configs"][c["cfg"]]
    obs = make_env(cfg["level"], cfg["A"], c)
    names = obs.get_agent_names()
    d = BayesianDelegator(c["self"], names, "bd", E2E_BRTDP(**fx["params"], **planner_kw), fx["none_action_prob"])
    allocs = [_alloc(a) for a, _ in c["before"]]
    d.probs = SubtaskAllocDistribution(allocs)
    for k, (_, p) in zip(allocs, c["before"]):
        d.probs.probs[k] = p
    random.seed(c["random_seed"])
    np.random.seed(c["np_seed"])
    try:
        d.bayes_update(obs_tm1=obs, actions_tm1={n: tuple(a) for n, a in c["actions"].items()}, beta=fx["beta"])
    except (AssertionError, AttributeError) as ex:
        return type(ex).__name__, c["raised"]
    got = [[[[None if t.subtask is None else str(t.subtask), list(t.subtask_agent_names)] for t in k], p]
           for k, p in d.probs.get_list()]
    return got, c["after"] if c["raised"] is None else c["raised"]


def run_batch(fx, calls, make_env, **planner_kw):
    """The recorded updates `calls` in ONE bayes_update_batch call, each delegator and planner
    with its own generators seeded as the recording was; returns [(got, want)] per call."""
    from gym_cooking_amd.delegation import BayesianDelegator, SubtaskAllocDistribution, bayes_update_batch
    from gym_cooking_amd.planner import E2E_BRTDP
    ds, obs, acts = [], [], []
    for c in calls:
        cfg = fx["configs"][c["cfg"]]
        o = make_env(cfg["level"], cfg["A"], c)
        planner = E2E_BRTDP(**fx["params"], rng=np.random.RandomState(c["np_seed"]), **planner_kw)
        d = BayesianDelegator(c["self"], o.get_agent_names(), "bd", planner, fx["none_action_prob"],
                              rng=random.Random(c["random_seed"]))
        allocs = [_alloc(a) for a, _ in c["before"]]
        d.probs = SubtaskAllocDistribution(allocs)
        for k, (_, p) in zip(allocs, c["before"]):
            d.probs.probs[k] = p
        ds.append(d)
        obs.append(o)
        acts.append({n: tuple(a) for n, a in c["actions"].items()})
    errs = bayes_update_batch(ds, obs, acts, fx["beta"])
    out = []
    for d, e, c in zip(ds, errs, calls):
        if e is not None:
            out.append((type(e).__name__, c["raised"]))
            continue
        got = [[[[None if t.subtask is None else str(t.subtask), list(t.subtask_agent_names)] for t in k], p]
               for k, p in d.probs.get_list()]
        out.append((got, c["after"] if c["raised"] is None else c["raised"]))
    return out


def test_host_bayes_update_batch_matches_reference():
    """Every recorded update (all configurations) in one bayes_update_batch call."""
    import test_planner_host as th
    fx = load()
    calls = fx["calls"]
    res = run_batch(fx, calls, th._env, expander=th.OracleExpander)
    bad = [i for i, (g, w) in enumerate(res) if g != w]
    assert not bad, "%d of %d batched updates differ: %s" % (len(bad), len(res), bad[:10])


def test_host_bayes_update_matches_reference():
    import test_planner_host as th
    fx = load()
    errs = []
    for i, c in enumerate(fx["calls"]):
        got, want = run_update(fx, c, th._env, expander=th.OracleExpander)
        if got != want:
            errs.append("update %d (cfg %d t %d self %s): got %s\n   want %s" % (i, c["cfg"], c["t"], c["self"],
                                                                          str(got)[:300], str(want)[:300]))
    assert fx["calls"]
    assert not errs, "%d of %d updates differ:\n%s" % (len(errs), len(fx["calls"]), "\n".join(errs[:6]))


def _plain(v):
    """A planner field as comparable data (arrays as bytes, subtasks and configurations as text)."""
    if isinstance(v, np.ndarray):
        return v.tobytes()
    if isinstance(v, (list, tuple)):
        return [_plain(x) for x in v]
    if isinstance(v, (bytes, frozenset, int, float, bool, str)) or v is None:
        return v
    return str(bytes(v)) if hasattr(v, "_fields_") else str(v)


def test_host_bayes_memo_changes_nothing():
    """The per-update memo (BayesianDelegator.use_memo) against the plain recomputation, on every
    recorded update in one batch: the same posteriors and exceptions, and the same state left
    behind -- both generators' states (the memo replays the argmin and get_max draws), the value
    tables in insertion order, the expansions and the other-agent planners' subtasks.  The
    recorded posteriors alone would not see a draw too many or too few."""
    import test_planner_host as th
    from gym_cooking_amd.delegation import BayesianDelegator, SubtaskAllocDistribution, bayes_update_batch
    from gym_cooking_amd.planner import E2E_BRTDP
    fx = load()
    calls = fx["calls"]

    def run(memo):
        ds, obs, acts = [], [], []
        for c in calls:
            cfg = fx["configs"][c["cfg"]]
            o = th._env(cfg["level"], cfg["A"], c)
            planner = E2E_BRTDP(**fx["params"], rng=np.random.RandomState(c["np_seed"]), expander=th.OracleExpander)
            d = BayesianDelegator(c["self"], o.get_agent_names(), "bd", planner, fx["none_action_prob"],
                                  rng=random.Random(c["random_seed"]))
            d.use_memo = memo
            allocs = [_alloc(a) for a, _ in c["before"]]
            d.probs = SubtaskAllocDistribution(allocs)
            for k, (_, p) in zip(allocs, c["before"]):
                d.probs.probs[k] = p
            ds.append(d)
            obs.append(o)
            acts.append({n: tuple(a) for n, a in c["actions"].items()})
        errs = bayes_update_batch(ds, obs, acts, fx["beta"])
        out = []
        for d, e in zip(ds, errs):
            p = d.planner
            st = p._rng.get_state()
            out.append((None if e is None else type(e).__name__, list(d.probs.probs.items()), d._rng.getstate(),
                        (st[0], st[1].tolist(), st[2:]), list(p.v_l.items()), list(p.v_u.items()), list(p._succ),
                        {n: (str(op.subtask), op.subtask_agent_names)
                         for n, op in getattr(p, "other_agent_planners", {}).items()},
                        sorted(k for k in p.__dict__ if not k.startswith("__")),
                        [(k, _plain(p.__dict__[k])) for k in ("_level", "subtask", "subtask_agent_names", "is_joint",
                                                              "_agents", "_sub_key", "cur_obj_count", "start",
                                                              "_start_goal", "_conf") if k in p.__dict__]))
        return out

    a, b = run(True), run(False)
    assert len(a) == len(b) == len(calls)
    bad = [i for i, (x, y) in enumerate(zip(a, b)) if x != y]
    assert not bad, "%d of %d updates leave a different state with the memo: %s" % (len(bad), len(a), bad[:10])
