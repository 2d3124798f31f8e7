"""GPU check of the Bayesian-delegation belief update (gym_cooking_amd.delegation.BayesianDelegator
.bayes_update): every Q, get_actions and doability query runs on the HIP engine (oc_rollout rows,
oc_subtask_bounds), and each of the reference's recorded updates (tests/golden/bayes.json) must
come out bit for bit -- the posterior, or the exception the reference raised."""
import time

import numpy as np
import pytest

import oc_testlib as tl
import test_delegation_host as td
from gym_cooking_amd import capi

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("obs", ["plan_env", "shim_env"])
def test_bayes_update_matches_reference(obs):
    """`obs`: the update's obs_tm1 as a PlanEnv (raw state bytes) or as the live reference-surface
    OvercookedEnvironment loaded with the recorded state."""
    from gym_cooking_amd.planner import PlanEnv
    from gym_cooking_amd import levels as _lv
    from test_planner_gpu import _STATIC, _env_at
    fx = td.load()

    def make_env(level_name, A, c):
        if obs == "shim_env":
            return _env_at(level_name, A, c)
        lv = _lv.load_level(level_name)
        K = capi.item_slots(lv)
        P = capi.pitch_for(1)
        s = tl.state_from_canonical(lv, A, K, P, np.array([c["agents"]], np.uint8),
                                    np.array([c["items"]], np.uint8), np.array([c["env_t"]]))
        return PlanEnv(lv, A, tl.env_view(s, A, K, P, 1)[:, 0], [g for g in c["groups"] if g not in _STATIC],
                       device="cuda:0")

    errs = []
    t0 = time.perf_counter()
    for i, c in enumerate(fx["calls"]):
        got, want = td.run_update(fx, c, make_env)
        if got != want:
            errs.append("update %d (cfg %d t %d self %s): got %s\n   want %s" % (i, c["cfg"], c["t"], c["self"],
                                                                          str(got)[:300], str(want)[:300]))
    dt = time.perf_counter() - t0
    print("\n%d bayes_update calls (%s): %.2f s on the engine; the reference took %.2f s on the build "
          "container's CPU" % (len(fx["calls"]), obs, dt, sum(c["ref_seconds"] for c in fx["calls"])))
    assert fx["calls"]
    assert not errs, "%d of %d updates differ:\n%s" % (len(errs), len(fx["calls"]), "\n".join(errs[:6]))


def test_bayes_update_batch_matches_reference():
    """All recorded updates (several levels and agent counts, 21 of them raising) in ONE
    bayes_update_batch call: shared oc_subtask_bounds and oc_rollout launches, each update
    bit for bit as recorded.  Prints the batched throughput beside the sequential one."""
    from gym_cooking_amd.planner import PlanEnv
    from gym_cooking_amd import levels as _lv
    from test_planner_gpu import _STATIC
    fx = td.load()

    def plan_env(level_name, A, c):  # one env per update (a live shim env would be shared)
        lv = _lv.load_level(level_name)
        K = capi.item_slots(lv)
        P = capi.pitch_for(1)
        s = tl.state_from_canonical(lv, A, K, P, np.array([c["agents"]], np.uint8),
                                    np.array([c["items"]], np.uint8), np.array([c["env_t"]]))
        return PlanEnv(lv, A, tl.env_view(s, A, K, P, 1)[:, 0], [g for g in c["groups"] if g not in _STATIC],
                       device="cuda:0")

    t0 = time.perf_counter()
    res = td.run_batch(fx, fx["calls"], plan_env)
    dt = time.perf_counter() - t0
    bad = [i for i, (g, w) in enumerate(res) if g != w]
    print("\n%d bayes_update calls in one batch: %.2f s (%.1f updates/s)" % (len(res), dt, len(res) / dt))
    assert not bad, "%d of %d batched updates differ: %s" % (len(bad), len(res), bad[:10])
