"""oc_cpu_step (include/oc_engine.h): the engine's step on the host, through the product
library's C-ABI, for callers without a GPU.  CPU tests, no device.

* every reference fixture (KATs, streams, greedy traces: overcooked_environment.py:255-306
  as the reference ran it, tests/golden/gen_golden.py) replayed through oc_cpu_step;
* random streams on every builtin level and agent count against the oracle, with the
  window statistics against the host restatement of the counters, several thread counts
  (the split over env ranges must not matter), in place and out of place;
* the user-level kernels (dup / many / edge levels: counts encoding, 8 and 16 item slots,
  border Floor) against the oracle."""
import numpy as np
import pytest

import oc_testlib as tl
from gym_cooking_amd import levels
from gym_cooking_amd.engine import CpuStepper

from oracle import oracle


def _step_fn(cs):
    def fn(state, acts):
        a = np.full(cs.A * cs.pitch, 4, np.uint8)
        a.reshape(cs.A, cs.pitch)[:, :cs.B] = acts
        out = np.zeros_like(state)
        ex = np.zeros(cs.A * cs.pitch, np.uint8)
        coll = np.zeros(cs.pitch, np.uint8)
        cs.step(state, out, a, ex, coll)
        return out, ex.reshape(cs.A, cs.pitch)[:, :cs.B], coll[:cs.B]
    return fn


@pytest.mark.parametrize("fixture", ["kat.npz", "streams.npz", "greedy.npz"])
def test_cpu_step_matches_reference_fixtures(fixture):
    fx = tl.load_fixture(fixture)
    for g in tl.episode_groups(fx):
        cs = CpuStepper(g.level, g.A, g.B, g.max_T, nthreads=2)
        ob = oracle.OracleBatch(g.level, g.A, g.max_T, g.B)
        s = ob.new_state()
        ob.reset(s)
        assert np.array_equal(tl.env_view(cs.new_state(), g.A, cs.K, cs.pitch, g.B),
                              tl.env_view(s, g.A, ob.K, ob.pitch, g.B)), "reset template"
        g.relocate(s, cs.pitch)
        errs = tl.compare_group(g, _step_fn(cs), s, cs.pitch, g.level.width)
        assert not errs, "\n".join(errs[:10])


def _random_vs_oracle(lv, A, B, steps, max_T, nthreads, seed, in_place=False):
    ob = oracle.OracleBatch(lv, A, max_T, B)
    cs = CpuStepper(lv, A, B, max_T, nthreads=nthreads)
    assert cs.pitch == ob.pitch and cs.K == ob.K
    P = ob.pitch
    s1, n1 = ob.new_state(), ob.new_state()
    ob.reset(s1)
    s2, n2 = s1.copy(), s1.copy()
    act = ob.new_actions()
    e1, e2 = np.zeros(A * P, np.uint8), np.zeros(A * P, np.uint8)
    c1, c2 = np.zeros(P, np.uint8), np.zeros(P, np.uint8)
    tot, want = np.zeros(5, np.uint64), np.zeros(5, np.int64)
    for t in range(steps):
        ob.gen_actions(act, 0, t, seed)
        fl_in = tl.planes_view(s1, A, ob.K, P)["fl"].copy()
        ob.step(s1, n1, act, e1, c1)
        s1, n1 = n1, s1
        want += tl.window_totals(fl_in, s1, c1, A, ob.K, P, B)
        if in_place:
            cs.step(s2, s2, act, e2, c2, tot)
        else:
            cs.step(s2, n2, act, e2, c2, tot)
            s2, n2 = n2, s2
        v1, v2 = tl.env_view(s1, A, ob.K, P, B), tl.env_view(s2, A, ob.K, P, B)
        if not np.array_equal(v1, v2):
            bad = np.argwhere(v1 != v2)
            raise AssertionError("step %d: %d bytes differ, first (plane, env) %s" % (t, len(bad), bad[:5].tolist()))
        assert np.array_equal(e1.reshape(A, -1)[:, :B], e2.reshape(A, -1)[:, :B]), t
        assert np.array_equal(c1[:B], c2[:B]), t
    assert np.array_equal(tot.astype(np.int64), want), (tot, want)
    return want


@pytest.mark.parametrize("level", sorted(levels.BUILTIN_LEVELS))
@pytest.mark.parametrize("A", [1, 2, 3, 4])
def test_cpu_step_matches_oracle_random(level, A):
    want = _random_vs_oracle(levels.load_level(level), A, 1003, 130, 60, nthreads=1, seed=A * 17 + 3)
    assert want[0] > 0  # episodes ended (max_T 60 < 130 steps)


@pytest.mark.parametrize("nthreads", [0, 3, 8])
def test_cpu_step_threads_and_in_place(nthreads):
    """40,003 envs over several threads (>= 16 Ki envs each: up to 3 ranges), in place."""
    _random_vs_oracle(levels.load_level("partial-divider_salad"), 2, 40003, 40, 25, nthreads, seed=5,
                      in_place=nthreads == 3)


@pytest.mark.parametrize("name,A", [("levels/dup-7x7_tomato2.txt", 2), ("levels/many-13x12_full16.txt", 3), ("levels/edge-8x7_tl.txt", 2),
                                    ("levels/big-15x17_salad.txt", 4)])
def test_cpu_step_user_levels(name, A):
    lv = tl.load_level(name)
    _random_vs_oracle(lv, A, 517, 90, 40, nthreads=2, seed=11)


def test_cpu_step_refuses_bad_arguments():
    cs = CpuStepper("open-divider_salad", 2, 10)
    s = cs.new_state()
    with pytest.raises(ValueError):
        cs.step(s, s, np.zeros(3, np.uint8))
