"""GPU parity at the bench's own shapes (BASELINE configs[1] and [3]).

* The headline kernel, oc_step_n, at the metric configuration (partial-divider_salad,
  2 agents, 2^20 envs) with the launch lengths bench.py uses (20 = the driver's
  `--steps 20`, 100 = the default launch cap), over 240 steps (auto-resets after the
  t = 100 timeouts at steps 101 and 202): every trajectory state, executed-action plane and
  collision mask against the 16-thread CPU oracle, byte for byte, plus the statistics.
* C4: 2^23 envs as 8 shards of 2^20 (global env ids r*2^20 + i, actions keyed by global id),
  each shard stepped by oc_step_n exactly as one bench rank does; every shard's checksum and
  final state against the oracle's single 2^23 batch, and the summed per-shard summaries
  (what the RCCL all-gather collects) against the oracle's totals.

Integer state: bit-exact, no tolerance."""
import numpy as np
import pytest

import oc_testlib as tl

from oracle import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

LEVEL, A, MAX_T = "partial-divider_salad", 2, 100


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from gym_cooking_amd import engine  # noqa: F401  (loads liboc_engine.so or raises)
    return torch.device("cuda:0")


def _batch(B):
    from gym_cooking_amd.engine import OvercookedBatch
    return OvercookedBatch(LEVEL, A, B, max_T=MAX_T, device="cuda:0")


def _segments(total, n):
    return [(i, min(n, total - i)) for i in range(0, total, n)]


@pytest.mark.parametrize("n", [20, 100])
def test_step_n_metric_shape_vs_oracle(dev, n):
    B, steps, seed = 1 << 20, 240, 2024 + n
    eb = _batch(B)
    P, S = eb.pitch, eb.layout.state_bytes
    ob = oracle.OracleBatch(eb.level, A, MAX_T, B)
    assert ob.pitch == P
    s, s2, stats = eb.new_state(), eb.new_state(), eb.new_stats()
    eb.reset(s)
    c, c2 = ob.new_state(), ob.new_state()
    ob.reset(c)
    cact, cex, ccoll = ob.new_actions(), np.zeros(A * P, np.uint8), np.zeros(P, np.uint8)
    traj = torch.empty(n * S, dtype=torch.uint8, device=dev)
    ex = torch.empty(n * A * P, dtype=torch.uint8, device=dev)
    coll = torch.empty(n * P, dtype=torch.uint8, device=dev)
    acts = torch.empty((n, A * P), dtype=torch.uint8, device=dev)
    tot = np.zeros(5, np.int64)
    totals = torch.full((5,), -1, dtype=torch.int64, device=dev)
    resets = 0
    for i0, m in _segments(steps, n):
        for r in range(m):
            eb.gen_actions(acts[r], step=i0 + r, seed=seed)
        eb.step_n(s, s2, acts[:m].reshape(-1), m, traj, ex, coll, stats, totals)  # in-launch fold, as bench.py
        s, s2 = s2, s
        h_traj = traj[:m * S].cpu().numpy().reshape(m, S)
        h_ex = ex[:m * A * P].cpu().numpy().reshape(m, A * P)
        h_coll = coll[:m * P].cpu().numpy().reshape(m, P)
        for r in range(m):
            t = i0 + r
            ob.gen_actions(cact, 0, t, seed)
            fl_in = tl.planes_view(c, A, ob.K, P)["fl"].copy()
            ob.step(c, c2, cact, cex, ccoll, nthreads=16)
            c, c2 = c2, c
            resets += int(((fl_in[:B] & 1) == 1).sum())
            tot += tl.window_totals(fl_in, c, ccoll, A, ob.K, P, B)
            assert np.array_equal(h_traj[r], c), "trajectory state differs at step %d (launch n=%d)" % (t, m)
            assert np.array_equal(h_ex[r].reshape(A, P)[:, :B], cex.reshape(A, P)[:, :B]), "exec at step %d" % t
            assert np.array_equal(h_coll[r][:B], ccoll[:B]), "collision mask at step %d" % t
        assert np.array_equal(totals.cpu().numpy(), tot), ("in-launch totals after step", i0 + m)
    assert np.array_equal(s.cpu().numpy(), c)
    got = eb.reduce_stats(stats).cpu().numpy()
    assert np.array_equal(got, tot), (got, tot)
    assert resets >= 2 * (B // 2), "expected two auto-reset waves (t=100 timeouts), saw %d resets" % resets
    assert tot[0] > 0 and tot[3] > 0


def test_c4_eight_shards_of_2_20(dev):
    """Config C4 on one GPU: the 8 ranks' shards, one after another, as bench.py steps them
    (oc_step_n launches of 100 / 100 / 30 steps, stats per shard, gen_actions with
    env_offset = r * 2^20)."""
    R, Bs, steps, seed = 8, 1 << 20, 230, 9
    Bg = R * Bs
    ob = oracle.OracleBatch(__import__("gym_cooking_amd").levels.load_level(LEVEL), A, MAX_T, Bg)
    c, c2 = ob.new_state(), ob.new_state()
    ob.reset(c)
    cact, ccoll = ob.new_actions(), np.zeros(ob.pitch, np.uint8)
    tot = np.zeros(5, np.int64)
    for t in range(steps):
        ob.gen_actions(cact, 0, t, seed)
        fl_in = tl.planes_view(c, A, ob.K, ob.pitch)["fl"].copy()
        ob.step(c, c2, cact, None, ccoll, nthreads=16)
        c, c2 = c2, c
        tot += tl.window_totals(fl_in, c, ccoll, A, ob.K, ob.pitch, Bg)
    ref_view = tl.env_view(c, A, ob.K, ob.pitch, Bg)

    eb = _batch(Bs)
    P = eb.pitch
    n = 100
    acts = torch.empty((n, A * P), dtype=torch.uint8, device=dev)
    s, s2 = eb.new_state(), eb.new_state()
    summed = np.zeros(5, np.int64)
    for r in range(R):
        stats = eb.new_stats()
        eb.reset(s)
        for i0, m in _segments(steps, n):
            for k in range(m):
                eb.gen_actions(acts[k], step=i0 + k, seed=seed, env_offset=r * Bs)
            eb.step_n(s, s2, acts[:m].reshape(-1), m, None, None, None, stats)
            s, s2 = s2, s
        got_sum = int(eb.checksum(s).item()) & (2**64 - 1)
        shard_ref = ref_view[:, r * Bs:(r + 1) * Bs]
        host = s.cpu().numpy()
        assert got_sum == tl.checksum(host, A, eb.K, P, Bs)
        assert np.array_equal(tl.env_view(host, A, eb.K, P, Bs), shard_ref), "shard %d differs" % r
        summed += eb.reduce_stats(stats).cpu().numpy()
    assert np.array_equal(summed, tot), (summed, tot)
    assert tot[0] >= Bg  # every env timed out at least once (max_T 100 < 230 steps)
