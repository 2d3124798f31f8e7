"""GPU parity of the C3 product kernel at its own shapes (BASELINE configs[2]).

C3 is 3-agent full-divider_tl; oc_step_n runs it as oc_step_n_kernel<3,4> with the loader wave
(a fifth wave per block that fills an LDS ring with the next steps' action words; DESIGN.md
3.2).  Checked against the 16-thread CPU oracle, byte for byte:

* the bench shape: 2^20 envs, 100-step launches (the bench's c3 line is one such launch),
  over 240 steps so that the t = 100 timeouts and the auto-resets after them fall inside
  launches;
* past one chunk per block: B = 2^20 + 2^18 + 17 envs.  The launcher caps the grid at 4
  blocks per CU (1,024 envs each), so on a 256-CU MI355X a quarter of the blocks step a second
  chunk: the loader's end-of-chunk hand-over and the ring refill for the next chunk run.  The
  batch is ragged (17 envs into the last 4,096-env page).  37-step launches (not a multiple
  of the ring's 4-step batches) and max_T = 7, so timeouts and auto-resets land mid-batch.

Every trajectory state, executed-action plane and collision mask of every step, the folded
totals of every launch, the final state and the reduced statistics.  Integer state:
bit-exact, no tolerance.  Reference: overcooked_environment.py:255-306.
"""
import numpy as np
import pytest

import oc_testlib as tl

from oracle import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

LEVEL, A = "full-divider_tl", 3


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from gym_cooking_amd import engine  # noqa: F401  (loads liboc_engine.so or raises)
    return torch.device("cuda:0")


def _segments(total, n):
    return [(i, min(n, total - i)) for i in range(0, total, n)]


def run_step_n_vs_oracle(dev, level, A, B, max_T, n, steps, seed):
    """oc_step_n launches of n steps (the last one shorter) against the oracle, every output
    of every step; returns (totals, resets seen)."""
    from gym_cooking_amd.engine import OvercookedBatch
    eb = OvercookedBatch(level, A, B, max_T=max_T, device=dev)
    P, S = eb.pitch, eb.layout.state_bytes
    ob = oracle.OracleBatch(eb.level, A, max_T, B)
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
        eb.step_n(s, s2, acts[:m].reshape(-1), m, traj, ex, coll, stats, totals)
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
            got = tl.env_view(h_traj[r], A, ob.K, P, B)  # envs [0, B): the pitch's padding is unspecified
            want = tl.env_view(c, A, ob.K, P, B)
            if not np.array_equal(got, want):
                bad = np.argwhere(got != want)
                raise AssertionError("trajectory state differs at step %d (launch of %d from %d): %d bytes, first "
                                     "(plane, env) %s" % (t, m, i0, len(bad), bad[:4].tolist()))
            assert np.array_equal(h_ex[r].reshape(A, P)[:, :B], cex.reshape(A, P)[:, :B]), "exec at step %d" % t
            assert np.array_equal(h_coll[r][:B], ccoll[:B]), "collision mask at step %d" % t
        assert np.array_equal(totals.cpu().numpy(), tot), ("in-launch totals after step", i0 + m)
    fin = tl.env_view(s.cpu().numpy(), A, ob.K, P, B)
    assert np.array_equal(fin, tl.env_view(c, A, ob.K, P, B)), "final state"
    got = eb.reduce_stats(stats).cpu().numpy()
    assert np.array_equal(got, tot), (got, tot)
    return tot, resets


def test_c3_bench_shape_100_step_launches(dev):
    """C3 as the bench launches it: 2^20 envs, 100-step launches (100 / 100 / 40 steps)."""
    B = 1 << 20
    tot, resets = run_step_n_vs_oracle(dev, LEVEL, A, B, 100, 100, 240, seed=3)
    assert resets >= B, "expected the auto-reset wave after the t = 100 timeouts, saw %d resets" % resets
    assert tot[0] >= B and tot[3] > 0


def test_c3_two_chunks_per_block_ragged_short_episodes(dev):
    """B past one grid pass (2^20 + 2^18 + 17 envs): a quarter of the blocks step two chunks,
    the loader refills the ring across the chunk boundary; 37-step launches, max_T = 7."""
    B = (1 << 20) + (1 << 18) + 17
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    blocks_needed = -(-B // 4096) * 4096 // 1024
    assert blocks_needed > 4 * cus, "batch must need more than one pass of the 4-blocks-per-CU grid"
    tot, resets = run_step_n_vs_oracle(dev, LEVEL, A, B, 7, 37, 111, seed=17)
    assert resets >= 10 * (B // 2), "expected many mid-launch auto-resets, saw %d" % resets
    assert tot[0] > 0 and tot[3] > 0


def test_c3_single_launch_many_chunks(dev):
    """4 chunks per block in one launch (B = 2^22 + 4,095 on 256 CUs), 13 steps."""
    B = (1 << 22) + 4095
    run_step_n_vs_oracle(dev, LEVEL, A, B, 5, 13, 13, seed=29)
