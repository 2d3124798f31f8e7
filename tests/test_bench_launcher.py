"""bench.py --gpus N without a torchrun wrapper starts N ranks itself (fresh child processes that
join a TCPStore the parent hosts on 127.0.0.1, port chosen at bind).  Run here on CPU with the
gloo self-test mode: every rank reports its env shard through the same all-gather the bench
uses, and runs the bench's timed_window with recording stand-ins, which pins what the timed
region holds at N > 1."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _selftest(n):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--batch", "4096",
                          "--cpu-budget", "1", "--selftest-ranks"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 alone prints
    return json.loads(lines[0])


def test_bench_gpus_2_starts_two_ranks():
    d = _selftest(2)
    assert d["n_gpus"] == 2
    ranks = d["ranks"]
    assert [r[0] for r in ranks] == [0, 1] and all(r[1] == 2 for r in ranks)
    assert [(r[2], r[3]) for r in ranks] == [(0, 4096), (4096, 4096)]  # contiguous global-id shards
    assert ranks[0][4] != ranks[1][4]  # two processes


def test_bench_line_at_2_ranks_has_cpu_baseline():
    """SURVEY 8(d) asks for the CPU path timed beside every line: at N > 1 too, rank 0 times the
    C restatement on its share of the job's host cores over one shard's workload."""
    d = _selftest(2)
    cb = d["cpu_baseline"]
    assert cb is not None and cb["value"] > 0 and cb["kind"] == "port"
    assert cb["cores"] >= 1 and cb["ranks_sharing_the_job_cores"] == 2
    assert "4096 envs" in cb["sample"]


def test_timed_window_holds_launches_gather_sync_only():
    """Between the two clock reads: the launches, the all-gather and the synchronize, in that
    order.  The barriers sit outside (entry barrier before the first read, closing barrier
    after the second), and the gather really ran across both ranks."""
    d = _selftest(2)
    tr = d["window_trace"]
    assert tr == ["barrier", "synchronize", "clock", "launch", "launch", "all_gather", "synchronize", "clock",
                  "barrier"], tr
    i0, i1 = tr.index("clock"), len(tr) - 1 - tr[::-1].index("clock")
    assert "barrier" not in tr[i0:i1]
    assert [r[0] for r in d["window_gathered"]] == [0, 1]


def test_timed_window_in_process():
    """The same function at world 1 with plain stand-ins: the elapsed time is the span between
    the clock reads, and the barrier after the closing read is not timed."""
    import bench
    ticks = iter([10.0, 12.5])
    calls = []
    dt, g = bench.timed_window([lambda: calls.append("L")], lambda: "G", lambda: calls.append("S"),
                               lambda: calls.append("B"), clock=lambda: next(ticks))
    assert dt == 2.5 and g == "G" and calls == ["B", "S", "L", "S", "B"]


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--selftest-ranks"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE 1" in out.stderr
