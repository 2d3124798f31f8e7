"""bench.py --gpus N without a torchrun wrapper starts N ranks itself (fresh child processes of
torch.distributed.run, rendezvous on 127.0.0.1).  Run here on CPU with the gloo self-test
mode: every rank reports its env shard through the same all-gather the bench uses."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus_2_starts_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch", "4096",
                          "--selftest-ranks"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    ranks = d["ranks"]
    assert [r[0] for r in ranks] == [0, 1] and all(r[1] == 2 for r in ranks)
    assert [(r[2], r[3]) for r in ranks] == [(0, 4096), (4096, 4096)]  # contiguous global-id shards
    assert ranks[0][4] != ranks[1][4]  # two processes


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--selftest-ranks"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE 1" in out.stderr
