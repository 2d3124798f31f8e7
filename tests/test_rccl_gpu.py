"""RCCL on the hardware path at world size 1 (the reference's counterpart is N
independent processes, gym_cooking/runpara.ps1:44-68).

bench.py creates its "nccl" process group at every world size, so the summary all-gather
and the max-over-ranks reduction of a single-GPU run are real RCCL calls.  This test starts a
fresh child interpreter (tests/rccl_child.py; started as a subprocess, nothing is exec'd) that
joins a world-1 RCCL group, steps 2^16 envs with oc_step_n and its in-launch statistics fold,
all-gathers the summary row through RCCL and compares it with reduce_stats and with the CPU
oracle's totals: bit-exact integers.  NCCL_DEBUG=INFO makes RCCL announce itself, which the
test checks, so a silent non-RCCL path cannot pass."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_rccl_world1_allgather_of_step_n_totals():
    env = dict(os.environ, NCCL_DEBUG="INFO", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_child.py"), str(1 << 16), "130", "50"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = next(x for x in r.stdout.splitlines() if x.startswith("RESULT "))
    out = json.loads(line[len("RESULT "):])
    assert out["backend"] == "nccl" and out["world"] == 1 and out["rccl_ranks"] == 1
    assert "NCCL INFO" in r.stdout + r.stderr, "RCCL did not initialise a communicator"
    g = out["gathered"]
    assert out["direct"] and out["via_process_group"] == g
    assert len(g) == 1 and len(g[0]) == 8
    assert g[0][:5] == out["reduced"] == out["oracle"], out
    assert out["oracle"][0] > 0 and out["oracle"][3] > 0
    assert out["state_equal"]
    assert out["max"] == 3.5
    assert out["summary"]["distinct_devices"] == 1
