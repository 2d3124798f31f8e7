# Round-4 GPU pass D: the planner / delegation GPU tests, the host-search breakdown
# (tools/prof_plan_gpu.py), the world-1 summary gather's cost, two default bench runs, and the
# staggered loader-wave hand-over A/B (OC_LW_STAGGER) with the C3 parity tests on its build.
# Usage: bash tools/gpu_r4d.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "planner or delegation or bayes" > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python tools/prof_plan_gpu.py > $O/prof_plan.jsonl 2> $O/prof_plan.err || { echo PROF_FAILED; tail -20 $O/prof_plan.err; exit 1; }
cat $O/prof_plan.jsonl
timeout -k 10 120 python - > $O/gather_probe.json 2>&1 <<'PY' || { echo PROBE_FAILED; cat $O/gather_probe.json; exit 1; }
import json, os, sys, torch
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "gym-cooking_amd")]
from gym_cooking_amd import dist as ocdist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
ocdist.init("nccl")
dev = torch.device("cuda:0")
allr, row = ocdist.summary_rows(8, dev)
for _ in range(20):
    ocdist.gather_summaries(row, allr)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(200):
    ocdist.gather_summaries(row, allr)
e1.record()
torch.cuda.synchronize()
print(json.dumps({"gather_us": e0.elapsed_time(e1) / 200 * 1e3, "rccl": ocdist.rccl() is not None}))
PY
cat $O/gather_probe.json
for i in 1 2; do
  timeout -k 10 600 python bench.py > $O/bench_default_$i.json 2> $O/bench_default_$i.err || { echo BENCH_FAILED; tail -20 $O/bench_default_$i.err; exit 1; }
done
timeout -k 10 600 python tools/step_ab.py --libs tools/_ab/liboc_stag0.so tools/_ab/liboc_stag1.so --rounds 4 --agents 3 > $O/step_ab_stagger.jsonl 2> $O/step_ab_stagger.err || { echo AB_FAILED; tail -20 $O/step_ab_stagger.err; exit 1; }
timeout -k 10 300 python tools/step_ab.py --per-step --libs tools/_ab/liboc_stag0.so tools/_ab/liboc_stepnt.so --rounds 3 > $O/step_ab_perstep_nt.jsonl 2> $O/step_ab_perstep.err || { echo AB2_FAILED; tail -20 $O/step_ab_perstep.err; exit 1; }
cp tools/_ab/liboc_stag1.so gym-cooking_amd/gym_cooking_amd/liboc_engine.so
timeout -k 10 600 python -u -m pytest tests/test_c3_stepn_gpu.py -x -v --timeout 300 --timeout-method thread > $O/gputest_c3_stag1.log 2>&1 || { echo C3_STAG1_FAILED; tail -30 $O/gputest_c3_stag1.log; exit 1; }
tail -1 $O/gputest_c3_stag1.log
echo done
