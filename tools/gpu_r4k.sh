# Round-4 GPU pass K (closing measurements of the final build): the full GPU suite + smoke, the
# headline rocprofv3 kernel trace and PMC traffic passes (tools/profile_round.sh), the C5
# counter passes (configuration-major rows), the host-search split, and the bench at the
# driver's shape (three runs) and at its default.
# Usage: bash tools/gpu_r4k.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 900 bash tools/profile_round.sh $TAG/round > $O/profile_round.log 2>&1 || { echo PROFILE_FAILED; tail -20 $O/profile_round.log; exit 1; }
OC_C5_ORDER=grouped timeout -k 10 900 bash tools/profile_c5.sh $TAG/c5 > $O/profile_c5.log 2>&1 || { echo PROFILE_C5_FAILED; tail -20 $O/profile_c5.log; exit 1; }
timeout -k 10 300 python tools/prof_plan_gpu.py > $O/prof_plan.jsonl 2> $O/prof_plan.err || { echo PROF_FAILED; tail -20 $O/prof_plan.err; exit 1; }
cat $O/prof_plan.jsonl
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || { echo BENCH_FAILED; tail -20 $O/bench_driver_$i.err; exit 1; }
done
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_FAILED; tail -20 $O/bench_default.err; exit 1; }
echo done
