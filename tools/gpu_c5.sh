# GPU check of the planner-table kernels after a change: their parity tests, then the bench's
# C5 lines, then the C5 counter passes (tools/profile_c5.sh).  Usage: bash tools/gpu_c5.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "rollout or bounds or likelihood or planner or delegation or dup or big or splits" > gpurun_out/$TAG/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; tail -30 gpurun_out/$TAG/gputest.log; exit 1; }
tail -2 gpurun_out/$TAG/gputest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-per-step --no-render --no-c3 --no-planner --no-cpu-baseline \
  > gpurun_out/$TAG/bench_c5.json 2> gpurun_out/$TAG/bench_c5.err || exit 1
OC_C5_ORDER=grouped bash tools/profile_c5.sh $TAG/pmc || exit 1
