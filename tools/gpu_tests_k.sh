# GPU tests selected by a -k expression, then (optionally) the headline bench three times.
# Usage: bash tools/gpu_tests_k.sh TAG "<-k expr>" [bench]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}; EXPR=${2:?expr}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$EXPR" \
  > gpurun_out/$TAG/gputest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/$TAG/gputest.log; exit 1; }
tail -2 gpurun_out/$TAG/gputest.log
if [ "$3" = bench ]; then
  for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-per-step --no-rollout --no-render --no-c3 --no-planner --no-cpu-baseline >> gpurun_out/$TAG/headline.jsonl 2>> gpurun_out/$TAG/headline.err || exit 1; done
  timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/$TAG/default.jsonl 2> gpurun_out/$TAG/default.err || exit 1
fi
