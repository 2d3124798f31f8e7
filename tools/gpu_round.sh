# End-of-milestone GPU pass: full GPU suite + smoke, the driver-shape bench (3x), the full
# default-shape bench, and tools/profile_round.sh (rocprofv3 stats + PMC traffic).
# Usage: bash tools/gpu_round.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; exit 1; }
for i in 1 2 3; do timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench_driver.jsonl 2>> $O/bench_driver.err || exit 1; done
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
bash tools/profile_round.sh $TAG/prof || exit 1
