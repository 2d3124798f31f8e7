# Round-4 GPU pass B: the full GPU suite + smoke, C5 counters and C5 under rocprofv3 (kernel
# means per bench measurement), the driver-shape bench (2x), the default bench, and the
# headline profile (rocprofv3 stats + PMC traffic).
# Usage: bash tools/gpu_r4b.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; exit 1; }
bash tools/profile_c5.sh $TAG/c5 > $O/profile_c5.log 2>&1 || { echo PROFILE_C5_FAILED; tail -20 $O/profile_c5.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5bench -o bench -- python3 bench.py --steps 20 --warmup 5 --no-per-step --no-render --no-c3 --no-planner --no-cpu-baseline > $O/c5bench.json 2> $O/c5bench.err || { echo C5BENCH_FAILED; tail -20 $O/c5bench.err; exit 1; }
python3 tools/c5_trace_split.py $(find $O/c5bench -name '*kernel_trace.csv' | head -1) $O/c5bench.json > $O/c5_trace_split.json || exit 1
for i in 1 2; do timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench_driver.jsonl 2>> $O/bench_driver.err || { echo BENCH_FAILED; tail -20 $O/bench_driver.err; exit 1; }; done
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_DEFAULT_FAILED; exit 1; }
bash tools/profile_round.sh $TAG/prof > $O/profile_round.log 2>&1 || { echo PROFILE_ROUND_FAILED; tail -20 $O/profile_round.log; exit 1; }
echo done
