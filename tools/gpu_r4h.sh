# Round-4 GPU pass H: the planner / delegation / shim GPU tests on the host-loop changes, the
# host-search split, the C5 kernel trace of the bench's own C5 lines split per measurement
# (tools/c5_trace_split.py: bench vs rocprofv3 means), and three bench runs at the driver's shape.
# Usage: bash tools/gpu_r4h.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "planner or delegation or bayes or shim or greedy" > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python tools/prof_plan_gpu.py > $O/prof_plan.jsonl 2> $O/prof_plan.err || { echo PROF_FAILED; tail -20 $O/prof_plan.err; exit 1; }
cat $O/prof_plan.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5bench -o bench -- python3 bench.py --steps 20 --warmup 5 --no-per-step --no-render --no-c3 --no-planner --no-cpu-baseline > $O/c5bench.json 2> $O/c5bench.err || { echo C5BENCH_FAILED; tail -20 $O/c5bench.err; exit 1; }
python3 tools/c5_trace_split.py $(find $O/c5bench -name '*kernel_trace.csv' | head -1) $O/c5bench.json > $O/c5_trace_split.json || exit 1
find $O/c5bench -name '*kernel_stats.csv' -exec cp {} $O/c5bench_kernel_stats.csv \;
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || { echo BENCH_FAILED; tail -20 $O/bench_driver_$i.err; exit 1; }
done
echo done
