# Round 6 closing pass: GPU suite + smoke, the bench at the driver's shape under rocprofv3 (kernel
# trace + stats, every secondary line but the host-bound planner ones), the PMC traffic passes,
# the C5 counter passes (cycle fields per tools/pmc_c5_report.py's round-6 rule), then the bench
# at the driver's shape three times and at its default once.
# Usage: bash tools/gpu_r6g.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; grep -E "FAILED|Error" $O/gputest.log | head -20; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
ARGS="--steps 20 --warmup 5 --no-planner --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py $ARGS \
  > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err || { echo ROCPROF_FAILED; tail -20 $O/bench_under_rocprof.err; exit 1; }
find $O/trace -name '*kernel_stats.csv' -exec cp {} $O/bench_kernel_stats.csv \;
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 tools/pmc_probe.py > $O/pmc_fetch.log 2>&1 || { echo PMC_FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 tools/pmc_probe.py > $O/pmc_write.log 2>&1 || { echo PMC_FAILED; exit 1; }
python3 tools/pmc_report.py $O/pmc_fetch $O/pmc_write $O/pmc_traffic.json > $O/pmc_report.log || { echo PMC_REPORT_FAILED; exit 1; }
OC_C5_ORDER=grouped timeout -k 10 900 bash tools/profile_c5.sh $TAG/c5 > $O/profile_c5.log 2>&1 || { echo PROFILE_C5_FAILED; tail -20 $O/profile_c5.log; exit 1; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || { echo BENCH_FAILED; tail -20 $O/bench_driver_$i.err; exit 1; }
  python tools/bench_summary.py $O/bench_driver_$i.json
done
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_FAILED; tail -20 $O/bench_default.err; exit 1; }
python tools/bench_summary.py $O/bench_default.json
echo done
