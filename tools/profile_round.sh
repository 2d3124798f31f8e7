#!/bin/bash
# Profiles for one round, run on the GPU box from the repo root:
#   tools/profile_round.sh OUT_TAG [BENCH_ARGS...]
# 1. rocprofv3 --kernel-trace --stats of bench.py at the driver's shape (default
#    --steps 20 --warmup 5, secondary lines off) -> gpurun_out/OUT_TAG/bench_*
# 2. two --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs, no trace domains) over
#    tools/pmc_probe.py -> gpurun_out/OUT_TAG/pmc_*, then tools/pmc_report.py -> pmc_traffic.json
# Each GPU step has its own time limit; the script stops at the first failure.
set -euo pipefail
TAG=${1:?tag}
shift || true
ARGS=${*:---steps 20 --warmup 5 --no-per-step --no-rollout --no-render --no-c3 --no-planner --no-cpu-baseline}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- python3 bench.py $ARGS > "$OUT/bench_under_rocprof.json" 2> "$OUT/bench_under_rocprof.err"
find "$OUT/trace" -name '*kernel_stats.csv' -exec cp {} "$OUT/bench_kernel_stats.csv" \;
find "$OUT/trace" -name '*kernel_trace.csv' -exec cp {} "$OUT/bench_kernel_trace.csv" \;
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o pmc -- python3 tools/pmc_probe.py > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o pmc -- python3 tools/pmc_probe.py > "$OUT/pmc_write.log" 2>&1
python3 tools/pmc_report.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_traffic.json" > "$OUT/pmc_report.log"
echo "profile_round $TAG done"
