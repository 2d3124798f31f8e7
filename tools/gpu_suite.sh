set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; exit 1; }
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-per-step --no-rollout --no-render --no-c3 --no-planner --no-cpu-baseline >> gpurun_out/headline.jsonl 2>> gpurun_out/headline.err || exit 1; done
timeout -k 10 200 python tools/rccl_window_ab.py --reps 300 > gpurun_out/rccl_ab.json 2> gpurun_out/rccl_ab.err
