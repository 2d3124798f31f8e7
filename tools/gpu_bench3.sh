set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/k16b
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-per-step --no-rollout --no-render --no-c3 --no-planner --no-cpu-baseline >> gpurun_out/k16b/headline.jsonl 2>> gpurun_out/k16b/headline.err || exit 1; done
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/k16b/default.jsonl 2> gpurun_out/k16b/default.err || exit 1
