# Round-4 GPU pass I: the driver-shape window, alternating: the product (auto host wait, fresh
# actions), spin host wait, and the window's own launch replayed right before it (as round 3's
# warmup did); four runs each.
# Usage: bash tools/gpu_r4i.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
L="--gpus 1 --steps 20 --warmup 5 --no-per-step --no-rollout --no-render --no-planner --no-cpu-baseline --no-c3"
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py $L >> $O/w_auto.jsonl 2>> $O/w.err || { echo BENCH_FAILED; tail -20 $O/w.err; exit 1; }
  timeout -k 10 300 python bench.py $L --host-wait spin >> $O/w_spin.jsonl 2>> $O/w.err || { echo BENCH_FAILED; tail -20 $O/w.err; exit 1; }
  timeout -k 10 300 python bench.py $L --window-actions replay >> $O/w_replay.jsonl 2>> $O/w.err || { echo BENCH_FAILED; tail -20 $O/w.err; exit 1; }
  timeout -k 10 300 python bench.py $L --window-actions replay --host-wait spin >> $O/w_replay_spin.jsonl 2>> $O/w.err || { echo BENCH_FAILED; tail -20 $O/w.err; exit 1; }
done
echo done
