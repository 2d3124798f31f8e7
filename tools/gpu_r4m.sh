# Round-4 GPU pass M: the driver-shape window on one box, alternating the current bench with the
# runtime's default host wait (fresh actions, and the window's own launch replayed before it)
# and the round-3 bench.py; four runs each, headline line only.
# Usage: bash tools/gpu_r4m.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
L="--gpus 1 --steps 20 --warmup 5 --no-per-step --no-rollout --no-render --no-planner --no-cpu-baseline --no-c3"
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py $L --host-wait auto >> $O/w_auto.jsonl 2>> $O/w.err || { echo BENCH_FAILED; tail -20 $O/w.err; exit 1; }
  timeout -k 10 300 python tools/_ab/bench_r03.py $L >> $O/w_r03.jsonl 2>> $O/w.err || { echo BENCH_FAILED; tail -20 $O/w.err; exit 1; }
  timeout -k 10 300 python bench.py $L --host-wait auto --window-actions replay >> $O/w_auto_replay.jsonl 2>> $O/w.err || { echo BENCH_FAILED; tail -20 $O/w.err; exit 1; }
  timeout -k 10 300 python bench.py $L >> $O/w_spin.jsonl 2>> $O/w.err || { echo BENCH_FAILED; tail -20 $O/w.err; exit 1; }
done
echo done
