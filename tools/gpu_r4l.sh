# Round-4 GPU pass L: the driver-shape window on one box, alternating the current bench, the
# round-3 bench.py (its window from a reset, the warmup replaying the timed launch; extracted
# with git show acc1784:bench.py into tools/_ab/) and the current bench with the window's own
# launch replayed before it; four runs each, headline line only.
# Usage: bash tools/gpu_r4l.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
L="--gpus 1 --steps 20 --warmup 5 --no-per-step --no-rollout --no-render --no-planner --no-cpu-baseline --no-c3"
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py $L >> $O/w_now.jsonl 2>> $O/w.err || { echo BENCH_FAILED; tail -20 $O/w.err; exit 1; }
  timeout -k 10 300 python tools/_ab/bench_r03.py $L >> $O/w_r03.jsonl 2>> $O/w.err || { echo BENCH_FAILED; tail -20 $O/w.err; exit 1; }
  timeout -k 10 300 python bench.py $L --window-actions replay >> $O/w_replay.jsonl 2>> $O/w.err || { echo BENCH_FAILED; tail -20 $O/w.err; exit 1; }
done
echo done
