# Round-4 GPU pass C: the full GPU suite (wide levels included) + smoke, the loader-wave batch
# A/B (4 / 6 / 8 steps per ring half), and the headline window with fresh vs replayed actions.
# Usage: bash tools/gpu_r4c.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; exit 1; }
timeout -k 10 600 python tools/step_ab.py --libs tools/_ab/liboc_lw4.so tools/_ab/liboc_lw6.so tools/_ab/liboc_lw8.so --rounds 3 --agents 3 > $O/step_ab_lwsteps.jsonl 2> $O/step_ab.err || { echo AB_FAILED; tail -20 $O/step_ab.err; exit 1; }
for i in 1 2; do
  for w in fresh replay; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --window-actions $w --no-per-step --no-rollout --no-render --no-planner --no-cpu-baseline >> $O/bench_window_$w.jsonl 2>> $O/bench_window.err || { echo BENCH_FAILED; tail -20 $O/bench_window.err; exit 1; }
  done
done
echo done
