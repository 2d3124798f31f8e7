# Round 6 pass B: (1) the window launched as one hipGraph vs one call per launch, alternating
# processes at the driver's shape (headline only); (2) rollout one-wave blocks for launches
# under 16 Ki rows vs 256-lane blocks everywhere (tools/bounds_ab.py, same box).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6b}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
FLAGS="--gpus 1 --steps 20 --warmup 5 --no-per-step --no-rollout --no-render --no-c3 --no-wide --no-planner --no-cpu-baseline"
for r in 1 2 3; do
  for m in graph call; do
    timeout -k 10 300 python bench.py $FLAGS --window-launch $m > $O/win_${m}_$r.json 2> $O/win_${m}_$r.err || { echo BENCH_FAILED $m; tail -30 $O/win_${m}_$r.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/win_${m}_$r.json')); r=d['roofline']
print('$m', $r, '%.4g' % d['value'], 'win %.1f us' % (d['ms_per_step']*20e3), 'kernel %.2f us' % (r['kernel_ms_mean']*1e3), 'wall %.3f cold %.3f' % (r['frac_wall'], r['frac_wall_cold']))"
  done
done
timeout -k 10 600 python tools/bounds_ab.py --libs gym-cooking_amd/gym_cooking_amd/liboc_engine.so tools/ab_libs/lib_roll256.so --rounds 3 > $O/ab_roll_small.jsonl 2> $O/ab_roll_small.err || { echo AB_FAILED; tail -20 $O/ab_roll_small.err; exit 1; }
cat $O/ab_roll_small.jsonl
timeout -k 10 600 python -u -m pytest tests/test_widegraph_gpu.py tests/test_widelevels_gpu.py tests/test_biglevels_gpu.py tests/test_rollout_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "not maze" > $O/gputest_graphs.log 2>&1 \
  || { echo PYTEST_FAILED; grep -E "FAILED|Error|error" $O/gputest_graphs.log | head -20; tail -30 $O/gputest_graphs.log; exit 1; }
tail -1 $O/gputest_graphs.log
