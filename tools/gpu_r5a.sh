set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/rolltl > $O/rolltl.log 2>&1 || { echo ROLLTL_FAILED; tail -20 $O/rolltl.log; exit 1; }
cat $O/rolltl.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --no-planner --no-render > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -30 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'wall', d['roofline']['frac_wall'], 'cold', d['roofline']['frac_wall_cold'])
print('c3', {k: d['c3'][k] for k in ('ms_per_step','frac_hbm','ms_per_launch_each','replay_from_reset')})
print('wide', {k: d['wide'][k] for k in ('ms_per_step','frac_hbm','state_bytes')})
r=d['rollout']; print('rollout', r['ms_per_launch'], r['planner_shape'], r['likelihood']['ms_per_launch'], r['subtask_bounds']['ms_per_launch'])
"
