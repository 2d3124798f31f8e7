# Round 6 pass O: the GPU suite and one default bench line (lane-group rollout kernel).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6o}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; grep -E "FAILED|Error" $O/gputest.log | head -20; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_FAILED; tail -20 $O/bench_default.err; exit 1; }
python -c "
import json; d = json.loads(open('$O/bench_default.json').read().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac']); r = d['rollout']; print('rollout', r['ms_per_launch'], 'planner_shape', r['planner_shape'])"
