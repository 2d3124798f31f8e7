# Round 6 pass E: the wide SWAR step (ocsw::step4w) on the GPU: the wide-level tests, then the
# bench's wide line twice (headline + wide only).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6e}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_widelevels_gpu.py tests/test_widegraph_gpu.py tests/test_maxt.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest_wide.log 2>&1 \
  || { echo PYTEST_FAILED; grep -E "FAILED|Error|error" $O/gputest_wide.log | head -20; tail -30 $O/gputest_wide.log; exit 1; }
tail -1 $O/gputest_wide.log
FLAGS="--gpus 1 --steps 20 --warmup 5 --no-per-step --no-rollout --no-render --no-c3 --no-planner --no-cpu-baseline"
for r in 1 2; do
  timeout -k 10 300 python bench.py $FLAGS > $O/bench_$r.json 2> $O/bench_$r.err || { echo BENCH_FAILED; tail -30 $O/bench_$r.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/bench_$r.json')); w=d['wide']
print('wide', w['ms_per_step']*1e3, 'us/step frac', w['frac_hbm'], 'headline', '%.4g' % d['value'])"
done
