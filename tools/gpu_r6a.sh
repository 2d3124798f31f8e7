# Round 6 pass A: C3 dynamic (chunk, segment) queue experiment (tools/c3tl.hip), the GPU suite
# (rollout one-wave blocks, wide padding columns, wide multi-launch test), one bench run.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6a}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
python -c "
import sys; sys.path.insert(0, 'gym-cooking_amd')
from gym_cooking_amd import capi, levels
open('$O/c3_level.bin', 'wb').write(bytes(capi.level_desc(levels.load_level('full-divider_tl'), 3)))" || exit 1
timeout -k 10 300 ./tools/c3tl $O/c3_level.bin > $O/c3tl.log 2>&1 || { echo C3TL_FAILED; tail -20 $O/c3tl.log; exit 1; }
grep -E "us/step" $O/c3tl.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; grep -E "FAILED|Error|error" $O/gputest.log | head -20; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --no-planner > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -30 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json
