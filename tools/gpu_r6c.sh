# Round 6 pass C: C3 block shapes (tools/c3tl.hip: 8 or 6 stepping waves per loader wave, launch
# bounds 6) against the product form, three alternating rounds; then the product library's
# rollout / bounds / likelihood rows (the reverted one-wave blocks) and the graph GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6c}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
python -c "
import sys; sys.path.insert(0, 'gym-cooking_amd')
from gym_cooking_amd import capi, levels
open('$O/c3_level.bin', 'wb').write(bytes(capi.level_desc(levels.load_level('full-divider_tl'), 3)))" || exit 1
timeout -k 10 400 ./tools/c3tl $O/c3_level.bin > $O/c3tl.log 2>&1 || { echo C3TL_FAILED; tail -20 $O/c3tl.log; exit 1; }
grep -E "us/step|per step: all|wave start" $O/c3tl.log
timeout -k 10 600 python -u -m pytest tests/test_widegraph_gpu.py tests/test_rollout_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "not maze and not corridor" > $O/gputest_graphs.log 2>&1 \
  || { echo PYTEST_FAILED; grep -E "FAILED|Error|error" $O/gputest_graphs.log | head -20; tail -30 $O/gputest_graphs.log; exit 1; }
tail -1 $O/gputest_graphs.log
