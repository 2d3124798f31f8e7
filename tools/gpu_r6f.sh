# Round 6 pass F: C3 stepping waves prefetching their own actions (tools/c3ahead.hip: compiler
# waits vs hand-counted vmcnt) against the loader-wave form and the no-load floor.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6f}
O=gpurun_out/$TAG
mkdir -p $O
python -c "
import sys; sys.path.insert(0, 'gym-cooking_amd')
from gym_cooking_amd import capi, levels
open('$O/c3_level.bin', 'wb').write(bytes(capi.level_desc(levels.load_level('full-divider_tl'), 3)))" || exit 1
timeout -k 10 300 ./tools/c3ahead $O/c3_level.bin > $O/c3ahead.log 2>&1 || { echo C3AHEAD_FAILED; tail -20 $O/c3ahead.log; exit 1; }
cat $O/c3ahead.log
