# Round 6 pass I: the planner-shape rollout launch phase by phase (tools/rollx.hip).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6i}
O=gpurun_out/$TAG
mkdir -p $O
python -c "
import sys; sys.path.insert(0, 'gym-cooking_amd')
from gym_cooking_amd import capi, levels
open('$O/c5_level.bin', 'wb').write(bytes(capi.level_desc(levels.load_level('full-divider_salad'), 4)))" || exit 1
timeout -k 10 300 ./tools/rollx $O/c5_level.bin > $O/rollx.log 2>&1 || { echo ROLLX_FAILED; tail -20 $O/rollx.log; exit 1; }
head -12 $O/rollx.log
tail -20 $O/rollx.log
