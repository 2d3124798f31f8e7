# Round 6 pass K: rocprofv3 kernel trace of tools/rollx (dispatch durations and gaps of the
# planner-shape rollout launches against the HIP-event per-launch times).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6k}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
python -c "
import sys; sys.path.insert(0, 'gym-cooking_amd')
from gym_cooking_amd import capi, levels
open('$O/c5_level.bin', 'wb').write(bytes(capi.level_desc(levels.load_level('full-divider_salad'), 4)))" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o rollx -- ./tools/rollx $O/c5_level.bin > $O/rollx.log 2>&1 || { echo ROLLX_FAILED; tail -20 $O/rollx.log; exit 1; }
head -14 $O/rollx.log
