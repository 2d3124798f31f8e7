# Round 6 pass S: tools/rollx.hip built with AMDGPU scheduler options (rollx_base / _ilp2 / _bias0).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6s}
O=gpurun_out/$TAG
mkdir -p $O
python -c "
import sys; sys.path.insert(0, 'gym-cooking_amd')
from gym_cooking_amd import capi, levels
open('$O/c5_level.bin', 'wb').write(bytes(capi.level_desc(levels.load_level('full-divider_salad'), 4)))" || exit 1
for v in base ilp2 bias0 base; do
  echo "== $v" >> $O/rollx.log
  timeout -k 10 120 ./tools/rollx_$v $O/c5_level.bin >> $O/rollx.log 2>&1 || { echo ROLLX_FAILED $v; tail -20 $O/rollx.log; exit 1; }
done
grep -E "^==|product \(|quads: bound split" $O/rollx.log
