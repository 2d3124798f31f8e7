# Round 5 pass D: C3 block-shape variants (tools/c3tl.hip), the rollout phase timeline
# (tools/rolltl.hip), and an A/B of the C5 kernels: node-distance table (round 4) vs Floor table.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r5d}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
python -c "
import sys; sys.path.insert(0, 'gym-cooking_amd')
from gym_cooking_amd import capi, levels
open('$O/c3_level.bin', 'wb').write(bytes(capi.level_desc(levels.load_level('full-divider_tl'), 3)))" || exit 1
timeout -k 10 300 ./tools/c3tl $O/c3_level.bin > $O/c3tl.log 2>&1 || { echo C3TL_FAILED; tail -20 $O/c3tl.log; exit 1; }
grep -E "us/step|per step: all|wave start" $O/c3tl.log
timeout -k 10 300 ./tools/rolltl > $O/rolltl.log 2>&1 || { echo ROLLTL_FAILED; tail -20 $O/rolltl.log; exit 1; }
grep -E "phases|product \(oc" $O/rolltl.log
timeout -k 10 600 python tools/bounds_ab.py --libs tools/ab_libs/lib_nodetable.so tools/ab_libs/lib_floor.so --rounds 3 > $O/ab_floor.jsonl 2> $O/ab_floor.err || { echo AB_FAILED; tail -20 $O/ab_floor.err; exit 1; }
cat $O/ab_floor.jsonl
