# Round 6 pass W: the node-to-square table for oc_subtask_bounds / oc_nav_likelihood at every
# launch size (tools/abx/liboc_sq.so, -DOC_SQ_GATE_ALL=0) against the product (gated like oc_rollout).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6w}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python tools/bounds_ab.py --libs gym-cooking_amd/gym_cooking_amd/liboc_engine.so tools/abx/liboc_sq.so --rounds 3 > $O/bounds_ab.jsonl 2> $O/bounds_ab.err || { echo BOUNDS_AB_FAILED; tail -20 $O/bounds_ab.err; exit 1; }
echo done
