# Round 6 pass Z: the agent-pair table also in the likelihood and rollout kernels
# (tools/abx/liboc_pt.so, -DOC_PT_LIK=1 -DOC_PT_ROLL=1) against the product (bounds only).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6z}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python tools/bounds_ab.py --libs gym-cooking_amd/gym_cooking_amd/liboc_engine.so tools/abx/liboc_pt.so --rounds 3 > $O/bounds_ab.jsonl 2> $O/bounds_ab.err || { echo BOUNDS_AB_FAILED; tail -20 $O/bounds_ab.err; exit 1; }
echo done
