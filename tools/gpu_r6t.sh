# Round 6 pass T: the product library against a build with -mllvm -amdgpu-sched-strategy=max-ilp
# (tools/abx/liboc_ilp.so): step kernels (tools/step_ab.py) and the C5 kernels (tools/bounds_ab.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6t}
O=gpurun_out/$TAG
mkdir -p $O
BASE=gym-cooking_amd/gym_cooking_amd/liboc_engine.so
ILP=tools/abx/liboc_ilp.so
timeout -k 10 400 python tools/bounds_ab.py --libs $BASE $ILP --rounds 3 > $O/bounds_ab.jsonl 2> $O/bounds_ab.err || { echo BOUNDS_AB_FAILED; tail -20 $O/bounds_ab.err; exit 1; }
timeout -k 10 700 python tools/step_ab.py --libs $BASE $ILP --rounds 2 > $O/step_ab.jsonl 2> $O/step_ab.err || { echo STEP_AB_FAILED; tail -20 $O/step_ab.err; exit 1; }
echo done
