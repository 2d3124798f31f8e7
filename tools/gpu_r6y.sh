# Round 6 pass Y: the agent-pair table in oc_bounds_kernel: C5 timings and output digest
# (tools/bounds_ab.py, compared with pass W's digest), then the GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6y}
O=gpurun_out/$TAG
mkdir -p $O
LIB=gym-cooking_amd/gym_cooking_amd/liboc_engine.so
timeout -k 10 300 python tools/bounds_ab.py --libs $LIB $LIB --rounds 2 > $O/bounds_ab.jsonl 2> $O/bounds_ab.err || { echo BOUNDS_AB_FAILED; tail -20 $O/bounds_ab.err; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; grep -E "FAILED|Error" $O/gputest.log | head -20; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
