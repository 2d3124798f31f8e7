# Round-4 GPU pass J: the full GPU suite on the build with wide-level rendering and device-memory
# distance tables for big graphs (the narrow blob layout changed too: nearest rows before the
# distances), minus the 605-node kitchen's tests (pass K, once its fixtures are recorded).
# Usage: bash tools/gpu_r4j.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "not widegraph" > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python tools/bounds_ab.py --libs gym-cooking_amd/gym_cooking_amd/liboc_engine.so --rounds 2 > $O/c5_after.jsonl 2> $O/c5_after.err || { echo C5_FAILED; tail -20 $O/c5_after.err; exit 1; }
cat $O/c5_after.jsonl
echo done
