# Round 6 pass D: the u16-distance kitchens (maze, corridor) on the GPU, then the whole GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6d}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_widegraph_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest_graphs.log 2>&1 \
  || { echo PYTEST_FAILED; grep -E "FAILED|Error|error" $O/gputest_graphs.log | head -20; tail -30 $O/gputest_graphs.log; exit 1; }
tail -1 $O/gputest_graphs.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; grep -E "FAILED|Error|error" $O/gputest.log | head -20; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
