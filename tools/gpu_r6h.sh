# Round 6 pass H: the wide SWAR step's branch variants on the device.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r6h}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_widelevels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k variants > $O/gputest_variants.log 2>&1 \
  || { echo PYTEST_FAILED; grep -E "FAILED|Error|error" $O/gputest_variants.log | head -20; tail -30 $O/gputest_variants.log; exit 1; }
tail -1 $O/gputest_variants.log
