# Round-4 GPU pass S: the GPU suite and smoke on the final tree; the compacted likelihood with each pending row's Level-0 view kept in LDS
# (OC_LIK_ROW_LDS) against the product build, C5 kernels, outputs digested; then the likelihood
# parity tests on that build.
# Usage: bash tools/gpu_r4s.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python tools/bounds_ab.py --libs tools/abx/liboc_prod.so tools/abx/liboc_likrow.so --rounds 3 > $O/lik_ab.jsonl 2> $O/lik_ab.err || { echo AB_FAILED; tail -20 $O/lik_ab.err; exit 1; }
cat $O/lik_ab.jsonl
cp tools/abx/liboc_likrow.so gym-cooking_amd/gym_cooking_amd/liboc_engine.so
timeout -k 10 300 python -u -m pytest tests/test_likelihood_gpu.py tests/test_widegraph_gpu.py tests/test_manylevels_gpu.py tests/test_widelevels_gpu.py -x -v --timeout 200 --timeout-method thread > $O/gputest_lik_row.log 2>&1 \
  || { echo LIK_FAILED; tail -40 $O/gputest_lik_row.log; exit 1; }
tail -1 $O/gputest_lik_row.log
echo done
