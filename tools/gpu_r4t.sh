# Round-4 GPU pass T: 32 rows per wave round for the compacted likelihood
# (OC_LIK_ROUND_SCALE=4) against the product build, C5 kernels, outputs digested; then the likelihood
# parity tests on that build.
# Usage: bash tools/gpu_r4t.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python tools/bounds_ab.py --libs tools/abx/liboc_prod.so tools/abx/liboc_likr4.so --rounds 3 > $O/lik_ab.jsonl 2> $O/lik_ab.err || { echo AB_FAILED; tail -20 $O/lik_ab.err; exit 1; }
cat $O/lik_ab.jsonl
cp tools/abx/liboc_likr4.so gym-cooking_amd/gym_cooking_amd/liboc_engine.so
timeout -k 10 300 python -u -m pytest tests/test_likelihood_gpu.py tests/test_widegraph_gpu.py tests/test_manylevels_gpu.py tests/test_widelevels_gpu.py -x -v --timeout 200 --timeout-method thread > $O/gputest_lik_r4.log 2>&1 \
  || { echo LIK_FAILED; tail -40 $O/gputest_lik_r4.log; exit 1; }
tail -1 $O/gputest_lik_r4.log
echo done
