# Round-4 GPU pass O: rows per round of the compacted likelihood (8 / 16 with 32-lane groups,
# OC_LIK_ROUND_SCALE=2) against the grouped form, C5 kernels, outputs digested; then the
# likelihood parity tests on the scale-2 build.
# Usage: bash tools/gpu_r4o.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python tools/bounds_ab.py --libs tools/_ab/liboc_likcompact.so tools/_ab/liboc_likr2.so tools/_ab/liboc_likgroup.so --rounds 3 > $O/lik_ab.jsonl 2> $O/lik_ab.err || { echo AB_FAILED; tail -20 $O/lik_ab.err; exit 1; }
cat $O/lik_ab.jsonl
cp tools/_ab/liboc_likr2.so gym-cooking_amd/gym_cooking_amd/liboc_engine.so
timeout -k 10 300 python -u -m pytest tests/test_likelihood_gpu.py tests/test_widegraph_gpu.py tests/test_manylevels_gpu.py -x -v --timeout 200 --timeout-method thread > $O/gputest_lik_r2.log 2>&1 \
  || { echo LIK_FAILED; tail -40 $O/gputest_lik_r2.log; exit 1; }
tail -1 $O/gputest_lik_r2.log
echo done
