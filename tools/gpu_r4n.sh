# Round-4 GPU pass N: the compacted likelihood kernel (OC_LIK_COMPACT, the product build): the
# likelihood parity tests, then the whole GPU suite, then the C5 kernels' A/B against the
# grouped form (tools/_ab/liboc_likgroup.so, -DOC_LIK_COMPACT=0), outputs digested.
# Usage: bash tools/gpu_r4n.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_likelihood_gpu.py -x -v --timeout 200 --timeout-method thread > $O/gputest_lik.log 2>&1 \
  || { echo LIK_FAILED; tail -40 $O/gputest_lik.log; exit 1; }
tail -1 $O/gputest_lik.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 600 python tools/bounds_ab.py --libs tools/_ab/liboc_likcompact.so tools/_ab/liboc_likgroup.so --rounds 4 > $O/lik_ab.jsonl 2> $O/lik_ab.err || { echo AB_FAILED; tail -20 $O/lik_ab.err; exit 1; }
cat $O/lik_ab.jsonl
echo done
