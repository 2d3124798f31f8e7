# Round-4 GPU pass F: the full GPU suite on the build with the wave-compacted bounds walk, the
# bounds A/B against the per-lane walk (tools/_ab/liboc_bnd0.so: times and output digests),
# the C5 counter passes (tools/profile_c5.sh, configuration-major rows), and the window prime A/B
# (bench at the driver's shape, --prime none / step alternating).
# Usage: bash tools/gpu_r4f.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 600 python tools/bounds_ab.py --libs gym-cooking_amd/gym_cooking_amd/liboc_engine.so tools/_ab/liboc_bnd0.so --rounds 3 > $O/bounds_ab.jsonl 2> $O/bounds_ab.err || { echo AB_FAILED; tail -20 $O/bounds_ab.err; exit 1; }
cat $O/bounds_ab.jsonl
OC_C5_ORDER=grouped timeout -k 10 900 bash tools/profile_c5.sh $TAG/c5 > $O/profile_c5.log 2>&1 || { echo PROFILE_FAILED; tail -20 $O/profile_c5.log; exit 1; }
for i in 1 2 3; do
  for p in none step; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --prime $p --no-per-step --no-rollout --no-render --no-planner --no-cpu-baseline --no-c3 >> $O/bench_prime_$p.jsonl 2>> $O/bench_prime.err || { echo BENCH_FAILED; tail -20 $O/bench_prime.err; exit 1; }
  done
done
echo done
