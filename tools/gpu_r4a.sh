# Round-4 first GPU pass: C3 step_n parity at the bench shapes (barrier hand-over, then the
# per-step LDS-flag hand-over), the loader-wave A/B, the C5 kernels' tests and counters after
# the uniform bound walk, C5 under rocprofv3, and the driver-shape bench.
# Usage: bash tools/gpu_r4a.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
LIBDIR=gym-cooking_amd/gym_cooking_amd
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_c3_stepn_gpu.py > $O/c3_barrier.log 2>&1 || { echo C3_BARRIER_FAILED; tail -30 $O/c3_barrier.log; exit 1; }
tail -1 $O/c3_barrier.log
timeout -k 10 600 $T tests/test_rollout_gpu.py tests/test_bounds_gpu.py tests/test_likelihood_gpu.py tests/test_planner_gpu.py tests/test_delegation_gpu.py > $O/c5_tests.log 2>&1 || { echo C5_TESTS_FAILED; tail -30 $O/c5_tests.log; exit 1; }
tail -1 $O/c5_tests.log
bash tools/profile_c5.sh $TAG/c5 > $O/profile_c5.log 2>&1 || { echo PROFILE_C5_FAILED; tail -20 $O/profile_c5.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5bench -o bench -- python3 bench.py --steps 20 --warmup 5 --no-per-step --no-render --no-c3 --no-planner --no-cpu-baseline > $O/c5bench.json 2> $O/c5bench.err || { echo C5BENCH_FAILED; tail -20 $O/c5bench.err; exit 1; }
timeout -k 10 600 python tools/step_ab.py --libs tools/_ab/liboc_barrier.so tools/_ab/liboc_flags.so --rounds 4 --agents 3 > $O/step_ab.jsonl 2> $O/step_ab.err || { echo AB_FAILED; tail -20 $O/step_ab.err; exit 1; }
cp $LIBDIR/liboc_engine.so /tmp/keep_engine.so && cp tools/_ab/liboc_flags.so $LIBDIR/liboc_engine.so
timeout -k 10 600 $T tests/test_c3_stepn_gpu.py > $O/c3_flags.log 2>&1 || { echo C3_FLAGS_FAILED; tail -30 $O/c3_flags.log; cp /tmp/keep_engine.so $LIBDIR/liboc_engine.so; exit 1; }
tail -1 $O/c3_flags.log
cp /tmp/keep_engine.so $LIBDIR/liboc_engine.so
for i in 1 2; do timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench_driver.jsonl 2>> $O/bench_driver.err || { echo BENCH_FAILED; tail -20 $O/bench_driver.err; exit 1; }; done
echo done
