# Round-4 GPU pass E: the full GPU suite + smoke on the current build, the oc_step store-policy
# A/B (sc1, the product, vs nt; hipGraphs of 20 oc_step launches), the host-search breakdown,
# the bench at the driver's shape (twice) and at its default, and the loader wave's 16-byte
# load A/B (OC_LW_X4) with the C3 parity tests on its build.
# Usage: bash tools/gpu_r4e.sh TAG
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
timeout -k 10 300 python tools/step_ab.py --per-step --libs tools/_ab/liboc_prod.so tools/_ab/liboc_stepnt.so --rounds 3 > $O/step_ab_perstep_nt.jsonl 2> $O/step_ab_perstep.err || { echo AB_FAILED; tail -20 $O/step_ab_perstep.err; exit 1; }
timeout -k 10 300 python tools/prof_plan_gpu.py > $O/prof_plan.jsonl 2> $O/prof_plan.err || { echo PROF_FAILED; tail -20 $O/prof_plan.err; exit 1; }
cat $O/prof_plan.jsonl
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || { echo BENCH_FAILED; tail -20 $O/bench_driver_$i.err; exit 1; }
done
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_FAILED; tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 600 python tools/step_ab.py --libs tools/_ab/liboc_prod.so tools/_ab/liboc_lwx4.so --rounds 4 --agents 3 > $O/step_ab_lwx4.jsonl 2> $O/step_ab_lwx4.err || { echo AB3_FAILED; tail -20 $O/step_ab_lwx4.err; exit 1; }
cp tools/_ab/liboc_lwx4.so gym-cooking_amd/gym_cooking_amd/liboc_engine.so
timeout -k 10 600 python -u -m pytest tests/test_c3_stepn_gpu.py -x -v --timeout 300 --timeout-method thread > $O/gputest_c3_lwx4.log 2>&1 || { echo C3_LWX4_FAILED; tail -30 $O/gputest_c3_lwx4.log; exit 1; }
tail -1 $O/gputest_c3_lwx4.log
echo done
