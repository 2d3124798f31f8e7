# GPU check of a step-kernel change: the step parity tests, then tools/step_ab.py against the
# baseline build in tools/_ab/.  Usage: bash tools/gpu_step.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "parity or c4 or step or envs or greedy or dup or big or rccl or many or edge" > gpurun_out/$TAG/gputest.log 2>&1 \
  || { echo PYTEST_FAILED; tail -30 gpurun_out/$TAG/gputest.log; exit 1; }
tail -2 gpurun_out/$TAG/gputest.log
timeout -k 10 600 python tools/step_ab.py --libs tools/_ab/liboc_engine_base.so gym-cooking_amd/gym_cooking_amd/liboc_engine.so \
  --rounds 3 > gpurun_out/$TAG/step_ab.jsonl 2> gpurun_out/$TAG/step_ab.err || exit 1
