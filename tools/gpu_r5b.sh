# Round 5 pass B: the rollout experiment (tools/rolltl.hip): variants and per-configuration cost.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5b}
mkdir -p $O
timeout -k 10 300 ./tools/rolltl > $O/rolltl.log 2>&1 || { echo ROLLTL_FAILED; tail -20 $O/rolltl.log; exit 1; }
cat $O/rolltl.log
