#!/bin/bash
# Counter passes for the C5 kernels (oc_rollout / oc_bounds / oc_likelihood) and the headline
# step kernel, run on the GPU box from the repo root:
#   [OC_C5_ORDER=grouped] tools/profile_c5.sh OUT_TAG
#   PROBE="python3 tools/pmc_render_probe.py" tools/profile_c5.sh OUT_TAG   (the render kernel)
# One rocprofv3 --pmc pass per counter group (SQ <= 8, TCC FETCH_SIZE or WRITE_SIZE alone,
# GRBM <= 2), no trace domains, each under its own time limit; then tools/pmc_c5_report.py.
set -euo pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PROBE=${PROBE:-python3 tools/pmc_c5_probe.py}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o c5 -- $PROBE > "$OUT/trace.log" 2>&1
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o pmc -- $PROBE > "$OUT/$name.log" 2>&1
}
pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
pass p2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE
pass p3 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VMEM
pass p4 FETCH_SIZE
pass p5 WRITE_SIZE
python3 tools/pmc_c5_report.py "$OUT" > "$OUT/pmc_c5.json"
echo "profile_c5 $TAG done"
