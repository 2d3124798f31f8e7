#!/bin/bash
# oc_step_n under the compiler's scheduling strategies (run on the GPU box from the repo root):
# tools/stepnexp.hip built with the default scheduler and with -mllvm --amdgpu-sched-strategy=S,
# each binary run on the same shapes, twice in alternating order; prints the product lines.
set -euo pipefail
OUT=${1:-gpurun_out/sched}
mkdir -p "$OUT"
STRATS="default max-ilp iterative-ilp max-memory-clause"
for s in $STRATS; do
  flag=""
  [ "$s" != default ] && flag="-mllvm --amdgpu-sched-strategy=$s"
  /opt/rocm/bin/hipcc -O3 -std=c++20 --offload-arch=gfx950 $flag -o /tmp/stepnexp_$s tools/stepnexp.hip
done
for round in 1 2; do
  for s in $STRATS; do
    for shape in "20 2" "100 2" "20 3"; do
      echo "== $s $shape round $round" >> "$OUT/sched.log"
      timeout -k 10 120 /tmp/stepnexp_$s $shape > "$OUT/tmp.log" 2>&1
      grep -E "^product oc_step_n|totals fold|identical|DIFFER" "$OUT/tmp.log" >> "$OUT/sched.log"
    done
  done
done
echo "sched_ab done"
