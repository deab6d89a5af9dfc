#!/bin/bash
# tools/output_path_probe.py under the three MPPI_DEBUG_OUT settings, 20- and 500-step batches
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in 20 500; do for o in 0 1 2 0; do
  MPPI_DEBUG_OUT=$o timeout -k 10 120 python tools/output_path_probe.py ${1:-arm_c3} $s || exit 1
done; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/output_path_${1:-arm_c3}.txt
exit ${PIPESTATUS[0]}
