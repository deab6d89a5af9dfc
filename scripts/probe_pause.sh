#!/bin/bash
# run_steps batches of 20: plain, with a host pause, with a host busy loop after each batch's sync
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for v in "0 0" "2 0" "0 2" "0 0"; do
  set -- $v
  MPPI_PROBE_PAUSE_MS=$1 MPPI_PROBE_SPIN_MS=$2 timeout -k 10 120 python tools/output_path_probe.py arm_c3 20 || exit 1
done; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/pause.txt
exit ${PIPESTATUS[0]}
