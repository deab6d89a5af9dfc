#!/bin/bash
# run_steps' host enqueue rate with the process on the GPU's socket vs the other one
export TMPDIR=/tmp
mkdir -p gpurun_out
{
for r in 1 2; do for c in local remote default; do
  MPPI_PROBE_CPUS=$c timeout -k 10 120 python tools/output_path_probe.py arm_c3 500 || exit 1
  MPPI_PROBE_CPUS=$c timeout -k 10 120 python tools/output_path_probe.py arm_c3 20 || exit 1
done; done
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/affinity.txt
