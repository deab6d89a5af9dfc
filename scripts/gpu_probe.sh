#!/bin/bash
# Rollout diagnostics on one box: phase stamps, K sweep and launch-geometry sweep.
#   scripts/gpu_probe.sh <tag>
# Every GPU step has its own time limit; the first failure ends the script.
tag=${1:-dev}
export TMPDIR=/tmp
mkdir -p gpurun_out
L=quadrotor_manipulator_mppi_amd/lib/libmppi_hip_stamps.so
{
  MPPI_HIP_LIB=$L MPPI_STAMPS=1 timeout -k 10 120 python tools/stamp_probe.py wholebody 8192 64 || exit 1
  MPPI_HIP_LIB=$L MPPI_STAMPS=1 timeout -k 10 120 python tools/stamp_probe.py arm 4096 32 || exit 1
  timeout -k 10 200 python tools/ksweep.py wholebody 64 4096,8192,16384,32768,65536 || exit 1
  timeout -k 10 300 python tools/geom_sweep.py wholebody 8192 64 256,512,1024 256,512 || exit 1
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/probe_$tag.txt
