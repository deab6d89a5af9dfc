#!/bin/bash
# Rollout phase stamps + wave timeline (stamps build):  scripts/gpu_stamps.sh <tag> "<model K H [threads nb]>" ...
tag=${1:-dev}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
L=quadrotor_manipulator_mppi_amd/lib/libmppi_hip_stamps.so
for a in "$@"; do
  MPPI_HIP_LIB=$L MPPI_STAMPS=1 timeout -k 10 120 python tools/stamp_probe.py $a || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/stamps_$tag.txt
