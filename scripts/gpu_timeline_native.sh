#!/bin/bash
# Step timelines of the timeline build under native dispatch and under HIP launches:
#   bash scripts/gpu_timeline_native.sh <tag> <workload> [<workload> ...]
tag=${1:-dev}; shift
L=quadrotor_manipulator_mppi_amd/lib/ab/timeline.so
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in "$@"; do
  for d in aql hip; do
    MPPI_DISPATCH=$d MPPI_HIP_LIB=$L MPPI_STAMPS=1 MPPI_EVENT_WAIT=1 MPPI_DEBUG_NO_FLAG=1 \
      timeout -k 10 120 python tools/timeline_probe.py $w 40 || exit 1
  done
done 2>&1 | grep -v "amdgpu.ids\|mppi stamps" | tee gpurun_out/timeline_native_$tag.txt
exit ${PIPESTATUS[0]}
