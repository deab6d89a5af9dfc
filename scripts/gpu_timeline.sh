#!/bin/bash
# Wall-clock step timelines (timeline build, tools/timeline_probe.py):
#   scripts/gpu_timeline.sh <tag> <lib.so> <workload> [<workload> ...]
tag=${1:-dev}; shift
L=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in "$@"; do
  MPPI_HIP_LIB=$L MPPI_STAMPS=1 MPPI_EVENT_WAIT=1 MPPI_DEBUG_NO_FLAG=1 timeout -k 10 120 python tools/timeline_probe.py $w 40 || exit 1
done 2>&1 | grep -v "amdgpu.ids\|mppi stamps" | tee gpurun_out/timeline_$tag.txt
exit ${PIPESTATUS[0]}
