#!/bin/bash
# Same-process A/B of library builds on the native dispatch path, both library orders:
#   [ABN_REPS=15] [ABN_RUNS="arm 4096 32;..."] scripts/gpu_abn.sh <tag> <lib.so> ...
tag=${1:-dev}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
RUNS=${ABN_RUNS:-"arm 4096 32;wholebody 8192 64"}
timeout -k 10 400 python tools/ab_native.py ${ABN_REPS:-15} "$RUNS" "$@" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/abn_$tag.txt
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
rev=(); for x in "$@"; do rev=("$x" "${rev[@]}"); done
echo "== reversed order" | tee -a gpurun_out/abn_$tag.txt
timeout -k 10 400 python tools/ab_native.py ${ABN_REPS:-15} "$RUNS" "${rev[@]}" 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/abn_$tag.txt
exit ${PIPESTATUS[0]}
