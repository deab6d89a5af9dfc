#!/bin/bash
# parity tests, then an optional tool command:  scripts/gpu_quick.sh <tag> [cmd...]
tag=${1:-dev}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/gt_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gt_$tag.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" gpurun_out/gt_$tag.log | head -120; exit $rc; }
if [ $# -gt 0 ]; then timeout -k 10 400 "$@" 2>&1 | grep -v amdgpu.ids; fi
