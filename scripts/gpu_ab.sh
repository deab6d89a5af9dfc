#!/bin/bash
# Same-box A/B of library builds (kernel times via tools/geom_sweep.py), optionally after
# the GPU parity tests.
#   [AB_TESTS=1] [AB_RUNS="wholebody 8192 64;..."] scripts/gpu_ab.sh <tag> <lib.so> [<lib.so> ...]
# Every GPU step has its own time limit; the first failure ends the script.
tag=${1:-dev}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${AB_TESTS:-1}" = 1 ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread \
      > gpurun_out/gt_$tag.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gt_$tag.log
  [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" gpurun_out/gt_$tag.log | head -150; exit $rc; }
fi
RUNS=${AB_RUNS:-"wholebody 8192 64;V8 wholebody 8192 64;arm 4096 32"}
LIBS=("$@")
for r in 1 2; do
  for L in "${LIBS[@]}"; do
    echo "== $L (rep $r)"
    IFS=';' read -ra RS <<< "$RUNS"
    for run in "${RS[@]}"; do
      read -ra A <<< "$run"
      if [ "${A[0]}" = V8 ]; then A=("${A[@]:1}"); GV=8; else GV=1; fi
      MPPI_CAPI_LENIENT=1 MPPI_HIP_LIB=$L GEOM_V=$GV timeout -k 10 120 python tools/geom_sweep.py "${A[@]}" || exit 1
    done
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_$tag.txt
