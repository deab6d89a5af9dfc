#!/bin/bash
# GPU parity tests, then a same-box A/B of library builds (kernel times via tools/geom_sweep.py).
#   scripts/gpu_ab.sh <tag> <lib.so> [<lib.so> ...]
# Every GPU step has its own time limit; the first failure ends the script.
tag=${1:-dev}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread \
    > gpurun_out/gt_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gt_$tag.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" gpurun_out/gt_$tag.log | head -150; exit $rc; }
for r in 1 2; do
  for L in "$@"; do
    echo "== $L (rep $r)"
    MPPI_HIP_LIB=$L timeout -k 10 120 python tools/geom_sweep.py wholebody 8192 64 || exit 1
    MPPI_HIP_LIB=$L GEOM_V=8 timeout -k 10 120 python tools/geom_sweep.py wholebody 8192 64 || exit 1
    MPPI_HIP_LIB=$L timeout -k 10 120 python tools/geom_sweep.py arm 4096 32 || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_$tag.txt
