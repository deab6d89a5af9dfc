#!/bin/bash
# GPU parity tests on the production build, then an interleaved same-process A/B of builds:
#   [AB_TESTS=0] [AB_REPS=15] [AB_RUNS="wholebody 8192 64;..."] scripts/gpu_abi.sh <tag> <lib.so> ...
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
RUNS=${AB_RUNS:-"wholebody 8192 64;wholebody 8192 64 8;wholebody 65536 64;arm 4096 32"}
# the first build loaded runs measurably slower in one process (engine memory placement:
# up to ~10% on the V=8 fleet), so the A/B runs twice, in the given and in reversed order
timeout -k 10 600 python tools/ab_interleave.py ${AB_REPS:-15} "$RUNS" "$@" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_$tag.txt
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
rev=(); for x in "$@"; do rev=("$x" "${rev[@]}"); done
echo "== reversed order" | tee -a gpurun_out/ab_$tag.txt
timeout -k 10 600 python tools/ab_interleave.py ${AB_REPS:-15} "$RUNS" "${rev[@]}" 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_$tag.txt
exit ${PIPESTATUS[0]}
