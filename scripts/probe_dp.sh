#!/bin/bash
# GPU tests, A/B of the kernel pair, then run_steps batches (GPU/enqueue/wall) per library
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_REPS=11 AB_RUNS="arm 4096 32;wholebody 8192 64;drone 4096 32" bash scripts/gpu_abi.sh dp "$@" || exit 1
for s in 20 500; do for L in "$@" "$@"; do
  echo "== $L"; MPPI_HIP_LIB=$L timeout -k 10 120 python tools/output_path_probe.py arm_c3 $s || exit 1
done; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/dp_runsteps.txt
exit ${PIPESTATUS[0]}
