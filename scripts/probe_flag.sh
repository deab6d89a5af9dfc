#!/bin/bash
# completion-flag protocol stress test (3000 calls per model) on the system-scope-fence build and on
# the store-acknowledgment build
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in flagwbl2 flagack; do
  MPPI_FLAG_STRESS_N=3000 MPPI_HIP_LIB=quadrotor_manipulator_mppi_amd/lib/ab/$L.so timeout -k 10 300 \
      python -u -m pytest tests/test_gpu_flag.py -v --timeout 250 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/flag_tests_$L.log 2>&1
  echo "$L rc=$?"; grep -E "passed|failed|AssertionError: " gpurun_out/flag_tests_$L.log | tail -5
done
exit 0
