#!/bin/bash
# completion-flag protocol: stress test (3000 calls per model) on the system-scope-fence build
# and on the system-scope-output-store build, then their control-call latency A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in flagwbl2 flagsys; do
  MPPI_FLAG_STRESS_N=3000 MPPI_HIP_LIB=quadrotor_manipulator_mppi_amd/lib/ab/$L.so timeout -k 10 300 \
      python -u -m pytest tests/test_gpu_flag.py -v --timeout 250 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/flag_tests_$L.log 2>&1
  echo "$L rc=$?"; grep -E "passed|failed|AssertionError: " gpurun_out/flag_tests_$L.log | tail -5
done
cd tools && timeout -k 10 300 python latency_lib_ab.py 20 ../quadrotor_manipulator_mppi_amd/lib/ab/flagwbl2.so \
    ../quadrotor_manipulator_mppi_amd/lib/ab/flagsys.so 2>&1 | grep -v amdgpu.ids | tee ../gpurun_out/flag_latency_ab.txt
