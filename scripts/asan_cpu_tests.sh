#!/bin/bash
# Host AddressSanitizer run of the CPU test suite (this container, no GPU):
#   scripts/asan_cpu_tests.sh [pytest args]
# Builds lib/libmppi_hip_asan.so (-Xarch_host -fsanitize=address on every translation
# unit: the C-ABI's config validation, host FK, SavGol taps, Philox restatement, the
# host dynamics) and runs `pytest -m "not gpu"` against it with the clang ASan runtime
# preloaded into python ahead of any preload already in the environment (our own process;
# python itself is not instrumented, so leak checking is off).  Any ASan report aborts the test process and fails the run.
set -e
cd "$(dirname "$0")/.."
python -m quadrotor_manipulator_mppi_amd.build --asan > /dev/null
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
LIB=$PWD/quadrotor_manipulator_mppi_amd/lib/libmppi_hip_asan.so
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1
LD_PRELOAD="$RT${LD_PRELOAD:+:$LD_PRELOAD}" MPPI_HIP_LIB=$LIB python - <<'EOF'
from quadrotor_manipulator_mppi_amd import _capi
_capi.lib()
maps = open("/proc/self/maps").read()
assert "libmppi_hip_asan.so" in maps and "libclang_rt.asan" in maps, "ASan library not mapped"
print("mapped:", _capi.LIB_PATH, "+ clang ASan runtime")
EOF
LD_PRELOAD="$RT${LD_PRELOAD:+:$LD_PRELOAD}" MPPI_HIP_LIB=$LIB timeout 900 python -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@"
