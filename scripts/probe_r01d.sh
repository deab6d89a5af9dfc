export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/gt.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gt.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/gt.log | head -80; exit $rc; }
timeout -k 10 100 python tools/ksweep.py arm 32 1024,4096,16384 2>&1 | grep K= || exit 1
timeout -k 10 100 python tools/ksweep.py wholebody 64 8192 2>&1 | grep K= || exit 1
timeout -k 10 100 python tools/step_rate.py arm 4096 32 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 100 python tools/step_rate.py drone 4096 32 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 100 python tools/step_rate.py wholebody 8192 64 2>&1 | grep -v amdgpu.ids || exit 1
S=$PWD/quadrotor_manipulator_mppi_amd/lib/libmppi_hip_stamps.so
MPPI_HIP_LIB=$S MPPI_STAMPS=1 timeout -k 10 60 python tools/stamp_probe.py arm 4096 32 2>&1 | grep -v amdgpu.ids
