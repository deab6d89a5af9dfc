export TMPDIR=/tmp
timeout -k 10 200 python tools/geom_sweep.py arm 4096 32 512,256 256 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python tools/geom_sweep.py arm 4096 32 1024,512 128 2>&1 | grep -v amdgpu.ids || exit 1
MPPI_HIP_LIB=$PWD/quadrotor_manipulator_mppi_amd/lib/libmppi_hip_stamps.so MPPI_STAMPS=1 timeout -k 10 120 python tools/stamp_probe.py arm 4096 32 2>&1 | grep -v amdgpu.ids
