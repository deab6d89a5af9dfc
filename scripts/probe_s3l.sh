export TMPDIR=/tmp
for T in 512 256 128; do
  if [ $T = 512 ]; then export MPPI_HIP_LIB=$PWD/quadrotor_manipulator_mppi_amd/lib/libmppi_hip.so; else export MPPI_HIP_LIB=$PWD/quadrotor_manipulator_mppi_amd/lib/libmppi_hip_fin$T.so; fi
  echo "== finalize threads $T"
  timeout -k 10 100 python tools/geom_sweep.py arm 4096 32 0 0 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 100 python tools/geom_sweep.py drone 4096 32 0 0 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 100 python tools/geom_sweep.py wholebody 8192 64 0 0 2>&1 | grep -v amdgpu.ids || exit 1
  GEOM_V=8 timeout -k 10 100 python tools/geom_sweep.py wholebody 8192 64 0 0 2>&1 | grep -v amdgpu.ids || exit 1
done
