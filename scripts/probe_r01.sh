export TMPDIR=/tmp
S=$PWD/quadrotor_manipulator_mppi_amd/lib/libmppi_hip_stamps.so
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/gt_split.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/gt_split.log
timeout -k 10 120 python tools/ksweep.py arm 32 1024,4096,8192,16384 > gpurun_out/ks_split.txt 2>&1 && cat gpurun_out/ks_split.txt | grep K=
for args in "arm 4096 32" "arm 4096 32 256" "arm 1024 32" "drone 4096 32" "wholebody 8192 64"; do
  MPPI_HIP_LIB=$S MPPI_STAMPS=1 timeout -k 10 60 python tools/stamp_probe.py $args > gpurun_out/st.txt 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/st.txt
done
