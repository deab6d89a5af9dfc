export TMPDIR=/tmp
S=$PWD/quadrotor_manipulator_mppi_amd/lib/libmppi_hip_stamps.so
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/gt.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gt.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/ksweep.py arm 32 1024,4096,8192,16384 > gpurun_out/ks.txt 2>&1 && grep K= gpurun_out/ks.txt || exit 1
timeout -k 10 120 python tools/ksweep.py wholebody 64 2048,8192 > gpurun_out/ks.txt 2>&1 && grep K= gpurun_out/ks.txt || exit 1
for args in "arm 4096 32" "wholebody 8192 64"; do
  MPPI_HIP_LIB=$S MPPI_STAMPS=1 timeout -k 10 60 python tools/stamp_probe.py $args > gpurun_out/st.txt 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/st.txt
done
timeout -k 10 300 python bench.py --secondary "" --cpu-budget 2 > gpurun_out/b.json 2> gpurun_out/b.err; rc=$?; cat gpurun_out/b.json; exit $rc
