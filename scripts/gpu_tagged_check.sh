export TMPDIR=/tmp
mkdir -p gpurun_out/tagged
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tagged/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/tagged/gpu_tests.log; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" gpurun_out/tagged/gpu_tests.log | head -120; exit $rc; }
MPPI_AQL_PROFILE=1 timeout -k 10 200 python tools/call_split_probe.py > gpurun_out/tagged/call_split.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/tagged/call_split.txt | grep -v "call setup\|step_call" | tail -8
timeout -k 10 150 python tools/call_probe.py hip,aql 2>&1 | grep -v amdgpu.ids > gpurun_out/tagged/call_probe.txt || exit 1
tail -8 gpurun_out/tagged/call_probe.txt
