# drop-in control-call latency beside Engine.step and the bare C call, in one process each
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/call_split_probe.py 2>&1 | grep -v "amdgpu.ids\|\[mppi" > gpurun_out/dropin_probe.txt || exit 1
timeout -k 10 200 python -c "
import bench
for i in range(3): print('dropin_latency', bench.dropin_latency(200))
" >> gpurun_out/dropin_probe.txt 2>&1 || exit 1
cat gpurun_out/dropin_probe.txt
