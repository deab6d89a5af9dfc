#!/bin/bash
# Native control calls: their parity tests, call latency (native vs HIP, and native with the
# arguments in pinned host memory), rocprof of the calls' kernels.  scripts/gpu_calls.sh <tag>
tag=${1:-dev}
export TMPDIR=/tmp
out=gpurun_out/calls_$tag
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_aql.py tests/test_gpu_flag.py -x -q --timeout 120 --timeout-method thread \
    > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $out/tests.log | head -80; exit $rc; }
timeout -k 10 150 python tools/call_probe.py hip,aql 2>&1 | grep -v amdgpu.ids | tee $out/call_probe.txt || exit 1
MPPI_AQL_CALL_HOSTMEM=1 timeout -k 10 150 python tools/call_probe.py aql 2>&1 | grep -v amdgpu.ids | tee -a $out/call_probe.txt || exit 1
cd /tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats -T --output-format csv -d $GRAFT_REPO_ROOT/$out/prof_aql -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/call_probe.py aql > /dev/null 2>&1 || exit 1
head -3 $GRAFT_REPO_ROOT/$out/prof_aql/run_kernel_stats.csv | cut -c1-120
