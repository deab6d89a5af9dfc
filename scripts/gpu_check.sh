#!/bin/bash
# One GPU call: the -m gpu suite, then a bench run at the driver's shape.
#   scripts/gpu_check.sh <tag> [extra bench.py args]
# Every GPU step has its own time limit; a crash/timeout ends the script.
tag=${1:-dev}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -v -rf --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/gpu_tests_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/gpu_tests_$tag.log | tail -25
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
rc=$?; echo "bench rc=$rc"; head -c 3000 gpurun_out/bench_$tag.json
if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_$tag.err; fi
exit $rc
