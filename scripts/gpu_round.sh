#!/bin/bash
# GPU check used with gpurun: parity tests, bench, rocprofv3 kernel stats.
#   scripts/gpu_round.sh <tag> [extra bench.py args]
# Every GPU step has its own time limit; a crash/timeout stops the script.
tag=${1:-dev}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests_$tag.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$tag.json
if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_$tag.err; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_$tag -o run -- \
    python3 bench.py --no-cpu-baseline --secondary "" --latency-steps 0 "$@" > gpurun_out/prof_$tag.json 2> gpurun_out/prof_$tag.err
rc=$?; echo "prof rc=$rc"; cat gpurun_out/prof_$tag/run_kernel_stats.csv
exit $rc
