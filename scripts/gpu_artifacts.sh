#!/bin/bash
# Round artifacts: GPU tests, bench lines (arm C3 + secondaries, fleet C5), rocprofv3 kernel
# stats, PMC traffic passes.  scripts/gpu_artifacts.sh <tag>
tag=${1:-dev}
export TMPDIR=/tmp
mkdir -p gpurun_out/art_$tag
o=gpurun_out/art_$tag
timeout -k 10 300 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $o/bench_arm_c3.json 2> $o/bench_arm_c3.err
rc=$?; echo "bench rc=$rc"; cat $o/bench_arm_c3.json; [ $rc -eq 0 ] || { tail -20 $o/bench_arm_c3.err; exit $rc; }
timeout -k 10 300 python bench.py --workload fleet_c5 --steps 200 --secondary "" --no-cpu-baseline > $o/bench_fleet_c5.json 2> $o/bench_fleet_c5.err
rc=$?; echo "fleet rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $o/prof -o run -- \
    python3 bench.py --no-cpu-baseline --secondary "" --latency-steps 0 > $o/prof.json 2> $o/prof.err
rc=$?; echo "prof rc=$rc"; cat $o/prof/run_kernel_stats.csv; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_traffic.sh $tag arm_c3 drone_c2 wholebody_c4 quadrotor_c2 fleet_c5
