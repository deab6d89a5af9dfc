#!/bin/bash
# HBM traffic passes (FETCH_SIZE and WRITE_SIZE cannot share a pass) per workload:
#   scripts/pmc_traffic.sh <tag> [workload ...]
# Counters only with --kernel-trace; every pass under its own time limit.
tag=${1:-dev}; shift
wls=${*:-arm_c3 drone_c2 wholebody_c4}
export TMPDIR=/tmp
for w in $wls; do
  d=gpurun_out/traffic_$tag/$w
  mkdir -p $d
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $d/$c -o run -- \
        python3 bench.py --workload $w --steps 100 --warmup 10 --latency-steps 0 --no-cpu-baseline --secondary "" \
        > $d/$c.json 2> $d/$c.err
    rc=$?; echo "$w $c rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $d/$c.err; exit $rc; fi
  done
  python3 scripts/pmc_traffic.py $d $w --merge gpurun_out/traffic_$tag/pmc_rollout.json || exit 1
done
