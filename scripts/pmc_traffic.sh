#!/bin/bash
# HBM traffic passes (FETCH_SIZE and WRITE_SIZE cannot share a pass) per launch shape:
#   scripts/pmc_traffic.sh <tag> [workload[:samples] ...]
# e.g. c4:32768 profiles the c4 rank shape at N=2.  Results merge into
# gpurun_out/traffic_<tag>/pmc_rollout.json under bench.shape_key(model, K, H, V).
# Counters only with --kernel-trace; every pass under its own time limit.
tag=${1:-dev}; shift
wls=${*:-arm_c3 drone_c2 wholebody_c4}
export TMPDIR=/tmp
for spec in $wls; do
  w=${spec%%:*}; k=""
  if [ "$spec" != "$w" ]; then k=${spec#*:}; fi
  d=gpurun_out/traffic_$tag/${w}${k:+_$k}
  mkdir -p $d
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $d/$c -o run -- \
        python3 bench.py --workload $w ${k:+--samples $k} --steps 100 --warmup 10 --latency-steps 0 \
        --no-cpu-baseline --secondary "" > $d/$c.json 2> $d/$c.err
    rc=$?; echo "$spec $c rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $d/$c.err; exit $rc; fi
  done
  key=$(python3 -c "import json,sys; r=json.load(open('$d/FETCH_SIZE.json'))['roofline']; print(r['launch_shape'])") || exit 1
  python3 scripts/pmc_traffic.py $d $key --merge gpurun_out/traffic_$tag/pmc_rollout.json --workload $spec || exit 1
done
