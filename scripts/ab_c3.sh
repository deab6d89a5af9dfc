#!/bin/bash
# A/B for the latency-bound small shapes (arm C3, drone C2): alternate two builds, fresh
# process each time.   scripts/ab_c3.sh <libA> <libB> [reps]
A=$1; B=$2; N=${3:-4}
export TMPDIR=/tmp
for r in $(seq $N); do
  for L in $A $B; do
    echo "== $L"
    MPPI_HIP_LIB=$L timeout -k 10 60 python tools/geom_sweep.py arm 4096 32 || exit 1
    MPPI_HIP_LIB=$L timeout -k 10 60 python tools/geom_sweep.py drone 4096 32 || exit 1
  done
done
