#!/bin/bash
# A/B kernel timing on one box: alternate two library builds (tools/geom_sweep.py).
#   scripts/ab_run.sh <libA> <libB> [reps]
A=$1; B=$2; N=${3:-3}
export TMPDIR=/tmp
for r in $(seq $N); do
  for L in $A $B; do
    echo "== $L"
    MPPI_HIP_LIB=$L GEOM_V=8 timeout -k 10 120 python tools/geom_sweep.py wholebody 8192 64 || exit 1
    MPPI_HIP_LIB=$L timeout -k 10 120 python tools/geom_sweep.py wholebody 8192 64 || exit 1
    MPPI_HIP_LIB=$L timeout -k 10 120 python tools/geom_sweep.py arm 4096 32 || exit 1
  done
done
