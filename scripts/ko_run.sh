#!/bin/bash
# Phase knockout timing (tools-only builds with -DMPPI_KO=n under lib/ko<n>/):
#   scripts/ko_run.sh n1 n2 ...      (the production lib first, as the reference)
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in lib "$@"; do
  if [ $v = lib ]; then L=quadrotor_manipulator_mppi_amd/lib/libmppi_hip.so; else L=quadrotor_manipulator_mppi_amd/lib/ko$v/libmppi_hip.so; fi
  echo "== $v"
  MPPI_HIP_LIB=$L GEOM_V=8 timeout -k 10 120 python tools/geom_sweep.py wholebody 8192 64 || exit 1
  MPPI_HIP_LIB=$L timeout -k 10 120 python tools/geom_sweep.py arm 4096 32 || exit 1
done
