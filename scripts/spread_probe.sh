#!/bin/bash
# Arm C3 rollout time across fresh processes, with and without an LDS floor that keeps
# one rollout block per CU (MPPI_LDS_FLOOR bytes).
export TMPDIR=/tmp
for r in 1 2 3 4 5; do
  timeout -k 10 60 python tools/geom_sweep.py arm 4096 32 || exit 1
  MPPI_LDS_FLOOR=83968 timeout -k 10 60 python tools/geom_sweep.py arm 4096 32 | sed 's/^/floor82K /' || exit 1
done
