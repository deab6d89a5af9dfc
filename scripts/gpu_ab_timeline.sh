#!/bin/bash
# GPU tests on the production build, an interleaved A/B of builds (both orders), then the
# timeline build's step timelines:
#   [AB_TESTS=0] [AB_REPS=15] [AB_RUNS=...] [TL_WORKLOADS="arm_c3 ..."] scripts/gpu_ab_timeline.sh <tag> <lib.so> ...
tag=${1:-dev}
AB_RUNS=${AB_RUNS:-"arm 4096 32;wholebody 8192 64;drone 4096 32"} bash scripts/gpu_abi.sh "$@" || exit $?
bash scripts/gpu_timeline.sh $tag quadrotor_manipulator_mppi_amd/lib/ab/timeline.so ${TL_WORKLOADS:-arm_c3 wholebody_c4 c4_shard_native1}
