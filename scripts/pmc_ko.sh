#!/bin/bash
# Dynamic per-section instruction counts of the whole-body rollout: one
# rocprofv3 counter pass (SQ_INSTS_VALU / SALU / LDS, SQ_WAVES) per knockout build of the C4 rank
# shard (whole-body K=8192 H=64), the baseline library first.  Knockouts (-DMPPI_KO, results wrong,
# timing / counting only): 2 Philox rounds, 32 Box-Muller, 1 integrator scans, 4 FK chain,
# 8 pose cost, 16 trajectory stores, 64 record-body fold.  Every pass runs under its own time limit
# and the first failure ends the script.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/pmc_ko
mkdir -p $out
for ko in 0 2 32 1 4 8 16 64; do
  lib=$PWD/quadrotor_manipulator_mppi_amd/lib/libmppi_hip.so
  [ $ko -ne 0 ] && lib=$PWD/ab_ko/libmppi_hip_ko$ko.so
  MPPI_FIN_DEBUG=0 MPPI_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --kernel-trace \
      --output-format csv -d $out/ko$ko -o run -- python3 bench.py --workload wholebody_c4 --steps 100 --warmup 10 \
      --latency-steps 0 --no-cpu-baseline --secondary "" > $out/ko$ko.json 2> $out/ko$ko.err \
      || { echo "ko $ko failed"; tail -5 $out/ko$ko.err; exit 1; }
  echo "ko $ko ok"
done
for ko in 0 2 32 1 4 8 16 64; do
  echo "== ko $ko" >> $out/summary.txt
  python3 scripts/pmc.py summary $out/ko$ko >> $out/summary.txt || exit 1
  rm -rf $out/ko$ko
done
