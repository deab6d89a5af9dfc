#!/bin/bash
# Instruction vs scalar-data requests the SQCs send to L2, per kernel, at arm C3 (production build
# and the 4-XCD finalize build): one counter per pass, each pass under its own time limit.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/fin_ifetch
mkdir -p $out
for lib in prod x4; do
  L=$PWD/quadrotor_manipulator_mppi_amd/lib/libmppi_hip.so; [ $lib = x4 ] && L=$PWD/ab_ko/libmppi_hip_x4.so
  for c in SQC_TC_INST_REQ SQC_TC_DATA_READ_REQ SQC_ICACHE_MISSES; do
    d=$out/${lib}_$c
    MPPI_HIP_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $d -o run -- \
        python3 bench.py --workload arm_c3 --steps 200 --warmup 20 --latency-steps 0 --no-cpu-baseline \
        --no-kernel-timing --secondary "" > $d.json 2> $d.err || { echo "pmc $lib $c failed"; tail -5 $d.err; exit 1; }
    echo "== $lib $c" >> $out/summary.txt
    python3 scripts/pmc.py summary $d | grep -A1 "k_rollout\|k_finalize" >> $out/summary.txt || exit 1
    rm -rf $d
  done
done
cat $out/summary.txt
