#!/bin/bash
# Whole-body rollout diagnosis: stamps, step rate (with/without trajectory), SQ counters.
export TMPDIR=/tmp
mkdir -p gpurun_out/probe_s2
L=quadrotor_manipulator_mppi_amd/lib/libmppi_hip_stamps.so
MPPI_HIP_LIB=$L MPPI_STAMPS=1 timeout -k 10 120 python tools/stamp_probe.py wholebody 8192 64 2>&1 | grep -v amdgpu.ids || exit 1
MPPI_HIP_LIB=$L MPPI_STAMPS=1 timeout -k 10 120 python tools/stamp_probe.py arm 4096 32 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 100 python tools/step_rate.py wholebody 8192 64 2>&1 | grep -v amdgpu.ids || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/probe_s2/p$i -o run -- \
      python3 bench.py --workload wholebody_c4 --steps 100 --warmup 10 --latency-steps 0 --no-cpu-baseline --secondary "" \
      > gpurun_out/probe_s2/p$i.json 2> gpurun_out/probe_s2/p$i.err
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/probe_s2/p$i.err; exit $rc; fi
done
python3 scripts/pmc_summary.py gpurun_out/probe_s2
