#!/bin/bash
# rocprofv3 PMC passes (counters only with --kernel-trace, one pass per group):
#   scripts/pmc_round.sh <tag> [bench.py args]
tag=${1:-dev}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$tag
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_$tag/p$i -o run -- \
      python3 bench.py --steps 100 --warmup 10 --latency-steps 0 --no-cpu-baseline --secondary "" "$@" \
      > gpurun_out/pmc_$tag/p$i.json 2> gpurun_out/pmc_$tag/p$i.err
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_$tag/p$i.err; exit $rc; fi
done
python3 scripts/pmc_summary.py gpurun_out/pmc_$tag > gpurun_out/pmc_$tag/summary.txt; cat gpurun_out/pmc_$tag/summary.txt
