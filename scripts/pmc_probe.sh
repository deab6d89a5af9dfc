#!/bin/bash
# One-off PMC groups for the rollout/finalize kernels: scripts/pmc_probe.sh <tag> "<grp1>" "<grp2>" ...
tag=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$tag
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_$tag/p$i -o run -- \
      python3 bench.py --steps 100 --warmup 10 --latency-steps 0 --no-cpu-baseline --secondary "" --workload ${WL:-arm_c3} \
      > gpurun_out/pmc_$tag/p$i.json 2> gpurun_out/pmc_$tag/p$i.err
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_$tag/p$i.err; exit $rc; fi
done
python3 scripts/pmc_summary.py gpurun_out/pmc_$tag > gpurun_out/pmc_$tag/summary.txt; cat gpurun_out/pmc_$tag/summary.txt
