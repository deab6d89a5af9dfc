#!/bin/bash
# Native dispatch: the 20-step bench line (the driver's --steps 20), and the step pair under
# packet fence-scope variants (diagnostic MPPI_AQL_FENCES) with a bit-exactness check against
# HIP dispatch.  scripts/gpu_aql_fences.sh <tag>
tag=${1:-dev}
export TMPDIR=/tmp
mkdir -p gpurun_out/aqlf_$tag
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 10 --secondary "" --no-cpu-baseline \
      > gpurun_out/aqlf_$tag/bench_s20_$i.json 2> gpurun_out/aqlf_$tag/bench_s20_$i.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/aqlf_$tag/bench_s20_$i.json'));t=d['timing'];print('s20', t['dispatch'], 'step %.2f us'%(d['ms_per_step']*1e3), 'batches', [round(x*1e3,2) for x in t['ms_per_step_batches']], 'enq', [round(x*1e3,2) for x in t['enqueue_ms_per_step_batches']])"
done
for f in 1111 1011 1101 1100 0101; do
  MPPI_AQL_FENCES=$f timeout -k 10 120 python tools/aql_fence_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/aqlf_$tag/fences.txt || exit 1
done
