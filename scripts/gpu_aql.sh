#!/bin/bash
# Native dispatch on the GPU: its parity tests, then the default bench line under both
# dispatch modes, alternating (scripts/gpu_aql.sh <tag>).  Each GPU step has its own limit.
tag=${1:-dev}
export TMPDIR=/tmp
mkdir -p gpurun_out/aql_$tag
timeout -k 10 300 python -u -m pytest tests/test_gpu_aql.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/aql_$tag/tests.log 2>&1
rc=$?; tail -15 gpurun_out/aql_$tag/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for m in hip aql; do
    MPPI_DISPATCH=$m timeout -k 10 240 python bench.py --steps ${STEPS:-500} --warmup 50 \
        > gpurun_out/aql_$tag/bench_${m}_$i.json 2> gpurun_out/aql_$tag/bench_${m}_$i.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/aql_$tag/bench_${m}_$i.json'));t=d['timing'];print('$m', 'step %.2f us'%(d['ms_per_step']*1e3), 'batches', [round(x*1e3,2) for x in t['ms_per_step_batches']], 'enq', [round(x*1e3,2) for x in t['enqueue_ms_per_step_batches']], 'p50 %.2f'%(d['latency_p50_ms']*1e3), 'pair %.2f'%d['kernels']['pair_us'])"
  done
done
