#!/bin/bash
# Rollout packets without a release fence (write-through outputs + store drain): the full GPU
# suite, the fence probe (default vs all-agent fences), and the default bench line.
tag=${1:-dev}
export TMPDIR=/tmp
out=gpurun_out/selfrel_$tag
mkdir -p $out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/gpu_tests.log; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" $out/gpu_tests.log | head -120; exit $rc; }
for f in "" 1011 1111 "" 1011 1111; do
  MPPI_AQL_FENCES=$f timeout -k 10 120 python tools/aql_fence_probe.py 2>&1 | grep -v amdgpu.ids | tee -a $out/fences.txt || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python bench.py > $out/bench_$i.json 2> $out/bench_$i.err || { tail -20 $out/bench_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/bench_$i.json'));t=d['timing'];print(t['dispatch'], 'step %.2f us'%(d['ms_per_step']*1e3), [round(x*1e3,2) for x in t['ms_per_step_batches']], 'p50 %.2f p99 %.2f'%(d['latency_p50_ms']*1e3, d['latency_p99_ms']*1e3), 'pair %.2f'%d['kernels']['pair_us'])"
done
