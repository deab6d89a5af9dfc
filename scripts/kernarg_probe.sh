export TMPDIR=/tmp
mkdir -p gpurun_out/kv
for i in 1 2; do
for v in 1 0; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python bench.py --workload arm_c3 --no-cpu-baseline --secondary "" --steps 500 --warmup 50 --latency-steps 400 > gpurun_out/kv/a_${v}_$i.json 2> gpurun_out/kv/a_${v}_$i.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/kv/a_${v}_$i.json'));print('DEV_KERNARG=$v', 'step %.2f us'%(d['ms_per_step']*1e3), 'p50 %.2f p99 %.2f us'%(d['latency_p50_ms']*1e3, d['latency_p99_ms']*1e3), {k:round(x,2) for k,x in d['kernels'].items() if isinstance(x,float)})"
done; done
