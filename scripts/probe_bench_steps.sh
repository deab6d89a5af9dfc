#!/bin/bash
# bench.py at the driver's 20-step shape (3 runs) and at 500 steps: per-batch step and host-enqueue times
export TMPDIR=/tmp
mkdir -p gpurun_out/b20
for i in 1 2 3; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --secondary '' --no-cpu-baseline --latency-steps 50 > gpurun_out/b20/s20_$i.json 2> gpurun_out/b20/s20_$i.err || exit 1
done
timeout -k 10 200 python bench.py --steps 500 --warmup 50 --secondary '' --no-cpu-baseline --latency-steps 50 > gpurun_out/b20/s500.json 2> gpurun_out/b20/s500.err || exit 1
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/b20/*.json')):
    d=json.load(open(f)); print(f, round(d['ms_per_step']*1e3,3), [round(x*1e3,2) for x in d['timing']['ms_per_step_batches']], 'enq', [round(x*1e3,2) for x in d['timing']['enqueue_ms_per_step_batches']], d['kernels']['pair_us'])
PY
