#!/bin/bash
# bench.py at the driver's shape with and without untimed warmup steps ahead of every batch
export TMPDIR=/tmp
mkdir -p gpurun_out/pr
for i in 1 2 3; do for pr in 0 1; do
  MPPI_BENCH_PRIME=$pr timeout -k 10 200 python bench.py --steps 20 --warmup 5 --secondary '' --no-cpu-baseline \
      --latency-steps 20 > gpurun_out/pr/p${pr}_$i.json 2> gpurun_out/pr/p${pr}_$i.err || exit 1
done; done
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/pr/*.json')):
    d=json.load(open(f)); t=d['timing']
    print(f, 'step', round(d['ms_per_step']*1e3,2), 'batches', [round(x*1e3,2) for x in t['ms_per_step_batches']], 'enq', [round(x*1e3,2) for x in t['enqueue_ms_per_step_batches']])
PY
