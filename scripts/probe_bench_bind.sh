#!/bin/bash
# bench.py at the driver's 20-step shape with and without the NUMA binding, interleaved
export TMPDIR=/tmp
mkdir -p gpurun_out/bb
for i in 1 2 3; do for b in bind nobind; do
  x=""; [ $b = nobind ] && x="--no-numa-bind"
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --secondary '' --no-cpu-baseline --latency-steps 100 $x \
      > gpurun_out/bb/${b}_$i.json 2> gpurun_out/bb/${b}_$i.err || exit 1
done; done
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/bb/*.json')):
    d=json.load(open(f)); t=d['timing']
    print(f, 'step', round(d['ms_per_step']*1e3,2), 'batches', [round(x*1e3,2) for x in t['ms_per_step_batches']], 'enq', [round(x*1e3,2) for x in t['enqueue_ms_per_step_batches']], 'p50', round(d['latency_p50_ms']*1e3,1), d.get('host_binding'))
PY
