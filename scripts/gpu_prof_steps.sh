#!/bin/bash
# rocprofv3 kernel traces of control steps only (bench.py --no-kernel-timing: no event-timed
# loops in the trace), next to the unprofiled bench line of the same workload:
#   scripts/gpu_prof_steps.sh <tag> [workload ...]
tag=${1:-dev}; shift
wls=${*:-arm_c3 wholebody_c4}
export TMPDIR=/tmp
out=gpurun_out/profsteps_$tag
mkdir -p $out
for w in $wls; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --secondary "" --latency-steps 0 --steps 500 \
      --warmup 50 > $out/bench_$w.json 2> $out/bench_$w.err
  rc=$?; echo "bench $w rc=$rc"; [ $rc -eq 0 ] || { tail -20 $out/bench_$w.err; exit $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $out/prof_$w -o run -- \
      python3 bench.py --workload $w --no-cpu-baseline --secondary "" --latency-steps 0 --no-kernel-timing \
      --steps 500 --warmup 50 > $out/prof_$w.json 2> $out/prof_$w.err
  rc=$?; echo "rocprof $w rc=$rc"; [ $rc -eq 0 ] || { tail -20 $out/prof_$w.err; exit $rc; }
  grep -h "k_rollout\|k_finalize" $out/prof_$w/run_kernel_stats.csv | cut -d, -f1-4
  python3 -c "import json,sys; d=json.load(open('$out/bench_$w.json')); print('$w unprofiled: step', round(d['ms_per_step']*1e3,2), 'us; kernels', {k: round(v,2) for k,v in d['kernels'].items() if isinstance(v,float)})"
done
