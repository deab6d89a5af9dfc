#!/bin/bash
# bench.py on one box: the default N=1 line, a 2-rank gloo rehearsal of the north-star
# (c4, strong-scaled) path, and rocprofv3 kernel-trace summaries of the bench commands.
#   scripts/gpu_bench.sh <tag>
# Every GPU step has its own time limit; the first failure ends the script.
tag=${1:-dev}
export TMPDIR=/tmp
out=gpurun_out/bench_$tag
mkdir -p $out
timeout -k 10 400 python bench.py --steps 500 --warmup 50 > $out/n1.json 2> $out/n1.err
rc=$?; echo "bench rc=$rc"; cat $out/n1.json
[ $rc -eq 0 ] || { tail -30 $out/n1.err; exit $rc; }
MPPI_DIST_BACKEND=gloo MPPI_NATIVE_COMM=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 50 --warmup 10 \
    --latency-steps 20 > $out/gloo2.json 2> $out/gloo2.err
rc=$?; echo "gloo rehearsal rc=$rc"; cat $out/gloo2.json
[ $rc -eq 0 ] || { tail -30 $out/gloo2.err; exit $rc; }
for w in arm_c3 wholebody_c4 fleet_c5 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $out/prof_$w -o run -- \
      python3 bench.py --workload $w --no-cpu-baseline --secondary "" --latency-steps 0 --steps 300 --warmup 30 \
      > $out/prof_$w.json 2> $out/prof_$w.err
  rc=$?; echo "rocprof $w rc=$rc"
  [ $rc -eq 0 ] || { tail -20 $out/prof_$w.err; exit $rc; }
  grep -h "k_rollout\|k_finalize" $out/prof_$w/run_kernel_stats.csv | cut -c1-200
done
