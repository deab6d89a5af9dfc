#!/bin/bash
# The round's evidence run on one box: GPU tests, the default bench line and the driver's
# 20-step shape, rocprofv3 kernel-trace summaries (the bench command, and control steps only),
# a 2-rank gloo rehearsal of the north-star path, and wall-clock step timelines.
#   scripts/gpu_final.sh <tag>
# Every GPU step has its own time limit; the first failure ends the script.
tag=${1:-dev}
export TMPDIR=/tmp
out=gpurun_out/final_$tag
mkdir -p $out
timeout -k 10 420 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $out/bench_default.json 2> $out/bench_default.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $out/bench_default.err; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $out/bench_s20_$i.json 2> $out/bench_s20_$i.err
  rc=$?; echo "bench s20 rc=$rc"; [ $rc -eq 0 ] || { tail -20 $out/bench_s20_$i.err; exit $rc; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $out/prof_bench -o run -- \
    python3 bench.py --steps 500 --warmup 50 --no-cpu-baseline --secondary "" --latency-steps 100 \
    > $out/prof_bench.json 2> $out/prof_bench.err
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $out/prof_bench.err; exit $rc; }
for w in arm_c3 wholebody_c4 c4_shard_native1 c4 drone_c2 quadrotor_c2 fleet_c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $out/profsteps_$w -o run -- \
      python3 bench.py --workload $w --no-cpu-baseline --secondary "" --latency-steps 0 --no-kernel-timing \
      --steps 500 --warmup 50 > $out/profsteps_$w.json 2> $out/profsteps_$w.err
  rc=$?; echo "rocprof steps $w rc=$rc"; [ $rc -eq 0 ] || { tail -20 $out/profsteps_$w.err; exit $rc; }
done
MPPI_DIST_BACKEND=gloo MPPI_NATIVE_COMM=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 50 --warmup 10 \
    --latency-steps 20 > $out/bench_gloo2.json 2> $out/bench_gloo2.err
rc=$?; echo "gloo rehearsal rc=$rc"; [ $rc -eq 0 ] || { tail -30 $out/bench_gloo2.err; exit $rc; }
if [ -f quadrotor_manipulator_mppi_amd/lib/ab/timeline.so ]; then   # (built by scripts/gpu_timeline.sh's recipe)
  bash scripts/gpu_timeline.sh $tag quadrotor_manipulator_mppi_amd/lib/ab/timeline.so arm_c3 wholebody_c4 c4_shard_native1 c4 \
      > $out/timeline.txt 2>&1
  rc=$?; echo "timeline rc=$rc"
fi
exit $rc
