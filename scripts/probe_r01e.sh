export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/gt.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gt.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/gt.log | head -80; exit $rc; }
timeout -k 10 100 python tools/step_rate.py arm 4096 32 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 100 python tools/step_rate.py wholebody 8192 64 2>&1 | grep -v amdgpu.ids || exit 1
MPPI_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 100 --warmup 10 --latency-steps 20 > gpurun_out/bench_w2.json 2> gpurun_out/bench_w2.err; rc=$?; echo "w2 rc=$rc"; cat gpurun_out/bench_w2.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_w2.err; exit $rc; }
timeout -k 10 300 python bench.py --workload fleet_c5 --steps 200 --secondary "" --no-cpu-baseline > gpurun_out/bench_fleet.json 2> gpurun_out/bench_fleet.err; rc=$?; echo "fleet rc=$rc"; cat gpurun_out/bench_fleet.json; [ $rc -eq 0 ] || tail -20 gpurun_out/bench_fleet.err
