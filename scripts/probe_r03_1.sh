set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/p1
timeout -k 10 120 python -u tools/bracket_probe.py --steps 20 --batches 15 > gpurun_out/p1/bracket20.txt 2>&1
timeout -k 10 120 python -u tools/bracket_probe.py --steps 500 --batches 5 > gpurun_out/p1/bracket500.txt 2>&1
timeout -k 10 200 python bench.py --workload c4_shard_native1 --steps 500 --no-cpu-baseline --secondary '' > gpurun_out/p1/native1.json 2> gpurun_out/p1/native1.err
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/p1/prof_native1 -o run -- python $GRAFT_REPO_ROOT/bench.py --workload c4_shard_native1 --steps 500 --no-kernel-timing --no-cpu-baseline --secondary '' --latency-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/p1/prof_native1.log 2>&1
echo ok
