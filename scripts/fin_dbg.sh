export TMPDIR=/tmp
for d in ${DBGS:-0 1 2 4 7}; do
  MPPI_FIN_DEBUG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/fin_$d -o run -- python3 bench.py --steps 200 --latency-steps 0 --no-cpu-baseline --secondary "" > /dev/null 2>&1 || exit 1
  echo "dbg=$d"; grep -E "k_finalize|k_rollout" gpurun_out/fin_$d/run_kernel_stats.csv
done
