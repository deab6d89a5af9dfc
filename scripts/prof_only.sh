export TMPDIR=/tmp
o=gpurun_out/art_s3o; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $o/prof -o run -- \
    python3 bench.py --no-cpu-baseline --secondary "" --latency-steps 0 > $o/prof.json 2> $o/prof.err
rc=$?; echo "prof rc=$rc"; cat $o/prof/run_kernel_stats.csv; cat $o/prof.json
