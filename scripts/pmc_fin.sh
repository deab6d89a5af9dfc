cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/pmc_fin2
mkdir -p $out
i=0
for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "FETCH_SIZE" "TCC_MISS_sum TCC_HIT_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out/p$i -o run -- \
      python3 bench.py --steps 100 --warmup 10 --latency-steps 0 --no-cpu-baseline --no-kernel-timing --secondary "" > $out/p$i.json 2> $out/p$i.err || { echo "pass $i failed"; tail -5 $out/p$i.err; exit 1; }
  echo "pass $i ($grp) ok"
done
python3 scripts/pmc.py summary $out > $out/summary.txt && rm -rf $out/p1 $out/p2 $out/p3 $out/p4
