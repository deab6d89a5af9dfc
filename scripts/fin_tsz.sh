#!/bin/bash
# Finalize slice width vs record fetch (profiles/r05/finalize_fetch): per MPPI_FIN_TSZ (t per slice)
# and workload, one steps-only kernel trace (durations) and one counter pass (the L2's 64 B and
# 128 B memory read requests: true bytes = 64 n64 + 128 n128).  Every pass has its own time limit
# and the first failure ends the script; the CSVs are summarised on the box and deleted.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/fin_tsz
mkdir -p $out
for w in arm_c3 wholebody_c4; do
  for tz in 8 16 32; do
    d=$out/${w}_$tz
    MPPI_FIN_TSZ=$tz timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d/t -o run -- \
        python3 bench.py --workload $w --steps 200 --warmup 20 --latency-steps 0 --no-cpu-baseline --no-kernel-timing \
        --secondary "" > $d.t.json 2> $d.t.err || { echo "trace $w $tz failed"; tail -5 $d.t.err; exit 1; }
    MPPI_FIN_TSZ=$tz timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace \
        --output-format csv -d $d/p -o run -- \
        python3 bench.py --workload $w --steps 200 --warmup 20 --latency-steps 0 --no-cpu-baseline --no-kernel-timing \
        --secondary "" > $d.p.json 2> $d.p.err || { echo "pmc $w $tz failed"; tail -5 $d.p.err; exit 1; }
    echo "== $w tsz=$tz" >> $out/summary.txt
    grep -h "k_rollout\|k_finalize" $d/t/run_kernel_stats.csv | cut -d, -f1-4 >> $out/summary.txt
    python3 scripts/pmc.py summary $d/p >> $out/summary.txt || exit 1
    python3 -c "import json;d=json.load(open('$d.t.json'));print('step us', round(d['ms_per_step']*1e3,2))" >> $out/summary.txt
    rm -rf $d
  done
done
cat $out/summary.txt
