#!/bin/bash
# Where the finalize's 64 B memory read requests come from (profiles/r05/finalize_fetch): the counter
# list of this box, then for the production build and a build whose finalize runs on 4 XCDs
# (-DMPPI_FIN_XCDS=4, ab_ko/libmppi_hip_x4.so) one counter pass of the L2's 64 B / 128 B read
# requests and, when the box lists it, one pass of SQ_IFETCH (instruction fetches), at arm C3.
# Every pass has its own time limit; the first failure ends the script.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/fin_fetch
mkdir -p $out
timeout -s KILL 60 rocprofv3 -L > $out/counters.txt 2>&1 || { echo "listing failed"; tail -5 $out/counters.txt; }
grep -o "SQC_[A-Z0-9_]*\|SQ_IFETCH[A-Z_]*\|TCC_EA0_RD[A-Z0-9_]*" $out/counters.txt | sort -u > $out/counters_grep.txt
cat $out/counters_grep.txt | tr '\n' ' '; echo
for lib in prod x4; do
  L=$PWD/quadrotor_manipulator_mppi_amd/lib/libmppi_hip.so; [ $lib = x4 ] && L=$PWD/ab_ko/libmppi_hip_x4.so
  groups=("TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum")
  grep -qx "SQ_IFETCH" $out/counters_grep.txt && groups+=("SQ_IFETCH SQ_WAVES")
  i=0
  for grp in "${groups[@]}"; do
    i=$((i+1)); d=$out/${lib}_p$i
    MPPI_HIP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $d -o run -- \
        python3 bench.py --workload arm_c3 --steps 200 --warmup 20 --latency-steps 0 --no-cpu-baseline \
        --no-kernel-timing --secondary "" > $d.json 2> $d.err || { echo "pmc $lib $i failed"; tail -5 $d.err; exit 1; }
    echo "== $lib pass $i ($grp)" >> $out/summary.txt
    python3 scripts/pmc.py summary $d >> $out/summary.txt || exit 1
    rm -rf $d
  done
  d=$out/${lib}_t
  MPPI_HIP_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
      python3 bench.py --workload arm_c3 --steps 500 --warmup 50 --latency-steps 0 --no-cpu-baseline \
      --no-kernel-timing --secondary "" > $d.json 2> $d.err || { echo "trace $lib failed"; tail -5 $d.err; exit 1; }
  python3 - "$d/run_kernel_stats.csv" "$lib" >> $out/summary.txt <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith(("void k_rollout", "void k_finalize", "k_rollout", "k_finalize")):
        print(sys.argv[2], "steps-only", r["Name"][:40], r["Calls"], "avg ns", r["AverageNs"])
PY
  rm -rf $d
done
cat $out/summary.txt | grep -v "copyBuffer\|fillBuffer"
