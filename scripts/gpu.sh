#!/bin/bash
# GPU runs used with gpurun, one subcommand per job:
#
#   scripts/gpu.sh tests    <tag> [pytest files]          GPU test suite (default: all -m gpu tests)
#   scripts/gpu.sh bench    <tag> [bench.py args]         default bench line + the driver's 20-step shape x2
#   scripts/gpu.sh prof     <tag> [workload ...]          rocprofv3 kernel traces of control steps only,
#                                                         beside the unprofiled line of the same workload
#   scripts/gpu.sh final    <tag>                         the round's evidence: tests, bench lines, rocprof of
#                                                         the bench command, the plain `bench.py --gpus 2` rehearsal
#                                                         (steps-only traces per workload: `prof`)
#   scripts/gpu.sh ab       <tag> <lib.so[@ENV=v,..]> ..  same-process A/B of builds, native dispatch,
#                                                         both library orders ([AB_REPS] [AB_RUNS])
#   scripts/gpu.sh abi      <tag> <lib.so> ..             same-process interleaved A/B, HIP launches
#   scripts/gpu.sh timeline <tag> <lib.so> <workload> ..  wall-clock step timelines (timeline build)
#   scripts/gpu.sh probe    <tag> <probe> [args]          one tools/probes.py probe
#   scripts/gpu.sh peer2    <tag>                         2-rank peer-exchange rehearsal of the N>1 bench path
#   scripts/gpu.sh gpus2    <tag>                         `python bench.py --gpus 2` (bench.py starts the ranks)
#   scripts/gpu.sh pmc      <tag> [bench.py args]         rocprofv3 counter passes, one group per pass
#   scripts/gpu.sh traffic  <tag> [workload[:K] ...]      FETCH_SIZE / WRITE_SIZE per launch shape ->
#                                                         gpurun_out/traffic_<tag>/pmc_rollout.json
#   scripts/gpu.sh counters <tag> <lib.so|prod> <workload> "<counters>" | trace ...
#                                                         one control-steps-only rocprofv3 pass per group
#                                                         (`trace`: a kernel trace with stats) of one build
#                                                         and workload, summarised into summary.txt and the
#                                                         CSVs deleted; the environment passes through
#                                                         (e.g. MPPI_FIN_TSZ, MPPI_FIN_DEBUG=0). Used for
#                                                         profiles/r05: finalize_fetch (RDREQ_64B/128B, SQC_*,
#                                                         a 4-XCD build, MPPI_FIN_TSZ=8/16/32) and
#                                                         wholebody_sections (SQ_INSTS_* per knockout build)
#
# Every GPU step runs under its own time limit and the first failure ends the script.
cmd=$1; tag=${2:-dev}; shift 2
export TMPDIR=/tmp
out=gpurun_out/${cmd}_$tag
mkdir -p $out
GPU_PYTEST="python -u -m pytest -q -rf --timeout 120 --timeout-method thread"

fail() { echo "$1 rc=$2"; [ -f "$3" ] && tail -30 "$3"; exit $2; }

run_tests() {   # $1 log, rest: files
  local log=$1; shift
  if [ $# -gt 0 ]; then timeout -k 10 600 $GPU_PYTEST -x "$@" > $log 2>&1
  else MPPI_ACCURACY_OUT=$out/acc.json timeout -k 10 600 $GPU_PYTEST -m gpu tests > $log 2>&1; fi
  local rc=$?; echo "pytest rc=$rc"; tail -4 $log
  [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" $log | head -150; exit $rc; }
}

bench_lines() {   # the default line and the driver's 20-step shape
  timeout -k 10 400 python bench.py "$@" > $out/bench_default.json 2> $out/bench_default.err \
      || fail bench $? $out/bench_default.err
  head -c 700 $out/bench_default.json; echo
  for i in 1 2; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $out/bench_s20_$i.json 2> $out/bench_s20_$i.err \
        || fail "bench s20" $? $out/bench_s20_$i.err
    python3 -c "import json;d=json.load(open('$out/bench_s20_$i.json'));t=d['timing'];print('s20', 'step %.2f us'%(d['ms_per_step']*1e3), 'batches', [round(x*1e3,2) for x in t['ms_per_step_batches']])"
  done
}

prof_steps() {   # $1 workload: rocprofv3 of control steps only (no event-timed loops in the trace)
  local w=$1
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --secondary "" --latency-steps 0 --steps 500 \
      --warmup 50 > $out/bench_$w.json 2> $out/bench_$w.err || fail "bench $w" $? $out/bench_$w.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $out/profsteps_$w -o run -- \
      python3 bench.py --workload $w --no-cpu-baseline --secondary "" --latency-steps 0 --no-kernel-timing \
      --steps 500 --warmup 50 > $out/profsteps_$w.json 2> $out/profsteps_$w.err || fail "rocprof $w" $? $out/profsteps_$w.err
  grep -h "k_rollout\|k_finalize" $out/profsteps_$w/run_kernel_stats.csv | cut -d, -f1-4
  python3 -c "import json; d=json.load(open('$out/bench_$w.json')); print('$w unprofiled: step', round(d['ms_per_step']*1e3,2), 'us; kernels', {k: round(v,2) for k,v in d['kernels'].items() if isinstance(v,float)})"
}

ab_both_orders() {   # $1 tool, rest: libs
  local tool=$1; shift
  local runs=${AB_RUNS:-"arm 4096 32;drone 4096 32;wholebody 8192 64;wholebody 65536 64;wholebody 8192 64 8"}
  timeout -k 10 500 python $tool ${AB_REPS:-7} "$runs" "$@" > $out/ab1.txt 2>&1
  local rc=$?; grep -v amdgpu.ids $out/ab1.txt; [ $rc -eq 0 ] || exit $rc
  local rev=(); for x in "$@"; do rev=("$x" "${rev[@]}"); done
  # the first build loaded can run slower in one process (memory placement), hence both orders
  timeout -k 10 500 python $tool ${AB_REPS:-7} "$runs" "${rev[@]}" > $out/ab2.txt 2>&1
  rc=$?; echo "== reversed order"; grep -v amdgpu.ids $out/ab2.txt; exit $rc
}

peer2() {   # the N>1 bench path through the peer exchange, 2 ranks on this one GPU (gloo carries
            # only the handle all-gather, the probe's barriers and the timing reductions)
  MPPI_DIST_BACKEND=gloo MPPI_EXCHANGE=peer timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 50 --warmup 10 \
      --latency-steps 20 > $out/bench_peer2.json 2> $out/bench_peer2.err || fail "peer rehearsal" $? $out/bench_peer2.err
  python3 -c "import json;d=json.load(open('$out/bench_peer2.json'));m=d['multi_gpu'];c=(d.get('secondary') or {}).get('c4') or {};print('peer2', d['config']['workload'], d['config']['parallelism'], 'step %.2f us'%(d['ms_per_step']*1e3), m['exchange'], m['native_comm_error'], '| c4', c.get('exchange'), ('step %.2f us'%(c.get('ms_per_step', 0)*1e3)) if c else None, '| fleet_c5', {k: f.get(k) for k in ('n_gpus', 'exchange', 'vehicles_per_gpu', 'vehicles_total', 'ms_per_step', 'value')} if (f := (d.get('secondary') or {}).get('fleet_c5')) else None)"
}

gpus2() {   # the N>1 bench line from ONE plain command: bench.py starts the 2 ranks itself (a child
           # torch.distributed.run; 2 ranks on this one GPU: gloo process group, peer exchange)
  timeout -k 10 600 python bench.py --gpus 2 --steps 50 --warmup 10 --latency-steps 20 > $out/bench_gpus2.json \
      2> $out/bench_gpus2.err || fail "bench --gpus 2" $? $out/bench_gpus2.err
  python3 -c "import json;d=json.load(open('$out/bench_gpus2.json'));m=d['multi_gpu'];print('gpus2 n_gpus', d['n_gpus'], m['exchange'], 'peer_ranks_connected', m['peer_ranks_connected'], m['process_group'], {k: (v.get('exchange'), v.get('rccl_nranks'), v.get('peer_ranks_connected'), (v.get('native_comm_error') or '')[:60]) for k, v in (d.get('secondary') or {}).items()})"
}

case $cmd in
tests)
  run_tests $out/gpu_tests.log "$@" ;;
bench)
  bench_lines "$@" ;;
prof)
  for w in ${*:-arm_c3 wholebody_c4}; do prof_steps $w; done ;;
final)
  run_tests $out/gpu_tests.log
  bench_lines
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $out/prof_bench -o run -- \
      python3 bench.py --steps 500 --warmup 50 --no-cpu-baseline --secondary "" --latency-steps 100 \
      > $out/prof_bench.json 2> $out/prof_bench.err || fail "rocprof bench" $? $out/prof_bench.err
  gpus2
  echo "final done" ;;
gpus2)
  gpus2 ;;
peer2)
  peer2 ;;
ab)
  ab_both_orders tools/ab_native.py "$@" ;;
abi)
  AB_RUNS=${AB_RUNS:-"wholebody 8192 64;wholebody 8192 64 8;wholebody 65536 64;arm 4096 32"} \
      ab_both_orders tools/ab_interleave.py "$@" ;;
timeline)
  L=$1; shift
  for w in "$@"; do
    MPPI_HIP_LIB=$L MPPI_STAMPS=1 MPPI_EVENT_WAIT=1 MPPI_DEBUG_NO_FLAG=1 timeout -k 10 120 \
        python tools/probes.py timeline $w 40 >> $out/timeline.txt 2> $out/timeline.err || fail "timeline $w" $? $out/timeline.err
  done
  cat $out/timeline.txt ;;
probe)
  timeout -k 10 300 python tools/probes.py "$@" > $out/probe.txt 2> $out/probe.err || fail "probe $1" $? $out/probe.err
  cat $out/probe.txt ;;
pmc)
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
             "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
             "${PMC_EXTRA:-SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES}" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $out/p$i -o run -- \
        python3 bench.py --steps 100 --warmup 10 --latency-steps 0 --no-cpu-baseline --secondary "" "$@" \
        > $out/p$i.json 2> $out/p$i.err || fail "pass $i ($grp)" $? $out/p$i.err
    echo "pass $i ($grp) ok"
  done
  python3 scripts/pmc.py summary $out | tee $out/summary.txt ;;
traffic)
  for spec in ${*:-arm_c3 drone_c2 wholebody_c4}; do
    w=${spec%%:*}; k=""
    if [ "$spec" != "$w" ]; then k=${spec#*:}; fi
    d=$out/${w}${k:+_$k}
    mkdir -p $d
    for c in FETCH_SIZE WRITE_SIZE; do   # the two cannot share a pass
      timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $d/$c -o run -- \
          python3 bench.py --workload $w ${k:+--samples $k} --steps 100 --warmup 10 --latency-steps 0 \
          --no-cpu-baseline --secondary "" > $d/$c.json 2> $d/$c.err || fail "$spec $c" $? $d/$c.err
      echo "$spec $c ok"
    done
    key=$(python3 -c "import json; print(json.load(open('$d/FETCH_SIZE.json'))['roofline']['launch_shape'])") || exit 1
    python3 scripts/pmc.py traffic $d $key --merge $out/pmc_rollout.json --workload $spec || exit 1
    rm -rf $d/FETCH_SIZE $d/WRITE_SIZE   # (the counter CSVs: gpurun copies back at most 64 MiB)
  done ;;
counters)
  lib=$1; w=$2; shift 2
  [ "$lib" = prod ] && lib=$PWD/quadrotor_manipulator_mppi_amd/lib/libmppi_hip.so
  i=0
  for grp in "$@"; do
    i=$((i+1)); d=$out/p$i
    if [ "$grp" = trace ]; then prof="--kernel-trace --stats"; else prof="--pmc $grp --kernel-trace"; fi
    MPPI_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 $prof --output-format csv -d $d -o run -- \
        python3 bench.py --workload $w --steps 200 --warmup 20 --latency-steps 0 --no-cpu-baseline \
        --no-kernel-timing --secondary "" > $d.json 2> $d.err || fail "pass $i ($grp)" $? $d.err
    echo "== $w $(basename $lib) pass $i ($grp)" >> $out/summary.txt
    if [ "$grp" = trace ]; then
      python3 - "$d/run_kernel_stats.csv" >> $out/summary.txt <<'PY' || exit 1
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_rollout" in r["Name"] or "k_finalize" in r["Name"]:
        print("   steps-only", r["Name"].split("(")[0], r["Calls"], "avg ns", r["AverageNs"])
PY
    else
      python3 scripts/pmc.py summary $d >> $out/summary.txt || exit 1
    fi
    rm -rf $d   # (the CSVs: gpurun copies back at most 64 MiB)
    echo "pass $i ($grp) ok"
  done
  grep -v "copyBuffer\|fillBuffer" $out/summary.txt ;;
*)
  sed -n '2,29p' "$0"; exit 2 ;;
esac
