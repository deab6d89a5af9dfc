#!/bin/bash
# round 4: GPU tests, default bench line, same-process A/B of library builds (both orders)
#   scripts/gpu_r04a.sh <tag> <lib.so[@ENV=..]> ...
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 $out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; head -c 600 $out/bench.json; echo
[ $rc -eq 0 ] || { tail -20 $out/bench.err; exit $rc; }
[ $# -gt 0 ] || exit 0
RUNS=${AB_RUNS:-"arm 4096 32;drone 4096 32;wholebody 8192 64;wholebody 65536 64;wholebody 8192 64 8"}
timeout -k 10 500 python tools/ab_native.py ${AB_REPS:-7} "$RUNS" "$@" > $out/ab1.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab1.txt
[ $rc -eq 0 ] || exit $rc
rev=(); for x in "$@"; do rev=("$x" "${rev[@]}"); done
timeout -k 10 500 python tools/ab_native.py ${AB_REPS:-7} "$RUNS" "${rev[@]}" > $out/ab2.txt 2>&1
rc=$?; echo "ab2 rc=$rc"; grep -v amdgpu.ids $out/ab2.txt
exit $rc
