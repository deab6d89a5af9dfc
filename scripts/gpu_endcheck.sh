export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_end.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_end.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_end.json 2> gpurun_out/bench_end.err || exit 1
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench_end.json"))
print(round(d["ms_per_step"] * 1e3, 3), "%.4g" % d["value"], round(d["roofline"]["frac"], 3), d["latency_p50_ms"], d["dropin_latency"]["p50_ms"], d.get("build"))
PY
