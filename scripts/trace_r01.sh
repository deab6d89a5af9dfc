export TMPDIR=/tmp
for w in "arm 4096 32" "drone 4096 32"; do
  set -- $w
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$1 -o run -- python3 tools/run_steps.py $w 500 > gpurun_out/trace_$1.txt 2>&1 || exit 1
  grep us/step gpurun_out/trace_$1.txt
  python3 - gpurun_out/trace_$1/run_kernel_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if 'k_' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
rows = rows[-400:]
import collections
d = collections.defaultdict(list); gaps = collections.defaultdict(list)
for a, b in zip(rows, rows[1:]):
    na = a['Kernel_Name'].split('(')[0].split('<')[0].split()[-1]; nb = b['Kernel_Name'].split('(')[0].split('<')[0].split()[-1]
    gaps[na + '->' + nb].append(int(b['Start_Timestamp']) - int(a['End_Timestamp']))
for r in rows:
    n = r['Kernel_Name'].split('(')[0].split('<')[0].split()[-1]
    d[n].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
for k, v in d.items(): print(f"  {k}: avg {sum(v)/len(v)/1e3:.2f} us  (n={len(v)})")
for k, v in gaps.items(): print(f"  gap {k}: avg {sum(v)/len(v)/1e3:.2f} us")
PY
done
