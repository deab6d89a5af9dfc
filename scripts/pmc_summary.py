"""Average rocprofv3 counter values per kernel over all dispatches of every pass
under a directory (counter_collection CSVs) and the kernel-trace durations."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
durs = defaultdict(list)
for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(path)):
        k = row.get("Kernel_Name", "?").split("(")[0]
        vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for path in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"].split("(")[0]
        durs[k].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
for k in sorted(vals):
    print(f"== {k}  (dispatches={len(durs.get(k, []))}, avg dur {sum(durs.get(k,[0]))/max(1,len(durs.get(k,[]))):.0f} ns)")
    for c in sorted(vals[k]):
        v = vals[k][c]
        print(f"   {c:24s} avg {sum(v)/len(v):16.1f}   n={len(v)}")
