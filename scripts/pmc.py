"""rocprofv3 counter summaries (scripts/gpu.sh pmc / traffic).

    python scripts/pmc.py summary <pmc dir>
        average counter values per kernel over all dispatches of every pass, with the
        kernel-trace durations
    python scripts/pmc.py traffic <pmc dir> <shape key> [--merge profiles/pmc_rollout.json] [--workload spec]
        HBM traffic per launch from FETCH_SIZE / WRITE_SIZE passes

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE reports half the bytes
of wide coalesced reads (MI355X_MICROARCH.md, HBM section), so it is doubled; WRITE_SIZE is taken
as is.  The per-launch figure is the average over all dispatches of the kernel.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _kernel(name):
    k = name.split("(")[0].split("<")[0].strip()
    return k.split()[-1].split("::")[-1] if k else "?"


def per_kernel(root):
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            vals[_kernel(row.get("Kernel_Name", "?"))][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def summary(root):
    vals = per_kernel(root)
    durs = defaultdict(list)
    for path in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            durs[_kernel(row["Kernel_Name"])].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    for k in sorted(vals):
        d = durs.get(k, [])
        print(f"== {k}  (dispatches={len(d)}, avg dur {sum(d) / max(1, len(d)):.0f} ns)")
        for c in sorted(vals[k]):
            v = vals[k][c]
            print(f"   {c:28s} avg {sum(v) / len(v):16.1f}   n={len(v)}")


def traffic(root, workload, out=None, spec=None):
    rec = {}
    for k, d in per_kernel(root).items():
        if "FETCH_SIZE" not in d and "WRITE_SIZE" not in d:
            continue
        avg = {c: sum(v) / len(v) for c, v in d.items()}
        fetch = avg.get("FETCH_SIZE", 0.0) * 1024.0 * 2.0
        write = avg.get("WRITE_SIZE", 0.0) * 1024.0
        rec[k] = {"fetch_kib_raw": avg.get("FETCH_SIZE"), "write_kib": avg.get("WRITE_SIZE"),
                  "fetch_bytes_corrected": fetch, "write_bytes": write,
                  "hbm_bytes_per_launch": fetch + write, "dispatches": max(len(v) for v in d.values())}
    print(json.dumps({workload: rec}, indent=1))
    if out:
        try:
            allw = json.load(open(out))
        except (OSError, ValueError):
            allw = {}
        roll = next((rec[k] for k in sorted(rec) if k.startswith("k_rollout")), {})
        try:   # the library build the counters were collected on (build.py writes BUILD_INFO.json)
            head = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "quadrotor_manipulator_mppi_amd", "lib", "BUILD_INFO.json")))["git_head"]
        except (OSError, ValueError, KeyError):
            head = "?"
        allw[workload] = {"hbm_bytes_per_launch": roll.get("hbm_bytes_per_launch"), "kernels": rec,
                          "build_head": head, "collected": root, "workload": spec or workload,
                          "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KiB->bytes, avg per dispatch"}
        json.dump(allw, open(out, "w"), indent=1)


if __name__ == "__main__":
    a = sys.argv
    if len(a) >= 3 and a[1] == "summary":
        summary(a[2])
    elif len(a) >= 4 and a[1] == "traffic":
        traffic(a[2], a[3], a[a.index("--merge") + 1] if "--merge" in a else None,
                a[a.index("--workload") + 1] if "--workload" in a else None)
    else:
        sys.exit(__doc__)
