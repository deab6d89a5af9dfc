"""HBM traffic per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    python scripts/pmc_traffic.py <pmc dir> <shape key> [--merge profiles/pmc_rollout.json] [--workload spec]

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE
reports half the bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM), so
it is doubled; WRITE_SIZE is taken as is.  The per-launch figure is the average
over all dispatches of the kernel.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kernel(root):
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            k = row.get("Kernel_Name", "?").split("(")[0].split("<")[0].strip()
            k = k.split()[-1].split("::")[-1] if k else "?"
            vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} | {"dispatches": max(len(v) for v in d.values())}
            for k, d in vals.items()}


def main():
    root, workload = sys.argv[1], sys.argv[2]
    out = sys.argv[sys.argv.index("--merge") + 1] if "--merge" in sys.argv else None
    ks = per_kernel(root)
    rec = {}
    for k, d in ks.items():
        if "FETCH_SIZE" not in d and "WRITE_SIZE" not in d:
            continue
        fetch = d.get("FETCH_SIZE", 0.0) * 1024.0 * 2.0
        write = d.get("WRITE_SIZE", 0.0) * 1024.0
        rec[k] = {"fetch_kib_raw": d.get("FETCH_SIZE"), "write_kib": d.get("WRITE_SIZE"),
                  "fetch_bytes_corrected": fetch, "write_bytes": write,
                  "hbm_bytes_per_launch": fetch + write, "dispatches": d["dispatches"]}
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
        spec = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else workload
        allw[workload] = {"hbm_bytes_per_launch": roll.get("hbm_bytes_per_launch"), "kernels": rec,
                          "build_head": head, "collected": root, "workload": spec,
                          "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KiB->bytes, avg per dispatch"}
        json.dump(allw, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
