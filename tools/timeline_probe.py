"""Wall-clock timeline of one control step on the GPU (tools/, not shipped).

    MPPI_HIP_LIB=.../lib/ab/timeline.so MPPI_STAMPS=1 MPPI_EVENT_WAIT=1 MPPI_DEBUG_NO_FLAG=1 \
        python tools/timeline_probe.py <workload> [trials]

The library is a timeline build (MPPI_HIPCC_EXTRA="-DMPPI_STAMPS -DMPPI_TIMELINE"): every
rollout wave and every finalize block stores s_memrealtime (100 MHz, one device clock) at
its start and end, nothing else, so the kernels run their own schedule.  Per trial the
engine runs n back-to-back steps (mppi_run_steps) and the stamps of the LAST step are read
(MPPI_DEBUG_NO_FLAG: that step skips the completion flag's system-scope fence like the others):
rollout first wave start .. last wave end, [PACK first block start .. last block end,]
FINAL first block start .. last block end, all relative to the rollout's first wave start.
Medians over the trials say where a step's time goes: the kernels' spans and the gaps
between them (launch boundary + ramp).  <workload> is a bench.py workload name."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def main():
    import bench
    from quadrotor_manipulator_mppi_amd.distributed import ShardedEngine
    name = sys.argv[1]
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    w = dict(bench.WORKLOADS[name])
    w.pop("desc")
    w.pop("strong", None)
    native = w.pop("native", None)
    se = ShardedEngine(seed=1234, native=native, **w)
    eng = se.engine
    V = w.get("n_vehicles", 1)
    bench.set_targets(eng, w["model"], V)
    eng.set_state(bench.make_state(w["model"], V))
    L = eng._L
    L.mppi_debug_stamps.restype = C.c_int64
    L.mppi_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    L.mppi_debug_fstamps.restype = C.c_int64
    L.mppi_debug_fstamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32]
    rb = np.zeros((1 << 18, 16), np.uint64)
    fb = np.zeros((4096, 16), np.uint64)
    se.run_steps(50)
    eng.synchronize()
    import time
    periods = []   # the step period of this build (the stamps' own cost included)
    for _ in range(5):
        t0 = time.perf_counter()
        se.run_steps(500)
        eng.synchronize()
        periods.append((time.perf_counter() - t0) / 500 * 1e9)
    rows = []
    for _ in range(trials):
        se.run_steps(10)
        eng.synchronize()
        n = L.mppi_debug_stamps(eng._h, rb.ctypes.data, rb.shape[0])
        r = rb[:n].astype(np.int64)
        t0 = r[:, 13].min()
        xcc = (r[:, 15] >> 32) & 0xF
        row = {"roll_last_start": (r[:, 13].max() - t0) * 10.0, "roll_first_end": (r[:, 14].min() - t0) * 10.0,
               "roll_end": (r[:, 14].max() - t0) * 10.0,
               "roll_life_med": float(np.median(r[:, 14] - r[:, 13])) * 10.0,
               # phases per wave: prologue (loads, LDS staging, barrier), the rollout groups, the
               # block combine + record (slots 1 and 5 of the timeline build)
               "roll_prologue_med": float(np.median(r[:, 1] - r[:, 13])) * 10.0,
               "roll_philox_med": float(np.median(r[:, 10] - r[:, 13])) * 10.0,      # loads issued + Philox
               "roll_staging_med": float(np.median(r[:, 1] - r[:, 10])) * 10.0,     # load wait + LDS + barrier
               "roll_groups_med": float(np.median(r[:, 5] - r[:, 1])) * 10.0,
               "roll_combine_med": float(np.median(r[:, 14] - r[:, 5])) * 10.0}
        for c in range(8):
            m = xcc == c
            if m.any():
                row[f"roll_xcd{c}_start"] = (r[m, 13].min() - t0) * 10.0
                row[f"roll_xcd{c}_end"] = (r[m, 14].max() - t0) * 10.0
        for which, key in ((1, "pack"), (0, "final")):
            m = L.mppi_debug_fstamps(eng._h, fb.ctypes.data, fb.shape[0], which)
            f = fb[:m].astype(np.int64)
            f = f[(f[:, 13] > 0) & (f[:, 14] >= f[:, 13])]
            if len(f) and (f[:, 13].min() >= t0 or key == "final"):
                row[key + "_start"] = (f[:, 13].min() - t0) * 10.0
                row[key + "_end"] = (f[:, 14].max() - t0) * 10.0
                row[key + "_life_med"] = float(np.median(f[:, 14] - f[:, 13])) * 10.0
                row[key + "_last_start"] = (f[:, 13].max() - t0) * 10.0
                row[key + "_records_med"] = float(np.median(f[:, 1] - f[:, 13])) * 10.0   # loads .. wave fold
                row[key + "_issue_med"] = float(np.median(f[:, 7] - f[:, 13])) * 10.0     # address math, issue, tail
                row[key + "_tail_med"] = float(np.median(f[:, 14] - f[:, 1])) * 10.0      # barrier .. end
                fx = f[:, 15] & 0xF
                for c in range(8):
                    m = fx == c
                    if m.any():
                        row[f"{key}_xcd{c}_start"] = (f[m, 13].min() - t0) * 10.0
        rows.append(row)
    keys = rows[0].keys()
    med = {k: float(np.median([r[k] for r in rows if k in r])) for k in keys}
    out = {"workload": name, "trials": trials, "dispatch": eng.dispatch_info(),
           "ns_median": {k: round(v) for k, v in med.items()}}
    if "final_start" in med:
        gaps = {"rollout_span": med["roll_end"]}
        prev = med["roll_end"]
        if "pack_start" in med:
            gaps["gap_rollout_pack"] = med["pack_start"] - prev
            gaps["pack_span"] = med["pack_end"] - med["pack_start"]
            prev = med["pack_end"]
        gaps["gap_to_final"] = med["final_start"] - prev
        gaps["final_span"] = med["final_end"] - med["final_start"]
        gaps["step_to_final_end"] = med["final_end"]
        gaps["step_period"] = float(np.median(periods))
        gaps["gap_final_to_next_rollout"] = gaps["step_period"] - med["final_end"]
        out["us"] = {k: round(v / 1e3, 3) for k, v in gaps.items()}
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
