"""Wall-clock split of the fused single-launch step (round-4 experiment, commit 610dd73, reverted).

    PYTHONPATH=<package built from 610dd73 with MPPI_HIPCC_EXTRA="-DMPPI_STAMPS -DMPPI_TIMELINE"
               and the fused tail's stamps (slots 2/3/4)> MPPI_STAMPS=1 \
        python timeline_probe_fused.py [trials]

Per trial: 10 back-to-back native steps, then the stamps of the LAST step (s_memrealtime, 100 MHz):
every rollout wave's start (13) and end of its rollout work (14); in a fused step the folding
blocks' waves also stamp the ticket (2), the moment every block had arrived (3) and the end of
the fold + finalize body (4).  The two-kernel step of the same build (MPPI_FUSED=0) reads the
finalize's own block stamps instead.  Medians over the trials, microseconds from the first
rollout wave's start."""
import ctypes as C
import json
import os
import sys

import numpy as np

from quadrotor_manipulator_mppi_amd.engine import Engine, make_config

HOME = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]
SHAPES = {"arm_c3": ("arm", 4096, 32, [0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 7),
          "drone_c2": ("drone", 4096, 32, [0.1, -0.2, 1.0, 0.0, 0.0, 0.0]),
          "wholebody_c4": ("wholebody", 8192, 64, [0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 10)}


def run(name, fused, trials):
    model, K, H, st = SHAPES[name]
    os.environ["MPPI_FUSED"] = "1" if fused else "0"
    e = Engine(make_config(model, n_samples=K, n_horizon=H, state_f64=(model == "arm")))
    e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5]) if model != "drone" else e.set_target([1.0, 2.0, 3.4])
    e.set_state(np.array(st, np.float64))
    L = e._L
    L.mppi_debug_stamps.restype = C.c_int64
    L.mppi_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    L.mppi_debug_fstamps.restype = C.c_int64
    L.mppi_debug_fstamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32]
    rb = np.zeros((1 << 16, 16), np.uint64)
    fb = np.zeros((4096, 16), np.uint64)
    e.run_steps(50)
    e.synchronize()
    rows = []
    for _ in range(trials):
        e.run_steps(10)
        e.synchronize()
        n = L.mppi_debug_stamps(e._h, rb.ctypes.data, rb.shape[0])
        r = rb[:n].astype(np.int64)
        t0 = r[:, 13].min()
        row = {"rollout_end": (r[:, 14].max() - t0) / 100.0}
        if fused:
            f = (r[:, 3] >= t0) & (r[:, 4] >= r[:, 3]) & (r[:, 2] >= t0)
            row.update(fold_waves=int(f.sum()),
                       last_ticket=(r[f, 2].max() - t0) / 100.0,
                       all_arrived_first=(r[f, 3].min() - t0) / 100.0,
                       all_arrived_last=(r[f, 3].max() - t0) / 100.0,
                       fold_end=(r[f, 4].max() - t0) / 100.0,
                       fold_life_med=float(np.median(r[f, 4] - r[f, 3])) / 100.0)
        else:
            m = L.mppi_debug_fstamps(e._h, fb.ctypes.data, fb.shape[0], 0)
            g = fb[:m].astype(np.int64)
            g = g[(g[:, 13] >= t0) & (g[:, 14] >= g[:, 13])]
            row.update(final_start=(g[:, 13].min() - t0) / 100.0, final_end=(g[:, 14].max() - t0) / 100.0)
        rows.append(row)
    e.close()
    return {k: round(float(np.median([x[k] for x in rows])), 3) for k in rows[0]}


if __name__ == "__main__":
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    for name in SHAPES:
        for fused in (False, True):
            print(json.dumps({"workload": name, "step": "fused" if fused else "two kernels",
                              "us_median": run(name, fused, trials)}), flush=True)
