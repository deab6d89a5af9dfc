"""Where the bench's short timed batches lose time (arm C3, 20-step batches).

For each of R batches of n control steps (mppi_run_steps) it records:
  wall      -- the bench bracket: synchronize + t0 ... run_steps ... synchronize + t1
  gpu       -- torch events on the engine stream around the n steps (device time)
  enqueue   -- host time of the run_steps call alone
  sync_wait -- host time of the closing synchronize
with three closing syncs: the engine stream (hipStreamSynchronize), torch.cuda.synchronize
(device), and a poll of the last step's completion flag (mppi_read_outputs) first.

    python tools/bracket_probe.py [--steps 20] [--batches 15]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batches", type=int, default=15)
    ap.add_argument("--workload", default="arm_c3")
    args = ap.parse_args()
    import torch
    import bench
    from quadrotor_manipulator_mppi_amd.distributed import ShardedEngine
    w = dict(bench.WORKLOADS[args.workload])
    w.pop("desc")
    se = ShardedEngine(seed=1234, **w)
    eng = se.engine
    bench.set_targets(eng, w["model"], 1)
    eng.set_state(bench.make_state(w["model"], 1))
    eng.run_steps(200)
    eng.synchronize()
    res = {}
    for mode in ("stream", "device", "flag", "stream", "device", "flag"):
        rows = []
        for _ in range(args.batches):
            eng.synchronize()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(se.stream)
            eng.run_steps(args.steps)
            e1.record(se.stream)
            t1 = time.perf_counter()
            if mode == "flag":
                eng.read_outputs()   # polls the last step's completion flag in mapped memory
            if mode in ("stream", "flag"):
                eng.synchronize()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            rows.append((t2 - t0, e0.elapsed_time(e1) * 1e-3, t1 - t0, t2 - t1))
        a = np.array(rows) * 1e6 / args.steps
        key = mode if mode not in res else mode + "_2"
        res[key] = {"wall_us_per_step": float(np.median(a[:, 0])), "gpu_us_per_step": float(np.median(a[:, 1])),
                    "enqueue_us_per_step": float(np.median(a[:, 2])), "sync_wait_us_per_step": float(np.median(a[:, 3])),
                    "wall_batches": [round(x, 2) for x in a[:, 0]]}
        print(key, json.dumps(res[key]), flush=True)
    print(json.dumps({"workload": args.workload, "steps": args.steps, "res": res}))


if __name__ == "__main__":
    main()
