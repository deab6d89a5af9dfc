#!/usr/bin/env python3
"""MPPI control-step benchmark (BASELINE.json metric: rollout-steps/s, K x H
state-steps, plus control-step p50 latency, at K=4096 H=32).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload arm_c3]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N ...

A "step" is one MPPI control step (noise -> rollout -> FK -> cost -> softmin ->
SavGol -> update) over one batch of synthetic state/goal input.
Scaling is WEAK: every rank owns K samples of the same controller (sample
sharding, one all-reduce per step), so the whole-job rate is N*K*H per step.
``value`` is measured with state and warm start resident on the GPU (async
steps, one sync at the end); the host-inclusive call latency (H2D state, D2H
outputs, check_reach) is reported separately as latency_p50/p99.

Rank 0 prints ONE JSON line on stdout; progress goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HOME_Q = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]                # kinova.py:135
ARM_TARGET = ([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])   # mppi.py:71-72
DRONE_TARGET = [1.0, 2.0, 3.4]                                   # drone_mppi.py:141
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

WORKLOADS = {
    # configs[2]: Kinova arm MPPI with on-GPU FK chain, K=4096 H=32 (BASELINE metric shape)
    "arm_c3": dict(model="arm", n_samples=4096, n_horizon=32, state_f64=True,
                   desc="Kinova-arm MPPI with on-GPU FK chain, K=4096 H=32 (BASELINE configs[2])"),
    # configs[1]: drone MPPI K=4096 H=32
    "drone_c2": dict(model="drone", n_samples=4096, n_horizon=32,
                     desc="Drone MPPI K=4096 H=32 (BASELINE configs[1])"),
    # configs[3] per-GPU shard: whole-body K=65536 H=64 over 8 GPUs -> 8192 per GPU
    "wholebody_c4": dict(model="wholebody", n_samples=8192, n_horizon=64,
                         desc="Whole-body MPPI, 8192 samples/GPU H=64 (BASELINE configs[3] shard)"),
    # configs[4] per-GPU share: 64 vehicles x K=8192 over 8 GPUs -> 8 vehicles per GPU
    # the 6-DoF rigid-body quadrotor (commented out in the reference), drone sizes
    "quadrotor_c2": dict(model="quadrotor", n_samples=4096, n_horizon=32,
                         desc="6-DoF quadrotor MPPI K=4096 H=32 (SURVEY §8f rank 3; configs[1] sizes)"),
    "fleet_c5": dict(model="wholebody", n_samples=8192, n_horizon=64, n_vehicles=8,
                     desc="64-vehicle whole-body fleet, 8 vehicles x K=8192 H=64 per GPU (configs[4] share)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_state(model: str, V: int) -> np.ndarray:
    rng = np.random.default_rng(0)
    rows = []
    for v in range(V):
        if model == "drone":
            rows.append([0.0, 0.0, 1.0, 0.0, 0.0, 0.0])
        elif model == "quadrotor":
            rows.append([0.0, 0.0, 1.0, 0.0, 0.0, 0.0] + [0.0] * 6)
        elif model == "arm":
            rows.append([0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0] + HOME_Q + [0.0] * 7)
        else:
            off = rng.uniform(-0.5, 0.5, 3) if v else np.zeros(3)
            joff = rng.uniform(-0.2, 0.2, 7) if v else np.zeros(7)
            rows.append(list(np.array([0.0, 0.0, 1.0]) + off) + [0.0, 0.0, 0.0, 1.0]
                        + list(np.array(HOME_Q) + joff) + [0.0] * 3 + [0.0] * 7)
    return np.asarray(rows, np.float64)


def set_targets(eng, model, V):
    rng = np.random.default_rng(1)
    for v in range(V):
        if model in ("drone", "quadrotor"):
            eng.set_target(DRONE_TARGET, vehicle=v)
        else:
            p = np.array(ARM_TARGET[0]) + (rng.uniform(-0.1, 0.1, 3) if v else 0.0)
            eng.set_target(p, ARM_TARGET[1], vehicle=v)


def load_traffic(workload: str):
    """Per-launch HBM bytes of the rollout kernel from the committed rocprofv3
    PMC summary (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), if present."""
    path = os.path.join(ROOT, "profiles", "pmc_rollout.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(workload, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(workload: str, budget_s: float):
    """The oracle (op-for-op torch-CPU restatement of the reference step, randn
    included) timed on the host cores on a bounded sample of the same workload."""
    import torch
    from oracle import mppi_oracle as O
    from quadrotor_manipulator_mppi_amd.robot.urdf_chain import load_chain
    w = WORKLOADS[workload]
    K, H, model = w["n_samples"], w["n_horizon"], w["model"]
    threads = torch.get_num_threads()
    times = []
    if model == "quadrotor":
        sig = torch.diag(torch.tensor([30.0, 1.0, 1.0, 1.0]))
        u = torch.zeros(H, 4)
        u[:, 0] = 14.7 * 9.81

        def one():
            return O.quad_step([0, 0, 1.0, 0, 0, 0], [0.0] * 6, u, O.draw_noise(K, H, sig), DRONE_TARGET)
    elif model == "drone":
        sig = torch.eye(3) * 30.0
        u = torch.zeros(H, 3)

        def one():
            return O.drone_step([0, 0, 1.0], [0, 0, 0.0], u, O.draw_noise(K, H, sig), DRONE_TARGET)
    elif model == "arm":
        chain = [O.Joint(j["name"], j["type"], j["xyz"], j["rpy"], j["axis"], j["q_index"]) for j in load_chain()]
        sig = torch.eye(7) * 0.1
        u = torch.zeros(H, 7)
        qf = np.array([0, 0, 1.0, 0, 0, 0, 1] + HOME_Q)
        vf = np.zeros(13)

        def one():
            return O.arm_step(chain, qf, vf, u, O.draw_noise(K, H, sig), *ARM_TARGET, f64=True)
    else:
        chain = [O.Joint(j["name"], j["type"], j["xyz"], j["rpy"], j["axis"], j["q_index"]) for j in load_chain()]
        sig = torch.diag(torch.tensor([30.0] * 3 + [0.1] * 7))
        u = torch.zeros(H, 10)
        rpy = O.base_rpy_from_quat([0, 0, 0, 1.0])

        def one():
            return O.wholebody_step(chain, [0, 0, 1.0], [0, 0, 0.0], HOME_Q, [0.0] * 7, rpy, u,
                                    O.draw_noise(K, H, sig), *ARM_TARGET)
    one()   # warm-up
    t_end = time.perf_counter() + budget_s
    while time.perf_counter() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        one()
        times.append(time.perf_counter() - t0)
    p50 = float(np.median(times))
    return {"value": K * H / p50, "unit": "rollout-steps/s", "cores": threads, "kind": "port",
            "p50_ms": p50 * 1e3,
            "sample": f"{len(times)} oracle control steps (torch-CPU restatement of the reference, randn "
                      f"included) at {workload} K={K} H={H}, {threads} threads, median"}


def run_workload(name, steps_n, warmup, rank, world, dist, lat_steps, timing=True):
    import torch
    from quadrotor_manipulator_mppi_amd.distributed import ShardedEngine
    w = dict(WORKLOADS[name])
    w.pop("desc")
    V = w.get("n_vehicles", 1)
    native = None if os.environ.get("MPPI_NATIVE_COMM", "1") != "0" else False
    se = ShardedEngine(seed=1234, native=native, **w)
    eng = se.engine
    set_targets(eng, w["model"], V)
    if w["model"] == "quadrotor":   # warm start at hover thrust (quadrotor_mppi.MPPI does the same)
        u = np.zeros((V, eng.H, eng.A), np.float32)
        u[..., 0] = eng.cfg.quad_mass * eng.cfg.quad_gravity
        eng.set_u_prev(u)
    state = make_state(w["model"], V)
    eng.set_state(state)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def steps(n):
        # one C call enqueues n control steps (rollout -> all-reduce over the engine's
        # RCCL communicator -> finalize when sharded); the gloo rehearsal path loops in Python
        se.run_steps(n)

    steps(warmup)
    barrier()
    t0 = time.perf_counter()
    steps(steps_n)
    eng.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    tim = None
    if timing:   # per-kernel HIP-event timing in its own region (events perturb the step rate)
        n_t = max(50, steps_n // 2)
        if world == 1:   # n launches of each kernel back to back between one event pair; the
            # median of 5 such batches (a transient clock dip on the box moves one batch, not the median)
            nb_ = max(50, n_t // 5)
            rs, fs = zip(*[eng.kernel_timing(nb_) for _ in range(5)])
            r_us, f_us = float(np.median(rs)), float(np.median(fs))
            tim = {"rollout_us": r_us, "finalize_us": f_us,
                   "method": f"HIP events around {nb_} back-to-back launches, median of 5 batches",
                   "rollout_us_batches": [round(x, 3) for x in rs]}
        else:            # sharded engines: an event pair around every launch (~2-3 us overhead each)
            eng.enable_timing(True)
            steps(n_t)
            eng.synchronize()
            t = eng.timing()
            eng.enable_timing(False)
            tim = {"rollout_us": 1e3 * t["rollout_ms_total"] / max(1, t["n_rollout"]),
                   "finalize_us": 1e3 * t["finalize_ms_total"] / max(1, t["n_finalize"]),
                   "method": "HIP event pair per launch"}
    if dist is not None:
        t = torch.tensor([dt], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # host-inclusive control-call latency (set_state H2D + step + D2H outputs + check_reach)
    lat = []
    for i in range(lat_steps + 20):
        t1 = time.perf_counter()
        se.step(state)
        if i >= 20:
            lat.append(time.perf_counter() - t1)
    out, u0, st = eng.read_outputs()
    if not os.environ.get("MPPI_FIN_DEBUG"):
        assert np.isfinite(out).all(), "non-finite control output"
    res = {"dt": dt, "tim": tim, "lat": lat, "K": eng.K, "H": eng.H, "A": eng.A, "V": V,
           "bytes": eng.rollout_bytes(), "ess": float(st[0].ess), "cfg": eng.cfg}
    eng.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--workload", default="arm_c3", choices=sorted(WORKLOADS))
    ap.add_argument("--latency-steps", type=int, default=200)
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of CPU baseline sampling")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--secondary", default="drone_c2,wholebody_c4,quadrotor_c2",
                    help="extra workloads reported (N=1 only), comma separated; '' for none")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # ranks beyond the visible devices wrap (rehearsing N ranks on fewer GPUs)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        backend = os.environ.get("MPPI_DIST_BACKEND", "nccl")   # nccl = RCCL; gloo only for rehearsal
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    if args.gpus != world:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    from quadrotor_manipulator_mppi_amd import _capi
    _capi.lib()

    r = run_workload(args.workload, args.steps, args.warmup, rank, world, dist, args.latency_steps)
    K, H, V = r["K"], r["H"], r["V"]
    per_step = r["dt"] / args.steps
    value = world * V * K * H / per_step
    tim = r["tim"]
    avg_roll_ms = tim["rollout_us"] * 1e-3
    avg_fin_ms = tim["finalize_us"] * 1e-3
    achieved = r["bytes"] / (avg_roll_ms * 1e-3) / 1e9
    lat = np.array(r["lat"]) * 1e3
    secondary = {}
    if world == 1 and args.secondary:
        for wname in [s for s in args.secondary.split(",") if s]:
            s = run_workload(wname, max(50, args.steps // 5), 20, rank, world, dist, 50)
            st = s["tim"]
            ms = st["rollout_us"] * 1e-3
            secondary[wname] = {
                "value": s["V"] * s["K"] * s["H"] / (s["dt"] / max(50, args.steps // 5)),
                "ms_per_step": 1e3 * s["dt"] / max(50, args.steps // 5),
                "latency_p50_ms": float(np.median(np.array(s["lat"]) * 1e3)) if s["lat"] else None,
                "rollout_kernel_us": ms * 1e3,
                "rollout_GBps": s["bytes"] / (ms * 1e-3) / 1e9,
                "roofline_frac": s["bytes"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
            log(f"secondary {wname}: {secondary[wname]}")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.workload, args.cpu_budget)
        log(f"cpu baseline: {cpu}")
    if rank == 0:
        traffic = load_traffic(args.workload)
        line = {
            "metric": "MPPI rollouts/sec (K x H state-steps) + control-step p50 latency, K=4096 H=32",
            "value": value, "unit": "rollout-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": per_step * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (reference C3 state/goal: home joints, base at (0,0,1), mppi.py target)",
            "config": {"workload": args.workload, "desc": WORKLOADS[args.workload]["desc"],
                       "samples_per_gpu": K, "horizon": H, "action_dim": r["A"], "vehicles_per_gpu": V,
                       "noise": "device Philox4x32-10", "state_dtype": "f64" if r["cfg"].state_f64 else "f32",
                       "parallelism": f"samples-sharded x{world}, 1 all-reduce/step" if world > 1 else "1 GPU"},
            "latency_p50_ms": float(np.median(lat)) if lat.size else None,
            "latency_p99_ms": float(np.percentile(lat, 99)) if lat.size else None,
            "kernels": {"rollout_us": avg_roll_ms * 1e3, "finalize_us": avg_fin_ms * 1e3,
                        "timing": tim["method"]},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_rollout_quad" if r["cfg"].model == 3 else "k_rollout",
                         "bytes_per_launch": r["bytes"]},
            "cpu_baseline": cpu,
            "secondary": secondary or None,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
