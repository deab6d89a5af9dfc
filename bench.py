#!/usr/bin/env python3
"""MPPI control-step benchmark (BASELINE.json metric: rollout-steps/s, K x H
state-steps, plus control-step p50 latency).

    python bench.py [--gpus 1] [--steps K] [--warmup W] [--workload arm_c3]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N ...
    python bench.py --gpus N ...      (no launcher: bench.py starts the N ranks itself, as a child)

A "step" is one MPPI control step (noise -> rollout -> FK -> cost -> softmin ->
SavGol -> update) over one batch of synthetic state/goal input.

Workloads (the same primary workload at every N, so the driver's per-N values form one curve):
* ``arm_c3`` -- the configuration BASELINE.json's metric is quoted on (Kinova arm, K=4096
  H=32, configs[2]).  At N=1 it is the plain control step.  Under torch.distributed.run
  (N ranks) every rank runs the K=4096 H=32 step as its shard of one K=4096*N controller
  (global samples [g*4096, (g+1)*4096), the ranks' softmin partials combined every step by
  the peer exchange): per-GPU work fixed, ``scaling`` "weak".
* ``secondary.c4`` -- the north star, whole-body K=65536 H=64 (configs[3]) with the samples
  split 65536/N per rank (strong scaling at the fixed K), at every N: in the plain N=1 run
  (one GPU, K=65536) and in every N>1 run (``--secondary-multi``).
``value`` is the whole job's rollout-steps per second with state and warm start resident
on the GPU (back-to-back steps, one host sync), bracketed by barrier + synchronize on
both sides and the max over ranks.  The host-inclusive call latency (state H2D, outputs,
check_reach) is ``latency_p50/p99_ms`` (never ``value``).

Rank 0 prints ONE JSON line on stdout; progress goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HOME_Q = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]                # kinova.py:135
ARM_TARGET = ([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])   # mppi.py:71-72
DRONE_TARGET = [1.0, 2.0, 3.4]                                   # drone_mppi.py:141
PREWARM_US = 200        # latency_100hz_prewarm's window (mppi_set_prewarm)
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
C4_K_TOTAL = 65536      # BASELINE configs[3]: whole-body K=65536 H=64 over the node

WORKLOADS = {
    # configs[2]: Kinova arm MPPI with on-GPU FK chain, K=4096 H=32 (BASELINE metric shape)
    "arm_c3": dict(model="arm", n_samples=4096, n_horizon=32, state_f64=True,
                   desc="Kinova-arm MPPI with on-GPU FK chain, K=4096 H=32 (BASELINE configs[2])"),
    # configs[1]: drone MPPI K=4096 H=32
    "drone_c2": dict(model="drone", n_samples=4096, n_horizon=32,
                     desc="Drone MPPI K=4096 H=32 (BASELINE configs[1])"),
    # configs[3], the north star: whole-body K=65536 H=64, samples split over the ranks
    "c4": dict(model="wholebody", n_samples=C4_K_TOTAL, n_horizon=64, strong=True,
               desc="Whole-body MPPI K=65536 H=64, samples split K/N per GPU (BASELINE configs[3])"),
    # configs[3] per-GPU shard at N=8: whole-body 8192 samples H=64 on one GPU
    "wholebody_c4": dict(model="wholebody", n_samples=8192, n_horizon=64,
                         desc="Whole-body MPPI, 8192 samples/GPU H=64 (BASELINE configs[3] shard at N=8)"),
    # the 6-DoF rigid-body quadrotor (commented out in the reference), drone sizes
    "quadrotor_c2": dict(model="quadrotor", n_samples=4096, n_horizon=32,
                         desc="6-DoF quadrotor MPPI K=4096 H=32 (SURVEY §8f rank 3; configs[1] sizes)"),
    # configs[4]: the 64-vehicle fleet, K=8192 H=64 each, its vehicles split over the ranks (SURVEY §8e:
    # "prefer vehicles across GPUs", no exchange; 8 per GPU at N=8, all 64 on one GPU at N=1)
    "fleet_c5": dict(model="wholebody", n_samples=8192, n_horizon=64, n_vehicles=64, mode="vehicles", strong=True,
                     desc="64-vehicle whole-body fleet K=8192 H=64, vehicles split over the GPUs, no exchange "
                          "(BASELINE configs[4])"),
    # configs[4] per-GPU share at N=8: 8 vehicles x K=8192 H=64 on one GPU
    "fleet_c5_share": dict(model="wholebody", n_samples=8192, n_horizon=64, n_vehicles=8,
                           desc="64-vehicle whole-body fleet, 8 vehicles x K=8192 H=64 per GPU (configs[4] share)"),
    # the N=8 rank's whole step on one GPU: the C4 shard through the engine-owned RCCL
    # communicator with one rank (rollout -> PACK -> ncclAllReduce -> finalize from C)
    "c4_shard_native1": dict(model="wholebody", n_samples=8192, n_horizon=64, native=True, mode="rccl",
                             desc="Whole-body 8192 samples H=64 through a 1-rank RCCL communicator "
                                  "(the N=8 rank's step of BASELINE configs[3])"),
    # the same rank step through the peer exchange (no collective: finalize blocks exchange their
    # partials through the ranks' exchange regions; one rank exchanges with itself)
    "c4_shard_peer1": dict(model="wholebody", n_samples=8192, n_horizon=64, native=True, mode="peer",
                           desc="Whole-body 8192 samples H=64 through the 1-rank peer exchange "
                                "(the N=8 rank's step of BASELINE configs[3])"),
    # configs[3] through the mechanism north_star names, "a single RCCL allreduce": the C4 split
    # 65536/N per rank, the engine-owned RCCL communicator over all N ranks (one ncclAllReduce per step)
    "c4_rccl": dict(model="wholebody", n_samples=C4_K_TOTAL, n_horizon=64, strong=True, native=True, mode="rccl",
                    desc="Whole-body MPPI K=65536 H=64, samples split K/N per GPU, one RCCL all-reduce per step "
                         "(BASELINE configs[3], the north star's mechanism)"),
}

# the CPU baseline's shapes (C4 K-reduced: the full C4 on CPU is impractical)
CPU_SHAPES = {
    "c1_drone_k128_h20": ("drone", 128, 20),
    "c2_drone_k4096_h32": ("drone", 4096, 32),
    "c3_arm_k4096_h32": ("arm", 4096, 32),
    "c4r_wholebody_k4096_h64": ("wholebody", 4096, 64),
}
CPU_HEADLINE = {"arm_c3": "c3_arm_k4096_h32", "drone_c2": "c2_drone_k4096_h32",
                "wholebody_c4": "c4r_wholebody_k4096_h64", "c4": "c4r_wholebody_k4096_h64",
                "fleet_c5": "c4r_wholebody_k4096_h64", "fleet_c5_share": "c4r_wholebody_k4096_h64"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ------------------------------------------------------------------------------ N ranks from one command
def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(n: int, argv, port: int = 0, script: str = ""):
    """The child that runs ``bench.py <argv>`` as N ranks on this node: torch.distributed.run with a
    static rendezvous on 127.0.0.1 (the driver's own launch line), every argument forwarded as given."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port or free_port()),
            script or os.path.abspath(__file__)] + list(argv)


def is_bench_line(s: str) -> bool:
    try:
        d = json.loads(s)
    except ValueError:
        return False
    return isinstance(d, dict) and "metric" in d and "value" in d


def spawn_ranks(cmd, out=None) -> int:
    """``bench.py --gpus N`` (N > 1) started without a launcher: run ``cmd`` (``launcher_cmd``) as a
    CHILD process -- never exec, this process has not touched the GPU and stays the parent -- relay
    exactly one bench line from the child's stdout (rank 0's; anything else there goes to stderr)
    and return the child's exit code.  SIGTERM / SIGINT to this process are passed on to the child's
    process group, so a driver that stops the parent stops the ranks too."""
    import signal
    import subprocess
    out = out or sys.stdout
    env = dict(os.environ, MPPI_BENCH_SPAWNED="1")
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    log(f"bench: no launcher in the environment, starting the ranks as a child: {' '.join(cmd)}")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env, start_new_session=True)

    def forward(sig, _frame):
        try:
            os.killpg(proc.pid, sig)
        except OSError:
            pass
    old = {s: signal.signal(s, forward) for s in (signal.SIGTERM, signal.SIGINT)}
    lines = []
    try:
        for ln in proc.stdout:
            s = ln.strip()
            if is_bench_line(s):
                lines.append(s)
            elif s:
                log(f"[child stdout] {s}")
        rc = proc.wait()
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    if len(lines) > 1:
        log(f"bench: the child printed {len(lines)} bench lines; relaying the last")
    if lines:
        print(lines[-1], file=out, flush=True)
    elif rc == 0:
        log("bench: the ranks exited 0 without a bench line")
        rc = 1
    return rc


def build_info():
    """The library build this run loaded (written by quadrotor_manipulator_mppi_amd/build.py)."""
    try:
        with open(os.path.join(ROOT, "quadrotor_manipulator_mppi_amd", "lib", "BUILD_INFO.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def make_state(model: str, V: int) -> np.ndarray:
    """Synthetic state rows of a fleet of V vehicles (row v = fleet-wide vehicle v: a vehicle-sharded
    rank takes its own rows of the whole fleet's array)."""
    rng = np.random.default_rng(0)
    rows = []
    for v in range(V):
        if model == "drone":
            rows.append([0.0, 0.0, 1.0, 0.0, 0.0, 0.0])
        elif model == "quadrotor":
            rows.append([0.0, 0.0, 1.0, 0.0, 0.0, 0.0] + [0.0] * 6)
        elif model == "arm":
            rows.append([0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0] + HOME_Q + [0.0] * 7)
        else:   # vehicle v > 0 offset by U(-0.5,0.5) m xyz, U(-0.2,0.2) rad joints
            off = rng.uniform(-0.5, 0.5, 3) if v else np.zeros(3)
            joff = rng.uniform(-0.2, 0.2, 7) if v else np.zeros(7)
            rows.append(list(np.array([0.0, 0.0, 1.0]) + off) + [0.0, 0.0, 0.0, 1.0]
                        + list(np.array(HOME_Q) + joff) + [0.0] * 3 + [0.0] * 7)
    return np.asarray(rows, np.float64)


def set_targets(eng, model, vehicles):
    """Targets of the fleet-wide vehicles ``vehicles`` (a range), set on the engine's vehicles 0..n-1."""
    rng = np.random.default_rng(1)
    for v in range(vehicles.stop):
        p = np.array(ARM_TARGET[0]) + (rng.uniform(-0.1, 0.1, 3) if v else 0.0)   # drawn for every v, in order
        if v not in vehicles:
            continue
        if model in ("drone", "quadrotor"):
            eng.set_target(DRONE_TARGET, vehicle=v - vehicles.start)
        else:   # targets jittered by +-0.1 m for v > 0
            eng.set_target(p, ARM_TARGET[1], vehicle=v - vehicles.start)


def shape_key(model: str, K: int, H: int, V: int = 1) -> str:
    """Key of one rollout launch shape in profiles/pmc_rollout.json (traffic is per shape:
    the c4 workload's per-rank K is 65536/N)."""
    return f"{model}_k{K}_h{H}" + (f"_v{V}" if V > 1 else "")


def load_traffic(key: str):
    """Per-launch HBM bytes of the rollout kernel at one launch shape (``shape_key``) from the
    committed rocprofv3 PMC summary (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), and where
    it came from; (None, None) for a shape without counters (never another shape's figure)."""
    path = os.path.join(ROOT, "profiles", "pmc_rollout.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    w = d.get(key)
    if not w or w.get("hbm_bytes_per_launch") is None:
        return None, None
    src = (f"profiles/pmc_rollout.json[{key}]: rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE, "
           f"separate passes, avg per k_rollout launch of this shape; collected on build {w.get('build_head', '?')}")
    return w["hbm_bytes_per_launch"], src


# ------------------------------------------------------------------------------ CPU baseline
def _cpu_step_fn(model: str, K: int, H: int):
    """One control step of the oracle (op-for-op torch-CPU restatement of the reference's
    compute_control_input, randn included) at a shape with the reference's C1-C4 inputs."""
    import torch
    from oracle import mppi_oracle as O
    from quadrotor_manipulator_mppi_amd.robot.urdf_chain import load_chain
    chain = [O.Joint(j["name"], j["type"], j["xyz"], j["rpy"], j["axis"], j["q_index"]) for j in load_chain()]
    if model == "quadrotor":
        sig = torch.diag(torch.tensor([30.0, 1.0, 1.0, 1.0]))
        u = torch.zeros(H, 4)
        u[:, 0] = 14.7 * 9.81
        return lambda: O.quad_step([0, 0, 1.0, 0, 0, 0], [0.0] * 6, u, O.draw_noise(K, H, sig), DRONE_TARGET)
    if model == "drone":
        sig = torch.eye(3) * 30.0
        u = torch.zeros(H, 3)
        return lambda: O.drone_step([0, 0, 1.0], [0, 0, 0.0], u, O.draw_noise(K, H, sig), DRONE_TARGET)
    if model == "arm":
        sig = torch.eye(7) * 0.1
        u = torch.zeros(H, 7)
        qf = np.array([0, 0, 1.0, 0, 0, 0, 1] + HOME_Q)
        vf = np.zeros(13)
        return lambda: O.arm_step(chain, qf, vf, u, O.draw_noise(K, H, sig), *ARM_TARGET, f64=True)
    sig = torch.diag(torch.tensor([30.0] * 3 + [0.1] * 7))
    u = torch.zeros(H, 10)
    rpy = O.base_rpy_from_quat([0, 0, 0, 1.0])
    return lambda: O.wholebody_step(chain, [0, 0, 1.0], [0, 0, 0.0], HOME_Q, [0.0] * 7, rpy, u,
                                    O.draw_noise(K, H, sig), *ARM_TARGET)


def _time_cell(fn, budget_s: float, min_steps: int = 3, warmup: int = 2):
    for _ in range(warmup):
        fn()
    times = []
    t_end = time.perf_counter() + budget_s
    while time.perf_counter() < t_end or len(times) < min_steps:
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
    return np.array(times)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(workload: str, cell_budget_s: float):
    """the oracle's control step (randn included) at C1, C2, C3 and a
    K-reduced C4, with torch's full thread pool (the job's share of the host cores) and
    with one thread, p50 and p99.  The headline is the cell of this run's workload."""
    import torch
    n_all = torch.get_num_threads()
    cells = {}
    # the thread counts: the job's share of the host (torch's pool = OMP_NUM_THREADS, 16 per GPU
    # on the GPU pool, whose rule is to stay within that share), 1, and a midpoint, so the cells
    # show how the oracle step scales with threads
    mid = max(2, n_all // 4) if n_all >= 4 else None
    counts = [("threads_all", n_all)] + ([(f"threads_{mid}", mid)] if mid and mid != n_all else []) + [("threads_1", 1)]
    for name, (model, K, H) in CPU_SHAPES.items():
        fn = _cpu_step_fn(model, K, H)
        cells[name] = {"model": model, "K": K, "H": H}
        for tag, nt in counts:
            torch.set_num_threads(nt)
            t = _time_cell(fn, cell_budget_s)
            p50, p99 = float(np.median(t)), float(np.percentile(t, 99))
            cells[name][tag] = {"threads": nt, "steps": int(t.size), "p50_ms": p50 * 1e3, "p99_ms": p99 * 1e3,
                                "rollout_steps_per_s": K * H / p50}
            log(f"cpu {name} {tag}={nt}: p50 {p50 * 1e3:.2f} ms p99 {p99 * 1e3:.2f} ms ({t.size} steps)")
        torch.set_num_threads(n_all)
    head = cells[CPU_HEADLINE.get(workload, "c3_arm_k4096_h32")]
    try:
        local = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        local = None
    host = {"os_cpu_count": os.cpu_count(), "cpu_model": cpu_model(), "torch_threads": n_all,
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"), "affinity_cpus": local,
            "note": ("threads_all = torch's pool = the job's CPU share (OMP_NUM_THREADS); the GPU pool asks a job "
                     "to stay within it, so the affinity set's remaining cores (other GPUs' shares) are not used")}
    hv = head["threads_all"]
    line = {"value": hv["rollout_steps_per_s"], "unit": "rollout-steps/s", "cores": n_all, "kind": "port",
            "p50_ms": hv["p50_ms"], "p99_ms": hv["p99_ms"],
            "value_1thread": head["threads_1"]["rollout_steps_per_s"],
            "sample": (f"{hv['steps']} oracle control steps (torch-CPU op-for-op restatement of the reference, "
                       f"randn included) at {head['model']} K={head['K']} H={head['H']}, {n_all} threads "
                       f"(os.cpu_count()={host['os_cpu_count']}, {host['cpu_model']}), median; "
                       f"{cell_budget_s:.1f} s per cell, all cells in cpu_baseline_all"),
            "host": host}
    return line, cells


# ------------------------------------------------------------------------------ GPU runs
def reduce_max(vals, dist, device):
    """Max over ranks of a list of floats (one all-reduce on the backend's device)."""
    if dist is None:
        return [float(v) for v in vals]
    import torch
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def timed_batches(run, n_batches, barrier, prime=None):
    """The contract's timed region, repeated: each batch is EXACTLY `steps` control steps
    bracketed by barrier + synchronize on both sides (wall clock); returns the per-batch
    seconds and the host time each batch's enqueue took (when that is close to the batch,
    the step was host-bound).  The line's ms_per_step is the median batch / steps (a 20-step
    batch is ~0.2 ms, so one host hiccup at a bracket would otherwise set the number)."""
    out, enq = [], []
    for _ in range(n_batches):
        if prime is not None:   # the warmup steps, untimed, ahead of every batch (not only the first)
            prime()
        barrier()
        t0 = time.perf_counter()
        run()
        enq.append(time.perf_counter() - t0)   # host time to enqueue the batch (diagnostic)
        barrier()
        out.append(time.perf_counter() - t0)
    return out, enq


def latency_at_rate(se, state, calls: int, period_s: float = 0.01, idle_s: float = 0.1):
    """Control calls at the node's cadence: the arm node ticks at 100 Hz (kinova.py:101,
    rospy.Rate(100)), so between calls the GPU idles ~10 ms and its clocks drop (profiles/r04/ramp).
    After ``idle_s`` of idle (no heat-up), ``calls`` control calls, each started on the next
    ``period_s`` tick as rospy.Rate.sleep does; host-inclusive wall time per call."""
    time.sleep(idle_s)
    lat = []
    nxt = time.perf_counter()
    for _ in range(calls):
        t1 = time.perf_counter()
        se.step(state)
        lat.append(time.perf_counter() - t1)
        nxt += period_s
        d = nxt - time.perf_counter()
        if d > 0:
            time.sleep(d)
        else:   # (a call longer than the period: the next tick starts now)
            nxt = time.perf_counter()
    return lat


class StepsGivenUp(RuntimeError):
    """A peer-exchange step was given up during a measurement.  Every rank raises it at the same
    point: the verdict comes from ShardedEngine.synchronize(), itself a collective."""


def run_workload(name, steps_n, warmup, world, dist, lat_steps, timing=True, batches=1, lat_rate_calls=0):
    import torch
    from quadrotor_manipulator_mppi_amd.distributed import ShardedEngine
    w = dict(WORKLOADS[name])
    w.pop("desc")
    strong = w.pop("strong", False)
    force_native = w.pop("native", None)
    mode = w.pop("mode", None)
    if strong and mode != "vehicles":   # (a vehicle-split fleet: ShardedEngine splits the vehicles)
        if w["n_samples"] % world:
            raise SystemExit(f"{name}: K={w['n_samples']} does not split over {world} ranks")
        w["n_samples"] //= world
    native = force_native if force_native is not None else (
        None if os.environ.get("MPPI_NATIVE_COMM", "1") != "0" else False)
    if native is None and world > 1:
        # the engine-owned exchange (peer, else RCCL, else the torch collective) over any process group:
        # a rehearsal's gloo group carries the peer exchange's handle all-gather just as RCCL's would
        native = True
    se = ShardedEngine(seed=1234, native=native, mode=mode, **w)
    try:
        eng = se.engine
        V = eng.V   # this rank's vehicles (the fleet-wide ones: se.vehicles)
        set_targets(eng, w["model"], se.vehicles)
        if w["model"] == "quadrotor":   # warm start at hover thrust (quadrotor_mppi.MPPI does the same)
            u = np.zeros((V, eng.H, eng.A), np.float32)
            u[..., 0] = eng.cfg.quad_mass * eng.cfg.quad_gravity
            eng.set_u_prev(u)
        state = make_state(w["model"], se.vehicles.stop)[se.vehicles.start:]
        eng.set_state(state)
        red_dev = "cuda" if dist is not None and dist.get_backend() == "nccl" else "cpu"

        def barrier():
            # torch's synchronize first: it covers torch's own streams (idle here: the steps run on
            # the engine's native queue or stream) and costs ~3 us of host time even on an idle
            # device, which it now spends while the batch still runs; eng.synchronize() then waits
            # for the batch's completion signal.  Both still bracket every batch.
            torch.cuda.synchronize()
            # on a multi-rank peer exchange se.synchronize() is itself a collective: the ranks agree that
            # no step was given up (a MAX all-reduce, which doubles as the barrier); a timeout would have
            # resynchronised the ranks and voids the measurement
            if se.synchronize():
                raise StepsGivenUp(f"{name}: a peer-exchange step timed out (ranks resynchronised): no valid timing")
            if dist is not None:
                if se.mode != "peer":
                    dist.barrier()
                torch.cuda.synchronize()

        se.run_steps(warmup)   # one C call enqueues n steps (rollout -> all-reduce -> finalize when sharded)
        barrier()
        tim = None
        if timing:   # per-kernel HIP-event timing in its own region, before the timed batches
            n_t = max(200, steps_n // 5)
            # n launches of each kernel back to back between one event pair, then n (rollout,
            # finalize) pairs as a step runs them; median of 7 batches (a transient clock dip on
            # the box moves one batch, not the median)
            rs, fs, ps = zip(*[eng.kernel_timing_ex(n_t) for _ in range(7)])
            r_us, f_us, p_us = float(np.median(rs)), float(np.median(fs)), float(np.median(ps))
            tim = {"rollout_us": r_us, "finalize_us": f_us, "pair_us": p_us,
                   "rollout_in_step_us": max(r_us, p_us - f_us),
                   "method": f"HIP events around {n_t} back-to-back launches (and {n_t} rollout+finalize pairs), "
                             f"median of 7 batches, on the engine stream",
                   "rollout_us_batches": [round(x, 3) for x in rs]}
            if se.mode == "rccl":   # the step's one collective alone (a collective call on every rank)
                tim["allreduce_us"] = float(np.median([eng.exchange_timing(n_t) for _ in range(3)]))
            se.run_steps(max(1, warmup))   # back to the control loop (repacks the slots the timing summed)
            barrier()
        # every batch follows its own W untimed warmup steps (the contract's warmup, repeated per
        # batch): the host's launch rate after a pause is what a batch then measures less of
        # (profiles/r03/bench_prime_probe.txt: 20-step lines 11.1-11.3 us primed vs 11.0-12.8 not)
        prime = None if os.environ.get("MPPI_BENCH_PRIME", "1") == "0" else (lambda: se.run_steps(max(1, warmup)))
        # GPU heat-up: the MI355X raises its clocks over ~10 ms of sustained load and drops them again
        # when idle (profiles/r04/ramp: C3 9.93 us/step in a 20-step batch after 50 ms idle, 9.42
        # after a 200-step burst, 9.02-9.05 after >= 1000 steps; consecutive 100-step chunks 9.33 ->
        # 8.73 over the first ~10 ms).  So ahead of each batch's W warmup steps the steps run back to
        # back for HEAT_MS first, and a batch measures the sustained rate, not the power-state ramp --
        # at 20 steps (0.2 ms) it would otherwise time mostly the ramp.  The same step count on every
        # rank (from the max-over-ranks step time), so peer-exchange ranks stay in lockstep.  The
        # batches without the heat-up are reported too (timing.ms_per_step_batches_no_heatup).
        heat_ms = float(os.environ.get("MPPI_BENCH_HEAT_MS", "15"))
        n_heat = 0
        if heat_ms > 0:
            # the step's wall time from one timed 20-step batch (a host-paced step -- the torch
            # collective's host round trip -- runs far longer than its kernel pair, and a heat-up sized
            # from the pair ran ~0.3 s of such steps per batch), never below the kernel pair's time
            barrier()
            t0 = time.perf_counter()
            se.run_steps(20)
            barrier()
            t_step = (time.perf_counter() - t0) / 20
            if tim is not None:
                t_step = max(t_step, tim["pair_us"] * 1e-6)
            t_step = reduce_max([t_step], dist, red_dev)[0]
            n_heat = int(min(20000, max(100, np.ceil(heat_ms * 1e-3 / t_step))))
        bt_cold, _ = timed_batches(lambda: se.run_steps(steps_n), batches, barrier, prime)
        bt_cold = reduce_max(bt_cold, dist, red_dev)
        heat_prime = prime
        if n_heat:
            heat_prime = (lambda: (se.run_steps(n_heat), se.run_steps(max(1, warmup)))) if prime is not None else \
                (lambda: se.run_steps(n_heat))
        bt, benq = timed_batches(lambda: se.run_steps(steps_n), batches, barrier, heat_prime)
        bt = reduce_max(bt, dist, red_dev)    # each batch: the slowest rank
        if tim is not None and dist is not None:   # the slowest rank's kernels
            tim["rollout_us_max_over_ranks"], tim["rollout_in_step_us_max_over_ranks"] = reduce_max(
                [tim["rollout_us"], tim["rollout_in_step_us"]], dist, red_dev)
        # host-inclusive control-call latency (set_state H2D + step + D2H outputs + check_reach)
        lat = []
        for i in range(lat_steps + 20 if lat_steps else 0):
            t1 = time.perf_counter()
            se.step(state)
            if i >= 20:
                lat.append(time.perf_counter() - t1)
        eng.synchronize()
        lat100 = latency_at_rate(se, state, lat_rate_calls) if lat_rate_calls else []
        lat100p, pw_touches = [], 0
        if lat_rate_calls:   # the same cadence with the engine's prewarm on (mppi_set_prewarm)
            eng.set_prewarm(PREWARM_US)
            lat100p = latency_at_rate(se, state, lat_rate_calls)
            pw_touches = eng.prewarm()[1]
            eng.set_prewarm(0)
        if not lat and not lat100:
            se.step(state)
        dispatch = eng.dispatch_info()   # "<aql | hip: why not>; calls: <aql | hip>" (batches; control calls)
        out, u0, st = eng.read_outputs()
        if not os.environ.get("MPPI_FIN_DEBUG"):
            assert np.isfinite(out).all(), "non-finite control output"
        comm = eng.comm_info() if se.mode == "rccl" else None
        # the peer exchange's own rank count: the ranks whose word reached this rank's region in the
        # connection probe's kernel phase (mppi_peer_info), min over ranks
        peer_n = None
        if se.mode == "peer":
            peer_n = int(-reduce_max([-float(eng.peer_info()[0])], dist, red_dev)[0])
        res = {"batches_s": bt, "enqueue_s": benq, "batches_s_no_heatup": bt_cold, "heat_steps": n_heat, "lat100": lat100,
               "lat100_prewarm": lat100p, "prewarm_touches": pw_touches,
               "heat_ms": heat_ms, "dispatch": dispatch, "dt": float(np.median(bt)), "tim": tim, "lat": lat,
               "K": eng.K, "H": eng.H,
               "A": eng.A, "V": V, "strong": strong, "bytes": eng.rollout_bytes(), "ess": float(st[0].ess),
               "model": w["model"], "state_f64": bool(eng.cfg.state_f64), "native": se.native, "exchange": se.mode,
               "native_error": se.native_error, "world": world,
               "backend": dist.get_backend() if dist is not None else None,
               "rccl_nranks": comm[0] if comm else None, "rccl_rank": comm[1] if comm else None,
               "peer_ranks_connected": peer_n, "agree_every": se.agree_every if se.mode == "peer" and world > 1 else None,
               "process_group": ({"backend": dist.get_backend(), "size": dist.get_world_size()} if dist is not None
                                 else None)}
    finally:   # (also when a step is given up or a call raises: the next workload gets a clean device)
        se.engine.close()
    return res


def roofline_of(r, steps_n):
    """Roofline of the dominant kernel (k_rollout) at this rank's launch shape, and the
    step-level fraction: the rank's rollout bytes per control step / the step time / peak
    (= N*bytes / step / (N*8 TB/s) for N ranks)."""
    tim = r["tim"]
    us = tim["rollout_in_step_us"]
    achieved = r["bytes"] / (us * 1e-6) / 1e9
    step_s = r["dt"] / steps_n
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "kernel": "k_rollout_quad" if r["model"] == "quadrotor" else "k_rollout",
            "bytes_per_launch": r["bytes"], "kernel_us": us,
            "launch_shape": shape_key(r["model"], r["K"], r["H"], r["V"]),
            "kernel_us_basis": "rollout in a control step: (rollout+finalize pair) - finalize, >= back-to-back",
            "frac_back_to_back": r["bytes"] / (tim["rollout_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS,
            "frac_step": r["bytes"] / step_s / 1e9 / HBM_PEAK_GBS,
            "frac_step_basis": "per-rank rollout bytes per control step / median step time (whole step: rollout, "
                              "[PACK, all-reduce,] finalize) / 8 TB/s; equals N*bytes/step/(N*8 TB/s)"}


def measured_hbm(local: int, nbytes: int = 1 << 30, reps: int = 10):
    """HBM bandwidth re-measured on this box: a write-only fill and a copy of
    1 GiB fp32 buffers (torch's own kernels), event-timed, median of ``reps``.  Reported next
    to the 8 TB/s spec peak, which stays the roofline's ``peak``."""
    import torch
    dev = torch.device(f"cuda:{local}")
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    out = {}
    for name, fn, moved in (("fill_GBps", lambda: a.fill_(1.0), nbytes),
                            ("copy_GBps", lambda: b.copy_(a), 2 * nbytes)):
        fn()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        out[name] = moved / float(np.median(ts)) / 1e9
    del a, b
    torch.cuda.empty_cache()
    out["method"] = "torch fill_ (write) and copy_ (read+write) of 1 GiB fp32, event-timed, median of 10"
    return out


def auto_batches(steps_n: int) -> int:
    """Timed batches for the median: 7 for short runs (the driver's --steps 20), fewer as
    each batch gets long enough to amortise its brackets."""
    return 7 if steps_n <= 100 else 3 if steps_n <= 1000 else 1


def make_line(workload, r, args, secondary=None, cpu=None, cpu_all=None, measured=None):
    """The one JSON line (bench contract) from rank 0's view of the max-over-ranks results."""
    world = r["world"]
    K, H, V = r["K"], r["H"], r["V"]
    per_step = r["dt"] / args.steps
    value = world * V * K * H / per_step
    tim = r["tim"]
    lat = np.array(r["lat"]) * 1e3
    rf = roofline_of(r, args.steps) if tim is not None else None
    if rf is not None:
        traffic, traffic_src = load_traffic(rf["launch_shape"])
        rf.update({"traffic": traffic, "traffic_source": traffic_src,
                   "traffic_over_algorithmic": traffic / r["bytes"] if traffic else None})
        if measured:
            rf.update({"peak_measured": measured, "frac_of_measured_fill": rf["achieved"] / measured["fill_GBps"]})
    w = WORKLOADS[workload]
    r.setdefault("exchange", "rccl" if r["native"] else "torch")
    line = {
        "metric": "MPPI rollouts/sec (K x H state-steps) + control-step p50 latency, K=4096 H=32",
        "value": value, "unit": "rollout-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": per_step * 1e3, "higher_is_better": True,
        "scaling": "strong" if r["strong"] else "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (reference state/goal: home joints, base at (0,0,1), mppi.py / drone_mppi.py targets; "
                "device Philox noise)",
        "config": {"workload": workload, "desc": w["desc"],
                   "samples_total": world * K * V if not r["strong"] else w["n_samples"], "samples_per_gpu": K,
                   "horizon": H, "action_dim": r["A"], "vehicles_per_gpu": V,
                   "noise": "device Philox4x32-10 (+2x32)", "state_dtype": "f64" if r["state_f64"] else "f32",
                   "parallelism": ((f"samples sharded over {world} GPUs, " +
                                    ("peer exchange inside each step's finalize" if r["exchange"] == "peer"
                                     else "1 all-reduce/step")) if world > 1 else "1 GPU")},
        "timing": {"timed_batches": len(r["batches_s"]), "steps_per_batch": args.steps,
                   "ms_per_step_batches": [round(1e3 * b / args.steps, 6) for b in r["batches_s"]],
                   "enqueue_ms_per_step_batches": [round(1e3 * b / args.steps, 6) for b in r.get("enqueue_s", [])],
                   "dispatch": r.get("dispatch"),
                   "heatup_steps_per_batch": r.get("heat_steps"),
                   "ms_per_step_batches_no_heatup": [round(1e3 * b / args.steps, 6) for b in r.get("batches_s_no_heatup", [])],
                   "ms_per_step_no_heatup": (1e3 * float(np.median(r["batches_s_no_heatup"])) / args.steps
                                             if r.get("batches_s_no_heatup") else None),
                   "basis": "median over the batches; each batch = a GPU heat-up (`heatup_steps_per_batch` back-to-back "
                            "steps, ~15 ms: the clocks' ramp under sustained load, profiles/r04/ramp), `warmup` untimed "
                            "steps, then exactly `steps` control steps bracketed by barrier + synchronize (wall clock), "
                            "max over ranks; the same batches without the heat-up: ms_per_step_no_heatup"},
        "latency_p50_ms": float(np.median(lat)) if lat.size else None,
        "latency_p99_ms": float(np.percentile(lat, 99)) if lat.size else None,
        "latency_100hz": latency_100hz(r.get("lat100"), lat),
        "latency_100hz_prewarm": latency_100hz(r.get("lat100_prewarm"), lat, prewarm_us=PREWARM_US,
                                               touches=r.get("prewarm_touches")),
        "kernels": {k: v for k, v in tim.items() if k != "rollout_us_batches"} if tim is not None else None,
        "roofline": rf,
        "cpu_baseline": cpu,
        "cpu_baseline_all": cpu_all,
        "secondary": secondary or None,
        "build": build_info(),
    }
    if world > 1 or r["native"]:
        line["multi_gpu"] = {
            "world_size": world, "backend": r["backend"],
            "rccl_nranks": r["rccl_nranks"], "rccl_rank": r["rccl_rank"],
            "rccl_nranks_source": "ncclCommCount of the engine's communicator" if r["exchange"] == "rccl" else
                                  "no RCCL communicator in this run",
            "exchange": r["exchange"],
            "collective": {"peer": "none: peer exchange (finalize blocks store tagged partials into every rank's "
                                   "IPC-mapped exchange region over xGMI and combine them from their own)",
                           "rccl": "engine-owned RCCL communicator: ncclAllReduce(SUM) of zero-padded "
                                   "partial-record slots",
                           "torch": f"torch.distributed ({r['backend']}) all_reduce(SUM) of the slots",
                           "vehicles": "none: the fleet's vehicles split over the ranks (each rank a whole "
                                       "controller of its vehicles), nothing exchanged"}[r["exchange"]],
            "allreduce_us": tim.get("allreduce_us") if tim else None,
            "peer_ranks_connected": r.get("peer_ranks_connected"),
            "peer_ranks_connected_source": ("mppi_peer_info: ranks whose tagged word reached this rank's region in the "
                                            "connection probe's kernel phase, min over ranks")
                                           if r.get("peer_ranks_connected") is not None else None,
            "peer_agree_every": r.get("agree_every"),
            "process_group": r.get("process_group"),
            "ranks_per_gpu": r.get("ranks_per_gpu"),
            "native_comm_error": r["native_error"],
            "rollout_us_max_over_ranks": tim.get("rollout_in_step_us_max_over_ranks") if tim else None,
            "payload_bytes_per_rank": int((4 + r["A"] * H + 3) // 4 * 4 * 4 * V)}
    return line


def latency_100hz(lat100, lat_b2b, prewarm_us=0, touches=None):
    """The control call at the node's 100 Hz cadence (latency_at_rate) beside the back-to-back one;
    with ``prewarm_us`` the engine's prewarm (mppi_set_prewarm) ran with that window."""
    if not lat100:
        return None
    x = np.array(lat100) * 1e3
    p50 = float(np.median(x))
    b2b = float(np.median(lat_b2b)) if len(lat_b2b) else None
    what = ("host-inclusive control call (state in, outputs, check_reach) started on every 10 ms tick after "
            "100 ms idle, no heat-up: the arm node's rospy.Rate(100) loop (kinova.py:101); the GPU idles "
            "~10 ms between calls")
    r = {"p50_ms": p50, "p99_ms": float(np.percentile(x, 99)), "mean_ms": float(x.mean()), "calls": int(x.size),
         "period_ms": 10.0, "vs_back_to_back_p50": p50 / b2b if b2b else None}
    if prewarm_us:
        what += (f"; the engine's prewarm on (mppi_set_prewarm, window {prewarm_us} us): its native queue touched "
                 "every 25 us from the window's start until the predicted call")
        r.update(prewarm_us=prewarm_us, prewarm_touches=touches)
    r["what"] = what
    return r


def secondary_entry(s, ns):
    rf = roofline_of(s, ns)
    e = {"value": s["world"] * s["V"] * s["K"] * s["H"] / (s["dt"] / ns), "unit": "rollout-steps/s",
         "ms_per_step": 1e3 * s["dt"] / ns,
         "latency_p50_ms": float(np.median(np.array(s["lat"]) * 1e3)) if s["lat"] else None,
         "n_gpus": s["world"], "scaling": "strong" if s["strong"] else "weak",
         "samples": s["K"], "samples_total": s["world"] * s["K"],
         "horizon": s["H"], "vehicles": s["V"],
         "rollout_kernel_us": rf["kernel_us"], "rollout_back_to_back_us": s["tim"]["rollout_us"],
         "finalize_us": s["tim"]["finalize_us"], "rollout_GBps": rf["achieved"],
         "roofline_frac": rf["frac"], "roofline_frac_back_to_back": rf["frac_back_to_back"],
         "roofline_frac_step": rf["frac_step"]}
    if s["native"]:
        e.update({"exchange": s.get("exchange", "rccl"), "allreduce_us": s["tim"].get("allreduce_us"),
                  "rccl_nranks": s["rccl_nranks"], "peer_ranks_connected": s.get("peer_ranks_connected")})
    if s["world"] > 1:
        e.update({"exchange": s["exchange"], "native_comm_error": s["native_error"],
                  "rccl_nranks": s["rccl_nranks"], "peer_ranks_connected": s.get("peer_ranks_connected"),
                  "process_group": s.get("process_group"),
                  "rollout_us_max_over_ranks": s["tim"].get("rollout_in_step_us_max_over_ranks")})
    if s.get("exchange") == "vehicles":   # the fleet split over the ranks: no exchange at all
        e.update({"exchange": "none", "split": "vehicles", "vehicles_total": s["world"] * s["V"], "samples_total": s["K"],
                  "vehicles_per_gpu": s["V"], "allreduce_us": None})
    return e


def guarded(what: str, fn):
    """One rank-local part of the line (N = 1 only: the drop-in latency, the CPU baseline, the
    HBM fill): its failure becomes {"error": ...} in the line instead of costing the whole line."""
    try:
        return fn()
    except Exception as ex:   # noqa: BLE001 -- reported in the line, never swallowed silently
        log(f"{what} failed: {type(ex).__name__}: {ex}")
        return {"error": f"{type(ex).__name__}: {ex}"}


def run_secondaries(names, steps, world, dist, ranks_per_gpu, run=None):
    """The secondary workloads, every rank in lockstep.  A failed secondary is reported in the line
    as {"error": ...} and the next one runs: at N = 1 any exception (no collective to desynchronise);
    at N > 1 only StepsGivenUp, which every rank raises at the same point (any other exception
    ends the run, as a one-rank failure leaves the ranks' collectives unpaired)."""
    run = run or run_workload
    out = {}
    for wname in names:
        ns = max(50, steps // 5)
        try:
            s = run(wname, ns, 20, world, dist, 50, batches=3)
        except Exception as ex:   # noqa: BLE001
            if world > 1 and not isinstance(ex, StepsGivenUp):
                raise
            out[wname] = {"error": f"{type(ex).__name__}: {ex}"}
            log(f"secondary {wname} failed: {out[wname]['error']}")
            continue
        s["ranks_per_gpu"] = ranks_per_gpu
        out[wname] = secondary_entry(s, ns)
        log(f"secondary {wname}: {out[wname]}")
    return out


def dropin_latency(n_calls):
    """The reference's own control call through the drop-in class (mppi_solver/mppi.py MPPI,
    the kinova node's tick: update_joint from the joint-state callback, then
    compute_control_input -> (qdes, vdes) numpy), arm C3 shape with an fp64 state, device
    noise: host-inclusive wall time per call, p50/p99 over n_calls after 20 untimed."""
    import torch
    from quadrotor_manipulator_mppi_amd.mppi_solver.mppi import MPPI
    m = MPPI(n_samples=4096, n_horizon=32, verbose=False)
    q = torch.tensor([0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0], dtype=torch.float64)
    v = torch.zeros(13, dtype=torch.float64)
    lat = []
    for i in range(n_calls + 20):
        t0 = time.perf_counter()
        m.update_joint(q, v)
        qdes, vdes = m.compute_control_input()
        if i >= 20:
            lat.append(time.perf_counter() - t0)
    assert np.isfinite(qdes).all() and np.isfinite(vdes).all()
    m._engine.close()
    lat = np.array(lat) * 1e3
    return {"p50_ms": float(np.median(lat)), "p99_ms": float(np.percentile(lat, 99)), "calls": int(lat.size),
            "what": "drop-in MPPI.update_joint + compute_control_input (mppi.py:196-200, :122-169), K=4096 H=32, "
                    "fp64 state, device noise, host-inclusive"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--batches", type=int, default=0, help="timed batches of --steps steps (0: auto)")
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help="default: arm_c3 for a plain run, c4 (north star, strong scaling) under torchrun")
    ap.add_argument("--samples", type=int, default=0,
                    help="override the workload's samples per GPU (profiling one launch shape, e.g. the c4 "
                         "rank shape 65536/N on one GPU)")
    ap.add_argument("--latency-steps", type=int, default=200)
    ap.add_argument("--cpu-budget", type=float, default=2.5, help="seconds of CPU sampling per baseline cell")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="skip the event-timed kernel loops (profiler runs: the trace then holds only the "
                         "control steps); no roofline in the line")
    ap.add_argument("--no-numa-bind", action="store_true",
                    help="leave the process's CPU affinity alone (default: bind to the GPU's local CPUs)")
    ap.add_argument("--secondary", default="drone_c2,wholebody_c4,c4_shard_native1,c4_shard_peer1,c4,fleet_c5,"
                                           "fleet_c5_share,quadrotor_c2",
                    help="extra workloads reported at N=1, comma separated; '' for none")
    ap.add_argument("--secondary-multi", default="c4,c4_rccl,fleet_c5",
                    help="extra workloads reported at N>1 (every rank runs them), comma separated; '' for none")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # N ranks from one command: the ranks run as a child (torch.distributed.run), this process
        # relays rank 0's line and exits with the child's code (nothing here has touched the GPU)
        if os.environ.get("MPPI_BENCH_SPAWNED"):
            raise SystemExit("bench.py: started by its own launcher without WORLD_SIZE")
        sys.exit(spawn_ranks(launcher_cmd(args.gpus, sys.argv[1:])))
    # the JSON line is the only thing on stdout: keep the real stdout for it and send fd 1 to
    # stderr, so native libraries that print there (RCCL's version banner at communicator
    # init) cannot add lines to it
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import torch
    launched = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one primary workload at every N (arm_c3: the metric's configuration; weak-scaled under
    # torchrun), so the N=1 point of a scaling curve measures what the N>1 points do
    workload = args.workload or "arm_c3"
    # ranks beyond the visible devices wrap (rehearsing N ranks on fewer GPUs)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    # the launching thread on the GPU's own socket (quadrotor_manipulator_mppi_amd.affinity);
    # threads created later (the CPU baseline's pool) inherit it
    binding = None
    if not args.no_numa_bind:
        from quadrotor_manipulator_mppi_amd.affinity import bind_to_gpu_numa
        binding = bind_to_gpu_numa(local)
        log(f"cpu binding: {binding}")
    dist = None
    ndev = torch.cuda.device_count()   # (no GPU initialisation on this image)
    ranks_per_gpu = -(-world // max(1, ndev))
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        # nccl = RCCL; with more ranks than GPUs (a rehearsal of N ranks on fewer GPUs, which RCCL
        # cannot pair) the process group is gloo
        backend = os.environ.get("MPPI_DIST_BACKEND", "nccl" if world <= ndev else "gloo")
        if world > ndev:
            log(f"note: {world} ranks on {ndev} GPU(s): a rehearsal, process group {backend}")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    if args.gpus != world:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    from quadrotor_manipulator_mppi_amd import _capi
    _capi.lib()

    if args.samples:
        WORKLOADS[workload] = dict(WORKLOADS[workload], n_samples=args.samples, strong=False)
    batches = args.batches or auto_batches(args.steps)
    r = run_workload(workload, args.steps, args.warmup, world, dist, args.latency_steps,
                     timing=not args.no_kernel_timing, batches=batches, lat_rate_calls=args.latency_steps)
    r["ranks_per_gpu"] = ranks_per_gpu
    extra = args.secondary if world == 1 else args.secondary_multi
    secondary = {}
    if extra and r["tim"] is not None:
        secondary = run_secondaries([s for s in extra.split(",") if s and s != workload], args.steps, world, dist,
                                    ranks_per_gpu)
    dropin = None
    if world == 1 and workload == "arm_c3" and args.latency_steps:
        dropin = guarded("drop-in latency", lambda: dropin_latency(args.latency_steps))
        log(f"drop-in latency: {dropin}")
    cpu, cpu_all = None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = guarded("cpu baseline", lambda: cpu_baseline(workload, args.cpu_budget))
        cpu, cpu_all = (cb, None) if isinstance(cb, dict) else cb   # (a dict: its error)
        log(f"cpu baseline: {cpu}")
    if rank == 0:
        measured = None
        if world == 1 and r["tim"] is not None:
            measured = guarded("measured HBM", lambda: measured_hbm(local))
            if "error" in measured:
                measured = None
            log(f"measured HBM: {measured}")
        line = make_line(workload, r, args, secondary, cpu, cpu_all, measured)
        line["host_binding"] = binding
        if dropin is not None:
            line["dropin_latency"] = dropin
        print(json.dumps(line), file=json_out, flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
