"""Timing validation of bench.py's CPU baseline against the reference itself (BASELINE.md §3,
SURVEY.md §8d: "the restatement must be validated in this container against the reference ...
timing within +-15%").

    PYTHONDONTWRITEBYTECODE=1 python tools/validate_cpu_baseline.py [--threads 1,8] [--rounds 15]
        [--out profiles/r06/cpu_baseline_validation.json]

Build container only: it imports the reference hot path READ-ONLY from /root/reference (with the
test-only import stand-ins of tests/golden/shims, as tests/golden/make_golden.py does); the GPU box
has no reference.  For every cell -- C1 drone K=128 H=20, C2 drone K=4096 H=32, C3 arm K=4096 H=32
(fp64 state, as the kinova node feeds it) and the whole-body K=4096 H=64 (composed from reference
primitives as make_golden.make_wholebody does: the reference has no whole-body controller) -- at each
thread count, it times ONE control step of

* the reference: drone ``MPPI.set_state`` + ``compute_control_input`` (drone_mppi.py:140-183), arm
  ``MPPI.update_joint`` + ``compute_control_input`` (mppi.py:122-200, check_reach included);
* the oracle step bench.py times (``bench._cpu_step_fn``: oracle/mppi_oracle.py, randn included);

interleaved round by round (the order alternating) so the shared host's slow phases hit both, and
reports the medians and the median of the per-round ratios oracle / reference.  The reference's stdout (the drone's per-step "Rho" print) goes
to /dev/null.
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import sys
import time

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("MPPI_REFERENCE_ROOT", "/root/reference")
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden", "shims"), os.path.join(ROOT, "tests", "golden"),
                os.path.join(REF, "src/mav_mppi/scripts"), os.path.join(REF, "src")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

CELLS = [("c1_drone_k128_h20", "drone", 128, 20), ("c2_drone_k4096_h32", "drone", 4096, 32),
         ("c3_arm_k4096_h32", "arm", 4096, 32), ("c4r_wholebody_k4096_h64", "wholebody", 4096, 64)]


def _devnull():
    return contextlib.redirect_stdout(open(os.devnull, "w"))


def reference_step_fn(model: str, K: int, H: int):
    """One reference control step at (K, H) with bench.py's C1-C4 inputs."""
    import make_golden as G
    if model == "drone":
        from mppi_solver.drone_mppi import MPPI as DroneMPPI
        m = DroneMPPI()
        m.n_samples, m.n_timestep = K, H
        m.u_prev = torch.zeros((H, 3))

        def step():
            m.set_state([0.0, 0.0, 1.0], [0.0, 0.0, 0.0])
            m.u_prev = torch.zeros((H, 3))   # (the oracle step starts from u_prev = 0 each time, too)
            with _devnull():
                return m.compute_control_input()
        return step
    if model == "arm":
        from mppi_solver.mppi import MPPI as ArmMPPI
        with _devnull():
            m = ArmMPPI()
        G._resize_arm(m, K, H)
        q_full = np.array([0, 0, 1.0, 0, 0, 0, 1] + bench.HOME_Q, np.float64)
        v_full = np.zeros(13)

        def step():
            m.update_joint(q_full, v_full)
            m.u_prev = torch.zeros((H, 7))
            with _devnull():
                return m.compute_control_input()
        return step
    # whole-body: the composition of reference primitives (make_golden.make_wholebody), one step
    from mppi_solver.mppi import MPPI as ArmMPPI
    from mav_mppi.scripts.sampling.standard_normal_noise import StandardSamplling
    from cost.cost_manager import CostManager
    from filter.svg_filter import SavGolFilter
    from utils.rotation_conversions import quaternion_to_matrix, matrix_to_euler_angles
    with _devnull():
        m = ArmMPPI()
    A = 10
    sg = StandardSamplling(K, H, A, device="cpu")
    sg.sigma = torch.diag(torch.tensor([30.0] * 3 + [0.1] * 7))
    cm = CostManager(K, H, A, m._lambda, "cpu")
    filt = SavGolFilter(A)
    robot = m.fk_urdf.robot
    ypr = matrix_to_euler_angles(quaternion_to_matrix(torch.tensor([0.0, 0.0, 0.0, 1.0])), "ZYX")
    rpy = torch.stack([ypr[2], ypr[1], ypr[0]])

    def step():
        u = torch.zeros((H, A))
        noise = sg.sampling()
        v = u.unsqueeze(0) + noise
        qs = sg.get_sample_joint(v, torch.tensor([0.0, 0.0, 1.0] + bench.HOME_Q), torch.zeros(A), m.dt)
        qfull = torch.cat([qs[..., :3], rpy.expand(K, H, 3), qs[..., 3:]], -1)
        robot._n_mobile_dof = 6
        robot._n_samples, robot._n_timestep = 1, 1
        ee = robot.forward_kinematics(qfull, base_movement=True)
        tp = type(m.target_pose)()
        tp.pose = torch.tensor(bench.ARM_TARGET[0])
        tp.orientation = torch.tensor(bench.ARM_TARGET[1])
        cm.update_pose_cost(qs, v, ee, torch.zeros((K, H, A)), tp)
        S = cm.compute_all_cost()
        w = m.compute_weights(S, m._lambda)
        w_eps = filt.savgol_filter_torch(torch.sum(w.view(-1, 1, 1) * noise, dim=0), window_size=9, polyorder=2)
        return u + w_eps
    return step


def time_pair(ref_fn, orc_fn, rounds: int, warmup: int = 2):
    """Per round one reference step and one oracle step back to back, the order alternating from
    round to round; returns both time arrays (the per-round ratio o_i / r_i pairs steps run within
    the same fraction of a second, so a slow phase of the shared host hits both)."""
    for _ in range(warmup):
        ref_fn()
        orc_fn()
    tr, to = [], []
    for i in range(rounds):
        first, second = (ref_fn, orc_fn) if i % 2 == 0 else (orc_fn, ref_fn)
        t0 = time.perf_counter()
        first()
        t1 = time.perf_counter()
        second()
        t2 = time.perf_counter()
        a, b = t1 - t0, t2 - t1
        tr.append(a if i % 2 == 0 else b)
        to.append(b if i % 2 == 0 else a)
    return np.array(tr), np.array(to)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default=f"1,{os.cpu_count()}")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--cells", default=",".join(c[0] for c in CELLS))
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    threads = [int(x) for x in a.threads.split(",") if x]
    res = {"cpu_model": bench.cpu_model(), "os_cpu_count": os.cpu_count(), "torch": torch.__version__,
           "rounds": a.rounds, "method": "one control step per round, reference and oracle interleaved; medians",
           "cells": {}}
    for name, model, K, H in CELLS:
        if name not in a.cells.split(","):
            continue
        ref_fn = reference_step_fn(model, K, H)
        orc_fn = bench._cpu_step_fn(model, K, H)
        res["cells"][name] = {}
        for nt in threads:
            torch.set_num_threads(nt)
            tr, to = time_pair(ref_fn, orc_fn, a.rounds)
            r, o = float(np.median(tr)), float(np.median(to))
            pr = float(np.median(to / tr))   # the median of the per-round ratios: the reported ratio
            res["cells"][name][f"threads_{nt}"] = {"reference_ms": r * 1e3, "oracle_ms": o * 1e3, "ratio": pr,
                                                   "ratio_of_medians": o / r,
                                                   "ratio_p25_p75": [float(np.percentile(to / tr, q)) for q in (25, 75)],
                                                   "reference_p10_p90_ms": [float(np.percentile(tr, q)) * 1e3
                                                                            for q in (10, 90)],
                                                   "oracle_p10_p90_ms": [float(np.percentile(to, q)) * 1e3
                                                                         for q in (10, 90)]}
            print(f"{name} threads={nt}: reference {r * 1e3:.2f} ms, oracle {o * 1e3:.2f} ms, "
                  f"oracle/reference {pr:.3f} (per-round median; ratio of medians {o / r:.3f})", flush=True)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return res


if __name__ == "__main__":
    with contextlib.redirect_stderr(io.StringIO()) if os.environ.get("QUIET") else contextlib.nullcontext():
        main()
