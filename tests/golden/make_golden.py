"""Generate the golden parity fixtures by running the REFERENCE itself.

Runs only in the build container (``/root/reference`` is read-only and does not
exist on the GPU box).  It imports the reference hot path
(``src/mav_mppi/scripts/{mppi_solver,sampling,robot,cost,filter,utils}``) with
two test-only import stand-ins (``tests/golden/shims``: a ``rospkg`` path map
and an xml.etree ``urdf_parser_py``), drives the reference's own classes at
small sizes with seeded ``torch.randn`` noise, and records every intermediate of
the MPPI control step into small ``.npz`` fixtures under ``tests/golden/``.
The fixtures are DATA (inputs + expected outputs); no reference source is
copied.  Regenerate with::

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Fixture map:
  drone_k128_h20.npz      F1  drone MPPI, 3 closed-loop steps (drone_mppi.py:140-176)
  drone_k256_h32.npz      F1b drone MPPI at H=32, 2 steps
  arm_k32_h32_f32.npz     F2  arm MPPI, fp32 state (mppi.py:122-169), 2 steps
  arm_k32_h32_f64.npz     F2  arm MPPI, fp64 state (the ROS node's dtype), 2 steps
  arm_k100_h32_f64.npz    F2b arm MPPI at the reference default K=100, 1 step
  fk_known_answer.npz     F3  URDFFK.compute_fk_gpu / compute_fk_cpu
  rotations.npz           F4  quaternion_to_matrix (xyzw) / matrix_to_euler_angles(ZYX)
  savgol.npz              F5  SavGol coefficients and filter I/O
  wholebody_k32_h64.npz   F6  whole-body composition, 2 steps
  arm_k64_h32_allcosts.npz F7 arm MPPI with every CostManager term the reference
                              ships disabled (cost_manager.py:83-87) switched on,
                              fp64 state near a joint limit, 2 steps
  arm_k32_h32_gap.npz     F2c arm MPPI with the sampler's Sigma at 1.0 I (10x the
                              default 0.1 I of standard_normal_noise.py:17), so the
                              top-2 cost gap is >= 20 lambda in both steps: the arm
                              path end to end at the plain 1e-4 rel bar, 2 steps

Regenerate one fixture only:  python tests/golden/make_golden.py --only arm_k32_h32_gap
Write into another directory: python tests/golden/make_golden.py --out DIR
(tests/test_golden_regen.py does that and compares every array with the committed ones.)
"""
import contextlib
import io
import math
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("MPPI_REFERENCE_ROOT", "/root/reference")
sys.path[:0] = [os.path.join(HERE, "shims"),
                os.path.join(REF, "src/mav_mppi/scripts"),
                os.path.join(REF, "src")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mppi_solver.mppi import MPPI as ArmMPPI  # noqa: E402
from mppi_solver.drone_mppi import MPPI as DroneMPPI  # noqa: E402
from mav_mppi.scripts.sampling.standard_normal_noise import StandardSamplling  # noqa: E402
from cost.cost_manager import CostManager  # noqa: E402
from filter.svg_filter import SavGolFilter  # noqa: E402
from utils.rotation_conversions import quaternion_to_matrix, matrix_to_euler_angles  # noqa: E402
from robot.transformation_matrix import make_transform_matrix  # noqa: E402

HOME_Q = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]          # kinova.py:135
ARM_TARGET_POS = [0.1029, 0.4055, 1.6498]                 # mppi.py:71
ARM_TARGET_QUAT = [-0.5, -0.5, 0.5, -0.5]                 # mppi.py:72 (xyzw)
DRONE_TARGET = [1.0, 2.0, 3.4]                            # drone_mppi.py:141


def _np(t):
    return t.detach().cpu().numpy().copy()


def _gap(S):
    s = np.sort(S.astype(np.float64))
    return float(s[1] - s[0]) if s.size > 1 else float("inf")


def _quiet():
    return contextlib.redirect_stdout(io.StringIO())


# --------------------------------------------------------------------------- arm
def _resize_arm(m, K, H):
    """Re-size the reference arm solver (mppi.py:37-41 hard-codes K=100, H=32)."""
    m.n_samples, m.n_horizon = K, H
    m.u_prev = torch.zeros((H, m.n_action))
    m.sample_gen = StandardSamplling(K, H, m.n_action, device=m.device)
    m.cost_manager = CostManager(K, H, m.n_action, m._lambda, m.device)


def _record_arm_step(m, seed):
    rec = {}
    orig_sampling = m.sample_gen.sampling
    orig_joint = m.sample_gen.get_sample_joint
    orig_fk = m.fk_urdf.compute_fk_gpu
    orig_cost = m.cost_manager.compute_all_cost
    orig_w = m.compute_weights
    orig_sg = m.svg_filter.savgol_filter_torch
    orig_reach = m.check_reach

    def sampling():
        n = orig_sampling(); rec["noise"] = _np(n); return n

    def get_sample_joint(v, q, qd, dt):
        rec["v"] = _np(v)
        out = orig_joint(v, q, qd, dt); rec["q_samples"] = _np(out); return out

    def compute_fk_gpu(q, base, base_movement=False):
        out = orig_fk(q, base, base_movement); rec["ee"] = _np(out); return out

    def compute_all_cost():
        S = orig_cost(); rec["S"] = _np(S); return S

    def compute_weights(S, lam):
        w = orig_w(S, lam); rec["w"] = _np(w); return w

    def savgol(seq, window_size, polyorder):
        rec["w_eps_raw"] = _np(seq)
        out = orig_sg(seq, window_size=window_size, polyorder=polyorder)
        rec["w_eps"] = _np(out); return out

    def check_reach(x):
        r = orig_reach(x); rec["reach"] = np.array(bool(r)); return r

    m.sample_gen.sampling = sampling
    m.sample_gen.get_sample_joint = get_sample_joint
    m.fk_urdf.compute_fk_gpu = compute_fk_gpu
    m.cost_manager.compute_all_cost = compute_all_cost
    m.compute_weights = compute_weights
    m.svg_filter.savgol_filter_torch = savgol
    m.check_reach = check_reach
    rec["u_prev_in"] = _np(m.u_prev)
    torch.manual_seed(seed)
    with _quiet():
        qdes, vdes = m.compute_control_input()
    rec["qdes"] = np.asarray(qdes).copy()
    rec["vdes"] = np.asarray(vdes).copy()
    rec["u_prev_out"] = _np(m.u_prev)
    for name, fn in (("sampling", orig_sampling), ("get_sample_joint", orig_joint)):
        setattr(m.sample_gen, name, fn)
    m.fk_urdf.compute_fk_gpu = orig_fk
    m.cost_manager.compute_all_cost = orig_cost
    m.compute_weights = orig_w
    m.svg_filter.savgol_filter_torch = orig_sg
    m.check_reach = orig_reach
    return rec


def _enable_all_costs(cm, rec_terms):
    """Switch on the terms compute_all_cost leaves commented out
    (cost_manager.py:83-87), in that order, calling the reference's own term
    implementations; each term's (K,) vector is recorded."""
    def compute_all_cost():
        S = torch.zeros((cm.n_sample), device=cm.device)
        terms = [("stage", lambda: cm.pose_cost.compute_stage_cost(cm.eef_trajectories, cm.target)),
                 ("terminal", lambda: cm.pose_cost.compute_terminal_cost(cm.eef_trajectories, cm.target)),
                 ("covar", lambda: cm.covar_cost.compute_covar_cost(cm.sigma_matrix, cm.u, cm.v)),
                 ("center", lambda: cm.joint_cost.compute_centering_cost(cm.qSamples)),
                 ("jtraj", lambda: cm.joint_cost.compute_jointTraj_cost(cm.qSamples, cm.joint_trajectories)),
                 ("action", lambda: cm.action_cost.compute_action_cost(cm.uSamples)),
                 ("limit", lambda: cm.joint_cost.compute_joint_limit_cost(cm.qSamples))]
        for name, fn in terms:
            t = fn()
            rec_terms[name] = _np(t)
            S += t
        return S
    cm.compute_all_cost = compute_all_cost


def make_arm(path, K, H, steps, f64, seed0, state, all_costs=False, sigma_scale=None):
    with _quiet():
        m = ArmMPPI()
    _resize_arm(m, K, H)
    if sigma_scale is not None:   # the sampler's own Sigma attribute (standard_normal_noise.py:17)
        m.sample_gen.sigma = torch.eye(m.n_action) * sigma_scale
    terms = {}
    if all_costs:
        _enable_all_costs(m.cost_manager, terms)
    base, q, v_base, qd = state
    q_full = list(base) + list(q)
    v_full = list(v_base) + list(qd)
    if f64:
        q_full, v_full = np.array(q_full, np.float64), np.array(v_full, np.float64)
    out = {"K": K, "H": H, "A": 7, "dt": m.dt, "lam": m._lambda, "state_f64": int(f64),
           "q_full": np.array(q_full, np.float64), "v_full": np.array(v_full, np.float64),
           "target_pos": np.array(ARM_TARGET_POS, np.float32),
           "target_quat": np.array(ARM_TARGET_QUAT, np.float32), "steps": steps,
           "sigma": _np(m.sample_gen.sigma)}
    gaps = []
    for s in range(steps):
        m.update_joint(q_full, v_full)
        rec = _record_arm_step(m, seed0 + s)
        for k, val in terms.items():
            rec[f"term_{k}"] = val
        gaps.append(_gap(rec["S"]))
        for k, val in rec.items():
            out[f"s{s}_{k}"] = val
    out["top2_gap"] = np.array(gaps)
    np.savez_compressed(path, **out)
    print(f"{os.path.basename(path)}: gaps={gaps}")


# ------------------------------------------------------------------------- drone
def make_drone(path, K, H, steps, seed0, x0, v0):
    m = DroneMPPI()
    m.n_samples, m.n_timestep = K, H
    m.u_prev = torch.zeros((H, 3))
    out = {"K": K, "H": H, "A": 3, "dt": m.dt, "lam": m.param_lambda, "steps": steps,
           "target": np.array(DRONE_TARGET, np.float32), "sigma": _np(m.sigma)}
    x, v = list(x0), list(v0)
    gaps = []
    for s in range(steps):
        rec = {}
        og, op, ow, of = (m.generateNoiseAndSampling, m.predict_trajectory,
                          m.compute_weights, m.filter.savgol_filter_torch)

        def gen():
            n = og(); rec["noise"] = _np(n); return n

        def pred(samples, q, qd, dt):
            t = op(samples, q, qd, dt); rec["traj"] = _np(t); return t

        def cw(S):
            rec["S"] = _np(S); w = ow(S); rec["w"] = _np(w); return w

        def sg(seq, window_size, polyorder):
            rec["w_eps_raw"] = _np(seq)
            o = of(seq, window_size=window_size, polyorder=polyorder)
            rec["w_eps"] = _np(o); return o

        m.generateNoiseAndSampling, m.predict_trajectory = gen, pred
        m.compute_weights, m.filter.savgol_filter_torch = cw, sg
        m.set_state(x, v)
        rec["x_in"] = np.array(x, np.float32); rec["v_in"] = np.array(v, np.float32)
        rec["u_prev_in"] = _np(m.u_prev)
        torch.manual_seed(seed0 + s)
        with _quiet():
            xo, vo = m.compute_control_input()
        rec["x_out"], rec["v_out"] = _np(xo), _np(vo)
        rec["u_prev_out"] = _np(m.u_prev)
        m.generateNoiseAndSampling, m.predict_trajectory = og, op
        m.compute_weights, m.filter.savgol_filter_torch = ow, of
        gaps.append(_gap(rec["S"]))
        for k, val in rec.items():
            out[f"s{s}_{k}"] = val
        x, v = xo.tolist(), vo.tolist()
    out["top2_gap"] = np.array(gaps)
    np.savez_compressed(path, **out)
    print(f"{os.path.basename(path)}: gaps={gaps}")


# ----------------------------------------------------------------- FK / rotations
def make_fk(path):
    with _quiet():
        m = ArmMPPI()
    g = torch.Generator().manual_seed(3)
    q32 = (torch.rand((16, 16, 7), generator=g) * 12.0 - 6.0)
    q32[0, 0] = torch.tensor(HOME_Q)
    bases = torch.tensor([[0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0],
                          [0.3, -0.2, 1.4, 0.0, 0.0, 0.3826834, 0.9238795],
                          [-1.0, 2.0, 0.5, 0.1, -0.2, 0.3, 0.9273618],
                          [0.0, 0.0, 0.0, 0.7071068, 0.0, 0.0, 0.7071068]])
    out = {"q32": _np(q32), "bases": _np(bases)}
    with _quiet():
        for b in range(bases.shape[0]):
            out[f"ee32_b{b}"] = _np(m.fk_urdf.compute_fk_gpu(q32, bases[b]))
            q64 = q32.double()
            out[f"ee64_b{b}"] = _np(m.fk_urdf.compute_fk_gpu(q64, bases[b].double()))
            out[f"eecpu_b{b}"] = np.stack([m.fk_urdf.compute_fk_cpu(bases[b], q32[0, j])
                                           for j in range(4)])
    # per-joint constant origin transforms (transformation_matrix.py:28-35)
    chain = m.fk_urdf.robot._joint_chain_list
    out["origins"] = np.stack([_np(make_transform_matrix(torch.tensor(j.origin.xyz),
                                                         torch.tensor(j.origin.rpy)))
                               for j in chain])
    np.savez_compressed(path, **out)
    print(os.path.basename(path))


def make_rotations(path):
    g = torch.Generator().manual_seed(4)
    quat = torch.randn((1024, 4), generator=g)
    quat = quat / quat.norm(dim=-1, keepdim=True)
    R = quaternion_to_matrix(quat)
    # near-gimbal (|m20| -> 1) and yaw ~ +-pi rotations, built from ZYX angles
    n = 256
    yaw = torch.rand(n, generator=g) * 2 * math.pi - math.pi
    yaw[:32] = math.pi - torch.rand(32, generator=g) * 1e-3
    yaw[32:64] = -math.pi + torch.rand(32, generator=g) * 1e-3
    pitch = torch.rand(n, generator=g) * math.pi - math.pi / 2
    pitch[64:128] = math.pi / 2 - torch.rand(64, generator=g) * 1e-3
    pitch[128:160] = -math.pi / 2 + torch.rand(32, generator=g) * 1e-3
    roll = torch.rand(n, generator=g) * 2 * math.pi - math.pi
    cy, sy, cp, sp, cr, sr = yaw.cos(), yaw.sin(), pitch.cos(), pitch.sin(), roll.cos(), roll.sin()
    R2 = torch.stack([torch.stack([cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr], -1),
                      torch.stack([sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr], -1),
                      torch.stack([-sp, cp * sr, cp * cr], -1)], -2)
    mats = torch.cat([R, R2], 0)
    np.savez_compressed(path, quat=_np(quat), quat_R=_np(R), mats=_np(mats),
                        euler=_np(matrix_to_euler_angles(mats, "ZYX")),
                        target_R=_np(quaternion_to_matrix(torch.tensor(ARM_TARGET_QUAT))))
    print(os.path.basename(path))


def make_savgol(path):
    g = torch.Generator().manual_seed(5)
    out = {}
    for (H, A, W, P) in ((20, 3, 5, 2), (32, 3, 5, 2), (32, 7, 9, 2), (64, 10, 9, 2),
                         (32, 7, 7, 3), (16, 4, 11, 2)):
        x = torch.randn((H, A), generator=g)
        f = SavGolFilter(A)
        out[f"x_{H}_{A}_{W}_{P}"] = _np(x)
        out[f"y_{H}_{A}_{W}_{P}"] = _np(f.savgol_filter_torch(x, window_size=W, polyorder=P))
        # impulse response on a long sequence -> the coefficients (svg_filter.py:52-55)
        imp = torch.zeros((4 * W, 1)); imp[2 * W, 0] = 1.0
        out[f"coef_{W}_{P}"] = _np(SavGolFilter(1).savgol_filter_torch(imp, window_size=W,
                                                                       polyorder=P))[2 * W - W // 2:2 * W + W // 2 + 1, 0]
    np.savez_compressed(path, **out)
    print(os.path.basename(path))


# ---------------------------------------------------------------- whole body (A16)
def make_wholebody(path, K, H, steps, seed0):
    """Whole-body MPPI composed from reference primitives.

    noise: StandardSamplling with Sigma = diag(30,30,30, 0.1 x7)
    rollout: get_sample_joint on all 10 dims (drone xyz acc + 7 joint acc)
    EE: URDFparser.forward_kinematics(base_movement=True, _n_mobile_dof=6) with
        q_mobile = (x, y, z, roll, pitch, yaw_meas) -- rotation held fixed as in
        drone_mppi.py:21-22
    cost: CostManager pose stage+terminal (cost_manager.py:78-89)
    weights: MPPI.compute_weights; SavGol window 9; u += w_eps
    outputs: drone (x, v) as drone_mppi.py:168-169 and arm (qdes, vdes) as mppi.py:157-158
    """
    with _quiet():
        m = ArmMPPI()
    A = 10
    lam, dt = m._lambda, m.dt
    sg = StandardSamplling(K, H, A, device="cpu")
    sg.sigma = torch.diag(torch.tensor([30.0] * 3 + [0.1] * 7))
    cm = CostManager(K, H, A, lam, "cpu")
    filt = SavGolFilter(A)
    robot = m.fk_urdf.robot
    base_quat = [0.0, 0.0, 0.1305262, 0.9914449]
    x = [0.1, -0.2, 1.0]; vx = [0.0, 0.05, 0.0]
    q = list(HOME_Q); qd = [0.0] * 7
    u_prev = torch.zeros((H, A))
    out = {"K": K, "H": H, "A": A, "dt": dt, "lam": lam, "steps": steps,
           "sigma": _np(sg.sigma), "base_quat": np.array(base_quat, np.float32),
           "target_pos": np.array(ARM_TARGET_POS, np.float32),
           "target_quat": np.array(ARM_TARGET_QUAT, np.float32)}
    ypr = matrix_to_euler_angles(quaternion_to_matrix(torch.tensor(base_quat)), "ZYX")
    rpy = torch.stack([ypr[2], ypr[1], ypr[0]])
    out["base_rpy"] = _np(rpy)
    gaps = []
    for s in range(steps):
        rec = {"x_in": np.array(x, np.float32), "vx_in": np.array(vx, np.float32),
               "q_in": np.array(q, np.float32), "qd_in": np.array(qd, np.float32),
               "u_prev_in": _np(u_prev)}
        u = u_prev.clone()
        u0_old = u[0].clone()
        torch.manual_seed(seed0 + s)
        noise = sg.sampling()
        v = u.unsqueeze(0) + noise
        state0 = torch.tensor(x + q); vel0 = torch.tensor(vx + qd)
        qs = sg.get_sample_joint(v, state0, vel0, dt)          # (K,H,10)
        qfull = torch.cat([qs[..., :3], rpy.expand(K, H, 3), qs[..., 3:]], -1)
        robot._n_mobile_dof = 6
        robot._n_samples, robot._n_timestep = 1, 1
        ee = robot.forward_kinematics(qfull, base_movement=True)
        tp = type(m.target_pose)()
        tp.pose = torch.tensor(ARM_TARGET_POS); tp.orientation = torch.tensor(ARM_TARGET_QUAT)
        cm.update_pose_cost(qs, v, ee, torch.zeros((K, H, A)), tp)
        S = cm.compute_all_cost()
        w = m.compute_weights(S, lam)
        w_eps_raw = torch.sum(w.view(-1, 1, 1) * noise, dim=0)
        w_eps = filt.savgol_filter_torch(w_eps_raw, window_size=9, polyorder=2)
        u += w_eps
        u_prev = u.clone()
        u0 = u[0].clone()
        xt, vt = torch.tensor(x), torch.tensor(vx)
        x_out = xt + vt * dt + 0.5 * u0[:3] * dt ** 2
        v_out = vt + dt * u0[:3]
        qt, qdt = torch.tensor(q), torch.tensor(qd)
        vdes = qdt + u0[3:] * dt
        qdes = qt + u0_old[3:] * dt + 0.5 * u0[3:] * dt * dt
        rec.update(noise=_np(noise), q_samples=_np(qs), ee=_np(ee), S=_np(S), w=_np(w),
                   w_eps_raw=_np(w_eps_raw), w_eps=_np(w_eps), u_prev_out=_np(u_prev),
                   x_out=_np(x_out), v_out=_np(v_out), qdes=_np(qdes), vdes=_np(vdes))
        gaps.append(_gap(rec["S"]))
        for k, val in rec.items():
            out[f"s{s}_{k}"] = val
        x, vx = x_out.tolist(), v_out.tolist()
        q, qd = qdes.tolist(), vdes.tolist()
    out["top2_gap"] = np.array(gaps)
    np.savez_compressed(path, **out)
    print(f"{os.path.basename(path)}: gaps={gaps}")


def main():
    torch.set_num_threads(1)
    d = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else HERE
    os.makedirs(d, exist_ok=True)
    if "--only" in sys.argv:
        only = sys.argv[sys.argv.index("--only") + 1]
        FIXTURES[only](d)
        return
    make_drone(os.path.join(d, "drone_k128_h20.npz"), 128, 20, 3, 100, [0.0, 0.0, 1.0], [0.0, 0.0, 0.0])
    make_drone(os.path.join(d, "drone_k256_h32.npz"), 256, 32, 2, 200, [0.2, -0.1, 1.5], [0.1, 0.0, -0.2])
    c3 = ([0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0], HOME_Q, [0.0] * 6, [0.0] * 7)
    pert = ([0.3, -0.2, 1.2, 0.0, 0.0, 0.3826834, 0.9238795],
            [1.4, 1.9, 0.2, 4.2, -0.1, 4.5, 0.3],
            [0.0] * 6, [0.05, -0.1, 0.02, 0.0, 0.1, -0.05, 0.2])
    make_arm(os.path.join(d, "arm_k32_h32_f32.npz"), 32, 32, 2, False, 300, c3)
    make_arm(os.path.join(d, "arm_k32_h32_f64.npz"), 32, 32, 2, True, 400, pert)
    make_arm(os.path.join(d, "arm_k100_h32_f64.npz"), 100, 32, 1, True, 500, c3)
    make_fk(os.path.join(d, "fk_known_answer.npz"))
    make_rotations(os.path.join(d, "rotations.npz"))
    make_savgol(os.path.join(d, "savgol.npz"))
    make_wholebody(os.path.join(d, "wholebody_k32_h64.npz"), 32, 64, 2, 600)
    near_limit = ([0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0],
                  [1.57, 1.7, 0.0, 4.4, 0.0, 5.1485, 0.0],         # joint 6 2e-4 under its 5.1487 limit
                  [0.0] * 6, [0.0, 0.3, 0.0, -0.2, 0.0, 0.0, 0.0])
    make_arm(os.path.join(d, "arm_k64_h32_allcosts.npz"), 64, 32, 2, True, 700, near_limit, all_costs=True)
    FIXTURES["arm_k32_h32_gap"](d)


FIXTURES = {
    "arm_k32_h32_gap": lambda d: make_arm(
        os.path.join(d, "arm_k32_h32_gap.npz"), 32, 32, 2, True, 800,
        ([0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0], HOME_Q, [0.0] * 6, [0.0] * 7), sigma_scale=1.0),
}


if __name__ == "__main__":
    main()
