"""CPU checks of the 6-DoF quadrotor model (parity unpinned:
the reference ships it only as commented code, drone_mppi.py:57-83).  The torch
restatement in the oracle is checked against closed-form motions, and the C-ABI
reports the model's layout.  No GPU calls."""
import ctypes as C
import math

import numpy as np
import torch

from oracle import mppi_oracle as O
from quadrotor_manipulator_mppi_amd import _capi as capi

M, G, DT = 14.7, 9.81, 0.01


def test_hover_thrust_holds_position():
    K, H = 4, 32
    u = torch.zeros(K, H, 4)
    u[..., 0] = M * G
    tr = O.quad_rollout(u, [0.3, -0.2, 1.0, 0, 0, 0.5], [0.0] * 6)
    assert torch.allclose(tr[..., :3], torch.tensor([0.3, -0.2, 1.0]).expand(K, H, 3), atol=2e-6)
    assert torch.allclose(tr[..., 5], torch.full((K, H), 0.5), atol=1e-7)


def test_free_fall_is_semi_implicit_euler():
    """z_t = z0 - g dt^2 sum_{i=1..t} (i+1): step 0 moves with the measured velocity
    (drone_mppi.py:70), later steps with the updated one (:78)."""
    H = 20
    tr = O.quad_rollout(torch.zeros(1, H, 4), [0, 0, 5.0, 0, 0, 0], [0.0] * 6)
    want = [5.0 - G * DT * DT * sum(i + 1 for i in range(1, t + 1)) for t in range(H)]
    assert np.allclose(tr[0, :, 2].numpy(), want, atol=2e-5)


def test_yaw_torque_spins_only_yaw():
    H = 16
    u = torch.zeros(1, H, 4)
    u[..., 0] = M * G
    u[..., 3] = 2.59     # tau_z = I_zz -> omega_z grows by dt per step
    tr = O.quad_rollout(u, [0, 0, 1.0, 0, 0, 0], [0.0] * 6)
    wz = [DT * (t + 1) for t in range(H)]
    yaw = [sum(DT * w for w in wz[1:t + 1]) for t in range(H)]   # step 0 integrates the measured rate
    assert np.allclose(tr[0, :, 5].numpy(), yaw, atol=1e-6)
    assert tr[0, :, 3:5].abs().max() == 0.0 and torch.allclose(tr[0, :, :3], torch.tensor([0, 0, 1.0]))


def test_jacobian_and_rotation_match_drone_py():
    """drone.py:114-154 at a generic attitude (float64 numpy restatement)."""
    phi, th, psi = 0.3, -0.4, 1.1
    J = O.quad_jacobian(torch.tensor([phi, th, psi], dtype=torch.float64)).numpy()
    Jr = np.array([[1, math.sin(phi) * math.tan(th), math.cos(phi) * math.tan(th)],
                   [0, math.cos(phi), -math.sin(phi)],
                   [0, math.sin(phi) / math.cos(th), math.cos(phi) / math.cos(th)]])
    assert np.allclose(J, Jr, atol=1e-12)
    R = O.quad_rotation(torch.tensor([phi, th, psi], dtype=torch.float64)).numpy()
    Rz = np.array([[math.cos(psi), -math.sin(psi), 0], [math.sin(psi), math.cos(psi), 0], [0, 0, 1]])
    Ry = np.array([[math.cos(th), 0, math.sin(th)], [0, 1, 0], [-math.sin(th), 0, math.cos(th)]])
    Rx = np.array([[1, 0, 0], [0, math.cos(phi), -math.sin(phi)], [0, math.sin(phi), math.cos(phi)]])
    assert np.allclose(R, Rz @ Ry @ Rx, atol=1e-12)


def test_literal_jinv_closed_form():
    """The device's literal mode (quad_literal_jinv) applies the closed-form inverse
    [[1, 0, -s_th], [0, c_ph, s_ph c_th], [0, -s_ph, c_ph c_th]] where the commented loop
    calls torch.linalg.inv(J) (drone_mppi.py:74); the oracle's literal rollout differs
    from the J rollout once the body rates are nonzero."""
    g = torch.Generator().manual_seed(5)
    e = (torch.rand((512, 3), generator=g, dtype=torch.float64) - 0.5) * torch.tensor([3.0, 2.6, 6.0], dtype=torch.float64)
    Ji = torch.linalg.inv(O.quad_jacobian(e))
    ph, th = e[:, 0], e[:, 1]
    z, o = torch.zeros_like(ph), torch.ones_like(ph)
    Jc = torch.stack([torch.stack([o, z, -torch.sin(th)], -1),
                      torch.stack([z, torch.cos(ph), torch.sin(ph) * torch.cos(th)], -1),
                      torch.stack([z, -torch.sin(ph), torch.cos(ph) * torch.cos(th)], -1)], -2)
    assert torch.allclose(Ji, Jc, atol=1e-9)
    u = torch.zeros((1, 16, 4))
    u[..., 0] = 14.7 * 9.81
    u[..., 1:] = 0.5
    a = O.quad_rollout(u, [0, 0, 1.0, 0.2, -0.3, 0.1], [0.0] * 6)
    b = O.quad_rollout(u, [0, 0, 1.0, 0.2, -0.3, 0.1], [0.0] * 6, literal_jinv=True)
    assert torch.equal(a[:, :1], b[:, :1])            # step 0 applies J in both (:69)
    assert (a[:, 1:, 3:] - b[:, 1:, 3:]).abs().max() > 1e-6


def test_tilted_thrust_accelerates_sideways():
    """Roll phi tilts body z toward -y: a_y = -g tan(phi) at the thrust that holds altitude."""
    phi = 0.2
    u = torch.zeros(1, 3, 4)
    u[..., 0] = M * G / math.cos(phi)
    tr = O.quad_rollout(u, [0, 0, 1.0, phi, 0, 0], [0.0] * 6)
    vy1 = (tr[0, 1, 1] - tr[0, 0, 1]) / DT
    assert abs(vy1.item() - (-2 * G * math.tan(phi) * DT)) < 1e-4
    assert abs(tr[0, 2, 2].item() - 1.0) < 1e-5


def test_step_improves_toward_target():
    torch.manual_seed(0)
    K, H = 512, 32
    u = torch.zeros(H, 4)
    u[:, 0] = M * G
    noise = O.draw_noise(K, H, torch.diag(torch.tensor([30.0, 1.0, 1.0, 1.0])))
    r = O.quad_step([0, 0, 3.0, 0, 0, 0], [0.0] * 6, u, noise, [0.0, 0.0, 3.4])
    assert r["u_prev_out"][0, 0] > M * G      # climbs toward z* = 3.4
    assert torch.isfinite(r["x_out"]).all() and torch.isfinite(r["v_out"]).all()


def test_capi_quadrotor_layout():
    L = capi.lib()
    c = capi.Config()
    L.mppi_config_default(C.byref(c), capi.MODEL_QUADROTOR)
    assert (c.n_action, c.n_horizon, c.savgol_window) == (4, 32, 5)
    assert (c.quad_mass, tuple(c.quad_inertia)) == (np.float32(14.7), tuple(np.float32([1.57, 3.93, 2.59])))
    assert c.sigma[0] == 30.0 and c.sigma[5] == 1.0 and c.sigma[1] == 0.0
    assert L.mppi_state_dim(C.byref(c)) == 12 and L.mppi_output_dim(C.byref(c)) == 12
    assert L.mppi_traj_channels(C.byref(c)) == 6
    c.n_samples, c.n_horizon = 4096, 32
    assert L.mppi_rollout_bytes(C.byref(c)) == 4096 * 32 * 6 * 4 + 4096 * 4
