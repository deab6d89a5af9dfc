"""GPU parity of the batched-vehicle path (BASELINE configs[4]) and of
the long-horizon lane maps (H > 64, the NCH = 2 DPP-scan integrator) against the CPU
oracle, on the same injected noise.

C5 is V vehicles in one launch: per-vehicle state, target, warm start and noise.  The
reference controller is per vehicle (``mppi.py:122-169``; whole-body composed from
``urdfparser.py:128-131``), so every vehicle v of a V > 1 launch is
checked against ``O.wholebody_step`` with vehicle v's own inputs -- trajectory, S, the
weighted noise, u_prev and the outputs -- at the F6 tolerances
(``test_gpu_parity.test_wholebody_matches_composed_fixture``).

Tolerances (written here, as in test_gpu_parity.py):
* positions atol 2e-5, EE atol 5e-5 (O(1) m / rad values);
* S rtol 2e-5;
* w_eps / u_prev rtol 1e-4 (the north star's 1e-4 rel) when the oracle's top-2 cost
  gap is >= 20 lambda; in a near tie the reduction is checked given the GPU's own S
  (rtol 1e-5) and end to end within the softmin's conditioning bound
  (``_amplified_bound``, as for the arm fixtures);
* drone outputs x atol 1e-6, v 1e-5; joint outputs qdes 1e-6, vdes 1e-5 (scaled by the
  u0 error in a near tie).
"""
import numpy as np
import pytest
import torch

from oracle import mppi_oracle as O

pytestmark = pytest.mark.gpu

LAM = 0.1
HOME_Q = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]            # kinova.py:135
ARM_TARGET = ([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])   # mppi.py:71-72
WB_SIGMA = np.diag([30.0] * 3 + [0.1] * 7).astype(np.float32)


def _engine(**kw):
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    return Engine(make_config(**kw))


def _chain():
    from quadrotor_manipulator_mppi_amd.robot.urdf_chain import load_chain
    return [O.Joint(j["name"], j["type"], j["xyz"], j["rpy"], j["axis"], j["q_index"]) for j in load_chain()]


def _close(got, want, rtol=0.0, atol=0.0, what=""):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    err = np.abs(got - want)
    bad = err > atol + rtol * np.abs(want)
    assert not bad.any(), f"{what}: {bad.sum()} / {bad.size} off, max err {err.max():.3e}"


def _gap(S):
    s = np.sort(np.asarray(S, np.float64))
    return float(s[1] - s[0])


def _amplified_bound(dS_max, w, noise, lam):
    """|d w_eps| <= (2/lam) max|dS| sum_k w_k |eps_k| (first order) + rounding."""
    return (2.0 / lam) * dS_max * np.einsum("k,kha->ha", w, np.abs(noise)) * 1.5 + 2e-6


def _check_reduction(S_gpu, raw, sm, u_prev_gpu, ref, noise, window, what):
    """The softmin-weighted noise, its SavGol and the update of one vehicle.  Returns
    the u0 tolerance the outputs inherit."""
    w_own = O.softmin(torch.from_numpy(S_gpu), LAM).numpy().astype(np.float64)
    _close(raw, np.einsum("k,kha->ha", w_own, noise), rtol=1e-5, atol=1e-7, what=f"{what}: w_eps | S_gpu")
    S_ref = ref["S"].numpy()
    if _gap(S_ref) >= 20 * LAM:
        _close(raw, ref["w_eps_raw"].numpy(), rtol=1e-4, atol=1e-5, what=f"{what}: w_eps")
        _close(sm, ref["w_eps"].numpy(), rtol=1e-4, atol=1e-5, what=f"{what}: w_eps savgol")
        _close(u_prev_gpu, ref["u_prev_out"].numpy(), rtol=1e-4, atol=1e-5, what=f"{what}: u_prev")
        return 1e-5
    dS = float(np.max(np.abs(S_gpu.astype(np.float64) - S_ref)))
    bound = _amplified_bound(dS, ref["w"].numpy().astype(np.float64), noise, LAM)
    assert np.all(np.abs(raw - ref["w_eps_raw"].numpy()) <= bound), f"{what}: w_eps beyond conditioning bound"
    sm_bound = np.abs(O.savgol(torch.from_numpy(bound.astype(np.float32)), window, 2).numpy()) + 4 * bound.max()
    assert np.all(np.abs(sm - ref["w_eps"].numpy()) <= sm_bound), f"{what}: savgol beyond bound"
    assert np.all(np.abs(u_prev_gpu - ref["u_prev_out"].numpy()) <= sm_bound + 1e-6), f"{what}: u_prev"
    return float(sm_bound.max()) + 1e-6


def _fleet_inputs(V, K, H, seed, sigma=WB_SIGMA):
    """C4 state + U(-0.5,0.5) m xyz and U(-0.2,0.2) rad joint offsets,
    targets jittered by +-0.1 m; here also a per-vehicle base yaw, base/joint rates and
    warm start so that every per-vehicle input of the launch differs."""
    rng = np.random.default_rng(seed)
    torch.manual_seed(seed)
    veh = []
    for v in range(V):
        x = (np.array([0.0, 0.0, 1.0]) + rng.uniform(-0.5, 0.5, 3)).tolist()
        yaw = rng.uniform(-0.6, 0.6)
        quat = [0.0, 0.0, float(np.sin(yaw / 2)), float(np.cos(yaw / 2))]
        q = (np.array(HOME_Q) + rng.uniform(-0.2, 0.2, 7)).tolist()
        vx = rng.uniform(-0.3, 0.3, 3).tolist()
        qd = rng.uniform(-0.4, 0.4, 7).tolist()
        tpos = (np.array(ARM_TARGET[0]) + rng.uniform(-0.1, 0.1, 3)).astype(np.float32)
        u_prev = (torch.randn(H, 10) * torch.tensor([2.0] * 3 + [0.2] * 7)).float()
        noise = O.draw_noise(K, H, torch.from_numpy(sigma))
        # the engine's state vector: base pos(3) quat(4) q(7) base vel(3) qd(7)
        state = np.array(x + quat + q + vx + qd, np.float64)
        veh.append(dict(x=x, quat=quat, q=q, vx=vx, qd=qd, tpos=tpos, u_prev=u_prev, noise=noise, state=state))
    return veh


def _run_fleet_vs_oracle(V, K, H, sigma=WB_SIGMA):
    chain = _chain()
    veh = _fleet_inputs(V, K, H, seed=1000 + V + H, sigma=sigma)
    e = _engine(model="wholebody", n_samples=K, n_horizon=H, n_vehicles=V, noise="injected",
                sigma=sigma)
    for v, d in enumerate(veh):
        e.set_target(d["tpos"], ARM_TARGET[1], vehicle=v)
    e.set_u_prev(np.stack([d["u_prev"].numpy() for d in veh]))
    noise = np.stack([d["noise"].numpy() for d in veh])
    out, u0, st = e.step(np.stack([d["state"] for d in veh]), noise)
    tr = e.get_trajectory()
    S = e.get_costs()
    raw, sm = e.get_weighted_noise()
    up = e.get_u_prev()
    e.close()
    dt = 0.01
    for v, d in enumerate(veh):
        what = f"vehicle {v}"
        ref = O.wholebody_step(chain, d["x"], d["vx"], d["q"], d["qd"], O.base_rpy_from_quat(d["quat"]),
                               d["u_prev"], d["noise"], d["tpos"], ARM_TARGET[1])
        _close(tr[v, ..., :10], ref["q_samples"].numpy(), atol=2e-5, what=f"{what}: positions")
        _close(tr[v, ..., 10:], ref["ee"].numpy().reshape(K, H, 16), atol=5e-5, what=f"{what}: EE")
        _close(S[v], ref["S"].numpy(), rtol=2e-5, what=f"{what}: S")
        u0_tol = _check_reduction(S[v], raw[v], sm[v], up[v], ref, d["noise"].numpy(), 9, what)
        _close(out[v, :3], ref["x_out"].numpy(), atol=max(1e-6, u0_tol * dt * dt), what=f"{what}: x")
        _close(out[v, 3:6], ref["v_out"].numpy(), atol=max(1e-5, u0_tol * dt), what=f"{what}: v")
        _close(out[v, 6:13], ref["qdes"].numpy(), atol=max(1e-6, u0_tol * dt * dt), what=f"{what}: qdes")
        _close(out[v, 13:20], ref["vdes"].numpy(), atol=max(1e-5, u0_tol * dt), what=f"{what}: vdes")
        assert not st[v].nonfinite


def test_fleet_c5_every_vehicle_matches_oracle():
    """V=8 vehicles x K=1024 x H=64 whole-body in one launch (the C5 layout at reduced
    K): every vehicle against its own oracle step.  A wrong per-vehicle offset of the
    records, targets, warm start or state (v >= 1) fails here."""
    _run_fleet_vs_oracle(8, 1024, 64)


def test_fleet_long_horizon_matches_oracle():
    """V=3 at H=128 (NCH = 2: DPP segment scans with a carry between the 64-step
    chunks) -- the batched path on the long-horizon lane map."""
    _run_fleet_vs_oracle(3, 256, 128)


@pytest.mark.parametrize("V", [1, 3])
def test_wholebody_full_sigma_extended_kernel(V):
    """A non-diagonal Sigma runs the whole-body rollout in the extended (XC) instantiation
    (its own register budget, the full z Sigma product): every vehicle against the oracle
    on the same injected noise, V == 1 (constants in the kernel arguments) and V > 1."""
    sig = WB_SIGMA.astype(np.float64).copy()
    sig[0, 1] = sig[1, 0] = 2.0          # xy correlation of the drone dims
    sig[4, 5] = sig[5, 4] = 0.02         # two arm joints
    _run_fleet_vs_oracle(V, 256, 64, sigma=sig.astype(np.float32))


def test_wholebody_ragged_k_looping_kernel():
    """K = 2999 on V = 2 vehicles runs the looping kernel (125 blocks x 3 groups of 8 waves per
    vehicle = 3000 rollout slots): the padding rollout of the last group must stay out of
    every vehicle's trajectory, S, records and weights."""
    _run_fleet_vs_oracle(2, 2999, 64)


def test_fleet_c5_full_size_properties():
    """C5 per-GPU share at full size: V=8 x K=8192 x H=64 whole-body with device Philox.
    Per vehicle: finite costs, sum w = 1, w_eps = sum_k w_k eps_k of the stored noise;
    a second engine with the same seed reproduces every output bit for bit; vehicles
    draw distinct noise (the Philox counter carries the vehicle id)."""
    V, K, H = 8, 8192, 64
    rng = np.random.default_rng(5)
    states = []
    for v in range(V):
        off = rng.uniform(-0.5, 0.5, 3) if v else np.zeros(3)
        joff = rng.uniform(-0.2, 0.2, 7) if v else np.zeros(7)
        states.append(list(np.array([0.0, 0.0, 1.0]) + off) + [0.0, 0.0, 0.0, 1.0]
                      + list(np.array(HOME_Q) + joff) + [0.0] * 10)
    states = np.array(states, np.float64)
    tg = [np.array(ARM_TARGET[0]) + (rng.uniform(-0.1, 0.1, 3) if v else 0.0) for v in range(V)]
    res = []
    for rep in range(2):
        e = _engine(model="wholebody", n_samples=K, n_horizon=H, n_vehicles=V, seed=31, store_noise=True)
        for v in range(V):
            e.set_target(tg[v], ARM_TARGET[1], vehicle=v)
        out, u0, st = e.step(states)
        S = e.get_costs()
        w = e.get_weights().astype(np.float64)
        raw, sm = e.get_weighted_noise()
        up = e.get_u_prev()
        if rep == 0:
            eps = e.get_noise()
            assert np.isfinite(S).all() and (S > 0).all()
            for v in range(V):
                assert abs(w[v].sum() - 1.0) < 1e-4, f"vehicle {v}: sum w = {w[v].sum()}"
                _close(raw[v], np.einsum("k,kha->ha", w[v], eps[v]), rtol=1e-4, atol=1e-7,
                       what=f"vehicle {v}: w_eps = sum w eps")
                assert st[v].ess >= 1.0 and not st[v].nonfinite
            assert not np.array_equal(eps[0], eps[1]), "vehicles must draw distinct noise"
            del eps
        res.append((out, u0, S, raw, sm, up))
        e.close()
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b), "same seed must reproduce bit-for-bit"


# ------------------------------------------------------------ long horizons (H > 64)
@pytest.mark.parametrize("H,f64,full", [(65, True, False), (100, True, False), (128, False, False), (128, True, False),
                                        (200, True, False), (256, False, False), (200, True, True), (256, False, True)])
def test_arm_long_horizons_match_oracle(H, f64, full):
    """Arm at H = 65..256 (NCH = 2 and 4 DPP-scan integrator, fp32 and fp64 state; NCH = 4
    runs the 2-wave register budget; H = 65 / 100 / 200 pad the trajectory rows to 64 B)
    against the oracle: trajectory, EE, S and the update (standard_normal_noise.py:41-48).
    ``full``: a full Sigma selects the extended (XC) kernel, whose NCH = 4 instantiation
    once ran its rollout group out of line (a 1.7 KB stack frame)."""
    chain = _chain()
    K = 256
    torch.manual_seed(300 + H)
    sig = np.eye(7, dtype=np.float32) * 0.1
    if full:
        sig[0, 1] = sig[1, 0] = 0.02
    noise = O.draw_noise(K, H, torch.from_numpy(sig))
    u_prev = torch.randn(H, 7) * 0.3
    q_full = np.array([0.1, -0.2, 1.1, 0.0, 0.0, 0.2588190, 0.9659258] + HOME_Q)
    v_full = np.array([0.0] * 6 + [0.8, -0.5, 0.3, -1.2, 0.4, 0.9, -0.7])
    r = O.arm_step(chain, q_full, v_full, u_prev, noise, *ARM_TARGET, f64=f64)
    e = _engine(model="arm", n_samples=K, n_horizon=H, noise="injected", state_f64=f64, sigma=sig)
    e.set_target(*ARM_TARGET)
    e.set_u_prev(u_prev.numpy())
    out, u0, st = e.step(np.concatenate([q_full[:7], q_full[7:], v_full[6:]]), noise.numpy()[None])
    tr = e.get_trajectory()[0]
    _close(tr[..., :7], r["q_samples"].numpy(), atol=2e-5, what="q")
    _close(tr[..., 7:], r["ee"].numpy().reshape(K, H, 16), atol=5e-5, what="EE")
    S = e.get_costs()[0]
    _close(S, r["S"].numpy(), rtol=2e-5, what="S")
    raw, sm = e.get_weighted_noise()
    _check_reduction(S, raw[0], sm[0], e.get_u_prev()[0], r, noise.numpy(), 9, f"arm H={H}")


@pytest.mark.parametrize("H", [65, 100, 128, 200])
def test_wholebody_long_horizons_match_oracle(H):
    """Whole-body at H = 65..200 (NCH = 2 and 4) against the oracle's composed step (A16)."""
    chain = _chain()
    K = 256
    torch.manual_seed(400 + H)
    noise = O.draw_noise(K, H, torch.from_numpy(WB_SIGMA))
    u_prev = torch.randn(H, 10) * 0.3
    x, vx, q, qd = [0.3, -0.1, 1.2], [0.5, -0.4, 0.2], HOME_Q, [0.8, -0.5, 0.3, -1.2, 0.4, 0.9, -0.7]
    quat = [0.0, 0.0, 0.1305262, 0.9914449]
    r = O.wholebody_step(chain, x, vx, q, qd, O.base_rpy_from_quat(quat), u_prev, noise, *ARM_TARGET)
    e = _engine(model="wholebody", n_samples=K, n_horizon=H, noise="injected", sigma=WB_SIGMA)
    e.set_target(*ARM_TARGET)
    e.set_u_prev(u_prev.numpy())
    e.step(np.array(x + quat + q + vx + qd, np.float64), noise.numpy()[None])
    tr = e.get_trajectory()[0]
    _close(tr[..., :10], r["q_samples"].numpy(), atol=2e-5, what="positions")
    _close(tr[..., 10:], r["ee"].numpy().reshape(K, H, 16), atol=5e-5, what="EE")
    S = e.get_costs()[0]
    _close(S, r["S"].numpy(), rtol=2e-5, what="S")
    raw, sm = e.get_weighted_noise()
    _check_reduction(S, raw[0], sm[0], e.get_u_prev()[0], r, noise.numpy(), 9, f"wholebody H={H}")


def test_output_sequence_survives_step_counter_rewind():
    """A step replayed with mppi_set_step_counter (same Philox counter) must still hand
    back its own outputs: the completion flag's sequence number is independent of the
    Philox counter (it used to be step_ctr + 1, so a rewound step matched the flags the
    previous step had left and read_outputs returned stale data)."""
    K, H = 1024, 32
    state = np.array([0, 0, 1, 0, 0, 0, 1] + HOME_Q + [0.0] * 7, np.float64)
    e = _engine(model="arm", n_samples=K, n_horizon=H, seed=17)
    e.set_target(*ARM_TARGET)
    e.set_step_counter(5)
    out1, u01, _ = e.step(state)
    e.set_step_counter(5)          # replay the same noise on the updated warm start
    out2, u02, _ = e.step(state)
    up = e.get_u_prev()[0]
    assert np.array_equal(u02[0], up[0]), "u0 must be the replayed step's u_prev[0]"
    assert not np.array_equal(u01, u02), "the replay moved u_prev, so u0 must differ"
    e.close()


# ------------------------------------------ SavGol windows (finalize template / generic path)
@pytest.mark.parametrize("model,H,window,order", [("arm", 32, 7, 3), ("arm", 16, 11, 2), ("arm", 32, 3, 1),
                                                  ("drone", 20, 9, 2), ("drone", 64, 13, 4),
                                                  ("wholebody", 64, 5, 2), ("arm", 32, 19, 2),
                                                  ("arm", 32, 31, 2), ("drone", 20, 19, 3),
                                                  ("wholebody", 64, 31, 4)])
def test_savgol_windows_match_oracle(model, H, window, order):
    """The finalize's SavGol for every window class: the templated 9- and 5-tap kernels
    and the generic one (3, 7, 11, 13, 19, 31 taps: half-widths up to MPPI_MAX_SAVGOL/2 = 15,
    the LDS pad's full depth), at horizons whose slices put the reflected
    pads (svg_filter.py:58) inside the window; checked as the reference filter of the
    device's own raw weighted noise (rtol 1e-5), and the update u += SavGol(w_eps)."""
    A = {"arm": 7, "drone": 3, "wholebody": 10}[model]
    K = 512
    torch.manual_seed(window * 31 + H)
    rng = np.random.default_rng(window)
    sig = np.eye(A, dtype=np.float32) * 0.2
    noise = O.draw_noise(K, H, torch.from_numpy(sig)).numpy()
    u_prev = rng.normal(0, 0.3, (H, A)).astype(np.float32)
    e = _engine(model=model, n_samples=K, n_horizon=H, noise="injected", sigma=sig, savgol_window=window,
                savgol_order=order)
    if model == "drone":
        e.set_target(np.asarray([0.5, 0.4, 2.0], np.float32))
        state = np.array([0.0, 0.0, 1.0, 0.1, -0.1, 0.0], np.float64)
    else:
        e.set_target(*ARM_TARGET)
        state = (np.array([0, 0, 1, 0, 0, 0, 1] + HOME_Q + [0.0] * 7, np.float64) if model == "arm" else
                 np.array([0, 0, 1, 0, 0, 0, 1] + HOME_Q + [0.0] * 10, np.float64))
    e.set_u_prev(u_prev)
    e.step(state, noise[None])
    raw, sm = e.get_weighted_noise()
    up = e.get_u_prev()[0]
    e.close()
    want = O.savgol(torch.from_numpy(raw[0].astype(np.float32)), window, order).numpy()
    scale = float(np.abs(raw[0]).max())
    # the engine's taps are the fp64 least-squares solution rounded to fp32; the reference
    # inverts A^T A in fp32 (svg_filter.py:52-55), which for a wide window of high order is
    # ill-conditioned (31 taps, order 4: its taps are 9e-6 off the exact ones, 1e-7 at the
    # reference's own 5/2 and 9/2).  The bar adds that tap error times the signal.
    half = window // 2
    x = np.arange(-half, half + 1, dtype=np.float64)
    Av = np.vander(x, order + 1, increasing=True)
    exact = (np.linalg.inv(Av.T @ Av) @ Av.T)[0]
    tap_err = float(np.abs(O.savgol_coefficients(window, order).numpy() - exact).sum())
    _close(sm[0], want, rtol=1e-5, atol=1e-6 * scale + 2.0 * tap_err * scale,
           what=f"{model} H={H} savgol({window},{order})")
    _close(up, u_prev + sm[0], rtol=1e-6, atol=1e-7, what="u_prev += w_eps")


# ----------------------------------------- extended (XC) kernel: drone full Sigma, generic chain
def test_drone_full_sigma_extended_kernel():
    """A non-diagonal Sigma sends the drone rollout to the extended (XC) instantiation
    (it used to stay on the common kernel): trajectory, S, the reduction, u_prev and the
    outputs against O.drone_step (drone_mppi.py:140-176) on the same injected noise; and in
    device-noise mode the stored eps equals z Sigma (row vector, drone_mppi.py:41-43) of the
    Philox normals."""
    K, H = 512, 32
    sig = np.diag([30.0, 30.0, 30.0]).astype(np.float32)
    sig[0, 1] = sig[1, 0] = 6.0
    sig[1, 2] = sig[2, 1] = -4.0
    torch.manual_seed(71)
    noise = O.draw_noise(K, H, torch.from_numpy(sig))
    u_prev = torch.randn(H, 3) * 2.0
    x, v, tgt = [0.0, 0.0, 1.0], [0.1, -0.1, 0.0], [1.0, 2.0, 3.4]
    ref = O.drone_step(x, v, u_prev, noise, tgt)
    e = _engine(model="drone", n_samples=K, n_horizon=H, noise="injected", sigma=sig)
    e.set_target(np.asarray(tgt, np.float32))
    e.set_u_prev(u_prev.numpy())
    out, u0, st = e.step(np.array(x + v, np.float64), noise.numpy()[None])
    _close(e.get_trajectory()[0], ref["traj"].numpy(), atol=2e-5, what="drone traj (full Sigma)")
    S = e.get_costs()[0]
    _close(S, ref["S"].numpy(), rtol=2e-5, what="drone S (full Sigma)")
    raw, sm = e.get_weighted_noise()
    u0_tol = _check_reduction(S, raw[0], sm[0], e.get_u_prev()[0], ref, noise.numpy(), 5, "drone full Sigma")
    _close(out[0, :3], ref["x_out"].numpy(), atol=max(1e-6, u0_tol * 1e-4), what="x")
    _close(out[0, 3:], ref["v_out"].numpy(), atol=max(1e-5, u0_tol * 1e-2), what="v")
    e.close()
    from quadrotor_manipulator_mppi_amd.engine import philox_normals
    e = _engine(model="drone", n_samples=K, n_horizon=H, sigma=sig, seed=3, store_noise=True)
    e.set_target(np.asarray(tgt, np.float32))
    e.step(np.array(x + v, np.float64))
    eps = e.get_noise()[0]
    e.close()
    _, z = philox_normals(3, 0, 0, 0, K, H, 3)
    _close(eps, z @ sig, rtol=1e-5, atol=1e-4, what="eps = z Sigma (device noise, full Sigma)")


@pytest.mark.parametrize("kinova_path_off", [False, True])
def test_arm_generic_chain_extended_kernel(kinova_path_off, monkeypatch):
    """Arm chains other than the Kinova axis-permutation chain run the generic FK (one 3x4
    affine product and one sincos per joint) in the extended (XC) instantiation: a URDF
    whose joint origins are not signed axis permutations (joint 3 tilted, joint 5 offset),
    and the shipped chain with the Kinova path disabled (MPPI_NO_KINOVA_PATH) -- each against
    the oracle's chain product (urdfparser.py:122-163) on the same injected noise."""
    from quadrotor_manipulator_mppi_amd.robot.urdf_chain import load_chain
    chain_d = [dict(j) for j in load_chain()]
    if kinova_path_off:
        monkeypatch.setenv("MPPI_NO_KINOVA_PATH", "1")
    else:
        chain_d[3]["rpy"] = [float(chain_d[3]["rpy"][0]) + 0.13, float(chain_d[3]["rpy"][1]) - 0.07,
                             float(chain_d[3]["rpy"][2])]
        chain_d[5]["xyz"] = [float(chain_d[5]["xyz"][0]) + 0.011, float(chain_d[5]["xyz"][1]),
                             float(chain_d[5]["xyz"][2]) - 0.02]
    chain = [O.Joint(j["name"], j["type"], j["xyz"], j["rpy"], j["axis"], j["q_index"]) for j in chain_d]
    K, H = 512, 32
    torch.manual_seed(91)
    noise = O.draw_noise(K, H, torch.eye(7) * 0.1)
    u_prev = torch.randn(H, 7) * 0.3
    q_full = np.array([0.1, -0.2, 1.1, 0.0, 0.0, 0.2588190, 0.9659258] + HOME_Q)
    v_full = np.array([0.0] * 6 + [0.8, -0.5, 0.3, -1.2, 0.4, 0.9, -0.7])
    r = O.arm_step(chain, q_full, v_full, u_prev, noise, *ARM_TARGET, f64=True)
    e = _engine(model="arm", n_samples=K, n_horizon=H, noise="injected", chain=chain_d)
    e.set_target(*ARM_TARGET)
    e.set_u_prev(u_prev.numpy())
    e.step(np.concatenate([q_full[:7], q_full[7:], v_full[6:]]), noise.numpy()[None])
    tr = e.get_trajectory()[0]
    _close(tr[..., :7], r["q_samples"].numpy(), atol=2e-6, what="q")
    _close(tr[..., 7:], r["ee"].numpy().reshape(K, H, 16), atol=2e-5, what="EE (generic chain)")
    S = e.get_costs()[0]
    _close(S, r["S"].numpy(), rtol=2e-5, what="S (generic chain)")
    raw, sm = e.get_weighted_noise()
    _check_reduction(S, raw[0], sm[0], e.get_u_prev()[0], r, noise.numpy(), 9, "arm generic chain")
    e.close()


# ------------------------------------------------------------------ vehicle sharding (C5 over GPUs)
def _fleet_state(V):
    """Fleet-wide states and targets as bench.py makes them (row / target v = vehicle v)."""
    import bench
    return bench.make_state("wholebody", V)


def _fleet_engine(V, K, H, offset=0, **kw):
    e = _engine(model="wholebody", n_samples=K, n_horizon=H, n_vehicles=V, seed=77, vehicle_offset=offset,
                blocks_per_vehicle=32, **kw)
    return e


def _set_fleet_targets(e, vehicles):
    import bench
    bench.set_targets(e, "wholebody", vehicles)


@pytest.mark.parametrize("dispatch", ["aql", "hip"])
def test_vehicle_split_equals_one_fleet_engine(dispatch, monkeypatch):
    """SURVEY §8e for C5 -- the fleet's vehicles split over engines with nothing exchanged
    (ShardedEngine mode "vehicles"): two engines over vehicles [0, 4) and [4, 8) (vehicle_offset 0
    and 4: the device noise is keyed by the fleet-wide vehicle index) equal ONE engine over all 8
    vehicles bit for bit -- costs, warm starts after a native batch, and control-call outputs --
    at the same per-vehicle geometry (blocks_per_vehicle pinned; the auto geometry depends on V)."""
    monkeypatch.setenv("MPPI_DISPATCH", dispatch)
    V, K, H = 8, 1024, 64
    full = _fleet_engine(V, K, H)
    halves = [_fleet_engine(4, K, H, offset=o) for o in (0, 4)]
    state = _fleet_state(V)
    _set_fleet_targets(full, range(V))
    full.set_state(state)
    for i, e in enumerate(halves):
        _set_fleet_targets(e, range(4 * i, 4 * i + 4))
        e.set_state(state[4 * i:4 * i + 4])
    try:
        for e in [full] + halves:
            e.run_steps(12)
            e.synchronize()
        assert np.array_equal(np.concatenate([e.get_u_prev() for e in halves]), full.get_u_prev())
        assert np.array_equal(np.concatenate([e.get_costs() for e in halves]), full.get_costs())
        st2 = state.copy()
        st2[:, 7:14] += 0.01
        o_f, u_f, s_f = full.step(st2)
        parts = [e.step(st2[4 * i:4 * i + 4]) for i, e in enumerate(halves)]
        assert np.array_equal(np.concatenate([p[0] for p in parts]), o_f)
        assert np.array_equal(np.concatenate([p[1] for p in parts]), u_f)
        assert [(s.rho, s.eta) for p in parts for s in p[2]] == [(s.rho, s.eta) for s in s_f]
    finally:
        for e in [full] + halves:
            e.close()


def _vehicle_rank(rank, world, port, V, K, H, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quadrotor_manipulator_mppi_amd.distributed import ShardedEngine
        se = ShardedEngine(mode="vehicles", model="wholebody", n_samples=K, n_horizon=H, n_vehicles=V, seed=77,
                           blocks_per_vehicle=32)
        _set_fleet_targets(se.engine, se.vehicles)
        se.engine.set_state(_fleet_state(V)[se.vehicles.start:se.vehicles.stop])
        se.run_steps(10)
        assert se.synchronize() is False
        out, u0, st = se.step(_fleet_state(V)[se.vehicles.start:se.vehicles.stop])
        q.put((rank, se.mode, se.vehicles.start, se.engine.V, se.engine.get_u_prev(), out, se.engine.dispatch_info()))
        se.engine.close()
    finally:
        dist.destroy_process_group()


def test_vehicle_split_two_processes_equal_one_engine():
    """The same through ShardedEngine(mode="vehicles") in two processes (gloo group, one GPU): each
    rank's engine runs its half of the fleet; nothing is exchanged; the ranks' warm starts and
    outputs, concatenated, equal one engine over the whole fleet bit for bit."""
    import socket
    import torch.multiprocessing as mp
    V, K, H = 8, 1024, 64
    full = _fleet_engine(V, K, H)
    _set_fleet_targets(full, range(V))
    full.set_state(_fleet_state(V))
    full.run_steps(10)
    full.synchronize()
    o_f, _, _ = full.step(_fleet_state(V))
    u_f = full.get_u_prev()
    full.close()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_vehicle_rank, args=(r, 2, port, V, K, H, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert [(r[1], r[2], r[3]) for r in res] == [("vehicles", 0, 4), ("vehicles", 4, 4)]
    assert all(r[6].startswith("aql;") for r in res), [r[6] for r in res]
    assert np.array_equal(np.concatenate([r[4] for r in res]), u_f)
    assert np.array_equal(np.concatenate([r[5] for r in res]), o_f)


def test_vehicle_offset_range():
    """The fleet-wide vehicle index rides in the noise argument's high half: an engine whose last
    vehicle is fleet vehicle 32767 is accepted and steps to finite outputs; one past it, or a
    negative offset, is rejected at create (MPPI_ERR_INVALID_ARG)."""
    from quadrotor_manipulator_mppi_amd._capi import MPPIError
    V, K, H = 2, 256, 64
    e = _fleet_engine(V, K, H, offset=32768 - V)
    _set_fleet_targets(e, range(V))
    e.set_state(_fleet_state(V))
    out, u0, st = e.step(_fleet_state(V))
    assert np.isfinite(out).all() and np.isfinite(u0).all() and not any(s.nonfinite for s in st)
    e.close()
    for bad in (32768 - V + 1, -1):
        with pytest.raises(MPPIError):
            _fleet_engine(V, K, H, offset=bad)
