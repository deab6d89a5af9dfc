"""GPU parity: the HIP engine (through the C-ABI) against the golden fixtures
and the CPU oracle, on the same injected noise.

Tolerances (fp32 path; the north star's bar is 1e-4 relative):
* trajectories (positions, joint angles, EE transforms): 2e-5 absolute
  (values are O(1) m / rad);
* per-rollout costs S: 2e-5 relative;
* weights / weighted noise / u / outputs: 1e-4 relative when the fixture's
  top-2 cost gap is >= 20*lambda.  In the near-tie regime (arm fixtures, gap
  0.1-0.8 with lambda = 0.1) the softmin amplifies any fp32 rounding of S by
  1/lambda: there the weighted noise is checked (a) against softmin(S_gpu)
  exactly (the reduction given the GPU's own costs, 1e-5 relative) and (b)
  end-to-end against a bound derived from the measured |dS| (see
  ``_amplified_bound``).  The reference itself cannot reproduce its own S
  bit-for-bit on other hardware (MKL LU in ``linalg.inv``).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import mppi_oracle as O

pytestmark = pytest.mark.gpu


def _engine(**kw):
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    return Engine(make_config(**kw))


def _close(got, want, rtol=0.0, atol=0.0, what=""):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    err = np.abs(got - want)
    lim = atol + rtol * np.abs(want)
    bad = err > lim
    assert not bad.any(), f"{what}: {bad.sum()} / {bad.size} off, max err {err.max():.3e}, " \
                          f"max rel {np.max(err / (np.abs(want) + 1e-30)):.3e}"


def _amplified_bound(dS_max, w, noise, lam):
    """|d w_eps| <= (2/lam) max|dS| sum_k w_k |eps_k| (first order) + rounding."""
    return (2.0 / lam) * dS_max * np.einsum("k,kha->ha", w, np.abs(noise)) * 1.5 + 2e-6


# ----------------------------------------------------------------------------- RNG
def test_device_philox_matches_restatement():
    from quadrotor_manipulator_mppi_amd.engine import philox_normals
    for (seed, step, veh, k0, K, H, A) in [(1234, 0, 0, 0, 64, 32, 7), (2**40 + 7, 5, 3, 4096, 32, 64, 10),
                                           (99, 1, 0, 7, 16, 20, 3), (5, 2, 2, 100, 8, 24, 4)]:
        raw, z = philox_normals(seed, step, veh, k0, K, H, A)
        raw_ref, z_ref = O.philox_normals(seed, step, veh, np.arange(k0, k0 + K), H, A)
        assert np.array_equal(raw, raw_ref), "Philox words must be bit-exact"
        _close(z, z_ref, rtol=2e-5, atol=2e-5, what="Box-Muller normals")


# --------------------------------------------------------------------------- drone
@pytest.mark.parametrize("name", ["drone_k128_h20.npz", "drone_k256_h32.npz"])
def test_drone_matches_reference_fixture(name):
    g = load_golden(name)
    K, H = int(g["K"]), int(g["H"])
    e = _engine(model="drone", n_samples=K, n_horizon=H, noise="injected", store_noise=True)
    e.set_target(g["target"])
    for s in range(int(g["steps"])):
        e.set_u_prev(g[f"s{s}_u_prev_in"])
        state = np.concatenate([g[f"s{s}_x_in"], g[f"s{s}_v_in"]]).astype(np.float64)
        out, u0, st = e.step(state, g[f"s{s}_noise"][None])
        assert g["top2_gap"][s] >= 20 * 0.1
        _close(e.get_trajectory()[0], g[f"s{s}_traj"], atol=2e-5, what="traj")
        _close(e.get_costs()[0], g[f"s{s}_S"], rtol=2e-5, what="S")
        _close(e.get_weights()[0], g[f"s{s}_w"], rtol=1e-4, atol=1e-12, what="w")
        raw, sm = e.get_weighted_noise()
        _close(raw[0], g[f"s{s}_w_eps_raw"], rtol=1e-4, atol=1e-5, what="w_eps raw")
        _close(sm[0], g[f"s{s}_w_eps"], rtol=1e-4, atol=1e-5, what="w_eps savgol")
        _close(e.get_u_prev()[0], g[f"s{s}_u_prev_out"], rtol=1e-4, atol=1e-5, what="u_prev")
        _close(out[0, :3], g[f"s{s}_x_out"], rtol=1e-6, atol=1e-6, what="x")
        _close(out[0, 3:], g[f"s{s}_v_out"], rtol=1e-5, atol=1e-6, what="v")
        assert not st[0].nonfinite


# ----------------------------------------------------------------------------- arm
@pytest.mark.parametrize("name,terms", [("arm_k32_h32_f32.npz", 0), ("arm_k32_h32_f64.npz", 0),
                                        ("arm_k100_h32_f64.npz", 0), ("arm_k64_h32_allcosts.npz", 31)])
def test_arm_matches_reference_fixture(name, terms):
    """F2 fixtures (pose cost, as the reference runs) and F7 (every CostManager
    term switched on: covar, centering, joint tracking, action, joint limit)."""
    g = load_golden(name)
    K, H = int(g["K"]), int(g["H"])
    f64 = bool(g["state_f64"])
    e = _engine(model="arm", n_samples=K, n_horizon=H, noise="injected", state_f64=f64, store_noise=True,
                cost_terms=terms)
    e.set_target(g["target_pos"], g["target_quat"])
    state = np.concatenate([g["q_full"][:7], g["q_full"][7:], g["v_full"][6:]])
    for s in range(int(g["steps"])):
        e.set_u_prev(g[f"s{s}_u_prev_in"])
        noise = g[f"s{s}_noise"]
        out, u0, st = e.step(state, noise[None])
        tr = e.get_trajectory()[0]
        _close(tr[..., :7], g[f"s{s}_q_samples"], atol=2e-6, what="q_samples")
        _close(tr[..., 7:], g[f"s{s}_ee"].reshape(K, H, 16), atol=2e-5, what="EE")
        S, S_ref = e.get_costs()[0], g[f"s{s}_S"]
        _close(S, S_ref, rtol=2e-5, what="S")
        # (a) reduction parity given the GPU's own costs
        w_own = O.softmin(torch.from_numpy(S), 0.1).numpy()
        raw, sm = e.get_weighted_noise()
        _close(e.get_weights()[0], w_own, rtol=1e-5, atol=1e-9, what="w | S_gpu")
        _close(raw[0], np.einsum("k,kha->ha", w_own.astype(np.float64), noise), rtol=1e-5, atol=1e-7,
               what="w_eps | S_gpu")
        # (b) end-to-end against the reference within the softmin's conditioning
        live = g[f"s{s}_w"] > 1e-12    # samples the 1e10 joint-limit penalty did not zero out
        dS = float(np.max(np.abs(S.astype(np.float64) - S_ref)[live]))
        bound = _amplified_bound(dS, g[f"s{s}_w"].astype(np.float64), noise, 0.1)
        assert np.all(np.abs(raw[0] - g[f"s{s}_w_eps_raw"]) <= bound), "w_eps beyond conditioning bound"
        sm_bound = np.abs(O.savgol(torch.from_numpy(bound.astype(np.float32)), 9, 2).numpy()) + 4 * bound.max()
        assert np.all(np.abs(sm[0] - g[f"s{s}_w_eps"]) <= sm_bound)
        dt = 0.01
        qdes_ref, vdes_ref = g[f"s{s}_qdes"], g[f"s{s}_vdes"]
        u0_ref = g[f"s{s}_u_prev_out"][0]
        u0_tol = np.abs(u0 - u0_ref).max() + 1e-7
        _close(u0[0], u0_ref, atol=float(sm_bound.max()) + 1e-6, what="u0")
        _close(out[0, 7:], vdes_ref, atol=u0_tol * dt + 1e-7, what="vdes")
        _close(out[0, :7], qdes_ref, atol=u0_tol * dt * dt + 1e-7, what="qdes")
        assert st[0].reach == bool(g[f"s{s}_reach"])


def test_arm_matches_reference_fixture_plain_tolerance():
    """F2c: the arm fixture whose top-2 cost gap is >= 20 lambda in both steps (the
    sampler's Sigma at 1.0 I), so the whole arm step -- w, w_eps, SavGol, u_prev,
    qdes, vdes -- meets the north star's plain 1e-4 rel against the reference, with
    no conditioning bound (mppi.py:122-169)."""
    g = load_golden("arm_k32_h32_gap.npz")
    K, H = int(g["K"]), int(g["H"])
    assert np.all(g["top2_gap"] >= 20 * 0.1)
    e = _engine(model="arm", n_samples=K, n_horizon=H, noise="injected", state_f64=True,
                sigma=g["sigma"])
    e.set_target(g["target_pos"], g["target_quat"])
    state = np.concatenate([g["q_full"][:7], g["q_full"][7:], g["v_full"][6:]])
    for s in range(int(g["steps"])):
        e.set_u_prev(g[f"s{s}_u_prev_in"])
        out, u0, st = e.step(state, g[f"s{s}_noise"][None])
        tr = e.get_trajectory()[0]
        _close(tr[..., :7], g[f"s{s}_q_samples"], atol=2e-6, what="q_samples")
        _close(tr[..., 7:], g[f"s{s}_ee"].reshape(K, H, 16), atol=2e-5, what="EE")
        _close(e.get_costs()[0], g[f"s{s}_S"], rtol=2e-5, what="S")
        _close(e.get_weights()[0], g[f"s{s}_w"], rtol=1e-4, atol=1e-12, what="w")
        raw, sm = e.get_weighted_noise()
        _close(raw[0], g[f"s{s}_w_eps_raw"], rtol=1e-4, atol=1e-6, what="w_eps raw")
        _close(sm[0], g[f"s{s}_w_eps"], rtol=1e-4, atol=1e-6, what="w_eps savgol")
        _close(e.get_u_prev()[0], g[f"s{s}_u_prev_out"], rtol=1e-4, atol=1e-6, what="u_prev")
        _close(out[0, :7], g[f"s{s}_qdes"], rtol=1e-6, atol=1e-9, what="qdes")
        _close(out[0, 7:], g[f"s{s}_vdes"], rtol=1e-4, atol=1e-9, what="vdes")
        assert st[0].reach == bool(g[f"s{s}_reach"])


def test_arm_trajectory_matches_oracle_large():
    """K=1024 H=32 fp64 state, seeded randn noise: oracle at the same inputs."""
    from quadrotor_manipulator_mppi_amd.robot.urdf_chain import load_chain
    chain = [O.Joint(j["name"], j["type"], j["xyz"], j["rpy"], j["axis"], j["q_index"]) for j in load_chain()]
    K, H = 1024, 32
    torch.manual_seed(7)
    noise = O.draw_noise(K, H, torch.eye(7) * 0.1)
    u_prev = torch.randn(H, 7) * 0.05
    q_full = np.array([0.1, -0.2, 1.1, 0.0, 0.0, 0.2588190, 0.9659258] + [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0])
    v_full = np.array([0.0] * 6 + [0.1, -0.1, 0.05, 0.0, 0.02, 0.0, -0.03])
    r = O.arm_step(chain, q_full, v_full, u_prev, noise, [0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    e = _engine(model="arm", n_samples=K, n_horizon=H, noise="injected", state_f64=True)
    e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    e.set_u_prev(u_prev.numpy())
    e.step(np.concatenate([q_full[:7], q_full[7:], v_full[6:]]), noise.numpy()[None])
    tr = e.get_trajectory()[0]
    _close(tr[..., :7], r["q_samples"].numpy(), atol=2e-6, what="q")
    _close(tr[..., 7:], r["ee"].numpy().reshape(K, H, 16), atol=2e-5, what="EE")
    _close(e.get_costs()[0], r["S"].numpy(), rtol=2e-5, what="S")


# ----------------------------------------------------------------------- whole-body
def test_wholebody_matches_composed_fixture():
    g = load_golden("wholebody_k32_h64.npz")
    K, H = int(g["K"]), int(g["H"])
    e = _engine(model="wholebody", n_samples=K, n_horizon=H, noise="injected", sigma=g["sigma"])
    e.set_target(g["target_pos"], g["target_quat"])
    for s in range(int(g["steps"])):
        e.set_u_prev(g[f"s{s}_u_prev_in"])
        state = np.concatenate([g[f"s{s}_x_in"], g["base_quat"], g[f"s{s}_q_in"], g[f"s{s}_vx_in"],
                                g[f"s{s}_qd_in"]]).astype(np.float64)
        noise = g[f"s{s}_noise"]
        out, u0, st = e.step(state, noise[None])
        tr = e.get_trajectory()[0]
        _close(tr[..., :10], g[f"s{s}_q_samples"], atol=2e-5, what="positions")
        _close(tr[..., 10:], g[f"s{s}_ee"].reshape(K, H, 16), atol=5e-5, what="EE")
        _close(e.get_costs()[0], g[f"s{s}_S"], rtol=2e-5, what="S")
        assert g["top2_gap"][s] >= 20 * 0.1
        raw, sm = e.get_weighted_noise()
        _close(raw[0], g[f"s{s}_w_eps_raw"], rtol=1e-4, atol=1e-5, what="w_eps")
        _close(e.get_u_prev()[0], g[f"s{s}_u_prev_out"], rtol=1e-4, atol=1e-5, what="u_prev")
        _close(out[0, :3], g[f"s{s}_x_out"], rtol=1e-6, atol=1e-6, what="x")
        _close(out[0, 3:6], g[f"s{s}_v_out"], rtol=1e-5, atol=1e-6, what="v")
        _close(out[0, 6:13], g[f"s{s}_qdes"], rtol=1e-6, atol=1e-6, what="qdes")
        _close(out[0, 13:20], g[f"s{s}_vdes"], rtol=1e-5, atol=1e-6, what="vdes")


# ------------------------------------------------------------- horizon chunks H>64
@pytest.mark.parametrize("H", [20, 64, 100, 128, 200, 256])
def test_drone_horizons_match_oracle(H):
    """Drone horizons over every lane map: L = 32, 64, NCH = 2 and NCH = 4 (H = 193..256,
    the 2-wave register budget), rows padded to 64 B (H = 20, 100, 200)."""
    K = 512
    torch.manual_seed(H)
    noise = O.draw_noise(K, H, torch.eye(3) * 30.0)
    u_prev = torch.randn(H, 3)
    r = O.drone_step([0.1, 0.2, 1.0], [0.3, 0.0, -0.1], u_prev, noise, [1.0, 2.0, 3.4])
    e = _engine(model="drone", n_samples=K, n_horizon=H, noise="injected")
    e.set_target([1.0, 2.0, 3.4])
    e.set_u_prev(u_prev.numpy())
    out, _, _ = e.step(np.array([0.1, 0.2, 1.0, 0.3, 0.0, -0.1]), noise.numpy()[None])
    _close(e.get_trajectory()[0], r["traj"].numpy(), atol=5e-5, what="traj")
    _close(e.get_costs()[0], r["S"].numpy(), rtol=2e-5, what="S")
    _close(e.get_u_prev()[0], r["u_prev_out"].numpy(), rtol=1e-4, atol=1e-4, what="u")


# -------------------------------------------------- full-size properties (Philox)
def test_full_size_arm_properties_and_determinism():
    """C3 shape K=4096 H=32 with device noise: finite costs, normalised weights,
    bit-identical reruns, weighted noise = sum_k w_k eps_k of the stored noise."""
    kw = dict(model="arm", n_samples=4096, n_horizon=32, seed=11, store_noise=True)
    state = np.array([0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7, np.float64)
    outs = []
    for _ in range(2):
        e = _engine(**kw)
        e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
        out, u0, st = e.step(state)
        outs.append((out, e.get_u_prev(), e.get_costs()))
        S = e.get_costs()[0]
        assert np.isfinite(S).all() and (S > 0).all()
        w = e.get_weights()[0].astype(np.float64)
        assert abs(w.sum() - 1.0) < 1e-4
        eps = e.get_noise()[0]
        raw, _ = e.get_weighted_noise()
        _close(raw[0], np.einsum("k,kha->ha", w, eps), rtol=1e-4, atol=1e-7, what="w_eps = sum w eps")
        assert st[0].ess >= 1.0
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b), "same seed must reproduce bit-for-bit"


@pytest.mark.parametrize("model,K,H", [("arm", 4096, 32), ("wholebody", 2048, 64), ("drone", 8192, 20)])
def test_launch_geometry_invariance(model, K, H):
    """The result does not depend on the block geometry: 1-wave blocks (2048+
    records -> multi-chunk finalize, several rollout groups per block) and
    capped block counts agree with the default launch; costs are bit-identical
    (a rollout's cost never depends on its block), the combine within fp32
    reordering."""
    state = {"arm": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7,
             "drone": [0, 0, 1, 0, 0, 0],
             "wholebody": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 10}[model]
    state = np.array(state, np.float64)
    tgt = ([1.0, 2.0, 3.4], None) if model == "drone" else ([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    res = []
    for bt, nbv in [(0, 0), (64, 0), (256, 7), (512, 1)]:
        e = _engine(model=model, n_samples=K, n_horizon=H, seed=21, block_threads=bt, blocks_per_vehicle=nbv)
        e.set_target(*tgt)
        out, u0, st = e.step(state)
        res.append((e.get_costs(), e.get_u_prev(), out, st[0]))
    S0, u_0, out0, st0 = res[0]
    for S, u, out, st in res[1:]:
        assert np.array_equal(S, S0), "per-rollout costs are geometry independent"
        _close(u, u_0, rtol=1e-4, atol=1e-6, what="u_prev across geometries")
        _close(out, out0, rtol=1e-5, atol=1e-7, what="outputs across geometries")
        assert st.rho == st0.rho
        assert abs(st.eta - st0.eta) <= 1e-4 * st0.eta


def test_kinova_fast_path_matches_generic_chain(monkeypatch):
    """The Kinova path drops the reference's float32 residuals of the origin
    rotations (sin(pi) = -8.7e-8, cos(pi/2) = -4.4e-8); against the generic
    chain product the EE moves by < 1e-6 and the costs by < 1e-7 relative."""
    K, H = 1024, 32
    state = np.array([0.1, -0.2, 1.0, 0.0, 0.0, 0.1305262, 0.9914449] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0]
                     + [0.0] * 7, np.float64)
    res = []
    for disable in (False, True):
        if disable:
            monkeypatch.setenv("MPPI_NO_KINOVA_PATH", "1")
        e = _engine(model="arm", n_samples=K, n_horizon=H, seed=3)
        e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
        e.step(state)
        res.append((e.get_trajectory()[0], e.get_costs()[0]))
    _close(res[0][0], res[1][0], atol=1e-6, what="EE/q Kinova path vs generic")
    _close(res[0][1], res[1][1], rtol=1e-6, what="S Kinova path vs generic")


def test_shards_combine_like_one_engine():
    """Sample sharding: two shard engines + a host sum of their
    exchange slots == one engine over all samples (same global Philox stream)."""
    import ctypes
    K, H = 2048, 32
    state = np.array([0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7, np.float64)
    tgt = ([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    full = _engine(model="arm", n_samples=2 * K, n_horizon=H, seed=5)
    full.set_target(*tgt)
    out_full, u0_full, _ = full.step(state)
    shards = [_engine(model="arm", n_samples=K, n_horizon=H, seed=5, shard_rank=r, shard_count=2)
              for r in range(2)]
    slot = shards[0].exchange_slot_floats()
    bufs = [torch.zeros(2 * slot, device="cuda") for _ in range(2)]
    for sh, b in zip(shards, bufs):
        sh.set_target(*tgt)
        sh.set_state(state)
        sh.bind_exchange(b.data_ptr())
        sh.rollout()
        sh.synchronize()
    total = bufs[0] + bufs[1]          # what the all-reduce computes
    for sh, b in zip(shards, bufs):
        b.copy_(total)
        torch.cuda.synchronize()
        sh.finalize()
    outs = [sh.read_outputs() for sh in shards]
    assert np.array_equal(outs[0][0], outs[1][0]), "every shard finalises identically"
    _close(outs[0][1], u0_full, rtol=1e-4, atol=1e-6, what="u0 sharded vs single")
    _close(shards[0].get_u_prev(), full.get_u_prev(), rtol=1e-4, atol=1e-6, what="u_prev")


def test_native_comm_one_rank_matches_plain_engine():
    """Engine-owned RCCL communicator (mppi_comm_init) with one rank: every step runs
    pack -> ncclAllReduce -> combine-from-slots, and must equal the plain engine
    (the slot combine of one record is the block combine of the same partials)."""
    K, H = 2048, 32
    state = np.array([0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7, np.float64)
    tgt = ([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    plain = _engine(model="arm", n_samples=K, n_horizon=H, seed=11)
    nat = _engine(model="arm", n_samples=K, n_horizon=H, seed=11)
    nat.comm_init(nat.comm_unique_id())
    for e in (plain, nat):
        e.set_target(*tgt)
    o1, u1, s1 = plain.step(state)
    o2, u2, s2 = nat.step(state)
    _close(u2, u1, rtol=1e-5, atol=1e-7, what="u0 native comm vs plain")
    _close(o2, o1, rtol=1e-6, atol=1e-9, what="qdes/vdes native comm vs plain")
    for e in (plain, nat):
        e.run_steps(5)
        e.synchronize()
    _close(nat.get_u_prev(), plain.get_u_prev(), rtol=1e-4, atol=1e-6, what="u_prev after run_steps")
    nat.close()
    plain.close()


def test_vehicle_batch_equals_single_vehicles():
    """V=4 vehicles in one launch == 4 single-vehicle engines (config C5 path)."""
    K, H = 1024, 64
    rng = np.random.default_rng(0)
    base = np.array([0.0, 0.0, 1.0, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 3 + [0.0] * 7)
    states = np.stack([base + np.concatenate([rng.uniform(-.5, .5, 3), [0] * 4, rng.uniform(-.2, .2, 7),
                                              [0] * 10]) for _ in range(4)])
    eb = _engine(model="wholebody", n_samples=K, n_horizon=H, n_vehicles=4, seed=9)
    for v in range(4):
        eb.set_target([0.1 + 0.05 * v, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5], vehicle=v)
    out_b, u0_b, _ = eb.step(states)
    for v in range(4):
        e1 = _engine(model="wholebody", n_samples=K, n_horizon=H, seed=9)
        e1.set_target([0.1 + 0.05 * v, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5])
        # vehicle v of the batch draws Philox counters with vehicle id v
        out_1, u0_1, _ = e1.step(states[v])
        if v == 0:
            _close(u0_b[0], u0_1[0], rtol=1e-4, atol=1e-6, what="vehicle 0")
            _close(out_b[0], out_1[0], rtol=1e-5, atol=1e-7, what="vehicle 0 outputs")
        assert np.isfinite(out_b[v]).all()


def test_empty_noise_zero_update():
    """With eps == 0 the update is exactly zero and u_prev is unchanged."""
    K, H = 256, 32
    e = _engine(model="drone", n_samples=K, n_horizon=H, noise="injected")
    e.set_target([1.0, 2.0, 3.4])
    u = np.random.default_rng(1).normal(size=(H, 3)).astype(np.float32)
    e.set_u_prev(u)
    e.step(np.array([0, 0, 1, 0, 0, 0.0]), np.zeros((1, K, H, 3), np.float32))
    assert np.array_equal(e.get_u_prev()[0], u)


def test_nan_cost_propagates_like_reference():
    """A NaN sample makes rho NaN in torch (S.min()) and the update NaN; the
    engine flags it (stats.nonfinite) and propagates NaN the same way."""
    K, H = 128, 20
    noise = np.zeros((1, K, H, 3), np.float32)
    noise[0, 5, 3, 1] = np.nan
    e = _engine(model="drone", n_samples=K, n_horizon=H, noise="injected")
    e.set_target([1.0, 2.0, 3.4])
    out, u0, st = e.step(np.array([0, 0, 1, 0, 0, 0.0]), noise)
    assert st[0].nonfinite
    assert np.isnan(e.get_u_prev()).all()


# ---------------------------------------------------------------- drop-in classes
def test_dropin_arm_class_reference_call_pattern():
    """kinova.py:116/182 call pattern with JointState-layout payloads
    (controller.cpp:305-333): update_joint(q(14), v(13)) -> (qdes, vdes)."""
    from quadrotor_manipulator_mppi_amd.mppi_solver.mppi import MPPI
    g = load_golden("arm_k100_h32_f64.npz")
    m = MPPI()
    m.update_joint(g["q_full"], g["v_full"])
    qdes, vdes = m.compute_control_input(noise=g["s0_noise"])
    assert isinstance(qdes, np.ndarray) and qdes.shape == (7,) and qdes.dtype == np.float64
    assert isinstance(vdes, np.ndarray) and vdes.shape == (7,) and vdes.dtype == np.float64
    _close(qdes, g["s0_qdes"], atol=1e-7, what="qdes")
    assert m.u_prev.shape == (32, 7)
    # production mode (device noise) keeps running and stays finite
    for _ in range(3):
        q, v = m.compute_control_input()
        assert np.isfinite(q).all() and np.isfinite(v).all()


def test_dropin_target_changes_reach_the_engine():
    """The drop-ins write the target into the engine only when it changed (mppi.py
    _sync_target, drone_mppi.py): a tensor modified in place, a tensor or Pose field
    reassigned, and a drone target list edited in place must each reach the next call."""
    from quadrotor_manipulator_mppi_amd.mppi_solver.mppi import MPPI
    from quadrotor_manipulator_mppi_amd.mppi_solver.drone_mppi import MPPI as DroneMPPI
    g = load_golden("arm_k100_h32_f64.npz")
    n = g["s0_noise"]
    a, b, c = MPPI(verbose=False), MPPI(verbose=False), MPPI(verbose=False)
    for m in (a, b, c):
        m.update_joint(g["q_full"], g["v_full"])
        m.compute_control_input(noise=n)
    a.target_pose.pose[0] += 0.05                                   # in place
    b.target_pose.pose = b.target_pose.pose + torch.tensor([0.05, 0.0, 0.0])   # reassigned
    qa, _ = a.compute_control_input(noise=n)
    qb, _ = b.compute_control_input(noise=n)
    qc, _ = c.compute_control_input(noise=n)                        # target unchanged
    np.testing.assert_array_equal(qa, qb)
    assert not np.array_equal(qa, qc)
    a.target_pose.orientation = torch.tensor([0.0, 0.0, 0.0, 1.0])  # reassigned
    b.target_pose.orientation[:] = torch.tensor([0.0, 0.0, 0.0, 1.0])   # in place
    np.testing.assert_array_equal(a.compute_control_input(noise=n)[0], b.compute_control_input(noise=n)[0])

    gd = load_golden("drone_k128_h20.npz")
    d1, d2 = DroneMPPI(n_samples=128, n_timestep=20), DroneMPPI(n_samples=128, n_timestep=20)
    for m in (d1, d2):
        m.verbose = False
        m.set_state(gd["s0_x_in"].tolist(), gd["s0_v_in"].tolist())
        m.compute_control_input(noise=gd["s0_noise"])
    d1.target[0] = 1.5                                              # list edited in place
    d2.target = [1.5, 2.0, 3.4]                                     # reassigned
    x1, _ = d1.compute_control_input(noise=gd["s1_noise"])
    x2, _ = d2.compute_control_input(noise=gd["s1_noise"])
    np.testing.assert_array_equal(x1.cpu().numpy(), x2.cpu().numpy())


def test_dropin_drone_class_reference_call_pattern():
    from quadrotor_manipulator_mppi_amd.mppi_solver.drone_mppi import MPPI
    g = load_golden("drone_k128_h20.npz")
    m = MPPI(n_samples=128, n_timestep=20)
    held = []
    for s in range(3):
        m.u_prev = torch.from_numpy(g[f"s{s}_u_prev_in"])
        m.set_state(g[f"s{s}_x_in"].tolist(), g[f"s{s}_v_in"].tolist())
        x, v = m.compute_control_input(noise=g[f"s{s}_noise"])
        assert isinstance(x, torch.Tensor) and x.shape == (3,) and x.device.type == "cuda"
        _close(x.cpu().numpy(), g[f"s{s}_x_out"], atol=1e-6, what="x")
        _close(v.cpu().numpy(), g[f"s{s}_v_out"], atol=1e-5, what="v")
        assert isinstance(x.to("cpu").tolist(), list)   # drone.py:240
        held.append((x, v))
    for _ in range(20):   # more calls than the staging ring is deep (one async H2D copy per call)
        m.compute_control_input()
    for s, (x, v) in enumerate(held):   # a returned tensor is the caller's: never overwritten later
        _close(x.cpu().numpy(), g[f"s{s}_x_out"], atol=1e-6, what="held x")
        _close(v.cpu().numpy(), g[f"s{s}_v_out"], atol=1e-5, what="held v")


# ------------------------------------------------------- multi-rank (gloo, 1 GPU)
def _sharded_rank(rank, world, port, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quadrotor_manipulator_mppi_amd.distributed import ShardedEngine
        se = ShardedEngine(model="arm", n_samples=1024, n_horizon=32, seed=77)
        se.engine.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
        state = np.array([0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7, np.float64)
        outs = []
        for _ in range(3):
            out, u0, st = se.step(state)
            outs.append(u0.copy())
        for _ in range(20):   # back-to-back, no host sync between steps
            se.step_async()
        out, u0, st = se.engine.read_outputs()
        outs.append(u0.copy())
        q.put((rank, np.stack(outs)))
    finally:
        dist.destroy_process_group()


def test_sharded_engine_two_ranks_gloo():
    """ShardedEngine end to end with 2 ranks (gloo collective on one GPU): every
    rank finalises the same u0 as one engine over all 2K samples, step after step."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sharded_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(res[0][1], res[1][1]), "ranks finalise identically"
    full = _engine(model="arm", n_samples=2048, n_horizon=32, seed=77)
    full.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    state = np.array([0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7, np.float64)
    ref = [full.step(state)[1] for _ in range(3)]
    full.run_steps(20)
    ref.append(full.read_outputs()[1])
    assert np.isfinite(res[0][1]).all()
    _close(res[0][1][:3], np.stack(ref[:3]), rtol=1e-4, atol=1e-6, what="sharded u0 vs single engine")
    # 20 more closed-loop steps: the two combine orders' fp32 rounding feeds back
    # through u_prev, so the bar is the drift of the loop, not one step's rounding
    _close(res[0][1][3], ref[3], rtol=5e-3, atol=1e-4, what="after 23 steps")


# ------------------------------------------- integrator lane maps (LDS transposition)
@pytest.mark.parametrize("H,f64", [(16, True), (32, False), (48, True), (64, False), (64, True)])
def test_arm_horizons_match_oracle(H, f64):
    """The transposed integrator's lane maps (L = 32: 2 rollouts x 7 dims x 4 chunks of 8;
    L = 64: 7 dims x 8 chunks of 8) with nonzero joint rates, fp32 and fp64 state."""
    from quadrotor_manipulator_mppi_amd.robot.urdf_chain import load_chain
    chain = [O.Joint(j["name"], j["type"], j["xyz"], j["rpy"], j["axis"], j["q_index"]) for j in load_chain()]
    K = 512
    torch.manual_seed(100 + H)
    noise = O.draw_noise(K, H, torch.eye(7) * 0.1)
    u_prev = torch.randn(H, 7) * 0.3
    q_full = np.array([0.1, -0.2, 1.1, 0.0, 0.0, 0.2588190, 0.9659258] + [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0])
    v_full = np.array([0.0] * 6 + [0.8, -0.5, 0.3, -1.2, 0.4, 0.9, -0.7])
    r = O.arm_step(chain, q_full, v_full, u_prev, noise, [0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5],
                   f64=f64)
    e = _engine(model="arm", n_samples=K, n_horizon=H, noise="injected", state_f64=f64)
    e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    e.set_u_prev(u_prev.numpy())
    e.step(np.concatenate([q_full[:7], q_full[7:], v_full[6:]]), noise.numpy()[None])
    tr = e.get_trajectory()[0]
    _close(tr[..., :7], r["q_samples"].numpy(), atol=2e-6, what="q")
    _close(tr[..., 7:], r["ee"].numpy().reshape(K, H, 16), atol=2e-5, what="EE")
    _close(e.get_costs()[0], r["S"].numpy(), rtol=2e-5, what="S")


@pytest.mark.parametrize("H", [16, 32, 64])
def test_wholebody_integrator_lane_maps(H):
    """Whole-body positions (drone xyz + 7 joints) against the oracle integrator, incl.
    L = 32 with 2 rollouts x 10 dims x 2 chunks of 16 per wave."""
    K = 256
    torch.manual_seed(200 + H)
    sigma = torch.diag(torch.tensor([30.0] * 3 + [0.1] * 7))
    noise = O.draw_noise(K, H, sigma)
    u_prev = torch.randn(H, 10) * 0.3
    x, vx = [0.3, -0.1, 1.2], [0.5, -0.4, 0.2]
    q, qd = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0], [0.8, -0.5, 0.3, -1.2, 0.4, 0.9, -0.7]
    ref = O.integrate(u_prev.unsqueeze(0) + noise, torch.tensor(x + q, dtype=torch.float32),
                      torch.tensor(vx + qd, dtype=torch.float32), 0.01)
    e = _engine(model="wholebody", n_samples=K, n_horizon=H, noise="injected", sigma=sigma.numpy())
    e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    e.set_u_prev(u_prev.numpy())
    state = np.array(x + [0.0, 0.0, 0.0, 1.0] + q + vx + qd, np.float64)
    e.step(state, noise.numpy()[None])
    pos = e.get_trajectory()[0][..., :10]
    assert np.isfinite(pos).all()
    _close(pos, ref.numpy(), atol=2e-5, rtol=2e-6, what="positions")


def test_trajectory_above_4gib_rejected_at_create():
    """The rollout kernels address one vehicle's trajectory planes through a buffer
    resource (32-bit offsets): a larger trajectory is refused before any allocation."""
    from quadrotor_manipulator_mppi_amd import _capi as capi
    with pytest.raises(capi.MPPIError, match="4 GiB"):
        _engine(model="wholebody", n_samples=1 << 20, n_horizon=256)
    e = _engine(model="wholebody", n_samples=1 << 20, n_horizon=256, store_trajectory=False)
    e.close()


def test_trajectory_between_2_and_4_gib():
    """One vehicle's trajectory planes above 2 GiB (arm K=2^20 H=32: 19 planes x 128 MiB
    = 2.4 GiB): the buffer-resource byte offsets past 2^31 (negative as the builtin's int)
    address the upper planes.  The first and last samples' stored joint positions equal the
    integration of their stored noise and their EE the oracle FK."""
    from quadrotor_manipulator_mppi_amd.robot.urdf_chain import load_chain
    chain = [O.Joint(j["name"], j["type"], j["xyz"], j["rpy"], j["axis"], j["q_index"]) for j in load_chain()]
    K, H = 1 << 20, 32
    q0 = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]
    base = [0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0]
    e = _engine(model="arm", n_samples=K, n_horizon=H, store_noise=True, seed=11, state_f64=False)
    e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    e.step(np.array(base + q0 + [0.0] * 7, np.float64))
    ks = np.r_[0:4, K - 4:K]
    eps = e.get_noise()[0][ks]
    tr = e.get_trajectory()[0][ks]
    e.close()
    q = O.integrate(torch.from_numpy(eps), torch.tensor(q0), torch.zeros(7), 0.01)
    _close(tr[..., :7], q.numpy(), atol=2e-6, what="q (K=2^20)")
    ee = O.ee_world(chain, q, torch.tensor(base))
    _close(tr[..., 7:], ee.numpy().reshape(len(ks), H, 16), atol=2e-5, what="EE (K=2^20)")
