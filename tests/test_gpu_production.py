"""Production mode against the oracle at the full BASELINE sizes (C2 drone K=4096 H=32, C3 arm
K=4096 H=32): device Philox noise, native control calls (mppi_step as AQL packets on the
engine's queue) and native batches -- the path the ROS nodes and bench.py run.  The stored
device noise of each call (``store_noise``) and the state go through the oracle's
``drone_step`` / ``arm_step`` (drone_mppi.py:140-176, mppi.py:122-169), and everything the call
produced is held to the parity tolerances of tests/test_gpu_parity.py:

* S rtol 2e-5, trajectories atol 2e-5 (drone positions) / 2e-6 (arm joint angles) / 2e-5 (EE);
* drone: the top-2 cost gap is >= 20 lambda (checked), so w, w_eps, u_prev, x and v meet the
  north star's plain 1e-4 rel;
* arm: the near-tie regime of the fixtures (gap ~ lambda): the reduction given the GPU's own
  costs at 1e-5 rel, end to end within the softmin's conditioning bound (``_amplified_bound``).

Full-size properties at C2 as at C3: sum w = 1 and w_eps = sum_k w_k eps_k of the stored noise.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import mppi_oracle as O
from test_gpu_parity import _amplified_bound, _close

pytestmark = pytest.mark.gpu

LAM = 0.1
ARM_T = ([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
DRONE_T = [1.0, 2.0, 3.4]


def _engine(**kw):
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    return Engine(make_config(device=0, **kw))


def _top2_gap(S):
    s = np.sort(np.asarray(S, np.float64))
    return float(s[1] - s[0])


def _drone_engine(seed, state):
    e = _engine(model="drone", n_samples=4096, n_horizon=32, seed=seed, store_noise=True)
    e.set_target(DRONE_T)
    e.set_state(state)
    return e


def test_c2_drone_production_matches_oracle():
    """C2 drone K=4096 H=32 in production mode: native control calls after a native batch, each
    call's stored noise through O.drone_step at the plain 1e-4 rel."""
    rng = np.random.default_rng(3)
    states = [np.array([0.1, -0.2, 1.0, 0.3, 0.0, -0.1]) + np.r_[rng.normal(0, 0.05, 3), [0.0] * 3]
              for _ in range(3)]
    # a seed whose calls all have top-2 gap >= 20 lambda (the plain-tolerance regime; the GPU's S
    # equals the oracle's within 2e-5 rel, checked below, so its gap stands for the oracle's)
    chosen = None
    for seed in range(1, 40):
        e = _drone_engine(seed, states[0])
        e.run_steps(20)
        gaps = []
        for st in states:
            e.step(st)
            gaps.append(_top2_gap(e.get_costs()[0]))
        e.close()
        if min(gaps) >= 40 * LAM:
            chosen = seed
            break
    assert chosen is not None, "no seed with a top-2 gap >= 40 lambda in 39 tries"
    e = _drone_engine(chosen, states[0])
    e.run_steps(20)   # native batch first: the calls continue its u_prev and step counter
    e.synchronize()
    assert e.dispatch_info().startswith("aql;"), e.dispatch_info()
    for i, st in enumerate(states):
        u_in = e.get_u_prev()[0]
        out, u0, sts = e.step(st)
        assert "calls: aql" in e.dispatch_info(), e.dispatch_info()
        eps = e.get_noise()[0]
        r = O.drone_step(st[:3], st[3:], torch.from_numpy(u_in), torch.from_numpy(eps), DRONE_T)
        S = e.get_costs()[0]
        _close(S, r["S"].numpy(), rtol=2e-5, what=f"call {i}: S")
        assert _top2_gap(r["S"].numpy()) >= 20 * LAM
        _close(e.get_trajectory()[0], r["traj"].numpy(), atol=2e-5, what=f"call {i}: traj")
        w = e.get_weights()[0]
        _close(w, r["w"].numpy(), rtol=1e-4, atol=1e-12, what=f"call {i}: w")
        raw, sm = e.get_weighted_noise()
        _close(raw[0], r["w_eps_raw"].numpy(), rtol=1e-4, atol=1e-5, what=f"call {i}: w_eps raw")
        _close(sm[0], r["w_eps"].numpy(), rtol=1e-4, atol=1e-5, what=f"call {i}: w_eps savgol")
        _close(e.get_u_prev()[0], r["u_prev_out"].numpy(), rtol=1e-4, atol=1e-5, what=f"call {i}: u_prev")
        _close(out[0, :3], r["x_out"].numpy(), rtol=1e-6, atol=1e-6, what=f"call {i}: x")
        _close(out[0, 3:], r["v_out"].numpy(), rtol=1e-5, atol=1e-6, what=f"call {i}: v")
        # full-size properties (C2): normalised weights, w_eps = sum_k w_k eps_k of the stored noise
        w64 = w.astype(np.float64)
        assert abs(w64.sum() - 1.0) < 1e-4
        _close(raw[0], np.einsum("k,kha->ha", w64, eps), rtol=1e-4, atol=1e-6, what=f"call {i}: w_eps = sum w eps")
        assert not sts[0].nonfinite and sts[0].ess >= 1.0
    e.close()


def _rel(got, exact):
    """Norm-wise relative error: max |got - exact| / max |exact|."""
    got, exact = np.asarray(got, np.float64), np.asarray(exact, np.float64)
    return float(np.abs(got - exact).max() / max(np.abs(exact).max(), 1e-300))


def _against_exact(chain, q_full, v_full, u_in, eps, r, S, raw, sm, u_prev, out, i, traj=None, records=None):
    """One arm call against the exact answer (the whole step in float64, ``O.float64_everywhere``, on
    the same noise), next to the reference arithmetic's own error (oracle fp32, ``r``).

    * S (not amplified): what the softmin sees is S up to a constant (mppi.py:184-188: S - min S), so
      the error that matters is the per-sample error about its mean over the K samples; its RMS for
      the GPU is at most twice the reference arithmetic's (fp32 rounding, LU inverse, fp64-promoted
      FK).  The plain RMS (a common shift included) is recorded too;
    * w_eps, u_prev (amplified by 1/lambda at near ties): within the softmin's conditioning bound
      computed from the GPU's OWN distance to the exact S -- the reduction adds nothing beyond what
      the S error implies; the errors and the reference's are recorded side by side (at a near tie
      their ratio is the luck of which samples' S errors lead the weights, either way).
    The record (relative errors: max |x - exact| / max |exact|) is appended to ``records`` before
    any assertion, so a failing call still leaves its numbers."""
    with O.float64_everywhere():
        ex = O.arm_step(chain, q_full, v_full, torch.from_numpy(u_in).double(), torch.from_numpy(eps).double(),
                        *ARM_T, f64=True)
    S_ex = ex["S"].numpy()
    dS_g, dS_r = S.astype(np.float64) - S_ex, r["S"].numpy().astype(np.float64) - S_ex
    rms = lambda x: float(np.sqrt(np.mean(x ** 2)))   # noqa: E731
    cg, cr = rms(dS_g - dS_g.mean()), rms(dS_r - dS_r.mean())
    rec = {"call": i, "top2_gap_exact": _top2_gap(S_ex), "top2_gap_over_lambda": _top2_gap(S_ex) / LAM,
           "S_centered_rms_err": {"gpu": cg, "reference_fp32": cr, "ratio": cg / cr},
           "S_rms_err": {"gpu": rms(dS_g), "reference_fp32": rms(dS_r), "ratio": rms(dS_g) / rms(dS_r)},
           "S_mean_err": {"gpu": float(dS_g.mean()), "reference_fp32": float(dS_r.mean())}}
    if traj is not None:   # where the S error comes from: joint angles, EE position, EE rotation
        K, H = S.shape[0], traj.shape[1]
        ee_x, ee_r = ex["ee"].numpy().reshape(K, H, 4, 4), r["ee"].numpy().reshape(K, H, 4, 4)
        ee_g = traj[..., 7:].reshape(K, H, 4, 4)
        q_x = ex["q_samples"].numpy()
        rec["q_rms_err"] = {"gpu": rms(traj[..., :7] - q_x), "reference_fp32": rms(r["q_samples"].numpy() - q_x)}
        rec["ee_pos_rms_err"] = {"gpu": rms(ee_g[..., :3, 3] - ee_x[..., :3, 3]),
                                 "reference_fp32": rms(ee_r[..., :3, 3] - ee_x[..., :3, 3])}
        rec["ee_rot_rms_err"] = {"gpu": rms(ee_g[..., :3, :3] - ee_x[..., :3, :3]),
                                 "reference_fp32": rms(ee_r[..., :3, :3] - ee_x[..., :3, :3])}
    w_ex = ex["w"].numpy().astype(np.float64)
    bound = _amplified_bound(float(np.abs(dS_g - dS_g.mean()).max()), w_ex, eps, LAM)
    rec["conditioning_bound_over_w_eps"] = float(bound.max() / np.abs(ex["w_eps_raw"].numpy()).max())
    pairs = {"S": (S, r["S"].numpy(), S_ex),
             "w_eps_raw": (raw, r["w_eps_raw"].numpy(), ex["w_eps_raw"].numpy()),
             "w_eps": (sm, r["w_eps"].numpy(), ex["w_eps"].numpy()),
             "u_prev": (u_prev, r["u_prev_out"].numpy(), ex["u_prev_out"].numpy()),
             "qdes": (out[:7], r["qdes"], ex["qdes"]), "vdes": (out[7:], r["vdes"], ex["vdes"])}
    for name, (gpu, ref32, exact) in pairs.items():
        rec[name] = {"gpu_rel_err": _rel(gpu, exact), "reference_fp32_rel_err": _rel(ref32, exact)}
    if records is not None:
        records.append(rec)
    assert cg <= 2.0 * cr, f"call {i}: S centered rms error GPU {cg:.3e} vs reference fp32 {cr:.3e}"
    assert np.all(np.abs(raw - ex["w_eps_raw"].numpy()) <= bound), f"call {i}: w_eps beyond the GPU's own bound"
    sm_bound = np.abs(O.savgol(torch.from_numpy(bound.astype(np.float32)), 9, 2).numpy()) + 4 * bound.max()
    assert np.all(np.abs(sm - ex["w_eps"].numpy()) <= sm_bound), f"call {i}: savgol beyond the GPU's own bound"
    assert np.all(np.abs(u_prev - ex["u_prev_out"].numpy()) <= sm_bound + 1e-6), f"call {i}: u_prev"
    return rec


def _dump(name, records, summary=None):
    out_path = os.environ.get("MPPI_ACCURACY_OUT")
    if out_path:
        with open(out_path.replace(".json", f"_{name}.json"), "w") as f:
            json.dump({"test": name, "summary": summary, "calls": records}, f, indent=1)


def test_c3_arm_production_matches_oracle():
    """C3 arm K=4096 H=32, fp64 state as the kinova node feeds it, in production mode: native
    control calls after a native batch; each call's stored noise through O.arm_step.

    Accuracy against the exact answer: the reference's own fp32 S is not
    reproducible bit for bit (LU ``inv`` at pose_cost.py:32, fp64 promotion at
    transformation_matrix.py:68-93), and near ties (gap ~ lambda) amplify any S rounding by 1/lambda
    (mppi.py:184-191).  So every call also runs the oracle with the WHOLE step in float64
    (``O.float64_everywhere``) on the same stored noise as the stand-in for the exact answer
    (``_against_exact``).  The achieved errors and the conditioning bound's size relative to |w_eps|
    go to $MPPI_ACCURACY_OUT when set."""
    from quadrotor_manipulator_mppi_amd.robot.urdf_chain import load_chain
    chain = [O.Joint(j["name"], j["type"], j["xyz"], j["rpy"], j["axis"], j["q_index"]) for j in load_chain()]
    e = _engine(model="arm", n_samples=4096, n_horizon=32, seed=17, store_noise=True)
    e.set_target(*ARM_T)
    base = np.array([0.1, -0.2, 1.1, 0.0, 0.0, 0.2588190, 0.9659258] + [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]
                    + [0.2, -0.1, 0.05, 0.0, 0.02, 0.0, -0.03])
    e.set_state(base)
    e.run_steps(20)
    e.synchronize()
    assert e.dispatch_info().startswith("aql;"), e.dispatch_info()
    rng = np.random.default_rng(11)
    records = []
    for i in range(3):
        st = base.copy()
        st[7:14] += rng.normal(0, 0.02, 7)
        u_in = e.get_u_prev()[0]
        out, u0, sts = e.step(st)
        assert "calls: aql" in e.dispatch_info(), e.dispatch_info()
        eps = e.get_noise()[0]
        q_full, v_full = st[:14], np.r_[[0.0] * 6, st[14:]]
        r = O.arm_step(chain, q_full, v_full, torch.from_numpy(u_in), torch.from_numpy(eps), *ARM_T, f64=True)
        tr = e.get_trajectory()[0]
        _close(tr[..., :7], r["q_samples"].numpy(), atol=2e-6, what=f"call {i}: q_samples")
        _close(tr[..., 7:], r["ee"].numpy().reshape(4096, 32, 16), atol=2e-5, what=f"call {i}: EE")
        S, S_ref = e.get_costs()[0], r["S"].numpy()
        _close(S, S_ref, rtol=2e-5, what=f"call {i}: S")
        # (a) the reduction given the GPU's own costs
        w_own = O.softmin(torch.from_numpy(S), LAM).numpy()
        raw, sm = e.get_weighted_noise()
        w = e.get_weights()[0]
        _close(w, w_own, rtol=1e-5, atol=1e-9, what=f"call {i}: w | S_gpu")
        _close(raw[0], np.einsum("k,kha->ha", w_own.astype(np.float64), eps), rtol=1e-5, atol=1e-7,
               what=f"call {i}: w_eps | S_gpu")
        # (b) end to end within the softmin's conditioning (near ties: gap ~ lambda)
        w_ref = r["w"].numpy().astype(np.float64)
        dS = float(np.max(np.abs(S.astype(np.float64) - S_ref)))
        bound = _amplified_bound(dS, w_ref, eps, LAM)
        assert np.all(np.abs(raw[0] - r["w_eps_raw"].numpy()) <= bound), f"call {i}: w_eps beyond conditioning bound"
        sm_bound = np.abs(O.savgol(torch.from_numpy(bound.astype(np.float32)), 9, 2).numpy()) + 4 * bound.max()
        assert np.all(np.abs(sm[0] - r["w_eps"].numpy()) <= sm_bound), f"call {i}: savgol"
        u_ref = r["u_prev_out"].numpy()
        _close(e.get_u_prev()[0], u_ref, atol=float(sm_bound.max()) + 1e-6, what=f"call {i}: u_prev")
        u0_tol = float(np.abs(u0[0] - u_ref[0]).max()) + 1e-7
        _close(out[0, 7:], r["vdes"], atol=u0_tol * 0.01 + 1e-7, what=f"call {i}: vdes")
        _close(out[0, :7], r["qdes"], atol=u0_tol * 1e-4 + 1e-7, what=f"call {i}: qdes")
        assert sts[0].reach == r["reach"]
        assert abs(w.astype(np.float64).sum() - 1.0) < 1e-4
        assert not sts[0].nonfinite
        # (c) against the exact answer: the whole step in float64 on the same noise
        try:
            _against_exact(chain, q_full, v_full, u_in, eps, r, S, raw[0], sm[0], e.get_u_prev()[0], out[0], i,
                           traj=tr, records=records)
        finally:
            _dump("production", records)
    e.close()


def test_c3_arm_accuracy_sweep_against_exact():
    """The same statement over 8 independent C3 calls (engine seeds 101..108, device Philox noise,
    fp64 state): per call, the GPU's S within twice the reference arithmetic's RMS error against the
    exact answer and w_eps / u_prev within the conditioning bound of the GPU's own S error
    (``_against_exact``); over the calls, the median ratio of the GPU's to the reference's w_eps
    error is recorded with the top-2 gaps ($MPPI_ACCURACY_OUT, ``_sweep`` suffix)."""
    from quadrotor_manipulator_mppi_amd.robot.urdf_chain import load_chain
    chain = [O.Joint(j["name"], j["type"], j["xyz"], j["rpy"], j["axis"], j["q_index"]) for j in load_chain()]
    st = np.array([0.1, -0.2, 1.1, 0.0, 0.0, 0.2588190, 0.9659258] + [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]
                  + [0.2, -0.1, 0.05, 0.0, 0.02, 0.0, -0.03])
    q_full, v_full = st[:14], np.r_[[0.0] * 6, st[14:]]
    records = []
    for seed in range(101, 109):
        e = _engine(model="arm", n_samples=4096, n_horizon=32, seed=seed, store_noise=True)
        e.set_target(*ARM_T)
        u_in = e.get_u_prev()[0]
        out, u0, sts = e.step(st)
        eps = e.get_noise()[0]
        r = O.arm_step(chain, q_full, v_full, torch.from_numpy(u_in), torch.from_numpy(eps), *ARM_T, f64=True)
        raw, sm = e.get_weighted_noise()
        tr = e.get_trajectory()[0]
        try:
            _against_exact(chain, q_full, v_full, u_in, eps, r, e.get_costs()[0], raw[0], sm[0], e.get_u_prev()[0],
                           out[0], seed, traj=tr, records=records)
        finally:
            e.close()
            ratios = [x["w_eps_raw"]["gpu_rel_err"] / max(x["w_eps_raw"]["reference_fp32_rel_err"], 1e-300)
                      for x in records]
            summary = {"median_w_eps_err_ratio_gpu_over_reference": float(np.median(ratios)),
                       "median_S_centered_rms_ratio": float(np.median([x["S_centered_rms_err"]["ratio"]
                                                                       for x in records])),
                       "calls_w_eps_gpu_within_1e-4": int(sum(x["w_eps_raw"]["gpu_rel_err"] <= 1e-4 for x in records)),
                       "calls_w_eps_reference_within_1e-4": int(sum(x["w_eps_raw"]["reference_fp32_rel_err"] <= 1e-4
                                                                    for x in records))}
            _dump("sweep", records, summary)
