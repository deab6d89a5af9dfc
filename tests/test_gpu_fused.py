"""The fused step (mppi_rollout.h fused_tail): k_rollout folds its block records and finalises the
control step itself -- one launch per step instead of k_rollout + k_finalize.  Same math as the
two-kernel step (mppi.py:144-158: the softmin-weighted noise, svg_filter.py's SavGol, u += w_eps and
the outputs); only the order of the softmin fold differs (records folded in groups of ~sqrt(nb), then
the groups, instead of k_finalize's per-lane chunks), so:

* costs S (the rollout itself) bit-identical to the two-kernel engine (MPPI_FUSED=0);
* u_prev, u0 and the outputs within fp32 rounding of the fold order: rtol 1e-5 (the north star's
  1e-4 with margin), stats rho exact (a min), eta / ess rtol 1e-5;
* native batches and native control calls bit-identical to the fused HIP launches (same kernel);
* a ragged K (groups of unequal size, nb not a power of two) and a one-block grid;
* the arrival counters are back to zero after every step (a batch of 500 steps stays right).
Parity against the reference oracle runs through every other GPU test: engines fuse by default.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HOME_Q = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]                 # kinova.py:135
ARM_TARGET = ([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])   # mppi.py:71-72
STATES = {"arm": [0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0] + HOME_Q + [0.0] * 7,
          "drone": [0.0, 0.0, 1.0, 0.0, 0.0, 0.0],
          "wholebody": [0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0] + HOME_Q + [0.0] * 10}


def _close(got, want, rtol, atol, what):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    err = np.abs(got - want)
    bad = err > atol + rtol * np.abs(want)
    assert not bad.any(), f"{what}: {bad.sum()} / {bad.size} off, max err {err.max():.3e}"


def _pair(monkeypatch, model, V=1, dispatch=None, **kw):
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    if dispatch:
        monkeypatch.setenv("MPPI_DISPATCH", dispatch)
    out = []
    for fused in (False, True):
        if fused:
            monkeypatch.delenv("MPPI_FUSED", raising=False)
        else:
            monkeypatch.setenv("MPPI_FUSED", "0")
        e = Engine(make_config(model=model, n_vehicles=V, seed=11, **kw))
        for v in range(V):
            if model == "drone":
                e.set_target([1.0, 2.0, 3.4], vehicle=v)
            else:
                e.set_target(np.array(ARM_TARGET[0]) + 0.02 * v, ARM_TARGET[1], vehicle=v)
        st = np.tile(np.array(STATES[model], np.float64), (V, 1))
        st[:, 0] += 0.05 * np.arange(V)
        e.set_state(st)
        out.append(e)
    monkeypatch.delenv("MPPI_FUSED", raising=False)
    two, one = out
    info = one.dispatch_info()
    assert "step: fused" in info and "step: rollout + finalize" in two.dispatch_info(), info
    return two, one, st


CASES = [
    ("arm", 1, dict(n_samples=4096, n_horizon=32, state_f64=True)),           # C3 (the metric's shape)
    ("drone", 1, dict(n_samples=4096, n_horizon=32)),                         # C2
    ("wholebody", 1, dict(n_samples=8192, n_horizon=64)),                     # the C4 rank's shard
    ("wholebody", 4, dict(n_samples=2048, n_horizon=64)),                     # a fleet (V > 1)
    ("arm", 1, dict(n_samples=2999, n_horizon=48, state_f64=False)),          # ragged K, H = 48
    ("drone", 1, dict(n_samples=48, n_horizon=20)),                           # one block (C1-sized)
]


@pytest.mark.parametrize("model,V,kw", CASES, ids=[f"{m}-V{v}-K{k['n_samples']}-H{k['n_horizon']}" for m, v, k in CASES])
def test_fused_step_matches_two_kernel_step(model, V, kw, monkeypatch):
    two, one, st = _pair(monkeypatch, model, V, **kw)
    try:
        for e in (two, one):   # a native batch, then control calls with a moving state
            e.run_steps(25)
            e.synchronize()
        assert np.array_equal(one.get_costs(), two.get_costs()), "costs (the rollout) bit-identical"
        _close(one.get_u_prev(), two.get_u_prev(), 1e-5, 1e-7, "u_prev after a batch")
        rng = np.random.default_rng(3)
        for i in range(4):
            s = st.copy()
            s[:, :3] += rng.normal(0, 0.01, (V, 3))
            o2, u2, s2 = two.step(s)
            o1, u1, s1 = one.step(s)
            _close(u1, u2, 1e-5, 1e-7, f"call {i}: u0")
            _close(o1, o2, 1e-6, 1e-9, f"call {i}: outputs")
            for a, b in zip(s1, s2):
                assert a.rho == b.rho and not a.nonfinite and not b.nonfinite
                _close(a.eta, b.eta, 1e-5, 0.0, "eta")
                _close(a.ess, b.ess, 1e-4, 0.0, "ess")
        _close(one.get_u_prev(), two.get_u_prev(), 1e-5, 1e-7, "u_prev after the calls")
        w1, w2 = one.get_weights(), two.get_weights()
        _close(w1, w2, 1e-5, 1e-9, "weights")
        r1, m1 = one.get_weighted_noise()
        r2, m2 = two.get_weighted_noise()
        _close(r1, r2, 1e-5, 1e-7, "w_eps readback")
    finally:
        one.close()
        two.close()


def test_fused_native_equals_hip_launches(monkeypatch):
    """The same fused kernel through native packets (one per step) and through HIP launches:
    bit-identical u_prev, costs and outputs, batches and calls (dispatch-id step counting with
    one packet per step)."""
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    es = {}
    for d in ("aql", "hip"):
        monkeypatch.setenv("MPPI_DISPATCH", d)
        e = Engine(make_config(model="arm", n_samples=4096, n_horizon=32, state_f64=True, seed=5))
        e.set_target(*ARM_TARGET)
        e.set_state(np.array(STATES["arm"]))
        es[d] = e
    try:
        for e in es.values():
            e.run_steps(40)
            e.synchronize()
        assert es["aql"].dispatch_info().startswith("aql;"), es["aql"].dispatch_info()
        assert np.array_equal(es["aql"].get_u_prev(), es["hip"].get_u_prev())
        assert np.array_equal(es["aql"].get_costs(), es["hip"].get_costs())
        for i in range(20):
            s = np.array(STATES["arm"])
            s[7:14] += 0.003 * i
            oa, ua, _ = es["aql"].step(s)
            oh, uh, _ = es["hip"].step(s)
            assert np.array_equal(oa, oh) and np.array_equal(ua, uh), f"call {i}"
        assert "calls: aql" in es["aql"].dispatch_info()
        for e in es.values():   # a long batch: every arrival counter must return to zero each step
            e.run_steps(500)
            e.synchronize()
        assert np.array_equal(es["aql"].get_u_prev(), es["hip"].get_u_prev())
        assert np.isfinite(es["aql"].get_u_prev()).all()
    finally:
        for e in es.values():
            e.close()
