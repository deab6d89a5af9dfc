"""The fused step (k_rollout FUSE, mppi_rollout.h fused_tail): one launch per control step whose
last-arriving blocks fold the block records and finalise -- or pack a shard's exchange slot -- in
the same launch, instead of a k_finalize launch after the rollout.  Every case runs the same
seeded steps on a fused engine (MPPI_FUSED=1) and on a two-kernel engine (MPPI_FUSED=0):

* the per-rollout costs are bit-identical (a cost never depends on who folds the records);
* u_prev, u0 and the outputs agree to fp32 reordering of the fold (the fused tail folds 8 rows
  per lane in 512-thread blocks, k_finalize 16 in 128-512: the same sums in another order);
* through native batches and calls, through HIP launches, and for the shard's fused pack.
The oracle comparisons of tests/test_gpu_parity.py and tests/test_gpu_production.py run on the
engines' default step (mppi_capi.cpp kFuseDefault)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HOME = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]


def _state(model, V=1, shift=0.0):
    s = {"arm": [0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 7, "drone": [0.0, 0.0, 1.0, 0.0, 0.0, 0.0],
         "wholebody": [0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 10}[model]
    s = np.tile(np.array(s, np.float64), (V, 1))
    s[:, 0] += shift
    return s


def _engines(monkeypatch, model, dispatch="auto", **kw):
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    out = []
    for fused in (False, True):
        monkeypatch.setenv("MPPI_DISPATCH", dispatch)
        monkeypatch.setenv("MPPI_FUSED", "1" if fused else "0")
        e = Engine(make_config(model, device=0, seed=13, **kw))
        for v in range(e.V):
            if model == "drone":
                e.set_target([1.0, 2.0, 3.4], vehicle=v)
            else:
                e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5], vehicle=v)
        e.set_state(_state(model, e.V))
        out.append(e)
    monkeypatch.delenv("MPPI_FUSED", raising=False)
    monkeypatch.delenv("MPPI_DISPATCH", raising=False)
    return out


def _agree(two, fused, what):
    two.synchronize()
    fused.synchronize()
    assert "step: fused" in fused.dispatch_info(), fused.dispatch_info()
    assert "step: two kernels: MPPI_FUSED=0" in two.dispatch_info(), two.dispatch_info()
    np.testing.assert_array_equal(fused.get_costs(), two.get_costs(), err_msg=what + ": costs")
    np.testing.assert_allclose(fused.get_u_prev(), two.get_u_prev(), rtol=1e-5, atol=1e-7, err_msg=what + ": u_prev")
    o2, u2, s2 = two.read_outputs()
    of, uf, sf = fused.read_outputs()
    np.testing.assert_allclose(of, o2, rtol=1e-6, atol=1e-9, err_msg=what + ": outputs")
    np.testing.assert_allclose(uf, u2, rtol=1e-5, atol=1e-7, err_msg=what + ": u0")
    for a, b in zip(sf, s2):
        assert a.rho == b.rho and abs(a.eta - b.eta) <= 1e-5 * b.eta and a.nonfinite == b.nonfinite, what


CASES = [("arm", dict(n_samples=4096, n_horizon=32)),                  # C3
         ("drone", dict(n_samples=4096, n_horizon=32)),                # C2
         ("wholebody", dict(n_samples=8192, n_horizon=64)),            # the C4 shard shape (looping kernel)
         ("wholebody", dict(n_samples=65536, n_horizon=64)),           # more blocks than fit at once
         ("arm", dict(n_samples=512, n_horizon=32, n_vehicles=4)),     # fleet: a counter per vehicle
         ("arm", dict(n_samples=3000, n_horizon=20, state_f64=False))]  # ragged K, H = 20


@pytest.mark.parametrize("dispatch", ["aql", "hip"])
@pytest.mark.parametrize("model,kw", CASES, ids=[f"{m}-{'-'.join(f'{k}{v}' for k, v in kw.items())}" for m, kw in CASES])
def test_fused_step_matches_two_kernel_step(monkeypatch, model, kw, dispatch):
    two, fused = _engines(monkeypatch, model, dispatch, **kw)
    for e in (two, fused):
        e.run_steps(9)
    _agree(two, fused, "9 steps")
    rng = np.random.default_rng(2)
    for i in range(6):   # control calls (native on the aql engines for one vehicle), changing state
        st = _state(model, two.V, shift=float(rng.normal(0, 0.02)))
        o2, u2, _ = two.step(st)
        of, uf, _ = fused.step(st)
        np.testing.assert_allclose(of, o2, rtol=1e-6, atol=1e-9, err_msg=f"call {i}")
        np.testing.assert_allclose(uf, u2, rtol=1e-5, atol=1e-7, err_msg=f"call {i}")
    for e in (two, fused):
        e.run_steps(3000)   # many steps: the arrival counters' epochs stay in step
    _agree(two, fused, "3000 more steps")
    two.close()
    fused.close()


def test_fused_pack_one_rank_communicator(monkeypatch):
    """The shard's pack in the rollout's own launch (engine-owned RCCL communicator, one rank):
    rollout+pack -> all-reduce -> finalize equals the plain fused engine and the unfused shard."""
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    kw = dict(n_samples=8192, n_horizon=64, seed=5)
    engines = {}
    for name, env in (("plain", "1"), ("shard_fused", "1"), ("shard_two", "0")):
        monkeypatch.setenv("MPPI_FUSED", env)
        e = Engine(make_config("wholebody", device=0, **kw))
        e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
        e.set_state(_state("wholebody"))
        if name != "plain":
            e.comm_init(e.comm_unique_id())
        engines[name] = e
    monkeypatch.delenv("MPPI_FUSED", raising=False)
    for e in engines.values():
        e.run_steps(12)
        e.synchronize()
    assert "step: fused rollout+pack" in engines["shard_fused"].dispatch_info()
    ref = engines["plain"].get_u_prev()
    for name in ("shard_fused", "shard_two"):
        np.testing.assert_array_equal(engines[name].get_costs(), engines["plain"].get_costs())
        np.testing.assert_allclose(engines[name].get_u_prev(), ref, rtol=1e-4, atol=1e-6, err_msg=name)
    o1 = engines["shard_fused"].step(_state("wholebody", shift=0.01))
    o2 = engines["shard_two"].step(_state("wholebody", shift=0.01))
    np.testing.assert_allclose(o1[0], o2[0], rtol=1e-6, atol=1e-9)
    for e in engines.values():
        e.close()
