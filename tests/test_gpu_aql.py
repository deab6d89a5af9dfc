"""Native dispatch (csrc/mppi_aql.cpp): mppi_run_steps and one-vehicle mppi_step as raw AQL
packets on the engine's own HSA queue must compute exactly what the HIP launches compute --
the same kernels (loaded from the library's code objects), the same arguments (captured from
the launchers), the Philox step counter taken from the dispatch id.  Every case runs one
engine per dispatch mode on identical inputs and compares bit for bit: u_prev, the outputs,
the costs, and the control call after a batch (it must continue the batch's counter)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HOME = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]


def _state(model, V=1, shift=0.0):
    if model == "arm":
        s = [0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 7
    elif model == "drone":
        s = [0.0, 0.0, 1.0, 0.0, 0.0, 0.0]
    elif model == "quadrotor":
        s = [0.0, 0.0, 1.0, 0.0, 0.0, 0.0] + [0.0] * 6
    else:
        s = [0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 10
    s = np.tile(np.array(s, np.float64), (V, 1))
    s[:, 0] += shift
    return s


def _pair(monkeypatch, model, **kw):
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    engines = []
    for mode in ("hip", "aql"):
        monkeypatch.setenv("MPPI_DISPATCH", mode)   # read at mppi_create
        e = Engine(make_config(model, device=0, seed=11, **kw))
        for v in range(e.V):
            if model in ("drone", "quadrotor"):
                e.set_target([1.0, 2.0, 3.4], vehicle=v)
            else:
                e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5], vehicle=v)
        e.set_state(_state(model, e.V))
        engines.append(e)
    monkeypatch.delenv("MPPI_DISPATCH")
    return engines


def _same(h, a, what):
    h.synchronize()
    a.synchronize()
    assert a.dispatch_info().startswith("aql;"), a.dispatch_info()
    assert h.dispatch_info().startswith("hip"), h.dispatch_info()
    np.testing.assert_array_equal(a.get_u_prev(), h.get_u_prev(), err_msg=what + ": u_prev")
    np.testing.assert_array_equal(a.get_costs(), h.get_costs(), err_msg=what + ": costs")
    oh, uh, sh = h.read_outputs()
    oa, ua, sa = a.read_outputs()
    np.testing.assert_array_equal(oa, oh, err_msg=what + ": outputs")
    np.testing.assert_array_equal(ua, uh, err_msg=what + ": u0")
    assert [s.rho for s in sa] == [s.rho for s in sh] and [s.eta for s in sa] == [s.eta for s in sh], what


CASES = [
    ("arm", dict(n_samples=4096, n_horizon=32)),                       # C3 (fp64 state)
    ("arm", dict(n_samples=1024, n_horizon=32, state_f64=False)),
    ("arm", dict(n_samples=2048, n_horizon=100)),                      # 2 chunks per rollout
    ("arm", dict(n_samples=512, n_horizon=32, n_vehicles=4)),          # fleet (vehicle block in memory)
    ("drone", dict(n_samples=4096, n_horizon=32)),
    ("wholebody", dict(n_samples=8192, n_horizon=64)),                 # the C4 shard shape, one group per wave
    ("wholebody", dict(n_samples=32768, n_horizon=64)),                # several groups per wave
    ("wholebody", dict(n_samples=65536, n_horizon=64)),                # C4 on one GPU: more blocks than fit at once
    ("quadrotor", dict(n_samples=1024, n_horizon=32)),
    ("arm", dict(n_samples=1024, n_horizon=32, cost_terms=("covar", "center", "action"))),   # extended kernel
]


@pytest.mark.parametrize("model,kw", CASES, ids=[f"{m}-{'-'.join(f'{k}{v}' for k, v in kw.items())}" for m, kw in CASES])
def test_native_dispatch_matches_hip(monkeypatch, model, kw):
    h, a = _pair(monkeypatch, model, **kw)
    for e in (h, a):
        e.run_steps(7)
    _same(h, a, "7 steps")
    # a control call after the batch (native on the aql engine for one vehicle) continues its counter
    st = _state(model, h.V, shift=0.01)
    oh, uh, _ = h.step(st)
    oa, ua, _ = a.step(st)
    np.testing.assert_array_equal(oa, oh)
    np.testing.assert_array_equal(ua, uh)
    # and a native batch after the call, at the call's new state (argument block re-uploaded)
    for e in (h, a):
        e.run_steps(5)
    _same(h, a, "after a control call")
    h.close()
    a.close()


def test_native_counter_rewind_and_many_batches(monkeypatch):
    """set_step_counter rewinds the device counter; back-to-back batches without a sync and
    a batch longer than the queue ring (4096 packets) stay in lock step with HIP."""
    h, a = _pair(monkeypatch, "arm", n_samples=1024, n_horizon=32)
    for e in (h, a):
        e.run_steps(3)
        e.set_step_counter(5)
        e.run_steps(4)
        e.run_steps(2)   # enqueued behind the previous batch (no host sync in between)
    _same(h, a, "rewind")
    for e in (h, a):
        e.run_steps(2500)   # 5000 packets: wraps the 4096-packet ring
    _same(h, a, "ring wrap")
    # outputs read straight after a batch (read_outputs waits on the batch's signal)
    for e in (h, a):
        e.run_steps(3)
    oh, _, _ = h.read_outputs()
    oa, _, _ = a.read_outputs()
    np.testing.assert_array_equal(oa, oh)
    h.close()
    a.close()


def test_native_is_the_default(monkeypatch):
    """auto mode (no MPPI_DISPATCH) dispatches natively on the GPU box; a sharded engine and
    timing mode say why they stay on HIP."""
    monkeypatch.delenv("MPPI_DISPATCH", raising=False)
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    e = Engine(make_config("arm", device=0, n_samples=1024, n_horizon=32))
    e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    e.set_state(_state("arm"))
    e.run_steps(3)
    e.synchronize()
    assert e.dispatch_info().startswith("aql;")
    e.enable_timing(True)
    e.run_steps(2)
    e.synchronize()
    assert e.dispatch_info().startswith("hip: per-launch timing"), e.dispatch_info()
    e.close()


def test_native_sees_host_writes_between_batches(monkeypatch):
    """Only a native submission's first packet acquires (mppi_aql.cpp); everything the host
    or the HIP stream writes between batches -- target, u_prev, state, the step counter, a
    HIP-path step in timing mode -- must be seen by the next batch's kernels.  Each change is
    made on both engines and the batches stay bit-identical with HIP."""
    h, a = _pair(monkeypatch, "arm", n_samples=2048, n_horizon=32)
    rng = np.random.default_rng(7)
    for i in range(4):
        for e in (h, a):
            e.run_steps(3)
        _same(h, a, f"round {i}: batch")
        tgt = [0.1 + 0.02 * i, 0.4 - 0.01 * i, 1.6]
        u = rng.normal(0.0, 0.2, (1, h.H, h.A)).astype(np.float32)
        st = _state("arm", 1, shift=0.01 * (i + 1))
        for e in (h, a):
            e.set_target(tgt, [-0.5, -0.5, 0.5, -0.5])
            e.run_steps(2)
            e.set_u_prev(u)
            e.run_steps(2)
            e.set_state(st)
            e.run_steps(1)
            e.set_step_counter(100 + 7 * i)
            e.run_steps(2)
        _same(h, a, f"round {i}: after host writes")
    for e in (h, a):   # a HIP-path batch in between (timing mode), then native again
        e.enable_timing(True)
        e.run_steps(2)
        e.synchronize()
        e.enable_timing(False)
        e.run_steps(3)
    _same(h, a, "after a HIP-path batch")
    h.close()
    a.close()


CALL_CASES = [("arm", dict(n_samples=4096, n_horizon=32)), ("arm", dict(n_samples=1024, n_horizon=32, state_f64=False)),
              ("drone", dict(n_samples=4096, n_horizon=32)), ("wholebody", dict(n_samples=8192, n_horizon=64)),
              ("quadrotor", dict(n_samples=1024, n_horizon=32))]


@pytest.mark.parametrize("model,kw", CALL_CASES, ids=[f"{m}-{kw['n_samples']}-{kw['n_horizon']}" for m, kw in CALL_CASES])
def test_native_control_calls_match_hip(monkeypatch, model, kw):
    """mppi_step as native packets (the state in the rollout's arguments in pinned host memory,
    completion by the bit-31 flags): every call's outputs, u0 and stats bit-identical to the HIP
    path's under a changing state, interleaved with native batches; the outputs read behind
    the flags equal a re-read after a full synchronize."""
    h, a = _pair(monkeypatch, model, **kw)
    rng = np.random.default_rng(5)
    base = _state(model)[0]
    for i in range(200):
        st = base.copy()
        st[:3] += rng.normal(0, 0.05, 3)
        oh, uh, sh = h.step(st)
        oa, ua, sa = a.step(st)
        np.testing.assert_array_equal(oa, oh, err_msg=f"call {i}")
        np.testing.assert_array_equal(ua, uh, err_msg=f"call {i}")
        assert sa[0].rho == sh[0].rho and sa[0].eta == sh[0].eta, i
        if i % 50 == 49:   # a batch between the calls, then a synchronised re-read
            for e in (h, a):
                e.run_steps(3)
            _same(h, a, f"batch after call {i}")
        elif i % 10 == 3:
            a.synchronize()
            oa2, ua2, _ = a.read_outputs()
            np.testing.assert_array_equal(oa2, oa)
            np.testing.assert_array_equal(ua2, ua)
    assert "calls: aql" in a.dispatch_info(), a.dispatch_info()
    assert h.dispatch_info().endswith("calls: hip"), h.dispatch_info()
    h.close()
    a.close()


@pytest.mark.parametrize("model,kw", [("arm", dict(n_samples=256, n_horizon=32)),
                                      ("quadrotor", dict(n_samples=256, n_horizon=32))],
                         ids=["arm-256-32", "quadrotor-256-32"])
def test_native_batch_readbacks_written_through(monkeypatch, model, kw):
    """The values read only after a native batch -- costs S, the readback copies of w_eps, the
    stored noise -- are written through at device scope (mppi_device.h st_dev / st_dev_run).  At
    a shape whose working set stays in the L2s (K=256, no trajectory), plain stores would leave
    their lines dirty across the batch's release-free packets in whichever XCD ran the writing
    block at each step, and which XCD runs a block is not fixed (MI355X_MICROARCH.md, workgroup
    placement): the readbacks after a 500-step batch must equal HIP's bit for bit."""
    h, a = _pair(monkeypatch, model, store_trajectory=False, store_noise=True, **kw)
    for rnd in range(3):
        for e in (h, a):
            e.run_steps(500)
        _same(h, a, f"500-step batch {rnd}")
        np.testing.assert_array_equal(a.get_weights(), h.get_weights(), err_msg="weights")
        ra, sa = a.get_weighted_noise()
        rh, sh = h.get_weighted_noise()
        np.testing.assert_array_equal(ra, rh, err_msg="w_eps raw")
        np.testing.assert_array_equal(sa, sh, err_msg="w_eps smoothed")
        np.testing.assert_array_equal(a.get_noise(), h.get_noise(), err_msg="stored noise")
        w = a.get_weights()[0].astype(np.float64)
        assert abs(w.sum() - 1.0) < 1e-4
    h.close()
    a.close()


def test_native_dispatch_refused_when_ids_are_not_packet_indices(monkeypatch):
    """The queue's creation probe (mppi_aql.cpp probe_dispatch_ids): when the dispatch ids the
    waves receive are not the queue's packet indices (a tool intercepting the queue; simulated
    here by skewing the probe's readback), the Philox step could not be derived from them, so
    the engine refuses native dispatch, says why, and the HIP path computes the same steps."""
    monkeypatch.delenv("MPPI_DISPATCH", raising=False)
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    ref = Engine(make_config("arm", device=0, seed=11, n_samples=1024, n_horizon=32))
    e = Engine(make_config("arm", device=0, seed=11, n_samples=1024, n_horizon=32))
    for x in (ref, e):   # (the queue -- and its probe -- comes with an engine's first native batch)
        x.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
        x.set_state(_state("arm"))
        if x is e:
            monkeypatch.setenv("MPPI_AQL_PROBE_SKEW", "6")
        x.run_steps(4)
        x.synchronize()
    monkeypatch.delenv("MPPI_AQL_PROBE_SKEW")
    assert "intercepted" in e.dispatch_info(), e.dispatch_info()
    assert ref.dispatch_info().startswith("aql;"), ref.dispatch_info()
    np.testing.assert_array_equal(e.get_u_prev(), ref.get_u_prev())
    oe, ue, _ = e.step(_state("arm", shift=0.01))
    orf, ur, _ = ref.step(_state("arm", shift=0.01))
    np.testing.assert_array_equal(oe, orf)
    assert e.dispatch_info().endswith("calls: hip"), e.dispatch_info()
    e.close()
    ref.close()


@pytest.mark.parametrize("model,kw", [("wholebody", dict(n_samples=8192, n_horizon=64)),
                                      ("arm", dict(n_samples=4096, n_horizon=32, state_f64=True)),
                                      ("wholebody", dict(n_samples=1024, n_horizon=64, n_vehicles=4))])
def test_overlapped_batches_bit_identical(monkeypatch, model, kw):
    """The overlapped native batch (experiment, MPPI_OVERLAP=1: every rollout after a batch's first
    dispatched while the finalize before it runs, drawing its first group's normals and then waiting
    on the finalize blocks' step counters before it reads u_prev) computes exactly what the HIP
    launches compute: 3 batches of 40 steps, then a control call, u_prev / costs / outputs bit for bit."""
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    engines = []
    for mode, ovl in (("hip", "0"), ("aql", "1")):
        monkeypatch.setenv("MPPI_DISPATCH", mode)
        monkeypatch.setenv("MPPI_OVERLAP", ovl)
        e = Engine(make_config(model, device=0, seed=23, **kw))
        for v in range(e.V):
            e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5], vehicle=v)
        e.set_state(_state(model, e.V))
        engines.append(e)
    monkeypatch.delenv("MPPI_DISPATCH")
    monkeypatch.delenv("MPPI_OVERLAP")
    h, a = engines
    try:
        for b in range(3):
            for e in engines:
                e.run_steps(40)
            _same(h, a, f"overlapped batch {b}")
        st = _state(model, h.V, shift=0.01)
        for e in engines:
            e.step(st)
        _same(h, a, "control call after overlapped batches")
    finally:
        for e in engines:
            e.close()
