"""The peer exchange (mppi_peer_open / mppi_peer_connect, csrc/mppi_finalize.hip): the sharded
step of SURVEY §8e without a collective.  What is sharded is the reference's softmin and
weighted sum (``mppi.py:143-148``, ``:184-191``); each finalize block stores its partial into
every rank's exchange region as tagged 8 B words and combines the ranks' partials from its own.

(a) one rank exchanging with itself reproduces the unsharded engine bit for bit -- native
    batches, native control calls, HIP launches, and the w_eps readback -- at the C4 shard shape;
(b) two ranks as two processes on this GPU (gloo only carries the handle all-gather and the
    probe's barrier), whole-body K = 2 x 4096, H = 64: per-global-k costs bit-identical to one
    engine over all 8192 samples, both ranks finalise bit-identically, and u0 / u_prev / outputs
    equal the one-engine step at the north star's rtol 1e-4 (the ranks' partials are combined in
    another order than the blocks' records);
(c) a probe word that never arrives fails the connection on every rank;
(d) 4 and 8 ranks as engines of ONE process on this GPU (mppi_peer_connect_ptrs: the regions'
    device addresses instead of IPC handles), each with its own native queue, every engine's
    batch in flight together: the rank counts of a node's scaling run on one GPU.
More than two ranks as separate processes are not run on one GPU (the box's process limits and
queue oversubscription; on a node each rank has its own GPU).
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

H = 64
HOME_Q = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]                 # kinova.py:135
TARGET = ([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])   # mppi.py:71-72
STATE = np.array([0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0] + HOME_Q + [0.0] * 10, np.float64)
SEED = 0xC4


def _engine(**kw):
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    e = Engine(make_config(model="wholebody", n_horizon=H, seed=SEED, **kw))
    e.set_target(*TARGET)
    return e


def _close(got, want, rtol=0.0, atol=0.0, what=""):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    err = np.abs(got - want)
    bad = err > atol + rtol * np.abs(want)
    assert not bad.any(), f"{what}: {bad.sum()} / {bad.size} off, max err {err.max():.3e}"


def _connect_self(e):
    e.peer_connect([e.peer_open()])
    e.peer_probe(0)
    e.peer_probe(1)
    e.peer_probe(2)


@pytest.mark.parametrize("dispatch", ["aql", "hip"])
def test_peer_one_rank_equals_unsharded(dispatch, monkeypatch):
    """(a) at the C4 shard shape (whole-body K=8192 H=64)."""
    monkeypatch.setenv("MPPI_DISPATCH", dispatch)
    plain = _engine(n_samples=8192)
    peer = _engine(n_samples=8192)
    _connect_self(peer)
    rng = np.random.default_rng(5)
    for e in (plain, peer):
        e.set_state(STATE)
        e.run_steps(30)
        e.synchronize()
    assert np.array_equal(peer.get_u_prev(), plain.get_u_prev()), "u_prev after a 30-step batch"
    assert np.array_equal(peer.get_costs(), plain.get_costs())
    if dispatch == "aql":
        assert peer.dispatch_info().startswith("aql;"), peer.dispatch_info()
    for i in range(3):
        st = STATE.copy()
        st[7:14] += rng.normal(0, 0.02, 7)
        o1, u1, s1 = plain.step(st)
        o2, u2, s2 = peer.step(st)
        assert np.array_equal(o2, o1) and np.array_equal(u2, u1), f"call {i}: outputs"
        assert (s2[0].rho, s2[0].eta, s2[0].ess) == (s1[0].rho, s1[0].eta, s1[0].ess)
        assert not s2[0].nonfinite
    r1, m1 = plain.get_weighted_noise()
    r2, m2 = peer.get_weighted_noise()
    assert np.array_equal(r2, r1) and np.array_equal(m2, m1), "w_eps readback through the exchange"
    assert np.array_equal(peer.get_u_prev(), plain.get_u_prev())
    peer.close()
    plain.close()


@pytest.mark.parametrize("model,kw,state", [
    ("arm", dict(n_samples=4096, n_horizon=32, state_f64=True),
     [0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0] + HOME_Q + [0.0] * 7),
    ("drone", dict(n_samples=2048, n_horizon=100, savgol_window=31), [0.1, -0.2, 1.0, 0.0, 0.0, 0.0]),
    ("quadrotor", dict(n_samples=1024, n_horizon=32), [0.0, 0.0, 1.0] + [0.0] * 9),
])
def test_peer_one_rank_equals_unsharded_models(model, kw, state):
    """(a) for the other kernel families and the widest SavGol window (a 38-column finalize
    window: the exchange's full 64-column word block), native batches and control calls."""
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    st = np.array(state, np.float64)
    engines = []
    for _ in range(2):
        e = Engine(make_config(model=model, seed=SEED, **kw))
        if model == "drone" or model == "quadrotor":
            e.set_target([1.0, 2.0, 3.4])
        else:
            e.set_target(*TARGET)
        if model == "quadrotor":
            u = np.zeros((1, e.H, e.A), np.float32)
            u[..., 0] = e.cfg.quad_mass * e.cfg.quad_gravity
            e.set_u_prev(u)
        e.set_state(st)
        engines.append(e)
    plain, peer = engines
    _connect_self(peer)
    for e in engines:
        e.run_steps(25)
        e.synchronize()
    assert np.array_equal(peer.get_u_prev(), plain.get_u_prev()), "u_prev after a native batch"
    for i in range(3):
        o1, u1, _ = plain.step(st)
        o2, u2, _ = peer.step(st)
        assert np.array_equal(o2, o1) and np.array_equal(u2, u1), f"call {i}"
    r1, m1 = plain.get_weighted_noise()
    r2, m2 = peer.get_weighted_noise()
    assert np.array_equal(r2, r1) and np.array_equal(m2, m1)
    peer.close()
    plain.close()


def test_peer_connect_errors():
    """Misuse is refused: connect before open, a second open, V > 1, an RCCL-bound engine."""
    from quadrotor_manipulator_mppi_amd import _capi
    e = _engine(n_samples=1024)
    with pytest.raises(_capi.MPPIError):
        e.peer_connect([b"\0" * _capi.PEER_HANDLE_BYTES])
    h = e.peer_open()
    with pytest.raises(_capi.MPPIError):
        e.peer_open()
    with pytest.raises(ValueError):
        e.peer_connect([h[:10]])
    e.close()
    fleet = _engine(n_samples=1024, n_vehicles=2)
    with pytest.raises(_capi.MPPIError):
        fleet.peer_open()
    fleet.close()


def _rank(rank, world, port, k_shard, u_ins, q, skew_probe):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quadrotor_manipulator_mppi_amd import distributed as D
        if skew_probe:
            if rank == 1:   # (c): this rank's probe words never reach the others
                real = D.Engine.peer_probe
                D.Engine.peer_probe = lambda self, phase: None if phase == 0 else real(self, phase)
            # (two processes on one GPU cannot pair in RCCL: the fallback goes to the torch collective)
            D.setup_native_comm = lambda *a, **k: "RCCL not tried in this test"
        se = D.ShardedEngine(mode="peer", model="wholebody", n_samples=k_shard, n_horizon=H, seed=SEED)
        if skew_probe:
            q.put((rank, se.mode, se.native_error))
            return
        se.engine.set_target(*TARGET)
        res = []
        for u_in in u_ins:
            se.engine.set_u_prev(u_in)
            out, u0, st = se.step(STATE)
            res.append((out.copy(), u0.copy(), se.engine.get_u_prev()[0], bool(st[0].nonfinite)))
        S = se.engine.get_costs()[0]
        se.engine.set_state(STATE)
        se.run_steps(40)
        se.engine.synchronize()
        q.put((rank, res, se.mode, S, se.engine.get_u_prev()[0], se.engine.dispatch_info(), se.engine.peer_info()))
    finally:
        dist.destroy_process_group()


def _spawn(world, k_shard, u_ins, skew_probe):
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, k_shard, u_ins, q, skew_probe)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return res


def test_peer_two_ranks_equal_one_engine():
    """(b) two processes, K = 4096 each, against one engine over K = 8192."""
    full = _engine(n_samples=8192)
    steps = []
    for s in range(2):
        u_in = full.get_u_prev()[0]
        out, u0, st = full.step(STATE)
        steps.append(dict(out=out, u0=u0, S=full.get_costs()[0], u_in=u_in, u_out=full.get_u_prev()[0]))
    full.close()
    res = _spawn(2, 4096, [steps[0]["u_in"], steps[1]["u_in"]], False)
    assert all(r[2] == "peer" for r in res), [r[2] for r in res]
    S = np.concatenate([r[3] for r in res])
    assert np.array_equal(S, steps[1]["S"]), "per-global-k costs (step 2)"
    for s in range(2):
        out, u0, up, nonfinite = res[0][1][s]
        assert not nonfinite
        for a, b in zip(res[1][1][s], res[0][1][s]):
            assert np.array_equal(a, b), f"step {s}: the ranks finalised differently"
        _close(u0[0], steps[s]["u0"][0], rtol=1e-4, atol=1e-6, what=f"step {s}: u0")
        _close(up, steps[s]["u_out"], rtol=1e-4, atol=1e-6, what=f"step {s}: u_prev")
        tol = 1e-4 * float(np.abs(steps[s]["u0"]).max()) * 0.01 + 1e-9
        _close(out, steps[s]["out"], atol=tol, what=f"step {s}: outputs")
    # a 40-step native batch on both ranks: still bit-identical across ranks, finite
    assert np.array_equal(res[0][4], res[1][4]) and np.isfinite(res[0][4]).all()
    assert all(r[5].startswith("aql;") for r in res), [r[5] for r in res]
    # mppi_peer_info: both ranks' words reached each rank's region in the probe's kernel phase
    assert [r[6][:2] for r in res] == [(2, 0), (2, 1)] and all(r[6][2] == 0 for r in res), [r[6] for r in res]


def _timeout_rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import time
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quadrotor_manipulator_mppi_amd.distributed import ShardedEngine
        se = ShardedEngine(mode="peer", model="wholebody", n_samples=1024, n_horizon=H, seed=SEED)
        se.engine.set_target(*TARGET)
        u_in = (np.arange(H * 10, dtype=np.float32).reshape(1, H, 10) % 7 - 3.0) * 0.01
        res = None
        if rank == 0:   # rank 1 never steps: this rank's finalize gives up after its 2 s bound
            se.engine.set_u_prev(u_in)
            t0 = time.perf_counter()
            out, u0, st = se.engine.step(STATE)   # (the engine alone: no agreement with rank 1)
            res = (time.perf_counter() - t0, (st[0].nonfinite, st[0].exchange_timeout), bool(np.isfinite(out).all()),
                   bool(np.array_equal(se.engine.get_u_prev(), u_in)), float(u0[0, 0]), float(u_in[0, 0, 0]))
        # both ranks: the agreement (ShardedEngine.synchronize) sees rank 0's timeout and resynchronises
        resynced = se.synchronize()
        u_after = se.engine.get_u_prev()
        sticky, reports, _ = se.engine.peer_status()
        q.put((rank, se.mode, res, resynced, u_after, sticky, reports, se.engine.get_step_counter()))
        se.engine.close()
    finally:
        dist.destroy_process_group()


def test_peer_timeout_keeps_warm_start():
    """A rank whose peer never steps: its finalize blocks wait out the 2 s bound, then the step
    keeps the warm start (u_prev unchanged, outputs from it, finite) and reports nonfinite = 2
    (StepStats.nonfinite and .exchange_timeout).  Then both ranks' ShardedEngine.synchronize agree
    on the timeout and resynchronise: rank 1 (which never stepped) ends with rank 0's warm start
    and step counter, and both exchanges are reset (no sticky word, no reports)."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_timeout_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=180) for _ in range(2)], key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert [r[1] for r in res] == ["peer", "peer"]
    dt, nonfinite, finite, kept, u0, u_in0 = res[0][2]
    assert nonfinite == (True, True) and finite and kept, res[0][2]
    assert u0 == u_in0, "u0 is the kept warm start's first step"
    assert 1.5 < dt < 30.0, dt
    assert res[0][3] and res[1][3], "every rank reports the timeout (ShardedEngine.synchronize)"
    assert np.array_equal(res[0][4], res[1][4]), "after the resync the ranks' warm starts are bit-identical"
    assert res[0][7] == res[1][7], "and their step counters"
    assert all(r[5] == 0 and not any(r[6]) for r in res), "the exchanges are reset"


def _pair(G=2, k=512, **kw):
    """G in-process peer ranks (mppi_peer_connect_ptrs) on this GPU, whole-body K = k each."""
    ranks = [_engine(n_samples=k, shard_rank=r, shard_count=G, **kw) for r in range(G)]
    for e in ranks:
        e.peer_open()
    addrs = [e.peer_region() for e in ranks]
    for e in ranks:
        e.peer_connect_ptrs(addrs)
        e.set_state(STATE)
    return ranks


def _sync_all(ranks):
    """Synchronise every engine; True per engine whose mppi_synchronize reported a timeout."""
    from quadrotor_manipulator_mppi_amd import _capi
    out = []
    for e in ranks:
        try:
            e.synchronize()
            out.append(False)
        except _capi.PeerTimeout:
            out.append(True)
    return out


def _resync_in_process(ranks):
    """ShardedEngine.resync for ranks in one process (no process group): rank 0's warm start, step
    counter and epoch + 1 on every rank, every region cleared with every engine idle."""
    _sync_all(ranks)
    u = ranks[0].get_u_prev()
    step = ranks[0].get_step_counter()
    epoch = ranks[0].peer_status(reports=False)[2]
    for e in ranks:
        e.peer_reset(step, epoch + 1)
    for e in ranks:
        e.set_u_prev(u)


def test_peer_timeout_rank_wide_and_resync():
    """Two in-process ranks; rank 1 runs ONE STEP FEWER in a native batch, so rank 0's last step
    times out.  After the batch every rank reports it -- rank 0 through its sticky word and
    mppi_synchronize's MPPI_ERR_PEER_TIMEOUT, rank 1 through the timeout report rank 0's blocks
    stored into rank 1's region (mppi_peer_status) -- and while the exchange stays unreset every
    further step on every rank is given up at once (no 2 s waits, warm starts held, reported by
    every block of every step).  After the in-process resync the ranks' u_prev are bit-identical,
    and further native batches stay bit-identical with no timeout."""
    import time
    ranks = _pair()
    try:
        for e in ranks:
            e.run_steps(3)
        assert _sync_all(ranks) == [False, False]
        n = 6
        ranks[0].run_steps(n)
        ranks[1].run_steps(n - 1)
        t0 = time.perf_counter()
        timed = _sync_all(ranks)
        dt = time.perf_counter() - t0
        assert timed[0] and 1.5 < dt < 30.0, (timed, dt)
        st0, rep0, _ = ranks[0].peer_status()
        st1, rep1, _ = ranks[1].peer_status()
        assert st0 != 0 and rep0[0] != 0, (st0, rep0)
        assert rep1[0] != 0, f"rank 1's region holds rank 0's timeout report: {rep1}"
        reported = [st != 0 or any(rep) for st, rep in ((st0, rep0), (st1, rep1))]
        assert reported == [True, True], "every rank reports the timeout after the batch"
        _, _, stats0 = ranks[0].read_outputs()
        assert stats0[0].exchange_timeout and stats0[0].nonfinite
        # broken until reset: both ranks give every step up at once and hold their warm starts
        held = [e.get_u_prev() for e in ranks]
        t0 = time.perf_counter()
        for e in ranks:
            e.run_steps(4)
        timed = _sync_all(ranks)
        dt = time.perf_counter() - t0
        assert timed == [True, True] and dt < 1.0, (timed, dt)
        assert all(np.array_equal(e.get_u_prev(), u) for e, u in zip(ranks, held)), "warm starts held"
        _resync_in_process(ranks)
        assert np.array_equal(ranks[0].get_u_prev(), ranks[1].get_u_prev())
        assert [e.peer_status()[0] for e in ranks] == [0, 0]
        for e in ranks:
            e.run_steps(8)
        assert _sync_all(ranks) == [False, False]
        u = [e.get_u_prev() for e in ranks]
        assert np.array_equal(u[0], u[1]) and np.isfinite(u[0]).all(), "ranks bit-identical after the resync"
        assert not np.array_equal(u[0], held[0]), "and stepping again"
        for e in ranks:
            _, _, st = e.read_outputs()
            assert not st[0].exchange_timeout
    finally:
        for e in ranks:
            e.close()


def test_peer_replay_in_lockstep_takes_no_stale_words():
    """both ranks rewind the step counter (mppi_set_step_counter) and replay a step from
    another warm start.  The replayed step's parity slots still hold the first run's words of the
    same step counter; the exchange epoch in the tags (moved by set_step_counter) keeps a rank that
    polls before its peer has rewritten them from taking them.  Rank 1's replay is enqueued 50 ms
    after rank 0's, so rank 0 polls while only stale words are there.  Result: bit-identical to a
    fresh pair run from the same warm start and counter."""
    import time
    rep_pair, fresh = _pair(), _pair()
    try:
        for e in rep_pair:
            e.run_steps(4)
        _sync_all(rep_pair)
        ctr = rep_pair[0].get_step_counter()
        for e in rep_pair:
            e.run_steps(2)
        assert _sync_all(rep_pair) == [False, False]
        u_alt = (rep_pair[0].get_u_prev() + np.float32(0.05)).astype(np.float32)   # another warm start
        for pair in (rep_pair, fresh):
            for e in pair:
                e.set_u_prev(u_alt)
                e.set_step_counter(ctr)
        for e in fresh:
            e.run_steps(2)
        rep_pair[0].run_steps(2)
        time.sleep(0.05)
        rep_pair[1].run_steps(2)
        assert _sync_all(fresh) == [False, False] and _sync_all(rep_pair) == [False, False]
        want = fresh[0].get_u_prev()
        assert np.array_equal(fresh[1].get_u_prev(), want)
        for r, e in enumerate(rep_pair):
            assert np.array_equal(e.get_u_prev(), want), f"rank {r}: the replay took stale partials"
    finally:
        for e in rep_pair + fresh:
            e.close()


def test_peer_probe_failure_falls_back_on_every_rank():
    """(c) rank 1 skips its probe stores: every rank's connection check fails the same way and
    every rank moves to the next exchange (RCCL, which then cannot pair two processes on one
    GPU, so the torch collective) -- no rank is left stepping alone."""
    res = _spawn(2, 1024, [], True)
    modes = {r[1] for r in res}
    assert len(modes) == 1 and "peer" not in modes, modes
    assert all("peer exchange" in (r[2] or "") for r in res), [r[2] for r in res]


@pytest.mark.parametrize("G", [4, 8])
def test_peer_in_process_ranks_equal_one_engine(G):
    """(d) G ranks as G engines in ONE process on this GPU (mppi_peer_region /
    mppi_peer_connect_ptrs): the rank counts of a node's scaling run, which separate processes
    cannot host on one GPU, with every engine's native batch in flight together.  Whole-body
    K = G x 512, H = 64, against one engine over all G x 512 samples: per-global-k costs
    bit-identical, every rank finalises bit-identically, u_prev at rtol 1e-4; then a 40-step batch
    on every engine, still bit-identical across ranks, and no exchange timeout."""
    k = 512
    full = _engine(n_samples=G * k)
    full.set_state(STATE)
    steps = []
    for s in range(2):
        u_in = full.get_u_prev()[0]
        full.run_steps(1)
        full.synchronize()
        steps.append(dict(u_in=u_in, S=full.get_costs()[0], u_out=full.get_u_prev()[0]))
    full.close()
    ranks = [_engine(n_samples=k, shard_rank=r, shard_count=G) for r in range(G)]
    try:
        for e in ranks:
            e.peer_open()
        addrs = [e.peer_region() for e in ranks]
        for e in ranks:
            e.peer_connect_ptrs(addrs)
            e.set_state(STATE)
        for s in range(2):
            for e in ranks:
                e.set_u_prev(steps[s]["u_in"])
            for e in ranks:   # queued on every engine's native queue, then waited for
                e.run_steps(1)
            for e in ranks:
                e.synchronize()
            S = np.concatenate([e.get_costs()[0] for e in ranks])
            assert np.array_equal(S, steps[s]["S"]), f"step {s}: per-global-k costs"
            ups = [e.get_u_prev()[0] for e in ranks]
            for r in range(1, G):
                assert np.array_equal(ups[r], ups[0]), f"step {s}: rank {r} finalised differently"
            _close(ups[0], steps[s]["u_out"], rtol=1e-4, atol=1e-6, what=f"step {s}: u_prev")
        for e in ranks:
            e.run_steps(40)
        for e in ranks:
            e.synchronize()
        ups = [e.get_u_prev()[0] for e in ranks]
        assert all(np.array_equal(u, ups[0]) for u in ups) and np.isfinite(ups[0]).all()
        for e in ranks:
            out, u0, st = e.read_outputs()
            assert not st[0].nonfinite and not st[0].exchange_timeout
        assert all(e.dispatch_info().startswith("aql;") for e in ranks), [e.dispatch_info() for e in ranks]
        with pytest.raises(Exception):   # another engine's address in this engine's own slot
            bad = _engine(n_samples=k, shard_rank=0, shard_count=2)
            bad.peer_open()
            try:
                bad.peer_connect_ptrs([addrs[1], addrs[0]])
            finally:
                bad.close()
    finally:
        for e in ranks:
            e.close()


def _stall(e, block, ms):
    """mppi_debug_peer_stall: the next FINAL's finalize block ``block`` stores its partial ``ms`` late."""
    import ctypes as C
    from quadrotor_manipulator_mppi_amd import _capi
    fn = _capi.lib().mppi_debug_peer_stall
    fn.restype, fn.argtypes = C.c_int32, [C.c_void_p, C.c_int32, C.c_int32]
    _capi.check(fn(e._h, block, ms), "debug_peer_stall")


# block 3 of the whole-body finalize grid (8 XCD lanes x 2 dim groups x 8 t-slices) is dim 3,
# t-slice 0 (t in [0, 8), the slice that also writes the dim's outputs): csrc/mppi_finalize.hip
STALL_BLOCK, STALL_DIM, STALL_T = 3, 3, slice(0, 8)


@pytest.mark.parametrize("stall_ms", [3000, 5000])
def test_peer_one_block_stalled_all_or_nothing(stall_ms):
    """ONE finalize block of rank 1 stores its partial ``stall_ms`` late (every
    other block of the step on time), so rank 0's matching block passes its 2 s bound while rank 0's
    other blocks have already updated their slices of u_prev.  Within a rank the step is all or
    nothing (mppi_dev.h kXDec: one decision per rank and step, a compare-and-swap before any slice is
    written): rank 0's late block finds its rank committed and keeps polling for a second bound.
    3000 ms: the partial arrives within it -- both ranks end FULLY UPDATED, bit-identical to a pair
    that never stalled, no step given up (the late block's report still asks for a resync, which
    follows).  5000 ms: two bounds pass -- rank 0's warm start
    is torn (that slice kept), which it reports (torn word, timeout report, nan flag 3) instead of
    leaving silently; rank 1 completes (its late block finds its rank committed, the words are in
    place) and is fully updated; the resync takes rank 1's warm start (the lowest rank not torn),
    after which both ranks equal the never-stalled pair and step on bit-identically."""
    ref, pair = _pair(), _pair()
    try:
        for p in (ref, pair):
            for e in p:
                e.run_steps(3)
            assert _sync_all(p) == [False, False]
        held = pair[0].get_u_prev()
        assert np.array_equal(held, ref[0].get_u_prev())
        for e in ref:
            e.run_steps(1)
        assert _sync_all(ref) == [False, False]
        want = ref[0].get_u_prev()
        assert not np.array_equal(want, held)
        _stall(pair[1], STALL_BLOCK, stall_ms)
        for e in pair:
            e.run_steps(1)
        timed = _sync_all(pair)
        u = [e.get_u_prev() for e in pair]
        torn = [e.peer_info()[2] for e in pair]
        assert [e.peer_info()[1] for e in pair] == [0, 1]
        assert np.array_equal(u[1], want), "rank 1 fully updated"
        # the late block reported the timeout either way (every region): the ranks resync before stepping on
        assert all(any(e.peer_status()[1]) for e in pair), "the timeout is reported in every rank's region"
        if stall_ms < 4000:
            assert timed == [False, False] and torn == [0, 0], (timed, torn)
            assert np.array_equal(u[0], want), "rank 0 fully updated (its late block completed)"
            for e in pair:
                _, _, st = e.read_outputs()
                assert not st[0].nonfinite and not st[0].exchange_timeout
        else:
            assert timed[0] and torn[0] != 0 and torn[1] == 0, (timed, torn)
            exp = want.copy()
            exp[0, STALL_T, STALL_DIM] = held[0, STALL_T, STALL_DIM]
            assert np.array_equal(u[0], exp), "rank 0: exactly the stalled block's slice kept, reported torn"
        # the resync (ShardedEngine.resync's choice, in process): the lowest rank that is not torn
        src = min(r for r in range(2) if not torn[r])
        assert src == (1 if stall_ms >= 4000 else 0)
        _sync_all(pair)
        u_src, step = pair[src].get_u_prev(), pair[src].get_step_counter()
        epoch = max(e.peer_status(reports=False)[2] for e in pair)
        for e in pair:
            e.peer_reset(step, epoch + 1)
        for e in pair:
            e.set_u_prev(u_src)
        assert [e.peer_info()[2] for e in pair] == [0, 0] and not any(any(e.peer_status()[1]) for e in pair)
        assert all(np.array_equal(e.get_u_prev(), want) for e in pair), "whole warm starts after the resync"
        for p in (ref, pair):   # and stepping on: bit-identical to the pair that never stalled
            for e in p:
                e.run_steps(5)
            assert _sync_all(p) == [False, False]
        assert all(np.array_equal(e.get_u_prev(), ref[0].get_u_prev()) for e in pair + ref[1:])
    finally:
        for e in ref + pair:
            e.close()
