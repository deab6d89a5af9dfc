"""CPU tests of the multi-GPU exchange protocol over gloo.

The device path is: every rank's rollout folds its samples into one partial
record per vehicle, PACK writes it into slot ``rank`` of a zeroed (G, V, P)
buffer, ONE ``all_reduce(SUM)`` hands every rank all G slots, and every rank's
finalize combines them.  These tests run the same protocol with the oracle's
fp64 shard partials standing in for the rollout (no GPU here): the slot layout,
the zero-padded SUM-as-gather, and the rescale-by-exp(-(rho_g - rho)/lambda)
combine are checked against the unsharded control step of the golden fixtures.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_golden
from oracle import mppi_oracle as O
from quadrotor_manipulator_mppi_amd.distributed import (HDR, all_reduce_slots, combine_slots, setup_native_comm,
                                                        share_comm_id)


def _slot_len(A, H):
    return (HDR + A * H + 3) & ~3   # P: header + N[a][t], rounded to 16 B (mppi_engine.cpp)


def _pack(S, eps, lam, P):
    """One shard's record in the engine's exchange layout: [rho, eta, eta2, nan | N a-major]."""
    rho, eta, N = O.shard_partial(torch.as_tensor(S), torch.as_tensor(eps), lam)
    f = torch.exp(-(torch.as_tensor(S).double() - rho) / lam)
    rec = np.zeros(P, np.float32)
    H, A = N.shape
    rec[0], rec[1], rec[2], rec[3] = float(rho), float(eta), float((f * f).sum()), 0.0
    rec[HDR:HDR + A * H] = N.numpy().T.reshape(-1)
    return rec


def _shards(K, G):
    b = np.linspace(0, K, G + 1).astype(int)
    return [(b[g], b[g + 1]) for g in range(G)]


@pytest.mark.parametrize("name,G", [("arm_k100_h32_f64.npz", 2), ("arm_k100_h32_f64.npz", 5),
                                    ("drone_k256_h32.npz", 4), ("wholebody_k32_h64.npz", 3)])
def test_combine_slots_matches_unsharded(name, G):
    d = load_golden(name)
    S, eps, lam = d["s0_S"], d["s0_noise"], float(d["lam"])
    K, H, A = eps.shape
    P = _slot_len(A, H)
    slots = np.stack([_pack(S[a:b], eps[a:b], lam, P) for a, b in _shards(K, G)])
    got = combine_slots(slots, lam, H, A)
    rho, eta, N = O.shard_partial(torch.as_tensor(S), torch.as_tensor(eps), lam)
    want = (N / eta).numpy()
    np.testing.assert_allclose(got, want, rtol=2e-5, atol=1e-6 * np.abs(want).max())
    # and the reference's own fp32 weighted sum (mppi.py:143) within its rounding
    np.testing.assert_allclose(got, d["s0_w_eps_raw"], rtol=1e-3, atol=2e-4 * np.abs(want).max())


def test_combine_slots_nan_and_empty_shard():
    """A shard whose samples all diverged has rho = inf and contributes 0."""
    d = load_golden("drone_k128_h20.npz")
    S, eps, lam = d["s0_S"], d["s0_noise"], float(d["lam"])
    K, H, A = eps.shape
    P = _slot_len(A, H)
    good = _pack(S, eps, lam, P)
    dead = np.zeros(P, np.float32)
    dead[0] = np.inf
    got = combine_slots(np.stack([good, dead]), lam, H, A)
    np.testing.assert_allclose(got, combine_slots(good[None], lam, H, A), rtol=0, atol=0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, name, V, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d = load_golden(name)
        S, eps, lam = d["s0_S"], d["s0_noise"], float(d["lam"])
        K, H, A = eps.shape
        P = _slot_len(A, H)
        a, b = _shards(K, world)[rank]
        # (G, V, P) zeroed exchange buffer; this rank fills only its slot.  Vehicle v
        # sees the fixture's costs shifted by v (a different, still valid, problem).
        buf = torch.zeros(world * V * P, dtype=torch.float32)
        view = buf.view(world, V, P)
        for v in range(V):
            view[rank, v] = torch.from_numpy(_pack(S[a:b] + v, eps[a:b], lam, P))
        mine = view[rank].clone()
        all_reduce_slots(buf)
        # SUM over zero padding is a gather: this rank's slot is bit-identical
        assert torch.equal(view[rank], mine)
        outs = [combine_slots(view[:, v].numpy(), lam, H, A) for v in range(V)]
        q.put((rank, view.numpy().copy(), outs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,V", [("arm_k100_h32_f64.npz", 1), ("wholebody_k32_h64.npz", 3)])
def test_gloo_world2_exchange(name, V):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, name, V, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    # every rank ends with the same slots and the same combined w_eps
    np.testing.assert_array_equal(res[0][1], res[1][1])
    d = load_golden(name)
    S, eps, lam = d["s0_S"], d["s0_noise"], float(d["lam"])
    for v in range(V):
        np.testing.assert_array_equal(res[0][2][v], res[1][2][v])
        rho, eta, N = O.shard_partial(torch.as_tensor(S + v), torch.as_tensor(eps), lam)
        want = (N / eta).numpy()
        np.testing.assert_allclose(res[0][2][v], want, rtol=2e-5, atol=1e-6 * np.abs(want).max())


# ----------------------------------------------------------- native RCCL path (host side)
def _uid_rank(rank, world, port, q, bad):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        made = []

        def make_id():
            made.append(rank)
            if bad == "raise":
                raise RuntimeError("librccl.so.1 not found")
            return b"x" * 7 if bad else bytes(range(128))
        try:
            q.put((rank, share_comm_id(rank, world, make_id=make_id), made))
        except RuntimeError as e:
            q.put((rank, str(e), made))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bad", [False, True, "raise"])
def test_comm_id_broadcast_world2(bad):
    """The engine-owned RCCL path's id hand-off (distributed.share_comm_id): only rank 0
    makes the ncclUniqueId, every rank receives the same 128 bytes over torch.distributed;
    a malformed id -- or rank 0 failing to make one -- is refused on every rank before
    ncclCommInitRank (no rank is left waiting in the broadcast)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_uid_rank, args=(r, world, port, q, bad)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][2] == [0] and res[1][2] == [], "only rank 0 makes the id"
    if bad:
        assert all("bad RCCL unique id" in r[1] for r in res)
        if bad == "raise":
            assert all("librccl.so.1 not found" in r[1] for r in res)
    else:
        assert res[0][1] == res[1][1] == bytes(range(128))


def test_native_comm_entry_points_reject_bad_arguments():
    """mppi_comm_unique_id / mppi_comm_init / mppi_exchange / mppi_exchange_timing check
    their arguments before touching RCCL or a device (CPU-callable)."""
    import ctypes as C
    from quadrotor_manipulator_mppi_amd import _capi as capi
    L = capi.lib()
    assert L.mppi_comm_unique_id(None) == capi.ERR_INVALID_ARG
    buf = (C.c_uint8 * capi.COMM_ID_BYTES)()
    assert L.mppi_comm_init(None, buf) == capi.ERR_INVALID_ARG
    assert L.mppi_comm_init_ex(None, buf, 100) == capi.ERR_INVALID_ARG
    n, r_ = C.c_int32(), C.c_int32()
    assert L.mppi_comm_info(None, C.byref(n), C.byref(r_)) == capi.ERR_INVALID_ARG
    assert L.mppi_exchange(None) == capi.ERR_INVALID_ARG
    us = C.c_double()
    assert L.mppi_exchange_timing(None, 10, C.byref(us)) == capi.ERR_INVALID_ARG
    r, f, pr = C.c_double(), C.c_double(), C.c_double()
    assert L.mppi_kernel_timing_ex(None, 10, C.byref(r), C.byref(f), C.byref(pr)) == capi.ERR_INVALID_ARG
    assert "bad arguments" in L.mppi_last_error().decode()
    # the peer exchange's entry points as well
    h = (C.c_uint8 * capi.PEER_HANDLE_BYTES)()
    assert L.mppi_peer_open(None, h) == capi.ERR_INVALID_ARG
    assert L.mppi_peer_connect(None, h) == capi.ERR_INVALID_ARG
    assert L.mppi_peer_probe(None, 0) == capi.ERR_INVALID_ARG
    addr = (C.c_uint64 * 8)()
    assert L.mppi_peer_region(None, addr) == capi.ERR_INVALID_ARG
    assert L.mppi_peer_connect_ptrs(None, addr) == capi.ERR_INVALID_ARG
    assert "null" in L.mppi_last_error().decode()


def _setup_rank(rank, world, port, q, fault):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = []

        def available():
            return "RCCL unavailable: librccl.so.1: cannot open" if (fault == "unavailable" and rank == 1) else None

        def init(uid):
            calls.append(len(uid))
            if fault == "timeout" and rank == 1:   # what mppi_comm_init_ex raises at its deadline
                raise RuntimeError("[mppi status -5] comm_init: ncclCommInitRankConfig(rank 1 of 2): "
                                   "not ready after 100 ms (aborted)")
        err = setup_native_comm(rank, world, None, 0, available, lambda: bytes(range(128)), init)
        q.put((rank, err, calls))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fault", [None, "unavailable", "timeout"])
def test_native_comm_setup_agreement_world2(fault):
    """distributed.setup_native_comm under gloo: the ranks agree on RCCL's availability
    before any of them enters the collective init (a rank without RCCL must not leave rank 0
    waiting in ncclCommInitRankConfig), and an init that times out on one rank (the
    non-blocking init's deadline) gives every rank the same failure -- the cue for all of
    them to take the torch.distributed collective -- instead of a stuck rank."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_setup_rank, args=(r, world, port, q, fault)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if fault is None:
        assert [r[1] for r in res] == [None, None]
        assert [r[2] for r in res] == [[128], [128]]
    elif fault == "unavailable":
        assert all(r[1] and "RCCL unavailable" in r[1] for r in res)
        assert [r[2] for r in res] == [[], []], "no rank may enter the init"
    else:
        assert all(r[1] for r in res)
        assert "not ready after" in res[1][1]
        assert [r[2] for r in res] == [[128], [128]]


class _FakePeerEngine:
    """The three peer-exchange calls of Engine, recording what the setup hands them."""

    def __init__(self, rank, fault):
        self.rank, self.fault, self.calls = rank, fault, []

    def peer_open(self):
        self.calls.append("open")
        if self.fault == "open" and self.rank == 1:
            raise RuntimeError("[mppi status -4] peer_open: peer exchange: one vehicle per engine (V = 2)")
        return bytes([self.rank]) * 64

    def peer_connect(self, handles):
        self.calls.append(("connect", [h[0] for h in handles]))

    def peer_probe(self, phase):
        self.calls.append(("probe", phase))
        if self.fault == "probe" and self.rank == 0 and phase == 2:
            raise RuntimeError("[mppi status -6] peer_probe: peer exchange: rank 1's word did not reach this "
                               "rank's region in the kernel probe")


def _peer_rank(rank, world, port, q, fault):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quadrotor_manipulator_mppi_amd.distributed import setup_peer_exchange
        e = _FakePeerEngine(rank, fault)
        err = setup_peer_exchange(rank, world, None, 0, e)
        q.put((rank, err, e.calls))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fault", [None, "open", "probe"])
def test_peer_exchange_setup_agreement_world2(fault):
    """distributed.setup_peer_exchange under gloo: every rank receives every rank's handle in
    rank order, runs the three probe phases in step with the others, and a failure on one rank
    (a region that cannot be opened, a probe word that never arrives) gives every rank the same
    verdict at the same phase -- the cue for all of them to take the RCCL path -- instead of a
    rank that steps alone."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_peer_rank, args=(r, world, port, q, fault)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = ["open", ("connect", [0, 1]), ("probe", 0), ("probe", 1), ("probe", 2)]
    if fault is None:
        assert [r[1] for r in res] == [None, None]
        assert [r[2] for r in res] == [full, full]
    elif fault == "open":
        assert all(r[1] for r in res) and "one vehicle" in res[1][1]
        assert [r[2] for r in res] == [["open"], ["open"]], "no rank may connect"
    else:
        assert all(r[1] for r in res) and "did not reach" in res[0][1]
        assert [r[2] for r in res] == [full, full]


def test_default_exchange(monkeypatch):
    from quadrotor_manipulator_mppi_amd.distributed import default_exchange
    monkeypatch.delenv("MPPI_EXCHANGE", raising=False)
    assert default_exchange(False, 2, 1) == "torch"
    assert default_exchange(True, 8, 1) == "peer"
    assert default_exchange(True, 16, 1) == "rccl"
    assert default_exchange(True, 2, 8) == "rccl"
    monkeypatch.setenv("MPPI_EXCHANGE", "rccl")
    assert default_exchange(True, 8, 1) == "rccl"
    monkeypatch.setenv("MPPI_EXCHANGE", "peer")
    assert default_exchange(False, 2, 1) == "peer"


# ---------------------------------------------------------------- vehicle sharding (config C5)
class _TargetSink:
    """Stands in for an Engine where bench.set_targets writes the per-vehicle targets."""
    def __init__(self):
        self.t = {}

    def set_target(self, pos, quat=None, vehicle=0):
        self.t[vehicle] = (np.asarray(pos, np.float32), np.asarray(quat, np.float32))


def _fleet_oracle_steps(vehicles, V_total, K=48, H=16, seed=77, steps=2):
    """The control steps of the fleet-wide vehicles ``vehicles`` as one rank of a vehicle split
    computes them: its rows of the fleet's state (bench.make_state), its targets (bench.set_targets
    with the rank's range), and the device noise keyed by the FLEET-WIDE vehicle index
    (O.philox_normals, the kernel's draw restated) -- through the oracle's whole-body step."""
    import bench
    from quadrotor_manipulator_mppi_amd.robot.urdf_chain import load_chain
    torch.set_num_threads(1)
    chain = [O.Joint(j["name"], j["type"], j["xyz"], j["rpy"], j["axis"], j["q_index"]) for j in load_chain()]
    state = bench.make_state("wholebody", vehicles.stop)[vehicles.start:]
    sink = _TargetSink()
    bench.set_targets(sink, "wholebody", vehicles)
    sig = np.diag([30.0] * 3 + [0.1] * 7).astype(np.float32)
    out = {}
    for i, v in enumerate(vehicles):
        s = state[i]
        tpos, tquat = sink.t[i]
        u = torch.zeros(H, 10)
        rpy = O.base_rpy_from_quat(s[3:7])
        res = []
        for step in range(steps):
            _, z = O.philox_normals(seed, step, v, np.arange(K), H, 10)
            noise = torch.from_numpy(z) @ torch.from_numpy(sig)
            r = O.wholebody_step(chain, s[0:3], s[14:17], s[7:14], s[17:24], rpy, u, noise, tpos, tquat)
            u = r["u_prev_out"]
            res.append((r["S"].numpy(), u.numpy(), r["qdes"].numpy()))
        out[v] = res
    return out


def _vehicle_split_main(rank, world, port, V, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quadrotor_manipulator_mppi_amd.distributed import vehicle_range
        vr = vehicle_range(V, world, rank)
        mine = _fleet_oracle_steps(vr, V)
        got = [None] * world
        dist.all_gather_object(got, (rank, list(vr), mine))   # (no collective on the step path: results only)
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_vehicle_split_equals_one_fleet():
    """Config C5 split over 2 ranks by vehicles (ShardedEngine mode "vehicles", SURVEY §8e "prefer
    vehicles across GPUs -- zero communication"): each rank takes vehicle_range(8, 2, rank), its rows
    of the fleet's state and its targets from bench.py, and the noise keyed by the fleet-wide vehicle
    index; every rank's vehicles equal one process over the whole fleet bit for bit (the GPU side of
    the same claim: tests/test_gpu_fleet.py test_vehicle_split_*)."""
    from quadrotor_manipulator_mppi_amd.distributed import vehicle_range
    V, world = 8, 2
    assert [list(vehicle_range(V, world, r)) for r in range(world)] == [[0, 1, 2, 3], [4, 5, 6, 7]]
    with pytest.raises(ValueError):
        vehicle_range(7, 2, 0)
    whole = _fleet_oracle_steps(range(V), V)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_vehicle_split_main, args=(r, world, port, V, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, got in res:
        owned = sorted(v for _, vs, _ in got for v in vs)
        assert owned == list(range(V)), "every vehicle owned by exactly one rank"
        for _, vs, mine in got:
            for v in vs:
                for (S, u, qd), (S1, u1, qd1) in zip(mine[v], whole[v]):
                    assert np.array_equal(S, S1) and np.array_equal(u, u1) and np.array_equal(qd, qd1), v


# ---------------------------------------------------------------- peer-exchange timeout agreement
class _FakeTimeoutEngine:
    """The engine calls ShardedEngine.synchronize / resync make, on the host only (no GPU here):
    rank ``late`` reports a timeout (mppi_synchronize's MPPI_ERR_PEER_TIMEOUT) until reset."""
    def __init__(self, rank, late, torn=None):
        from quadrotor_manipulator_mppi_amd import _capi
        self._exc = _capi.PeerTimeout
        self.timed_out = rank == late
        self.rank, self.torn = rank, (0x80000007 if rank == torn else 0)
        self.u = np.full((1, 4, 3), float(rank + 1), np.float32)
        self.ctr, self.epoch = 10 + rank, 3 + rank
        self.resets = []

    def synchronize(self):
        if self.timed_out:
            raise self._exc(-6, "peer exchange: a step was given up")

    def get_u_prev(self):
        return self.u.copy()

    def set_u_prev(self, u):
        self.u = np.asarray(u, np.float32).copy()

    def get_step_counter(self):
        return self.ctr

    def peer_status(self, reports=True):
        return (1 if self.timed_out else 0), None, self.epoch

    def peer_info(self):
        return 2, self.rank, self.torn

    def step(self, state):   # (the control call: its stats report this rank's sticky word)
        from quadrotor_manipulator_mppi_amd.engine import StepStats
        return None, None, [StepStats(0.0, 1.0, 1.0, self.timed_out, False, self.timed_out)]

    def peer_reset(self, step, epoch):
        self.timed_out = False
        self.torn = 0
        self.ctr, self.epoch = step, epoch
        self.resets.append((step, epoch))


def _fake_sharded(rank, world, late, torn=None, agree_every=100):
    from quadrotor_manipulator_mppi_amd.distributed import ShardedEngine
    se = object.__new__(ShardedEngine)   # (the host protocol only: no Engine, no HIP stream)
    se.group, se.rank, se.world, se.local, se.mode, se.resyncs = None, rank, world, 0, "peer", 0
    se.agree_every, se._calls = agree_every, 0
    se.engine = _FakeTimeoutEngine(rank, late, torn)
    return se


def _agree_main(rank, world, port, late, q, torn=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        se = _fake_sharded(rank, world, late, torn)
        first = se.synchronize()
        second = se.synchronize()
        e = se.engine
        q.put((rank, first, second, e.u, e.ctr, e.epoch, e.resets, se.resyncs))
    finally:
        dist.destroy_process_group()


def _step_agree_main(rank, world, port, late, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        se = _fake_sharded(rank, world, late, agree_every=3)
        seen = []
        for _ in range(6):   # calls 3 and 6 are the agreements (collectives); 1, 2, 4, 5 are local
            st = se.step(None)[2]
            seen.append((bool(st[0].exchange_timeout), se.resyncs))
        q.put((rank, seen, se.engine.u))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("late", [0, 1, None])
def test_gloo_world2_peer_timeout_agreement_and_resync(late):
    """ShardedEngine.synchronize on a multi-rank peer exchange (the host side of the failure
    handling; the device side is tests/test_gpu_peer.py): the ranks MAX-agree on any rank's
    timeout, so EVERY rank reports it (True) even when only one rank's engine saw it, and every
    rank resynchronises -- rank 0's warm start and step counter, epoch + 1, its region reset -- so
    the warm starts are identical afterwards; no timeout: nothing happens on any rank."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_main, args=(r, world, port, late, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if late is None:
        assert all(r[1] is False and r[2] is False and r[6] == [] for r in res)
        return
    for rank, first, second, u, ctr, epoch, resets, n in res:
        assert first is True and second is False and n == 1, (rank, first, second, n)
        assert np.array_equal(u, np.full((1, 4, 3), 1.0, np.float32)), "rank 0's warm start on every rank"
        assert (ctr, epoch) == (10, 4) and resets == [(10, 4)]


def _run2(target, *args):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _agree_torn_main(rank, world, port, q):
    _agree_main(rank, world, port, 0, q, torn=0)


def test_gloo_world2_resync_source_skips_a_torn_rank():
    """A rank whose warm start came out of a step torn (mppi_peer_info: a finalize block that timed
    out twice while the rank's other blocks had updated their slices) is not the resync's source:
    the lowest rank that is not torn is (rank 1 here), so every rank ends with a whole warm start."""
    res = _run2(_agree_torn_main)
    for rank, first, second, u, ctr, epoch, resets, n in res:
        assert first is True and n == 1
        assert np.array_equal(u, np.full((1, 4, 3), 2.0, np.float32)), "rank 1's warm start on every rank"
        assert (ctr, epoch) == (11, 5) and resets == [(11, 5)]


def test_gloo_world2_step_agrees_every_n_calls():
    """ShardedEngine.step keeps the control call collective-free between agreements: a
    rank whose step was given up reports it at once on that rank, and the ranks agree (and resync)
    only on every ``agree_every``-th call -- here the 3rd -- on every rank alike."""
    res = _run2(_step_agree_main, 1)
    r0, r1 = res[0][1], res[1][1]
    assert r0 == [(False, 0), (False, 0), (True, 1), (False, 1), (False, 1), (False, 1)], r0
    assert r1 == [(True, 0), (True, 0), (True, 1), (False, 1), (False, 1), (False, 1)], r1
    assert np.array_equal(res[0][2], res[1][2])
