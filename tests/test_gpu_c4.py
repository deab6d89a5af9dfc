"""The north-star configuration C4 on one GPU: whole-body MPPI, K = 65536, H = 64, the
samples sharded 8 ways (BASELINE.json configs[3]).

What is sharded is the reference's softmin and weighted sum (``mppi.py:143-148``,
``:184-191``) on the whole-body composition of ``urdfparser.py:128-131`` (SURVEY §8a
A16).  Rank g owns the global samples [g*8192, (g+1)*8192); its Philox counters carry the
global sample index, so a shard draws exactly the noise the one-engine run draws for
those samples.  Three runs of the same step are compared:

(a) 8 shard engines (``shard_rank`` 0..7, K = 8192 each) whose exchange slots are summed
    on the host -- the value ONE all-reduce(SUM) of the zero-padded slots computes;
(b) the same 8 shards as 8 processes of ``ShardedEngine`` (gloo collective: one GPU
    cannot hold 8 RCCL ranks, RCCL rejects a duplicate device), and the engine-owned
    RCCL communicator at the 8192 x 64 shard shape with one rank;
(c) one engine over all K = 65536 samples.

Asserted: per-global-k costs bit-identical across (a) and (c) (same arithmetic per
rollout, whatever the block geometry); every shard finalises bit-identically; u0 and
u_prev of (a)/(b) agree with (c) at rtol 1e-4 (the north star's bar; the two runs
combine the same partial records in a different order); the K = 65536 step satisfies
size-independent properties: finite costs, sum w = 1, w_eps = sum_k w_k eps_k of the
stored noise, u_prev += SavGol(w_eps).
"""
import numpy as np
import pytest
import torch

from oracle import mppi_oracle as O

pytestmark = pytest.mark.gpu

K_ALL, H, A, G = 65536, 64, 10, 8
K_SHARD = K_ALL // G
HOME_Q = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]            # kinova.py:135
TARGET = ([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])   # mppi.py:71-72
# C4 synthetic state: drone at (0, 0, 1), level, arm at home, at rest
STATE = np.array([0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0] + HOME_Q + [0.0] * 10, np.float64)
SEED = 0xC4


def _engine(**kw):
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    return Engine(make_config(**kw))


def _close(got, want, rtol=0.0, atol=0.0, what=""):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    err = np.abs(got - want)
    bad = err > atol + rtol * np.abs(want)
    assert not bad.any(), f"{what}: {bad.sum()} / {bad.size} off, max err {err.max():.3e}"


@pytest.fixture(scope="module")
def c4_full():
    """(c): one whole-body engine over all 65536 samples, two control steps (the second
    runs on the first's warm start), with the noise stored for the property checks."""
    e = _engine(model="wholebody", n_samples=K_ALL, n_horizon=H, seed=SEED, store_noise=True)
    e.set_target(*TARGET)
    steps = []
    for s in range(2):
        u_in = e.get_u_prev()[0]
        out, u0, st = e.step(STATE)
        raw, sm = e.get_weighted_noise()
        steps.append(dict(out=out, u0=u0, st=st[0], S=e.get_costs()[0], w=e.get_weights()[0],
                          raw=raw[0], sm=sm[0], u_in=u_in, u_out=e.get_u_prev()[0],
                          eps=e.get_noise()[0] if s == 0 else None))
    e.close()
    return steps


def test_c4_one_engine_full_size_properties(c4_full):
    """(c) at full size: finite costs, sum w = 1, w_eps = sum_k w_k eps_k of the stored
    noise (mppi.py:148), u_prev_out = u_prev_in + SavGol(w_eps) (mppi.py:149-153)."""
    s = c4_full[0]
    assert np.isfinite(s["S"]).all() and (s["S"] > 0).all()
    w = s["w"].astype(np.float64)
    assert abs(w.sum() - 1.0) < 1e-4, w.sum()
    want = np.tensordot(w, s["eps"].astype(np.float64), axes=(0, 0))
    _close(s["raw"], want, rtol=1e-4, atol=1e-7, what="w_eps = sum w eps (K=65536)")
    sm = O.savgol(torch.from_numpy(s["raw"]), 9, 2).numpy()
    _close(s["sm"], sm, rtol=1e-5, atol=1e-6 * float(np.abs(s["raw"]).max()), what="SavGol(w_eps)")
    _close(s["u_out"], s["u_in"] + s["sm"], rtol=1e-6, atol=1e-7, what="u += w_eps")
    assert s["st"].ess >= 1.0 and not s["st"].nonfinite
    assert not c4_full[1]["st"].nonfinite


def test_c4_eight_shards_host_sum_equal_one_engine(c4_full):
    """(a): 8 shard engines, their exchange slots summed on the host (what the one
    all-reduce(SUM) computes), finalised on every shard; two consecutive steps."""
    shards = [_engine(model="wholebody", n_samples=K_SHARD, n_horizon=H, seed=SEED, shard_rank=r,
                      shard_count=G) for r in range(G)]
    slot = shards[0].exchange_slot_floats()
    bufs = [torch.zeros(G * slot, device="cuda") for _ in range(G)]
    for sh, b in zip(shards, bufs):
        sh.set_target(*TARGET)
        sh.bind_exchange(b.data_ptr())
    for s in range(2):
        for sh in shards:
            # step 2 starts from the one engine's warm start, so its rollouts are the same
            # arithmetic again (the combine order leaves u_prev a few ulps apart)
            sh.set_u_prev(c4_full[s]["u_in"])
            sh.set_state(STATE)
            sh.rollout()
            sh.synchronize()
        # each shard wrote only its own slot and zeroed the rest
        for r, b in enumerate(bufs):
            v = b.view(G, slot)
            assert torch.count_nonzero(v[torch.arange(G) != r]).item() == 0, f"shard {r} left another slot dirty"
        total = torch.stack(bufs).sum(0)
        for sh, b in zip(shards, bufs):
            b.copy_(total)
            torch.cuda.synchronize()
            sh.finalize()
        outs = [sh.read_outputs() for sh in shards]
        ref = c4_full[s]
        S = np.concatenate([sh.get_costs()[0] for sh in shards])
        assert np.array_equal(S, ref["S"]), \
            f"step {s}: per-global-k costs differ ({int((S != ref['S']).sum())} samples)"
        ups = [sh.get_u_prev()[0] for sh in shards]
        for r in range(1, G):
            assert np.array_equal(outs[r][0], outs[0][0]) and np.array_equal(outs[r][1], outs[0][1]), \
                f"step {s}: shard {r} finalised differently"
            assert np.array_equal(ups[r], ups[0]), f"step {s}: shard {r} u_prev differs"
        _close(outs[0][1][0], ref["u0"][0], rtol=1e-4, atol=1e-6, what=f"step {s}: u0 sharded vs one engine")
        _close(ups[0], ref["u_out"], rtol=1e-4, atol=1e-6, what=f"step {s}: u_prev sharded vs one engine")
        _close(outs[0][0], ref["out"], atol=_out_tol(ref), what=f"step {s}: outputs")
        assert abs(outs[0][2][0].rho - ref["st"].rho) == 0.0, "rho = min over all samples"
    for sh in shards:
        sh.close()


def test_c4_shard_native_comm_one_rank():
    """(b), engine-owned path at the C4 shard shape (whole-body K=8192 H=64): with a
    1-rank RCCL communicator every step runs rollout -> PACK -> ncclAllReduce ->
    combine-from-slots; it must equal the plain engine's block combine, step and
    back-to-back steps alike."""
    plain = _engine(model="wholebody", n_samples=K_SHARD, n_horizon=H, seed=SEED)
    nat = _engine(model="wholebody", n_samples=K_SHARD, n_horizon=H, seed=SEED)
    nat.comm_init(nat.comm_unique_id())
    info = nat.comm_info()
    assert info == (1, 0), info
    for e in (plain, nat):
        e.set_target(*TARGET)
    o1, u1, s1 = plain.step(STATE)
    o2, u2, s2 = nat.step(STATE)
    _close(u2, u1, rtol=1e-5, atol=1e-7, what="u0 native comm vs plain")
    _close(o2, o1, rtol=1e-6, atol=1e-9, what="outputs native comm vs plain")
    assert np.array_equal(nat.get_costs(), plain.get_costs())
    for e in (plain, nat):
        e.run_steps(10)
        e.synchronize()
    _close(nat.get_u_prev(), plain.get_u_prev(), rtol=1e-4, atol=1e-6, what="u_prev after run_steps")
    assert nat.exchange_timing(20) > 0.0
    nat.close()
    plain.close()


def _out_tol(ref):
    """x/v and qdes/vdes move by u0*dt (u0*dt^2/2): the u0 bar (rtol 1e-4) times dt."""
    return 1e-4 * float(np.abs(ref["u0"]).max()) * 0.01 + 1e-9


def _c4_rank(rank, world, port, u_ins, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from quadrotor_manipulator_mppi_amd.distributed import ShardedEngine
        se = ShardedEngine(model="wholebody", n_samples=K_SHARD, n_horizon=H, seed=SEED)
        se.engine.set_target(*TARGET)
        res = []
        for u_in in u_ins:
            se.engine.set_u_prev(u_in)
            out, u0, st = se.step(STATE)
            res.append((out.copy(), u0.copy(), se.engine.get_u_prev()[0]))
        q.put((rank, res, se.native, se.engine.get_costs()[0]))
    finally:
        dist.destroy_process_group()


def test_c4_eight_ranks_gloo_equal_one_engine(c4_full):
    """(b): C4 as configured -- 8 ranks of ShardedEngine (K = 8192 each, one collective per
    step) on this GPU, gloo carrying the all-reduce.  Every rank finalises the same
    outputs, equal to the one-engine step."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    u_ins = [c4_full[s]["u_in"] for s in range(2)]
    procs = [ctx.Process(target=_c4_rank, args=(r, G, port, u_ins, q)) for r in range(G)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=240) for _ in range(G)], key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    assert not any(r[2] for r in res), "gloo ranks take the torch.distributed collective"
    S = np.concatenate([r[3] for r in res])
    assert np.array_equal(S, c4_full[1]["S"]), "per-global-k costs (step 2)"
    for s in range(2):
        for r in range(1, G):
            for a, b in zip(res[r][1][s], res[0][1][s]):
                assert np.array_equal(a, b), f"step {s}: rank {r} finalised differently"
        out, u0, up = res[0][1][s]
        _close(u0[0], c4_full[s]["u0"][0], rtol=1e-4, atol=1e-6, what=f"step {s}: u0")
        _close(up, c4_full[s]["u_out"], rtol=1e-4, atol=1e-6, what=f"step {s}: u_prev")
        _close(out, c4_full[s]["out"], atol=_out_tol(c4_full[s]), what=f"step {s}: outputs")


_DEADLINE_PROBE = r"""
import sys, time
sys.path.insert(0, sys.argv[1])
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
from quadrotor_manipulator_mppi_amd import _capi
e = Engine(make_config(model="wholebody", n_samples=1024, n_horizon=64, shard_rank=0, shard_count=2))
uid = Engine.comm_unique_id()
t0 = time.time()
try:
    e.comm_init(uid, timeout_ms=3000)
    print("JOINED")
except _capi.MPPIError as x:
    print("ERR", x.status, round(time.time() - t0, 3), x)
e.close()
print("CLOSED")
"""


def test_native_comm_init_deadline_aborts():
    """mppi_comm_init_ex's deadline on hardware: rank 0 of a declared 2-rank communicator
    whose peer never joins returns MPPI_ERR_COMM after the deadline (the half-made
    communicator aborted) instead of blocking forever in ncclCommInitRank, and the engine
    closes cleanly.  Run in a child process under its own time limit."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _DEADLINE_PROBE, root], capture_output=True, text=True,
                       timeout=100)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith(("ERR", "JOINED", "CLOSED"))]
    assert r.returncode == 0, r.stderr[-2000:]
    assert lines and lines[0].startswith("ERR -5"), (lines, r.stderr[-2000:])
    elapsed = float(lines[0].split()[2])
    assert 2.9 <= elapsed < 30.0, elapsed
    assert "not ready after 3000 ms" in lines[0]
    assert lines[-1] == "CLOSED"
