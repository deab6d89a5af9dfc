"""Sample sharding over GPUs: one process per GPU, one all-reduce per step.

SURVEY.md §8e: rollouts are independent until the softmin, so rank g owns the
global samples [g*K, (g+1)*K) (the device Philox stream is keyed by the global
sample index, so the noise does not depend on the GPU count).  Each rank folds
its rollouts into one partial record (rho_g, eta_g, eta2_g, N_g[A*H]) and writes
it into slot g of a zero-initialised (G, V, P) exchange buffer; ONE
``all_reduce(SUM)`` over RCCL/xGMI (backend "nccl") then hands every rank all G
slots (x + 0 is exact, so the sum is a gather), and every rank runs the same
finalize: rho = min_g rho_g, rescale by exp(-(rho_g - rho)/lambda), SavGol,
u += w_eps.  The payload is (4 + A*H) floats per vehicle per rank -- 2.6 KB at
H=64, A=10 -- so the collective is latency-bound; ring bandwidth is irrelevant.

Three ways to run the exchange:

* ``exchange="peer"`` (``native=True`` on a one-vehicle shard; ``MPPI_EXCHANGE=peer``): no
  collective at all.  Each rank's engine opens an exchange region in its own GPU memory, the ranks
  all-gather the regions' IPC handles once, and every finalize block stores its partial into every
  rank's region over xGMI as tagged 8 B words and combines the ranks' partials from its own
  (``mppi_peer_open`` / ``mppi_peer_connect``, csrc/mppi_finalize.hip).  A step is the unsharded
  step's two kernels -- native dispatch, no PACK launch, nothing enqueued by the host between
  them; a connection probe runs before the first step;
* ``exchange="rccl"`` (``native=True``, the default for ``native`` otherwise): the engine owns an
  RCCL communicator (``mppi_comm_init``; rank 0's unique id is broadcast over torch.distributed)
  and a whole control step -- rollout, pack, all-reduce, finalize -- is enqueued from C with no
  Python in between (``Engine.run_steps`` / ``Engine.step`` work unchanged on a shard);
* ``native=False``: the engine packs into a torch buffer and ``torch.distributed``
  does the all-reduce (any backend; the gloo tests on CPU and rehearsals use it).

If the engine-owned exchange cannot be set up on some rank (no peer mapping, no loadable RCCL, a
bad unique id, peers that do not join before the init deadline), every rank learns it (MIN
all-reduces of an ok flag) and all of them take the next way down -- peer, then RCCL, then the
torch.distributed collective -- on a fresh engine; ``native_error`` says why.  RCCL's
availability is agreed on before any rank enters the collective init.

The reference has no distributed code (single process, ``CUDA_VISIBLE_DEVICES='0'``
at ``mppi.py:31``); there is no reference collective to mirror.
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist

from .engine import Engine, make_config

HDR = 4   # partial record header: rho, eta, eta2, nan-flag


def all_reduce_slots(buf: torch.Tensor, group=None) -> torch.Tensor:
    """The single collective of a control step (SUM over a zero-padded slot buffer)."""
    dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return buf


def share_comm_id(rank: int, world: int, group=None, make_id: Optional[Callable[[], bytes]] = None) -> bytes:
    """Rank 0 makes the RCCL unique id (``mppi_comm_unique_id``) and every rank receives it
    over torch.distributed (any backend), as ncclCommInitRank requires.  Raises on a
    malformed id, so no rank enters the collective init with a bad one."""
    from . import _capi
    make_id = make_id or Engine.comm_unique_id
    uid = [None]
    if rank == 0:
        try:
            uid[0] = make_id()
        except Exception as exc:   # still broadcast: the other ranks must not wait forever
            uid[0] = f"rank 0 could not make the RCCL unique id: {exc}"
    if world > 1:
        dist.broadcast_object_list(uid, src=0, group=group)
    if not isinstance(uid[0], (bytes, bytearray)) or len(uid[0]) != _capi.COMM_ID_BYTES:
        why = uid[0] if isinstance(uid[0], str) else (
            f"{type(uid[0]).__name__}, {len(uid[0]) if uid[0] is not None else 0} bytes")
        raise RuntimeError(f"rank {rank}: bad RCCL unique id from rank 0 ({why})")
    return bytes(uid[0])


def _all_ranks_ok(ok: bool, group, device: int) -> bool:
    """True only if every rank passes ok (one MIN all-reduce over the process group)."""
    t = torch.tensor([1 if ok else 0], dtype=torch.int32,
                     device=f"cuda:{device}" if dist.get_backend(group) == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


def _any_rank(flag: bool, group, device: int) -> bool:
    """True if any rank passes flag (one MAX all-reduce; every rank returns the same verdict, and
    every rank has joined it when it returns: it doubles as a barrier)."""
    t = torch.tensor([1 if flag else 0], dtype=torch.int32,
                     device=f"cuda:{device}" if dist.get_backend(group) == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return bool(t.item())


def setup_native_comm(rank: int, world: int, group, device: int, available: Callable[[], Optional[str]],
                      make_id: Callable[[], bytes], init: Callable[[bytes], None]) -> Optional[str]:
    """Agree on, then build, the engine-owned RCCL communicator.  Returns None when every
    rank has it, else the reason (the same verdict on every rank).

    1. every rank checks that RCCL is loadable (``available``: mppi_comm_available) and the
       ranks agree on it (MIN all-reduce) BEFORE any rank enters the collective init, so a
       rank without RCCL cannot leave its peers waiting in ncclCommInitRankConfig;
    2. rank 0 makes the unique id and broadcasts it (a failure is broadcast too);
    3. every rank joins (``init``: mppi_comm_init, non-blocking with a deadline, so a rank
       whose peers never arrive gets an error instead of hanging);
    4. the ranks agree on the outcome (MIN all-reduce)."""
    err = available()
    if world > 1 and not _all_ranks_ok(err is None, group, device):
        return err or "RCCL unavailable on another rank"
    if err is not None:
        return err
    try:
        init(share_comm_id(rank, world, group, make_id=make_id))
    except Exception as exc:   # a bad id (every rank sees it), an init error or timeout
        err = str(exc)
    if world > 1 and not _all_ranks_ok(err is None, group, device):
        return err or "another rank failed mppi_comm_init"
    return err


def combine_slots(slots: np.ndarray, lam: float, H: int, A: int) -> np.ndarray:
    """Host restatement of the finalize combine for a (G, P) slot array -> raw
    w_eps (H, A).  Used by the CPU (gloo) tests of the exchange protocol; the
    device path is ``k_finalize`` in csrc/mppi_finalize.hip."""
    rho = slots[:, 0].astype(np.float64)
    r = rho.min()
    f = np.exp(-(rho - r) / lam)
    eta = float((f * slots[:, 1]).sum())
    N = (f[:, None] * slots[:, HDR:HDR + A * H].astype(np.float64)).sum(0)
    return (N / eta).reshape(A, H).T


def setup_peer_exchange(rank: int, world: int, group, device: int, engine: Engine) -> Optional[str]:
    """Open this rank's exchange region, all-gather the IPC handles, map every rank's region and
    probe the mapping (``mppi_peer_probe``).  Returns None when every rank is connected, else the
    reason (the same verdict on every rank)."""
    def agreed(err):
        if world > 1 and not _all_ranks_ok(err is None, group, device):
            return err or "peer exchange failed on another rank"
        return err

    handle, err = None, None
    try:
        handle = engine.peer_open()
    except Exception as exc:
        err = str(exc)
    if (err := agreed(err)) is not None:
        return err
    handles = [None] * world
    if world > 1:
        dist.all_gather_object(handles, handle, group=group)
    else:
        handles = [handle]
    try:
        engine.peer_connect(handles)
        engine.peer_probe(0)
    except Exception as exc:
        err = str(exc)
    if (err := agreed(err)) is not None:
        return err
    for phase in (1, 2):   # 1: the copied words arrived; 2: the finalize's stores and polls
        if world > 1:
            dist.barrier(group=group)
        try:
            engine.peer_probe(phase)
        except Exception as exc:
            err = str(exc)
        if (err := agreed(err)) is not None:
            return err
    return None


def vehicle_range(n_vehicles: int, world: int, rank: int) -> range:
    """The fleet-wide vehicles rank ``rank`` owns when a fleet of ``n_vehicles`` is split over
    ``world`` GPUs ("prefer vehicles across GPUs -- zero communication"):
    consecutive blocks of n_vehicles / world.  The engine is made with vehicle_offset = the range's
    start, so its device noise is keyed by the fleet-wide index and each rank's vehicles draw, roll
    out and finalise exactly as in one engine over the whole fleet."""
    if n_vehicles % world:
        raise ValueError(f"{n_vehicles} vehicles do not split over {world} ranks")
    n = n_vehicles // world
    return range(rank * n, (rank + 1) * n)


def default_exchange(native: bool, world: int, n_vehicles: int) -> str:
    """MPPI_EXCHANGE (peer | rccl | torch; also over a gloo group, for rehearsals on one GPU) or,
    for an engine-owned exchange, peer on one-vehicle shards of at most 8 ranks and RCCL otherwise.
    ("vehicles" -- the fleet split over the ranks, no exchange -- is chosen explicitly.)"""
    env = os.environ.get("MPPI_EXCHANGE")
    if env in ("peer", "rccl", "torch"):
        return env
    if not native:
        return "torch"
    return "peer" if n_vehicles == 1 and world <= 8 else "rccl"


class ShardedEngine:
    """One rank's engine of a sample-sharded MPPI controller -- or, with ``mode="vehicles"``, of a
    vehicle-sharded fleet: ``n_vehicles`` is then the whole fleet, this rank's engine runs
    ``vehicle_range(n_vehicles, world, rank)`` of it over all K samples, and nothing is exchanged
    (each vehicle's softmin is its own; ``set_state`` / ``set_target`` take this rank's vehicles)."""

    def __init__(self, group=None, exchange: Callable = all_reduce_slots, native: Optional[bool] = None,
                 mode: Optional[str] = None, **engine_kw):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if native is None:
            native = self.world > 1 and dist.get_backend(group) == "nccl" and exchange is all_reduce_slots
        self.native = bool(native)
        # the exchange: "peer" (no collective), "rccl" (engine-owned communicator), "torch"
        self.mode = mode or default_exchange(self.native, self.world, int(engine_kw.get("n_vehicles", 1) or 1))
        if self.mode not in ("peer", "rccl", "torch", "vehicles"):
            raise ValueError(f"exchange mode {self.mode!r}")
        self.native = self.mode != "torch"
        device = engine_kw.pop("device", 0)
        self.local = int(os.environ.get("LOCAL_RANK", device))
        self.local %= max(1, torch.cuda.device_count())   # more ranks than devices: wrap
        torch.cuda.set_device(self.local)
        self.vehicles = range(int(engine_kw.get("n_vehicles", 1) or 1))   # the fleet-wide vehicles this rank runs
        if self.mode == "vehicles":   # every rank a whole controller over its share of the fleet
            self.vehicles = vehicle_range(len(self.vehicles), self.world, self.rank)
            engine_kw = dict(engine_kw, n_vehicles=len(self.vehicles), vehicle_offset=self.vehicles.start)
            cfg = make_config(device=self.local, shard_rank=0, shard_count=1, **engine_kw)
        else:
            cfg = make_config(device=self.local, shard_rank=self.rank, shard_count=self.world, **engine_kw)
        self.engine = Engine(cfg)
        # one dedicated stream carries rollout -> collective -> finalize (the default
        # stream's handle is 0, which mppi_set_stream reads as "engine-owned stream")
        self.stream = torch.cuda.Stream(device=self.local)
        self.engine.set_stream(self.stream.cuda_stream)
        self._exchange = exchange
        self.buf: Optional[torch.Tensor] = None
        self.native_error: Optional[str] = None
        self.resyncs = 0   # peer-exchange recoveries (resync) so far
        # On a multi-rank peer exchange the ranks agree on a timeout (a collective) every
        # ``agree_every`` control calls of ``step`` and in every ``synchronize``; in between a step
        # is collective-free (a timeout is rank-wide on the device already: the other ranks' steps
        # are given up too, warm starts held, until the agreement resyncs them).  1 = every call.
        self.agree_every = max(1, int(os.environ.get("MPPI_PEER_AGREE_EVERY", "100")))
        self._calls = 0

        def fresh_engine():
            self.engine.close()
            self.engine = Engine(cfg)
            self.engine.set_stream(self.stream.cuda_stream)

        if self.mode == "peer":
            err = setup_peer_exchange(self.rank, self.world, group, self.local, self.engine)
            if err is not None:   # every rank takes the RCCL communicator instead, on a fresh engine
                self.native_error = f"peer exchange: {err}"
                self.mode = "rccl"
                fresh_engine()
        if self.mode == "rccl":   # engine-owned RCCL communicator: the whole step is enqueued from C
            err = setup_native_comm(self.rank, self.world, group, self.local, Engine.comm_available,
                                    Engine.comm_unique_id, self.engine.comm_init)
            if err is not None and self.world > 1:
                # a failure on any rank: every rank takes the torch.distributed collective
                # instead (same slots, same finalize) on a fresh engine, so no rank is left
                # waiting in a collective alone
                self.native_error = (self.native_error + "; " if self.native_error else "") + err
                self.native = False
                self.mode = "torch"
                fresh_engine()
            elif err is not None:
                raise RuntimeError(err)
        if not self.native and self.world > 1 and self.mode != "vehicles":
            slot = self.engine.exchange_slot_floats()
            with torch.cuda.stream(self.stream):
                self.buf = torch.zeros(self.world * slot, dtype=torch.float32, device=f"cuda:{self.local}")
            self.engine.bind_exchange(self.buf.data_ptr())
        self.stream.synchronize()

    def step_async(self, d_noise_ptr: int = 0):
        """rollout -> (all-reduce) -> finalize, all ordered on self.stream, no host sync."""
        if self.native or self.mode == "vehicles":
            self.engine.rollout(d_noise_ptr)
            if self.mode == "rccl":
                self.engine.exchange()
            self.engine.finalize()
            return
        with torch.cuda.stream(self.stream):
            self.engine.rollout(d_noise_ptr)
            if self.world > 1:
                self._exchange(self.buf, self.group)
            self.engine.finalize()

    def run_steps(self, n: int):
        """n back-to-back control steps; on a native shard one C call enqueues them all."""
        if self.native or self.world == 1:
            self.engine.run_steps(n)
        else:
            for _ in range(n):
                self.step_async()

    def step(self, state, d_noise_ptr: int = 0):
        """One control step -> (out, u0, [StepStats]).  A step given up by the peer exchange reports
        ``exchange_timeout`` (and ``nonfinite``) on this rank at once; on a multi-rank peer exchange
        every ``agree_every``-th call is also a collective -- the ranks agree on whether any of them
        gave a step up since the last agreement (one MAX all-reduce of the sticky word) and, if so,
        resynchronise (``resync``), every rank then reporting ``exchange_timeout``.  Every rank must
        make the same calls (the control loop runs in lockstep on the ranks)."""
        if (self.world == 1 or self.mode in ("peer", "vehicles")) and not d_noise_ptr:   # one C call, as the drop-in classes step
            out, u0, st = self.engine.step(state)
        else:
            self.engine.set_state(state)
            self.step_async(d_noise_ptr)
            out, u0, st = self.engine.read_outputs()
        if self._checks_exchange():
            self._calls += 1
            if self._calls % self.agree_every == 0:
                local = any(s.exchange_timeout for s in st) or self.engine.peer_status(reports=False)[0] != 0
                if _any_rank(local, self.group, self.local):
                    self.resync()
                    for s in st:
                        s.exchange_timeout = True
                        s.nonfinite = True
        return out, u0, st

    # ------------------------------------------------------------- failure handling (peer)
    def _checks_exchange(self) -> bool:
        return self.mode == "peer" and self.world > 1

    def synchronize(self) -> bool:
        """Wait for this rank's steps.  On a multi-rank peer exchange it is a collective (and a
        barrier): the ranks agree whether any of them gave a step up since the last check -- this
        rank's sticky timeout word (any block of any step of a batch, mppi_synchronize's
        MPPI_ERR_PEER_TIMEOUT) MAX-reduced over the process group -- and if one did, every rank
        resynchronises (``resync``).  Returns True when it did (then every rank returns True)."""
        from ._capi import PeerTimeout
        local = False
        try:
            self.engine.synchronize()
        except PeerTimeout:
            local = True
        if not self._checks_exchange():
            if local:   # (one rank exchanging with itself cannot time out; a bad state all the same)
                raise RuntimeError("peer exchange timeout on a one-rank exchange")
            return False
        if not _any_rank(local, self.group, self.local):
            return False
        self.resync()
        return True

    def resync(self):
        """Collective recovery after a peer-exchange timeout (every rank calls it): every rank takes
        the warm start u_prev and step counter of the lowest rank whose warm start is not torn
        (rank 0 normally) and a fresh exchange epoch, and its exchange
        region is cleared between two barriers (no kernel writes into any region while it is
        cleared, and no rank steps before every region is clear).  Afterwards the ranks' warm starts
        are bit-identical and the exchange runs again (the sharded reduction is
        mppi.py:143-148)."""
        from ._capi import PeerTimeout
        eng = self.engine
        try:
            eng.synchronize()
        except PeerTimeout:
            pass
        dev = f"cuda:{self.local}" if dist.get_backend(self.group) == "nccl" else "cpu"
        u = torch.from_numpy(eng.get_u_prev()).to(dev)
        _, _, epoch = eng.peer_status(reports=False)
        ctl = torch.tensor([eng.get_step_counter(), epoch], dtype=torch.int64, device=dev)
        # the source: the lowest rank whose warm start is not torn (mppi_peer_info; a step's blocks
        # all update or all keep their slices unless a peer stayed silent through two bounds)
        torn = bool(eng.peer_info()[2])
        first = torch.tensor([self.world if torn else self.rank], dtype=torch.int64, device=dev)
        dist.all_reduce(first, op=dist.ReduceOp.MIN, group=self.group)
        g0 = int(first.item())
        g0 = 0 if g0 >= self.world else g0   # (every rank torn: rank 0's, as before)
        self.resync_source = g0
        src = dist.get_global_rank(self.group, g0) if self.group is not None else g0
        dist.broadcast(u, src=src, group=self.group)
        dist.broadcast(ctl, src=src, group=self.group)
        step, epoch = (int(x) for x in ctl.tolist())
        dist.barrier(group=self.group)
        eng.peer_reset(step, epoch + 1)
        dist.barrier(group=self.group)
        eng.set_u_prev(u.cpu().numpy())
        self.resyncs += 1

    def __getattr__(self, name):
        if name == "engine":
            raise AttributeError(name)
        return getattr(self.engine, name)
