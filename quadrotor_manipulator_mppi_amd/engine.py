"""Python handle on one libmppi_hip.so engine.

Thin host-side plumbing over the C-ABI (``include/mppi_hip.h``): it fills the
config struct, keeps numpy staging arrays, and turns status codes into
exceptions.  All arithmetic of the control step runs in the HIP kernels.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _capi as capi
from .robot.urdf_chain import load_chain

MODELS = {"drone": capi.MODEL_DRONE, "arm": capi.MODEL_ARM, "wholebody": capi.MODEL_WHOLEBODY,
          "quadrotor": capi.MODEL_QUADROTOR}
QUAD_FIELDS = ("quad_mass", "quad_kd", "quad_gravity")
JOINT_TYPES = {"fixed": capi.JOINT_FIXED, "revolute": capi.JOINT_REVOLUTE,
               "continuous": capi.JOINT_REVOLUTE, "prismatic": capi.JOINT_PRISMATIC}


@dataclass(slots=True)
class StepStats:
    rho: float
    eta: float
    ess: float
    nonfinite: bool
    reach: bool
    exchange_timeout: bool = False   # a peer-exchange step gave up waiting for a rank (u_prev kept)


def fill_joints(cfg: capi.Config, chain: Sequence[Dict]) -> None:
    if len(chain) > capi.MAX_JOINTS:
        raise ValueError(f"chain has {len(chain)} joints (max {capi.MAX_JOINTS})")
    cfg.n_joints = len(chain)
    for i, j in enumerate(chain):
        J = cfg.joints[i]
        J.type = JOINT_TYPES.get(j["type"], capi.JOINT_FIXED)
        J.q_index = int(j.get("q_index", -1))
        for d in range(3):
            J.xyz[d] = float(j["xyz"][d])
            J.rpy[d] = float(j["rpy"][d])
        ax = j.get("axis")
        J.has_axis = 0 if ax is None else 1
        if ax is not None:
            for d in range(3):
                J.axis[d] = float(ax[d])


def make_config(model: str = "arm", n_samples: Optional[int] = None, n_horizon: Optional[int] = None,
                n_vehicles: int = 1, n_action: Optional[int] = None, dt: float = 0.01, lam: float = 0.1,
                sigma=None, weights: Optional[Sequence[float]] = None, chain=None,
                savgol_window: Optional[int] = None, savgol_order: int = 2, noise: str = "philox",
                seed: int = 0x5EED, device: int = 0, shard_rank: int = 0, shard_count: int = 1,
                state_f64: Optional[bool] = None, store_trajectory: bool = True, store_noise: bool = False,
                check_reach: Optional[bool] = None, reach_tol: float = 0.005, blocks_per_vehicle: int = 0,
                block_threads: int = 0, cost_terms=0, cost_weights: Optional[Dict[str, float]] = None,
                quad: Optional[Dict] = None, vehicle_offset: int = 0) -> capi.Config:
    """``cost_terms``: bitmask of ``capi.COST_*`` or an iterable of names among
    ``covar, center, joint_track, action, joint_limit`` -- the CostManager terms the
    reference ships disabled (cost_manager.py:83-87).  ``cost_weights`` overrides
    ``w_covar, cost_alpha, cost_gamma, w_center, w_joint_track, w_action,
    joint_limit_penalty``.  ``quad`` overrides the QUADROTOR rigid body: ``quad_mass``,
    ``quad_inertia`` (3,), ``quad_kd``, ``quad_gravity``, ``quad_literal_jinv``.  ``vehicle_offset``:
    the fleet-wide index of vehicle 0 (vehicle sharding: the device noise is keyed by it)."""
    L = capi.lib()
    cfg = capi.Config()
    L.mppi_config_default(C.byref(cfg), MODELS[model])
    cfg.n_vehicles = n_vehicles
    if n_samples is not None:
        cfg.n_samples = n_samples
    if n_horizon is not None:
        cfg.n_horizon = n_horizon
    if n_action is not None:
        cfg.n_action = n_action
    cfg.dt, cfg.lambda_ = dt, lam
    A = cfg.n_action
    if sigma is not None:
        s = np.asarray(sigma, np.float32)
        if s.ndim == 1:
            s = np.diag(s)
        if s.shape != (A, A):
            raise ValueError(f"sigma must be ({A},{A})")
        for i in range(A * A):
            cfg.sigma[i] = float(s.reshape(-1)[i])
    if weights is not None:
        cfg.w_stage_pos, cfg.w_stage_ori, cfg.w_term_pos, cfg.w_term_ori = map(float, weights)
    if model in ("arm", "wholebody"):
        fill_joints(cfg, chain if chain is not None else load_chain())
    for k, val in (quad or {}).items():
        if k == "quad_inertia":
            for d in range(3):
                cfg.quad_inertia[d] = float(val[d])
        elif k in QUAD_FIELDS:
            setattr(cfg, k, float(val))
        elif k == "quad_literal_jinv":   # drone_mppi.py:73-76 taken literally (inv(J) for t >= 1)
            cfg.quad_literal_jinv = 1 if val else 0
        else:
            raise ValueError(f"unknown quadrotor parameter {k!r}")
    if savgol_window is not None:
        cfg.savgol_window = savgol_window
    cfg.savgol_order = savgol_order
    cfg.noise_mode = capi.NOISE_INJECTED if noise == "injected" else capi.NOISE_PHILOX
    cfg.seed = seed
    cfg.device = device
    cfg.shard_rank, cfg.shard_count = shard_rank, shard_count
    cfg.vehicle_offset = vehicle_offset
    if state_f64 is not None:
        cfg.state_f64 = int(state_f64)
    cfg.store_trajectory = int(store_trajectory)
    cfg.store_noise = int(store_noise)
    if check_reach is not None:
        cfg.check_reach = int(check_reach)
    cfg.reach_tol = reach_tol
    cfg.blocks_per_vehicle = blocks_per_vehicle
    cfg.block_threads = block_threads
    cfg.cost_terms = cost_term_bits(cost_terms)
    for k, val in (cost_weights or {}).items():
        if k not in COST_WEIGHT_FIELDS:
            raise ValueError(f"unknown cost weight {k!r}")
        setattr(cfg, k, float(val))
    return cfg


COST_TERMS = {"covar": capi.COST_COVAR, "center": capi.COST_CENTER, "joint_track": capi.COST_JOINT_TRACK,
              "action": capi.COST_ACTION, "joint_limit": capi.COST_JOINT_LIMIT}
COST_WEIGHT_FIELDS = ("w_covar", "cost_alpha", "cost_gamma", "w_center", "w_joint_track", "w_action",
                      "joint_limit_penalty")


def cost_term_bits(terms) -> int:
    if isinstance(terms, int):
        return terms
    bits = 0
    for t in terms:
        if t not in COST_TERMS:
            raise ValueError(f"unknown cost term {t!r} (known: {sorted(COST_TERMS)})")
        bits |= COST_TERMS[t]
    return bits


class Engine:
    """One MPPI engine on one GPU (V vehicles x K samples x H steps)."""

    def __init__(self, cfg: Optional[capi.Config] = None, **kw):
        self._L = capi.lib()
        self.cfg = cfg if cfg is not None else make_config(**kw)
        h = C.c_void_p()
        capi.check(self._L.mppi_create(C.byref(self.cfg), C.byref(h)), "mppi_create")
        self._h = h
        c = self.cfg
        self.V, self.K, self.H, self.A = c.n_vehicles, c.n_samples, c.n_horizon, c.n_action
        self.state_dim = self._L.mppi_state_dim(C.byref(c))
        self.out_dim = self._L.mppi_output_dim(C.byref(c))
        self.traj_channels = self._L.mppi_traj_channels(C.byref(c))
        self._out = np.zeros((self.V, self.out_dim), np.float64)
        self._u0 = np.zeros((self.V, self.A), np.float32)
        self._stats = (capi.Stats * self.V)()
        # persistent host buffers with their ctypes pointers made once: ndarray.ctypes.data_as
        # costs ~3-4 us per call, several of them per control call (the latency path)
        self._state_buf = np.zeros((self.V, self.state_dim), np.float64)
        self._tgt_pos = np.zeros(3, np.float32)
        self._tgt_quat = np.zeros(4, np.float32)
        self._p_out, self._p_u0 = capi.dptr(self._out), capi.fptr(self._u0)
        self._p_state = capi.dptr(self._state_buf)
        self._state_flat = self._state_buf.reshape(-1)   # a view: the per-call fast path below
        self._p_tpos, self._p_tquat = capi.fptr(self._tgt_pos), capi.fptr(self._tgt_quat)

    # ------------------------------------------------------------------ admin
    def close(self):
        if getattr(self, "_h", None):
            self._L.mppi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------- native collective
    @staticmethod
    def comm_unique_id() -> bytes:
        """A fresh RCCL unique id (rank 0 makes it; the caller broadcasts it)."""
        buf = (C.c_uint8 * capi.COMM_ID_BYTES)()
        capi.check(capi.lib().mppi_comm_unique_id(buf), "comm_unique_id")
        return bytes(buf)

    @staticmethod
    def comm_available() -> Optional[str]:
        """None if RCCL is loadable with every entry point the engine binds, else why not."""
        L = capi.lib()
        if L.mppi_comm_available() == capi.OK:
            return None
        return L.mppi_last_error().decode(errors="replace")

    def comm_init(self, uid: bytes, timeout_ms: int = 0):
        """Join the shard communicator (collective over cfg.shard_count ranks).  Non-blocking
        init polled until ``timeout_ms`` (0: MPPI_COMM_INIT_TIMEOUT_MS, default 60 s); raises
        MPPIError(ERR_COMM) when the peers do not join in time."""
        if len(uid) != capi.COMM_ID_BYTES:
            raise ValueError("comm id must be %d bytes" % capi.COMM_ID_BYTES)
        buf = (C.c_uint8 * capi.COMM_ID_BYTES).from_buffer_copy(uid)
        capi.check(self._L.mppi_comm_init_ex(self._h, buf, int(timeout_ms)), "comm_init")

    def comm_info(self):
        """(nranks, rank) as the RCCL communicator itself reports them."""
        n, r = C.c_int32(), C.c_int32()
        capi.check(self._L.mppi_comm_info(self._h, C.byref(n), C.byref(r)), "comm_info")
        return n.value, r.value

    def exchange(self):
        capi.check(self._L.mppi_exchange(self._h), "exchange")

    def peer_open(self) -> bytes:
        """Open this rank's peer-exchange region; returns its IPC handle (mppi_peer_open)."""
        buf = (C.c_uint8 * capi.PEER_HANDLE_BYTES)()
        capi.check(self._L.mppi_peer_open(self._h, buf), "peer_open")
        return bytes(buf)

    def peer_connect(self, handles):
        """Map every rank's region (handles in rank order, this rank's own included)."""
        blob = b"".join(bytes(h) for h in handles)
        if any(len(h) != capi.PEER_HANDLE_BYTES for h in handles):
            raise ValueError("peer handles must be %d bytes each" % capi.PEER_HANDLE_BYTES)
        buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        capi.check(self._L.mppi_peer_connect(self._h, buf), "peer_connect")

    def peer_region(self) -> int:
        """This engine's exchange region as a device address (after peer_open; mppi_peer_region)."""
        x = C.c_uint64(0)
        capi.check(self._L.mppi_peer_region(self._h, C.byref(x)), "peer_region")
        return int(x.value)

    def peer_connect_ptrs(self, addresses):
        """In-process ranks: every rank's region address in rank order (mppi_peer_connect_ptrs)."""
        buf = (C.c_uint64 * len(addresses))(*[int(a) for a in addresses])
        capi.check(self._L.mppi_peer_connect_ptrs(self._h, buf), "peer_connect_ptrs")

    def peer_probe(self, phase: int):
        """Connection check (collective): phase 0 on every rank, a barrier, then phase 1."""
        capi.check(self._L.mppi_peer_probe(self._h, int(phase)), "peer_probe")

    def peer_status(self, reports: bool = True):
        """(sticky, reports, epoch) of the peer exchange (mppi_peer_status): ``sticky`` = this
        engine's timeout word (the given-up step's tag, 0 = none; host memory), ``reports`` = the
        timeout reports in this rank's region (one per rank, 0 = none; a device read, None when
        ``reports`` is False), ``epoch`` = the exchange epoch of the tags."""
        st, ep = C.c_uint32(0), C.c_uint32(0)
        rep = (C.c_uint64 * capi.MAX_PEERS)() if reports else None
        capi.check(self._L.mppi_peer_status(self._h, C.byref(st), rep, C.byref(ep)), "peer_status")
        return st.value, (list(rep) if reports else None), ep.value

    def peer_info(self):
        """(connected, rank, torn) of the peer exchange (mppi_peer_info): ``connected`` = the ranks whose
        word reached this rank's region in the connection probe's kernel phase, ``rank`` = this
        engine's shard rank, ``torn`` = the step tag of a step this rank's warm start came out of torn
        (some slices updated, others kept; 0 = none)."""
        n, r, t = C.c_int32(0), C.c_int32(0), C.c_uint32(0)
        capi.check(self._L.mppi_peer_info(self._h, C.byref(n), C.byref(r), C.byref(t)), "peer_info")
        return n.value, r.value, t.value

    def peer_reset(self, step: int, epoch: int):
        """Clear this rank's region and sticky word, take the agreed step counter and epoch
        (collective recovery: every rank synchronised, a barrier before and after)."""
        capi.check(self._L.mppi_peer_reset(self._h, step & 0xFFFFFFFF, epoch & 0xFFFFFFFF), "peer_reset")

    def get_step_counter(self) -> int:
        x = C.c_uint32(0)
        capi.check(self._L.mppi_get_step_counter(self._h, C.byref(x)), "get_step_counter")
        return x.value

    def set_stream(self, stream_handle: int):
        capi.check(self._L.mppi_set_stream(self._h, C.c_void_p(stream_handle)), "set_stream")

    def set_target(self, pos, quat=None, vehicle: int = 0):
        self._tgt_pos[:] = np.reshape(pos, 3)
        if quat is not None:
            self._tgt_quat[:] = np.reshape(quat, 4)
        capi.check(self._L.mppi_set_target(self._h, vehicle, self._p_tpos,
                                           None if quat is None else self._p_tquat), "set_target")

    def set_joint_trajectory(self, traj=None, vehicle: int = 0):
        """Joint tracking target (H, nq) of the joint_track cost term (None = zeros)."""
        t = None if traj is None else np.ascontiguousarray(traj, np.float32).reshape(self.H, -1)
        capi.check(self._L.mppi_set_joint_trajectory(self._h, vehicle, capi.fptr(t)), "set_joint_trajectory")

    def set_u_prev(self, u):
        u = np.ascontiguousarray(u, np.float32).reshape(self.V, self.H, self.A)
        capi.check(self._L.mppi_set_u_prev(self._h, capi.fptr(u)), "set_u_prev")

    def get_u_prev(self) -> np.ndarray:
        u = np.empty((self.V, self.H, self.A), np.float32)
        capi.check(self._L.mppi_get_u_prev(self._h, capi.fptr(u)), "get_u_prev")
        return u

    def set_state(self, state):
        self._state_buf[...] = np.reshape(state, (self.V, self.state_dim))
        capi.check(self._L.mppi_set_state(self._h, self._p_state), "set_state")

    def set_step_counter(self, step: int):
        capi.check(self._L.mppi_set_step_counter(self._h, step & 0xFFFFFFFF), "set_step_counter")

    # ------------------------------------------------------------------- step
    def step(self, state=None, noise=None):
        """One control step: returns (out (V,out_dim) float64, u0 (V,A), [StepStats])."""
        ps = None
        if state is not None:
            # (the control call's host overhead: a flat ndarray of the right size is copied
            #  with one slice assignment, ~1.6 us less than the reshape + broadcast)
            if type(state) is np.ndarray and state.shape == self._state_flat.shape:
                self._state_flat[:] = state
            else:
                self._state_buf[...] = np.reshape(state, (self.V, self.state_dim))
            ps = self._p_state
        n = None if noise is None else np.ascontiguousarray(noise, np.float32).reshape(
            self.V, self.K, self.H, self.A)
        capi.check(self._L.mppi_step(self._h, ps, capi.fptr(n), self._p_out, self._p_u0, self._stats),
                   "mppi_step")
        return self._out.copy(), self._u0.copy(), self.stats()

    def rollout(self, d_noise_ptr: int = 0):
        capi.check(self._L.mppi_rollout(self._h, C.c_void_p(d_noise_ptr or None)), "rollout")

    def finalize(self):
        capi.check(self._L.mppi_finalize(self._h), "finalize")

    def read_outputs(self):
        capi.check(self._L.mppi_read_outputs(self._h, self._p_out, self._p_u0, self._stats), "read_outputs")
        return self._out.copy(), self._u0.copy(), self.stats()

    def run_steps(self, n: int):
        """n asynchronous back-to-back control steps (no host sync)."""
        capi.check(self._L.mppi_run_steps(self._h, n), "run_steps")

    def synchronize(self):
        capi.check(self._L.mppi_synchronize(self._h), "synchronize")

    def set_prewarm(self, window_us: int):
        """Warm the native queue before each predicted control call (mppi_set_prewarm): for a node
        that ticks with idle gaps (100 Hz).  ``window_us`` 50 .. 5000; 0 turns it off."""
        capi.check(self._L.mppi_set_prewarm(self._h, int(window_us)), "set_prewarm")

    def prewarm(self):
        """(window_us, queue touches so far) of the prewarm."""
        us, n = C.c_int32(), C.c_int64()
        capi.check(self._L.mppi_get_prewarm(self._h, C.byref(us), C.byref(n)), "get_prewarm")
        return us.value, n.value

    def dispatch_info(self) -> str:
        """How the last run_steps / step were dispatched: "<aql | hip: why>; calls: <aql | hip>"."""
        buf = C.create_string_buffer(256)
        capi.check(self._L.mppi_dispatch_info(self._h, buf, len(buf)), "dispatch_info")
        return buf.value.decode(errors="replace")

    def stats(self) -> List[StepStats]:
        st = self._stats
        return [StepStats(s.rho, s.eta, s.ess, bool(s.nonfinite), bool(s.reach), s.nonfinite == 2)
                for s in ((st[0],) if self.V == 1 else st)]

    # -------------------------------------------------------------- exchange
    def exchange_slot_floats(self) -> int:
        n = C.c_int64()
        capi.check(self._L.mppi_exchange_slot_floats(self._h, C.byref(n)), "exchange_slot_floats")
        return n.value

    def bind_exchange(self, d_ptr: int):
        capi.check(self._L.mppi_bind_exchange(self._h, C.c_void_p(d_ptr)), "bind_exchange")

    # -------------------------------------------------------------- readback
    def get_costs(self) -> np.ndarray:
        S = np.empty((self.V, self.K), np.float32)
        capi.check(self._L.mppi_get_costs(self._h, capi.fptr(S)), "get_costs")
        return S

    def get_weights(self) -> np.ndarray:
        w = np.empty((self.V, self.K), np.float32)
        capi.check(self._L.mppi_get_weights(self._h, capi.fptr(w)), "get_weights")
        return w

    def get_noise(self) -> np.ndarray:
        e = np.empty((self.V, self.K, self.H, self.A), np.float32)
        capi.check(self._L.mppi_get_noise(self._h, capi.fptr(e)), "get_noise")
        return e

    def get_trajectory(self) -> np.ndarray:
        t = np.empty((self.V, self.K, self.H, self.traj_channels), np.float32)
        capi.check(self._L.mppi_get_trajectory(self._h, capi.fptr(t)), "get_trajectory")
        return t

    def get_weighted_noise(self):
        raw = np.empty((self.V, self.H, self.A), np.float32)
        sm = np.empty_like(raw)
        capi.check(self._L.mppi_get_weighted_noise(self._h, capi.fptr(raw), capi.fptr(sm)), "get_weighted_noise")
        return raw, sm

    # ---------------------------------------------------------------- timing
    def enable_timing(self, on: bool = True):
        capi.check(self._L.mppi_enable_timing(self._h, int(on)), "enable_timing")

    def timing(self):
        r, f = C.c_double(), C.c_double()
        rn, fn = C.c_int64(), C.c_int64()
        capi.check(self._L.mppi_get_timing(self._h, C.byref(r), C.byref(f), C.byref(rn), C.byref(fn)), "timing")
        return {"rollout_ms_total": r.value, "finalize_ms_total": f.value,
                "n_rollout": rn.value, "n_finalize": fn.value}

    def kernel_timing(self, n: int = 200):
        """(rollout_us, finalize_us): average device time per launch, launched back to back."""
        r, f = C.c_double(), C.c_double()
        capi.check(self._L.mppi_kernel_timing(self._h, n, C.byref(r), C.byref(f)), "kernel_timing")
        return r.value, f.value

    def kernel_timing_ex(self, n: int = 200):
        """(rollout_us, finalize_us, pair_us): back-to-back averages of each kernel, and of
        (rollout, finalize) pairs as a control step runs them.  Also on a shard."""
        r, f, pr = C.c_double(), C.c_double(), C.c_double()
        capi.check(self._L.mppi_kernel_timing_ex(self._h, n, C.byref(r), C.byref(f), C.byref(pr)),
                   "kernel_timing_ex")
        return r.value, f.value, pr.value

    def exchange_timing(self, n: int = 100) -> float:
        """Average all-reduce time (us) of the engine's RCCL communicator (collective)."""
        us = C.c_double()
        capi.check(self._L.mppi_exchange_timing(self._h, n, C.byref(us)), "exchange_timing")
        return us.value

    def rollout_bytes(self) -> int:
        return int(self._L.mppi_rollout_bytes(C.byref(self.cfg)))


def philox_normals(seed: int, step: int, vehicle: int, k0: int, K: int, H: int, A: int, device: int = 0):
    L = capi.lib()
    z = np.empty((K, H, A), np.float32)
    raw = np.empty((K, H, L.mppi_philox_words(A)), np.uint32)   # the words in consumption order
    capi.check(L.mppi_philox_normals(seed, step, vehicle, k0, K, H, A, device, capi.fptr(z),
                                     raw.ctypes.data_as(C.POINTER(C.c_uint32))), "philox_normals")
    return raw, z


def host_fk(chain, q, xyzquat, f64: bool = True) -> np.ndarray:
    """Single-configuration FK on the host (the check_reach path)."""
    L = capi.lib()
    cfg = capi.Config()
    fill_joints(cfg, chain)
    qq = np.ascontiguousarray(q, np.float64)
    b = np.ascontiguousarray(xyzquat, np.float64)
    T = np.empty(16, np.float32)
    capi.check(L.mppi_host_fk(cfg.joints, cfg.n_joints, capi.dptr(qq), capi.dptr(b), int(f64),
                              capi.fptr(T)), "host_fk")
    return T.reshape(4, 4)
