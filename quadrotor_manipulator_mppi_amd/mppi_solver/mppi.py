"""Drop-in replacement for the reference's arm solver ``mppi_solver/mppi.py``.

Same class name, constructor (no required arguments), methods and attributes as
``MPPI`` at ``src/mav_mppi/scripts/mppi_solver/mppi.py:27-200``:

* ``update_joint(q_full(14,), v_full(13,))``  (mppi.py:196-200)
* ``compute_control_input() -> (qdes: np.ndarray(7,), vdes: np.ndarray(7,))``
  (mppi.py:122-169; fp64 arrays when the state was fp64, as the reference)
* ``compute_weights(S, _lambda)`` (mppi.py:173-193), ``check_reach`` (:95-120)
* attributes ``n_action, n_samples, n_horizon, dt, _lambda, u_prev, u, qdes,
  vdes, target_pose, base_pose, device``

The control step itself runs in libmppi_hip.so (noise, rollout, FK, cost,
softmin, SavGol, update: two gfx950 kernels); this class only stages state in
and results out.  ``update_joint`` snapshots the state under a lock -- the
reference's rospy callback thread writes ``_q/_qdot/base_pose`` with no lock
while the main loop reads them (kinova.py:106-116 vs :182).
"""
from __future__ import annotations

import threading
from typing import Optional

import numpy as np
import torch

from ..engine import Engine, host_fk, make_config
from ..robot.urdf_chain import load_chain, parse_urdf_chain
from ..utils.pose import Pose
from ._outputs import LazyU


def _is_f64(x) -> bool:
    """The dtype ``torch.tensor(x)`` would infer (mppi.py:197-200)."""
    if isinstance(x, torch.Tensor):
        return x.dtype == torch.float64
    if isinstance(x, np.ndarray):
        return x.dtype == np.float64
    return False   # Python floats -> torch default dtype float32


def _host_view(x, dtype) -> np.ndarray:
    """x as a host array of dtype without a copy where it can be (a CPU tensor's own memory;
    np.array on a tensor goes through the array protocol, ~2.5 us): the caller copies the
    slices it keeps."""
    if isinstance(x, torch.Tensor):
        if x.device.type == "cpu" and not x.requires_grad:
            a = x.numpy()
        else:
            a = x.detach().cpu().numpy()
        return a if a.dtype == dtype else a.astype(dtype)
    return np.asarray(x, dtype=dtype)


class MPPI(LazyU):
    def __init__(self, n_samples: int = 100, n_horizon: int = 32, device: Optional[int] = None,
                 noise: str = "philox", seed: int = 0x5EED, urdf_path: Optional[str] = None,
                 root_link: str = "base", end_link: str = "j2s7s300_link_7", verbose: bool = True,
                 cost_terms=(), cost_weights=None, prewarm_us: int = 0):
        """``cost_terms``: CostManager terms to switch on beyond the pose cost the
        reference runs (cost_manager.py:83-87): any of ``covar, center, joint_track,
        action, joint_limit`` (engine.COST_TERMS); ``cost_weights`` overrides their
        weights (defaults: cost_manager.py:21-43).  ``prewarm_us`` > 0: the engine's queue
        prewarm with that window (mppi_set_prewarm), for a node ticking with idle gaps such as
        kinova.py:101's rospy.Rate(100); results are unchanged."""
        self.device = torch.device(f"cuda:{device or 0}" if torch.cuda.is_available() else "cpu")
        self._dev_index = device or 0
        # mppi.py:37-42
        self.n_action = 7
        self.n_manipulator_dof = 7
        self.n_mobile_dof = 0
        self.n_samples = n_samples
        self.n_horizon = n_horizon
        self.dt = 0.01
        self._lambda = 0.1
        self._noise, self._seed = noise, seed
        self._cost_terms, self._cost_weights = cost_terms, cost_weights
        self._prewarm_us = int(prewarm_us)
        self.verbose = verbose
        self.chain = parse_urdf_chain(urdf_path, root_link, end_link) if urdf_path else load_chain()
        # mppi.py:45-58
        self._q = np.zeros(7, np.float32)
        self._qdot = np.zeros(7, np.float32)
        self.base_pose = np.zeros(7, np.float32)
        self._f64 = False
        self.u = torch.zeros(self.n_action)
        self.qdes = None
        self.vdes = None
        # mppi.py:70-72
        self.target_pose = Pose()
        self.target_pose.pose = torch.tensor([0.1029, 0.4055, 1.6498])
        self.target_pose.orientation = torch.tensor([-0.5, -0.5, 0.5, -0.5])
        self._lock = threading.Lock()
        self._engine: Optional[Engine] = None
        self._u_prev_host = np.zeros((self.n_horizon, self.n_action), np.float32)
        self.cnt = 0
        self._row = np.zeros(21, np.float64)   # base xyzquat(7) + q(7) + qdot(7)
        self._last_target = None               # (engine, target bytes) last written (_sync_target)
        self._target_views = None              # (pose tensor, quat tensor, their numpy views)

    # -------------------------------------------------------------- engine
    def _ensure_engine(self, f64: bool, noise: Optional[str] = None) -> Engine:
        noise = noise or self._noise
        e = self._engine
        if e is not None and bool(e.cfg.state_f64) == f64 and (e.cfg.noise_mode == 1) == (noise == "injected"):
            return e
        u = self._u_prev_host if e is None else e.get_u_prev()[0]
        if e is not None:
            e.close()
        cfg = make_config("arm", n_samples=self.n_samples, n_horizon=self.n_horizon, dt=self.dt,
                          lam=self._lambda, chain=self.chain, noise=noise, seed=self._seed,
                          device=self._dev_index, state_f64=f64, check_reach=True,
                          cost_terms=self._cost_terms, cost_weights=self._cost_weights)
        self._engine = Engine(cfg)
        self._engine.set_u_prev(u)
        if self._prewarm_us:
            self._engine.set_prewarm(self._prewarm_us)
        return self._engine

    @property
    def u_prev(self) -> torch.Tensor:
        if self._engine is None:
            return torch.from_numpy(self._u_prev_host.copy())
        return torch.from_numpy(self._engine.get_u_prev()[0])

    @u_prev.setter
    def u_prev(self, value):
        u = np.ascontiguousarray(torch.as_tensor(value).detach().cpu().numpy(), np.float32)
        self._u_prev_host = u.reshape(self.n_horizon, self.n_action).copy()
        if self._engine is not None:
            self._engine.set_u_prev(self._u_prev_host)

    # ------------------------------------------------------------ reference API
    def update_joint(self, q_full, v_full):
        """mppi.py:196-200: q_full = base xyzquat(7) + q(7); v_full = base twist(6) + qdot(7)."""
        f64 = _is_f64(q_full)
        q = _host_view(q_full, np.float64 if f64 else np.float32)
        v = _host_view(v_full, np.float64 if _is_f64(v_full) else np.float32)
        # fresh arrays (sliced copies), rebound under the lock: _snapshot takes references
        qn, vn, bn = q[7:].copy(), v[6:].copy(), q[:7].copy()
        with self._lock:
            self._q, self._qdot, self.base_pose = qn, vn, bn
            self._f64 = f64

    def _snapshot(self):
        # update_joint rebinds fresh arrays (never writes into the current ones), so the
        # references taken under the lock are a consistent snapshot without copies
        with self._lock:
            return self._q, self._qdot, self.base_pose, self._f64

    def _state_row(self, q, qd, base):
        row = self._row   # the engine copies it in mppi_step: one preallocated row
        row[:7] = base
        row[7:14] = q
        row[14:21] = qd
        return row

    def _sync_target(self, eng: Engine) -> None:
        """The target into the engine when it changed since the last call (the control call's
        host time: a target write rebuilds the vehicle constants through one more C call).
        The tensors' numpy views are cached per tensor object and their bytes compared, so an
        unchanged target costs ~1 us instead of two .numpy() calls and two array_equal."""
        pt, qt = self.target_pose.pose, self.target_pose.orientation
        views = self._target_views
        if views is None or views[0] is not pt or views[1] is not qt:
            views = self._target_views = (pt, qt, pt.numpy(), qt.numpy())
        key = views[2].tobytes() + views[3].tobytes()
        last = self._last_target
        if last is None or last[0] is not eng or last[1] != key:
            eng.set_target(views[2], views[3])
            self._last_target = (eng, key)

    def compute_control_input(self, noise: Optional[np.ndarray] = None):
        """mppi.py:122-169.  ``noise`` (K,H,A) switches to injected-noise mode
        (parity with the reference's torch.randn draws)."""
        q, qd, base, f64 = self._snapshot()
        eng = self._ensure_engine(f64, "injected" if noise is not None else None)
        self._sync_target(eng)
        out, u0, stats = eng.step(self._state_row(q, qd, base), noise)
        dt = np.float64 if f64 else np.float32
        self.qdes = out[0, :7].astype(dt)
        self.vdes = out[0, 7:14].astype(dt)
        self._set_u0(u0[0])   # the tensor is made on first read (LazyU)
        self.last_stats = stats[0]
        self.cnt += 1
        if stats[0].reach and self.verbose:   # mppi.py:165-167
            print("Reach !")
        return self.qdes.copy(), self.vdes.copy()

    def compute_weights(self, S: torch.Tensor, _lambda) -> torch.Tensor:
        """mppi.py:173-193 (host helper; the engine computes the same weights on device)."""
        rho = S.min()
        scaled_S = (-1.0 / _lambda) * (S - rho)
        return torch.exp(scaled_S) / torch.exp(scaled_S).sum()

    def check_reach(self, q_full=None) -> bool:
        """mppi.py:95-120: host FK at qdes, L1 position error < 0.005."""
        q, qd, base, f64 = self._snapshot()
        if self.qdes is None:
            return False
        T = host_fk(self.chain, self.qdes, base, f64)
        err = float(np.abs(T[:3, 3] - self.target_pose.pose.numpy()).sum())
        return err < 0.005

    # ------------------------------------------------------- build extras
    def get_trajectory(self) -> np.ndarray:
        """(K,H,7+16): q_samples and the EE 4x4 per (k,t) of the last step."""
        return self._engine.get_trajectory()[0]

    def get_costs(self) -> np.ndarray:
        return self._engine.get_costs()[0]
