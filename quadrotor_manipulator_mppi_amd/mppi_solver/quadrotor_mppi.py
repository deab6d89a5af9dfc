"""6-DoF rigid-body quadrotor MPPI, shaped like the drone solver.

The reference ships this controller only as the commented-out ``predict_trajectory``
of ``src/mav_mppi/scripts/mppi_solver/drone_mppi.py:57-83`` (thrust along body z plus
body torques, Euler-angle attitude; J and R from ``drone.py:114-154``; m and I from
``aerial_manipulation/urdf/drone.urdf:15-16``).  This class gives it the drone
solver's surface: ``MPPI()``, ``set_state(x, v)`` with x = (xyz, rpy) and
v = (world velocity, body rates), and ``compute_control_input() -> (x_des, v_des)``
as torch (6,) tensors on ``self.device``: the model's first step under the new u[0].
The action is (thrust [N], tau_x, tau_y, tau_z [N m]); the warm start begins at
hover thrust m*g.  Parity is unpinned (no reference output exists): the GPU path is
checked against the torch restatement ``oracle.mppi_oracle.quad_step``.
"""
from __future__ import annotations

import threading
from typing import Optional

import numpy as np
import torch

from ..engine import Engine, make_config
from ._outputs import LazyU, OutputRing


class MPPI(LazyU):
    def __init__(self, n_samples: int = 1000, n_timestep: int = 32, device: Optional[int] = None,
                 noise: str = "philox", seed: int = 0x5EED, mass: float = 14.7,
                 inertia=(1.57, 3.93, 2.59), kd: float = 0.0, gravity: float = 9.81, verbose: bool = False, prewarm_us: int = 0):
        self.device = torch.device(f"cuda:{device or 0}" if torch.cuda.is_available() else "cpu")
        self._out_ring = OutputRing(self.device, 12)   # (x_des, v_des): one async H2D copy per call
        self._prewarm_us = int(prewarm_us)
        self._dev_index = device or 0
        self.n_samples = n_samples
        self.n_timestep = n_timestep
        self.dt = 0.01
        self.n_action = 4
        self.x_prev = torch.zeros(6)
        self.v_prev = torch.zeros(6)
        self.u = torch.zeros(self.n_action)
        self.sigma = torch.diag(torch.tensor([30.0, 1.0, 1.0, 1.0]))
        self.param_lambda = 0.1
        self.target = [1.0, 2.0, 3.4]          # drone_mppi.py:141
        self._row = np.zeros(12, np.float64)   # x(6) + v(6) of the control call
        self._last_target = None               # (engine, target bytes) last written
        self.params = dict(quad_mass=mass, quad_inertia=tuple(inertia), quad_kd=kd, quad_gravity=gravity)
        self.verbose = verbose
        self._noise, self._seed = noise, seed
        self._lock = threading.Lock()
        self._engine: Optional[Engine] = None
        self._u_prev_host = np.zeros((n_timestep, 4), np.float32)
        self._u_prev_host[:, 0] = np.float32(mass * gravity)   # hover thrust

    def _ensure_engine(self, noise: str) -> Engine:
        e = self._engine
        if e is not None and (e.cfg.noise_mode == 1) == (noise == "injected") \
                and e.K == self.n_samples and e.H == self.n_timestep:
            return e
        u = self._u_prev_host if e is None else e.get_u_prev()[0]
        if e is not None:
            e.close()
        cfg = make_config("quadrotor", n_samples=self.n_samples, n_horizon=self.n_timestep, dt=self.dt,
                          lam=self.param_lambda, sigma=self.sigma.numpy(), noise=noise, seed=self._seed,
                          device=self._dev_index, quad=self.params)
        self._engine = Engine(cfg)
        self._engine.set_u_prev(u)
        if self._prewarm_us:   # (mppi_set_prewarm: for a loop ticking with idle gaps)
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
        self._u_prev_host = u.reshape(self.n_timestep, 4).copy()
        if self._engine is not None:
            self._engine.set_u_prev(self._u_prev_host)

    def set_state(self, x, v):
        """x = (xyz, rpy), v = (world velocity, body rates); float32 like drone_mppi.py:179-183."""
        with self._lock:
            self.x_prev = torch.tensor(np.asarray(x, np.float64).reshape(6), dtype=torch.float32)
            self.v_prev = torch.tensor(np.asarray(v, np.float64).reshape(6), dtype=torch.float32)

    def compute_control_input(self, noise: Optional[np.ndarray] = None):
        row = self._row   # x, v into one preallocated fp64 row (the engine copies it)
        with self._lock:
            row[:6] = self.x_prev.numpy()
            row[6:] = self.v_prev.numpy()
        eng = self._ensure_engine("injected" if noise is not None else self._noise)
        # the target into the engine only when it changed (a target write rebuilds the
        # vehicle constants through one more C call)
        tgt = np.asarray(self.target, np.float32)
        key = tgt.tobytes()
        last = self._last_target
        if last is None or last[0] is not eng or last[1] != key:
            eng.set_target(tgt)
            self._last_target = (eng, key)
        out, u0, stats = eng.step(row, noise)
        self._set_u0(u0[0])   # the tensor is made on first read (LazyU)
        self.last_stats = stats[0]
        if self.verbose:
            print("Rho :", torch.tensor(stats[0].rho))
        t = self._out_ring.to_device(out[0, :12])   # one async H2D copy per call
        xo, vo = t[:6], t[6:12]
        return xo, vo

    def compute_weights(self, S: torch.Tensor) -> torch.Tensor:
        rho = S.min()
        scaled_S = (-1.0 / self.param_lambda) * (S - rho)
        return torch.exp(scaled_S) / torch.exp(scaled_S).sum()

    def get_trajectory(self) -> np.ndarray:
        """(K, H, 6): xyz, rpy per sample and step (the commented loop's trajectory)."""
        return self._engine.get_trajectory()[0]

    def get_costs(self) -> np.ndarray:
        return self._engine.get_costs()[0]
