"""Drop-in replacement for the reference's drone solver ``mppi_solver/drone_mppi.py``.

Same surface as ``MPPI`` at ``src/mav_mppi/scripts/mppi_solver/drone_mppi.py:7-183``:
``MPPI()``, ``set_state(x(3,), v(3,))`` (:179-183),
``compute_control_input() -> (x: torch(3,), v: torch(3,))`` on ``self.device``
(:140-176; the caller does ``xdes.to('cpu').tolist()``, drone.py:240),
``compute_weights(S)`` (:111-130) and the attributes ``n_samples, n_timestep,
dt, n_action, sigma, param_lambda, param_gamma, u_prev, u, x_prev, v_prev``.

The step runs in libmppi_hip.so.  The reference prints ``Rho`` on every step
(:123); set ``verbose=True`` to get the same line (off by default: it is I/O in
the control loop).
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
                 noise: str = "philox", seed: int = 0x5EED, verbose: bool = False, prewarm_us: int = 0):
        self.device = torch.device(f"cuda:{device or 0}" if torch.cuda.is_available() else "cpu")
        self._prewarm_us = int(prewarm_us)
        self._dev_index = device or 0
        self.n_samples = n_samples
        self.n_timestep = n_timestep
        self.dt = 0.01
        self.n_action = 3
        self.v_prev = torch.zeros(3)
        self.x_prev = torch.zeros(3)
        self.u = torch.zeros(self.n_action)
        self.sigma = torch.eye(self.n_action) * 30.0
        self.param_lambda = 0.1
        self.param_gamma = self.param_lambda * (1.0 - 0.9)
        self.target = [1.0, 2.0, 3.4]          # drone_mppi.py:141
        self._row = np.zeros(6, np.float64)   # x(3) + v(3) of the control call
        self._last_target = None               # (engine, target bytes) last written
        self.verbose = verbose
        self._noise, self._seed = noise, seed
        self._lock = threading.Lock()
        self._engine: Optional[Engine] = None
        self._u_prev_host = np.zeros((n_timestep, 3), np.float32)
        self._out_ring = OutputRing(self.device, 6)   # (x, v): one async H2D copy per call

    def _ensure_engine(self, noise: str) -> Engine:
        e = self._engine
        if e is not None and (e.cfg.noise_mode == 1) == (noise == "injected") \
                and e.K == self.n_samples and e.H == self.n_timestep:
            return e
        u = self._u_prev_host if e is None else e.get_u_prev()[0]
        if e is not None:
            e.close()
        cfg = make_config("drone", n_samples=self.n_samples, n_horizon=self.n_timestep, dt=self.dt,
                          lam=self.param_lambda, sigma=self.sigma.numpy(), noise=noise, seed=self._seed,
                          device=self._dev_index)
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
        self._u_prev_host = u.reshape(self.n_timestep, 3).copy()
        if self._engine is not None:
            self._engine.set_u_prev(self._u_prev_host)

    def set_state(self, x, v):
        """drone_mppi.py:179-183 (stored as float32 like the reference)."""
        with self._lock:
            self.x_prev = torch.tensor(np.asarray(x, np.float64), dtype=torch.float32)
            self.v_prev = torch.tensor(np.asarray(v, np.float64), dtype=torch.float32)

    def compute_control_input(self, noise: Optional[np.ndarray] = None):
        row = self._row   # x, v into one preallocated fp64 row (the engine copies it)
        with self._lock:
            row[:3] = self.x_prev.numpy()
            row[3:] = self.v_prev.numpy()
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
        t = self._out_ring.to_device(out[0, :6])
        return t[:3], t[3:6]

    def compute_weights(self, S: torch.Tensor) -> torch.Tensor:
        rho = S.min()
        scaled_S = (-1.0 / self.param_lambda) * (S - rho)
        return torch.exp(scaled_S) / torch.exp(scaled_S).sum()

    def apply_constraint(self, u: torch.Tensor) -> torch.Tensor:
        """drone_mppi.py:131-137 (unused by the reference's step)."""
        lim = torch.tensor([10.0, 10.0, 10.0], device=u.device)
        return torch.clamp(u, min=-lim, max=lim)

    def get_trajectory(self) -> np.ndarray:
        return self._engine.get_trajectory()[0]

    def get_costs(self) -> np.ndarray:
        return self._engine.get_costs()[0]
