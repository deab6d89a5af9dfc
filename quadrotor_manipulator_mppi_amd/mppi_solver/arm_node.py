"""The arm node's per-tick MPPI + computed-torque step, without ROS.

Mirrors the MPPI branch of ``controller`` in ``src/mav_mppi/scripts/kinova.py``:

* ``joint_state(position, velocity)`` = ``joint_state_callback`` (``kinova.py:106-116``):
  q (14) = base xyz + quaternion xyzw + 7 joints; v (13); the base linear velocity is
  rotated local -> world with the base rotation (``kinova.py:113-114``, as the node does
  before both the MPPI and Pinocchio see it); then ``MPPI.update_joint(q, v)``;
* ``tick()`` = one pass of the MPPI branch of ``main`` (``kinova.py:180-190``):
  ``qdes, vdes = mppi.compute_control_input()`` and
  ``torque = M[6:,6:] @ (400 (qdes - q[7:]) + 40 (-v[6:])) + nle[6:]``, with M and nle of
  the node's Pinocchio model (``kinova.py:126-131``) from the host dynamics in
  libmppi_hip.so (``robot/dynamics.py``), evaluated as one recursive Newton-Euler pass.

The joint-space warm-up trajectory and the SE3 trajectory manager of the node
(``trajManager.py``) stay out of scope: the node only feeds their output
to the same torque law.
"""
from __future__ import annotations

import threading
from typing import Optional

import numpy as np

from ..robot.dynamics import RobotDynamics
from .mppi import MPPI


def _quat_R(x, y, z, w):
    n = np.sqrt(x * x + y * y + z * z + w * w)
    x, y, z, w = x / n, y / n, z / n, w / n
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


class ArmTorqueNode:
    def __init__(self, mppi: Optional[MPPI] = None, dynamics: Optional[RobotDynamics] = None,
                 kp: float = 400.0, kd: float = 40.0):
        self.mppi = mppi if mppi is not None else MPPI()
        self.dyn = dynamics if dynamics is not None else RobotDynamics()
        self.kp, self.kd = kp, kd
        self.q: Optional[np.ndarray] = None
        self.v: Optional[np.ndarray] = None
        self._lock = threading.Lock()

    def joint_state(self, position, velocity):
        """kinova.py:106-116."""
        q = np.array(position, np.float64)
        v = np.array(velocity, np.float64)
        v[:3] = _quat_R(*q[3:7]) @ v[:3]
        with self._lock:
            self.q, self.v = q, v
        self.mppi.update_joint(q, v)

    def tick(self, noise: Optional[np.ndarray] = None):
        """One MPPI-branch tick: returns (torque (7,), qdes (7,), vdes (7,))."""
        with self._lock:
            if self.q is None:
                return None
            q, v = self.q.copy(), self.v.copy()
        qdes, vdes = self.mppi.compute_control_input(noise)
        tau = self.dyn.computed_torque(q, v, np.asarray(qdes, np.float64), self.kp, self.kd)
        return tau, qdes, vdes
