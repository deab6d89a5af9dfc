"""Host rigid-body dynamics of the arm node (the Pinocchio calls of ``kinova.py:54-184``).

``RobotDynamics`` wraps ``mppi_dyn_*`` in libmppi_hip.so (``include/mppi_hip.h``):

* ``compute_all_terms(q, v) -> (M, nle)``: what the node reads from
  ``pin.computeAllTerms(model, data, q, v)``: ``data.M`` (nv x nv) and ``data.nle``
  (``kinova.py:126, 131``);
* ``computed_torque(q, v, qdes, kp=400, kd=40)``: the node's MPPI-branch law
  ``M[6:,6:] @ (kp (qdes - q[7:]) - kd v[6:]) + nle[6:]`` (``kinova.py:184``), as one
  recursive Newton-Euler pass;
* ``rnea(q, v, a)``: inverse dynamics.

The model defaults to ``full_robot_floating2.urdf`` (the node's Pinocchio URDF), shipped as
``robot/full_robot_floating2.json`` (``robot/urdf_tree.py``).  Conventions are
Pinocchio's free-flyer: q = base xyz + quaternion xyzw + 7 joints (14), v = base linear +
angular velocity in the base frame + joint rates (13).  Parity with Pinocchio is
unpinned (Pinocchio is not installed); ``tests/test_dynamics_cpu.py`` checks these terms
against an independent numpy Lagrangian restatement in the oracle.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence

import numpy as np

from .. import _capi as capi
from .urdf_tree import load_tree


def link_table(tree: Sequence[Dict]):
    arr = (capi.Link * len(tree))()
    for i, l in enumerate(tree):
        L = arr[i]
        L.parent, L.type = int(l["parent"]), int(l["type"])
        for d in range(3):
            L.xyz[d], L.rpy[d], L.axis[d], L.com[d] = l["xyz"][d], l["rpy"][d], l["axis"][d], l["com"][d]
        L.mass = float(l["mass"])
        for k in range(9):
            L.inertia[k] = float(l["inertia"][k])
    return arr


class RobotDynamics:
    def __init__(self, tree: Optional[List[Dict]] = None, gravity: float = 9.81):
        self._L = capi.lib()
        tree = tree if tree is not None else load_tree()
        links = link_table(tree)
        h = C.c_void_p()
        capi.check(self._L.mppi_dyn_create(links, len(tree), gravity, C.byref(h)), "mppi_dyn_create")
        self._h = h
        nq, nv, nb = C.c_int32(), C.c_int32(), C.c_int32()
        self._L.mppi_dyn_dims(h, C.byref(nq), C.byref(nv), C.byref(nb))
        self.nq, self.nv, self.n_bodies = nq.value, nv.value, nb.value

    def close(self):
        if getattr(self, "_h", None):
            self._L.mppi_dyn_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _qv(self, q, v):
        q = np.ascontiguousarray(q, np.float64).reshape(self.nq)
        v = np.ascontiguousarray(v, np.float64).reshape(self.nv)
        return q, v

    def compute_all_terms(self, q, v):
        q, v = self._qv(q, v)
        M = np.empty((self.nv, self.nv), np.float64)
        nle = np.empty(self.nv, np.float64)
        capi.check(self._L.mppi_dyn_terms(self._h, capi.dptr(q), capi.dptr(v), capi.dptr(M), capi.dptr(nle)),
                   "mppi_dyn_terms")
        return M, nle

    def rnea(self, q, v, a=None):
        q, v = self._qv(q, v)
        aa = None if a is None else np.ascontiguousarray(a, np.float64).reshape(self.nv)
        tau = np.empty(self.nv, np.float64)
        capi.check(self._L.mppi_dyn_rnea(self._h, capi.dptr(q), capi.dptr(v), capi.dptr(aa), capi.dptr(tau)),
                   "mppi_dyn_rnea")
        return tau

    def computed_torque(self, q, v, qdes, kp: float = 400.0, kd: float = 40.0, first_v: int = 6):
        q, v = self._qv(q, v)
        qd = np.ascontiguousarray(qdes, np.float64).reshape(self.nv - first_v)
        tau = np.empty(self.nv - first_v, np.float64)
        capi.check(self._L.mppi_computed_torque(self._h, capi.dptr(q), capi.dptr(v), capi.dptr(qd), kp, kd,
                                                first_v, capi.dptr(tau)), "mppi_computed_torque")
        return tau
