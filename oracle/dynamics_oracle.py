"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the arm node's Pinocchio terms.

PARITY UNPINNED: the reference gets M and nle from Pinocchio
(``pin.computeAllTerms``, ``kinova.py:126``), which is not installed here and has no
committed outputs in the reference.  This module is an independent formulation used to
check the C++ recursive Newton-Euler (``csrc/mppi_dynamics.cpp``): per-link geometric
Jacobians in the world frame and the Lagrangian

    M(q)      = sum_i m_i Jv_i^T Jv_i + Jw_i^T I_i Jw_i
    g(q)      = sum_i m_i Jv_i^T (0, 0, g)
    nle_j     = (Mdot v)_j - 1/2 d(v^T M v)/dq_j + g_j       (rows of true coordinates)

with Pinocchio's free-flyer conventions (q = xyz + quaternion xyzw + joints; v = base
linear + angular velocity in the base frame + joint rates).  Mdot and d/dq_j are central
differences.  Only ``tests/`` imports it.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np


def _rpy(r, p, y):
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    return np.array([[cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr],
                     [sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr],
                     [-sp, cp * sr, cp * cr]])


def _axis_angle(a, q):
    a = np.asarray(a, float) / np.linalg.norm(a)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(q) * K + (1 - np.cos(q)) * K @ K


def _quat(qx, qy, qz, qw):
    n = np.sqrt(qx * qx + qy * qy + qz * qz + qw * qw)
    x, y, z, w = qx / n, qy / n, qz / n, qw / n
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


class TreeModel:
    """Floating-base tree from ``robot/urdf_tree.py`` entries (no fixed-link merging:
    every link is kept with its own Jacobian)."""

    def __init__(self, tree: Sequence[Dict], gravity: float = 9.81):
        self.tree = list(tree)
        self.g = gravity
        self.jidx = {}
        n = 0
        for i, l in enumerate(self.tree):
            if l["type"] in (1, 2):
                self.jidx[i] = n
                n += 1
        self.nj = n
        self.nq, self.nv = 7 + n, 6 + n

    def frames(self, q):
        """World rotation/origin of every link frame, and of every joint frame (for axes)."""
        R, p, jz, jo = [], [], {}, {}
        for i, l in enumerate(self.tree):
            if l["type"] == 3:
                Ri, pi = _quat(*q[3:7]), np.asarray(q[:3], float)
            else:
                Rp, pp = R[l["parent"]], p[l["parent"]]
                Ro = Rp @ _rpy(*l["rpy"])
                po = pp + Rp @ np.asarray(l["xyz"], float)
                if l["type"] == 1:
                    ax = np.asarray(l["axis"], float) / np.linalg.norm(l["axis"])
                    jz[i], jo[i] = Ro @ ax, po
                    Ri, pi = Ro @ _axis_angle(ax, q[7 + self.jidx[i]]), po
                elif l["type"] == 2:
                    ax = np.asarray(l["axis"], float) / np.linalg.norm(l["axis"])
                    jz[i], jo[i] = Ro @ ax, po
                    Ri, pi = Ro, po + Ro @ ax * q[7 + self.jidx[i]]
                else:
                    Ri, pi = Ro, po
            R.append(Ri)
            p.append(pi)
        return R, p, jz, jo

    def _ancestors(self, i):
        out = []
        while i >= 0:
            out.append(i)
            i = self.tree[i]["parent"]
        return out

    def jacobians(self, q):
        R, p, jz, jo = self.frames(q)
        Rb, pb = R[0], p[0]
        out = []
        for i, l in enumerate(self.tree):
            c = p[i] + R[i] @ np.asarray(l["com"], float)
            Jv, Jw = np.zeros((3, self.nv)), np.zeros((3, self.nv))
            Jv[:, 0:3] = Rb
            d = c - pb
            Jv[:, 3:6] = -np.array([[0, -d[2], d[1]], [d[2], 0, -d[0]], [-d[1], d[0], 0]]) @ Rb
            Jw[:, 3:6] = Rb
            for a in self._ancestors(i):
                if a in jz:
                    k = 6 + self.jidx[a]
                    if self.tree[a]["type"] == 1:
                        Jw[:, k] = jz[a]
                        Jv[:, k] = np.cross(jz[a], c - jo[a])
                    else:
                        Jv[:, k] = jz[a]
            Iw = R[i] @ np.asarray(l["inertia"], float).reshape(3, 3) @ R[i].T
            out.append((l["mass"], Jv, Jw, Iw))
        return out

    def mass_matrix(self, q):
        M = np.zeros((self.nv, self.nv))
        for m, Jv, Jw, Iw in self.jacobians(q):
            M += m * Jv.T @ Jv + Jw.T @ Iw @ Jw
        return M

    def gravity(self, q):
        gz = np.array([0.0, 0.0, self.g])
        return sum(m * Jv.T @ gz for m, Jv, Jw, Iw in self.jacobians(q))

    def integrate(self, q, v, h):
        """q (+) h v on the free-flyer manifold (first order in h for the base, exact joints)."""
        q = np.array(q, float)
        Rb = _quat(*q[3:7])
        q[:3] += h * Rb @ v[:3]
        Rn = Rb @ _axis_angle(v[3:6], h * np.linalg.norm(v[3:6])) if np.linalg.norm(v[3:6]) > 0 else Rb
        w = np.sqrt(max(1e-300, 1 + Rn[0, 0] + Rn[1, 1] + Rn[2, 2])) / 2
        q[3:7] = [(Rn[2, 1] - Rn[1, 2]) / (4 * w), (Rn[0, 2] - Rn[2, 0]) / (4 * w), (Rn[1, 0] - Rn[0, 1]) / (4 * w), w]
        q[7:] += h * v[6:]
        return q

    def nle_joint_rows(self, q, v, h=1e-6):
        """nle rows 6.. (the joint coordinates) from the Lagrangian, central differences."""
        Mp, Mm = self.mass_matrix(self.integrate(q, v, h)), self.mass_matrix(self.integrate(q, v, -h))
        Mdot_v = (Mp - Mm) @ v / (2 * h)
        out = np.zeros(self.nj)
        for j in range(self.nj):
            qp, qm = np.array(q, float), np.array(q, float)
            qp[7 + j] += h
            qm[7 + j] -= h
            dT = (v @ self.mass_matrix(qp) @ v - v @ self.mass_matrix(qm) @ v) / (2 * h)
            out[j] = Mdot_v[6 + j] - 0.5 * dT
        return out + self.gravity(q)[6:]

    def mdot(self, q, v, h=1e-6):
        return (self.mass_matrix(self.integrate(q, v, h)) - self.mass_matrix(self.integrate(q, v, -h))) / (2 * h)
