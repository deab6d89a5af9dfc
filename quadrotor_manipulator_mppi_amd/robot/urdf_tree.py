"""URDF -> kinematic tree with inertias, for the node's rigid-body dynamics.

The reference's arm node builds a Pinocchio model from
``aerial_manipulation/urdf/full_robot_floating2.urdf`` (``kinova.py:54-61``):
a ``floating`` world joint (Pinocchio's free-flyer: q = xyz + quaternion xyzw,
v = local linear + local angular velocity), the drone body, the Kinova arm fixed
under it, 7 revolute joints and fixed finger / end-effector links.  Each tick it
calls ``pin.computeAllTerms(model, data, q, v)`` and uses ``data.M[6:, 6:]`` and
``data.nle[6:]`` in the computed-torque law (``kinova.py:126-184``).

This module flattens that URDF into the entry table ``mppi_dyn_create`` takes
(``include/mppi_hip.h``): one entry per link in topological order, with its
parent entry, the joint that attaches it (type, origin, axis) and its inertial
(mass, COM and inertia about the COM, rotated into the link frame).  The C++
side merges fixed-joint links into their movable ancestor, as Pinocchio does.
Parsing is pure ``xml.etree``.
"""
from __future__ import annotations

import json
import math
import os
import xml.etree.ElementTree as ET
from typing import Dict, List

DEFAULT_TREE_JSON = os.path.join(os.path.dirname(os.path.abspath(__file__)), "full_robot_floating2.json")
TYPES = {"fixed": 0, "revolute": 1, "continuous": 1, "prismatic": 2, "floating": 3}


def _vec(text, default):
    return [float(v) for v in text.split()] if text is not None else list(default)


def _rpy(r, p, y):
    """Rz(y) Ry(p) Rx(r), row-major 3x3 (URDF convention)."""
    cr, sr, cp, sp, cy, sy = math.cos(r), math.sin(r), math.cos(p), math.sin(p), math.cos(y), math.sin(y)
    return [[cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr],
            [sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr],
            [-sp, cp * sr, cp * cr]]


def parse_urdf_tree(path: str) -> List[Dict]:
    root = ET.parse(path).getroot()
    links = {}
    for le in root.findall("link"):
        ent = {"name": le.get("name"), "mass": 0.0, "com": [0.0, 0.0, 0.0], "inertia": [0.0] * 9}
        ine = le.find("inertial")
        if ine is not None:
            o = ine.find("origin")
            ent["mass"] = float(ine.find("mass").get("value"))
            ent["com"] = _vec(None if o is None else o.get("xyz"), [0, 0, 0])
            R = _rpy(*_vec(None if o is None else o.get("rpy"), [0, 0, 0]))
            ie = ine.find("inertia")
            g = {k: float(ie.get(k, "0")) for k in ("ixx", "ixy", "ixz", "iyy", "iyz", "izz")}
            Ic = [[g["ixx"], g["ixy"], g["ixz"]], [g["ixy"], g["iyy"], g["iyz"]], [g["ixz"], g["iyz"], g["izz"]]]
            # inertia about the COM in the link frame: R Ic R^T
            RI = [[sum(R[i][k] * Ic[k][j] for k in range(3)) for j in range(3)] for i in range(3)]
            ent["inertia"] = [sum(RI[i][k] * R[j][k] for k in range(3)) for i in range(3) for j in range(3)]
        links[ent["name"]] = ent
    joint_of = {}
    for je in root.findall("joint"):
        o, ax = je.find("origin"), je.find("axis")
        joint_of[je.find("child").get("link")] = {
            "joint": je.get("name"), "type": je.get("type"), "parent_link": je.find("parent").get("link"),
            "xyz": _vec(None if o is None else o.get("xyz"), [0, 0, 0]),
            "rpy": _vec(None if o is None else o.get("rpy"), [0, 0, 0]),
            "axis": _vec(None if ax is None else ax.get("xyz"), [1, 0, 0])}
    roots = [n for n in links if n not in joint_of]
    if len(roots) != 1:
        raise ValueError(f"URDF must have exactly one root link, found {roots}")
    children = {}
    for child, j in joint_of.items():
        children.setdefault(j["parent_link"], []).append(child)
    order, index = [], {}
    stack = [(c, -1) for c in reversed(children.get(roots[0], []))]   # the root link itself is the world
    while stack:
        name, parent = stack.pop()
        j = joint_of[name]
        index[name] = len(order)
        order.append({"link": name, "joint": j["joint"], "parent": parent, "type": TYPES[j["type"]],
                      "xyz": j["xyz"], "rpy": j["rpy"], "axis": j["axis"], "mass": links[name]["mass"],
                      "com": links[name]["com"], "inertia": links[name]["inertia"]})
        for c in reversed(children.get(name, [])):
            stack.append((c, index[name]))
    return order


def load_tree(path: str = DEFAULT_TREE_JSON) -> List[Dict]:
    with open(path) as f:
        return json.load(f)["links"]


if __name__ == "__main__":   # regenerate the shipped table from the robot model
    import sys
    urdf = sys.argv[1] if len(sys.argv) > 1 else \
        "/root/reference/src/aerial_manipulation/urdf/full_robot_floating2.urdf"
    tree = parse_urdf_tree(urdf)
    with open(DEFAULT_TREE_JSON, "w") as f:
        json.dump({"source": "aerial_manipulation/urdf/full_robot_floating2.urdf (the Pinocchio model of "
                             "kinova.py:54-61): floating base, drone, Kinova j2s7s300 arm, fixed fingers",
                   "links": tree}, f, indent=1)
    print(f"{len(tree)} links -> {DEFAULT_TREE_JSON}")
