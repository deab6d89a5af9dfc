"""URDF -> active joint chain table for the on-device FK.

Host-side mirror of what the reference's ``robot/urdfparser.py`` extracts from
``aerial_manipulator_gpu.urdf`` before every FK call:

* active joints: walk ``parent_map`` from the end link up to ``root_link`` or the
  absolute root (``urdfparser.py:62-69``);
* actuated-joint index map in URDF document order (``urdfparser.py:71-89``);
* chain from the absolute root to the tip, filtered to active joints
  (``urdfparser.py:110-120``).

The reference re-reads these tensors from Python objects on every call
(``urdfparser.py:133-161``); here they are parsed once into a flat table that
the C-ABI engine uploads to the device (``mppi_joint`` in ``include/mppi_hip.h``).
Parsing is pure ``xml.etree``; ``urdf_parser_py`` (ROS) is not needed.
"""
from __future__ import annotations

import json
import os
import xml.etree.ElementTree as ET
from typing import Dict, List

ACTUATED = ("prismatic", "revolute", "continuous")
DEFAULT_CHAIN_JSON = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kinova_j2s7s300.json")


def _vec(text, default):
    return [float(v) for v in text.split()] if text is not None else list(default)


def parse_urdf_chain(path: str, root_link: str, end_link: str) -> List[Dict]:
    root = ET.parse(path).getroot()
    joints, parent_of, links = [], {}, [le.get("name") for le in root.findall("link")]
    for je in root.findall("joint"):
        origin, axis = je.find("origin"), je.find("axis")
        j = {"name": je.get("name"), "type": je.get("type"),
             "parent": je.find("parent").get("link"), "child": je.find("child").get("link"),
             "xyz": _vec(None if origin is None else origin.get("xyz"), [0, 0, 0]),
             "rpy": _vec(None if origin is None else origin.get("rpy"), [0, 0, 0]),
             "axis": None if axis is None else _vec(axis.get("xyz"), [1, 0, 0])}
        joints.append(j)
        parent_of[j["child"]] = j
    roots = [l for l in links if l not in parent_of]
    if len(roots) != 1:
        raise ValueError(f"URDF must have exactly one root link, found {roots}")
    abs_root = roots[0]
    if end_link not in parent_of:
        raise ValueError(f"end link {end_link!r} not found in {path}")
    active, link = set(), end_link
    while link not in (root_link, abs_root):
        j = parent_of[link]
        active.add(j["name"])
        link = j["parent"]
    qmap, idx = {}, 0
    for j in joints:
        if j["type"] in ACTUATED and j["name"] in active:
            qmap[j["name"]] = idx
            idx += 1
    chain, link = [], end_link
    while link != abs_root:
        j = parent_of[link]
        if j["name"] in active:
            chain.append(j)
        link = j["parent"]
    chain.reverse()
    return [{"name": j["name"], "type": j["type"], "xyz": j["xyz"], "rpy": j["rpy"],
             "axis": j["axis"], "q_index": qmap.get(j["name"], -1)} for j in chain]


def load_chain(path: str = DEFAULT_CHAIN_JSON) -> List[Dict]:
    with open(path) as f:
        return json.load(f)["joints"]


if __name__ == "__main__":   # regenerate the shipped table from the robot model
    import sys
    urdf = sys.argv[1] if len(sys.argv) > 1 else \
        "/root/reference/src/aerial_manipulation/urdf/aerial_manipulator_gpu.urdf"
    chain = parse_urdf_chain(urdf, "base", "j2s7s300_link_7")
    with open(DEFAULT_CHAIN_JSON, "w") as f:
        json.dump({"source": "aerial_manipulation/urdf/aerial_manipulator_gpu.urdf:67-365 "
                             "(root 'base' -> end 'j2s7s300_link_7', mppi.py:84-88)",
                   "joints": chain}, f, indent=1)
    print(json.dumps(chain, indent=1))
