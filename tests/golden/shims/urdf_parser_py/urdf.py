"""Test-only stand-in for ``urdf_parser_py.urdf`` (ROS urdfdom_py, not installed).

Only the attributes the reference's ``robot/urdfparser.py:50-120`` touches are
provided: ``links``, ``joints`` (name, type, parent, child, origin.xyz/rpy,
axis), ``joint_map``, ``parent_map``, ``get_root()`` and ``get_chain()``.  It
does XML parsing only (no arithmetic); the floats it yields are pinned by the
FK fixture (``fk_known_answer.npz``).  Used ONLY by ``tests/golden/make_golden.py``.
"""
import xml.etree.ElementTree as ET


def _floats(text, default):
    if text is None:
        return list(default)
    return [float(v) for v in text.split()]


class _Origin:
    def __init__(self, elem):
        self.xyz = _floats(None if elem is None else elem.get("xyz"), [0.0, 0.0, 0.0])
        self.rpy = _floats(None if elem is None else elem.get("rpy"), [0.0, 0.0, 0.0])


class _Link:
    def __init__(self, name):
        self.name = name


class _Joint:
    def __init__(self, elem):
        self.name = elem.get("name")
        self.type = elem.get("type")
        self.parent = elem.find("parent").get("link")
        self.child = elem.find("child").get("link")
        origin = elem.find("origin")
        self.origin = _Origin(origin)
        axis = elem.find("axis")
        self.axis = None if axis is None else _floats(axis.get("xyz"), [1.0, 0.0, 0.0])


class URDF:
    def __init__(self):
        self.links = []
        self.joints = []
        self.joint_map = {}
        self.link_map = {}
        self.parent_map = {}
        self.child_map = {}

    @classmethod
    def from_xml_file(cls, path):
        root = ET.parse(path).getroot()
        robot = cls()
        for le in root.findall("link"):
            link = _Link(le.get("name"))
            robot.links.append(link)
            robot.link_map[link.name] = link
        for je in root.findall("joint"):
            joint = _Joint(je)
            robot.joints.append(joint)
            robot.joint_map[joint.name] = joint
            robot.parent_map[joint.child] = (joint.name, joint.parent)
            robot.child_map.setdefault(joint.parent, []).append((joint.name, joint.child))
        return robot

    def get_root(self):
        roots = [l.name for l in self.links if l.name not in self.parent_map]
        assert len(roots) == 1, roots
        return roots[0]

    def get_chain(self, root, tip, joints=True, links=True, fixed=True):
        chain = []
        if links:
            chain.append(tip)
        link = tip
        while link != root:
            joint, parent = self.parent_map[link]
            if joints and (fixed or self.joint_map[joint].type != "fixed"):
                chain.append(joint)
            if links:
                chain.append(parent)
            link = parent
        chain.reverse()
        return chain
