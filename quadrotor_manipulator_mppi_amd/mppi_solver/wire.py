"""ROS1 wire formats around the control step, without ROS.

The MPPI nodes talk to the Gazebo plugin over three topics.  This module packs and
unpacks those messages in the ROS1 serialization (little-endian; ``uint32`` length
prefix for strings and variable arrays), so a bridge or a recorded bag can drive the
drop-in solvers without ``rospy``:

* ``/harrierD7/robot_states`` ``sensor_msgs/JointState`` (plugin -> nodes).  The plugin
  fills ``position[14] = [x, y, z, qx, qy, qz, qw, q1..q7]`` and ``velocity[13] =
  [v(3), omega(3), qdot(7)]`` (``aerial_manipulation/src/controller.cpp:305-333``);
  without the manipulator the joint entries stay 0 (``:327-335``).
* ``/harrierD7/robot_cmd`` ``sensor_msgs/JointState`` (arm node -> plugin): only
  ``effort[:7]`` is set (``kinova.py:189-191``) and read (``controller.cpp:659-665``).
* ``/harrierD7/drone_pose`` ``std_msgs/Float64MultiArray`` (nodes -> plugin):
  ``data = xdes.to('cpu').tolist()`` (``drone.py:239-241``); the plugin reads
  ``data[0:3]`` as the desired position (``controller.cpp:667-672``).

``DroneNode`` replays the drone node's loop body (``drone.py:99-112, 160-241``) on these
payloads; ``ArmTorqueNode`` (``arm_node.py``) is the arm node's, and
``arm_tick_message`` wraps its torque into the ``/robot_cmd`` payload.

Host code only: the messages are a few hundred bytes per 10 ms tick.
"""
from __future__ import annotations

import struct
import threading
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

N_POSITION = 14   # controller.cpp:306
N_VELOCITY = 13   # controller.cpp:307
N_EFFORT = 7      # controller.cpp:661, kinova.py:190


class WireError(ValueError):
    """A payload that does not parse as the named message (truncated, trailing bytes)."""


# ----------------------------------------------------------------- primitives
class _Reader:
    def __init__(self, buf: bytes):
        self.buf = memoryview(bytes(buf))
        self.off = 0

    def take(self, n: int) -> memoryview:
        if n < 0 or self.off + n > len(self.buf):
            raise WireError(f"truncated payload: need {n} bytes at offset {self.off}, "
                            f"have {len(self.buf) - self.off}")
        m = self.buf[self.off:self.off + n]
        self.off += n
        return m

    def u32(self) -> int:
        return struct.unpack_from("<I", self.take(4))[0]

    def string(self) -> str:
        return bytes(self.take(self.u32())).decode("utf-8")

    def f64_array(self) -> np.ndarray:
        n = self.u32()
        return np.frombuffer(self.take(8 * n), dtype="<f8").astype(np.float64)

    def string_array(self) -> List[str]:
        return [self.string() for _ in range(self.u32())]

    def done(self):
        if self.off != len(self.buf):
            raise WireError(f"{len(self.buf) - self.off} trailing bytes")


def _string(s: str) -> bytes:
    b = s.encode("utf-8")
    return struct.pack("<I", len(b)) + b


def _f64_array(x) -> bytes:
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1), dtype="<f8")
    return struct.pack("<I", a.size) + a.tobytes()


def _string_array(xs: Sequence[str]) -> bytes:
    return struct.pack("<I", len(xs)) + b"".join(_string(s) for s in xs)


# ------------------------------------------------------------ message types
@dataclass
class Header:
    """std_msgs/Header: uint32 seq, time stamp (secs, nsecs), string frame_id."""
    seq: int = 0
    secs: int = 0
    nsecs: int = 0
    frame_id: str = ""


@dataclass
class JointState:
    """sensor_msgs/JointState: Header, string[] name, float64[] position/velocity/effort."""
    header: Header = field(default_factory=Header)
    name: List[str] = field(default_factory=list)
    position: np.ndarray = field(default_factory=lambda: np.zeros(0))
    velocity: np.ndarray = field(default_factory=lambda: np.zeros(0))
    effort: np.ndarray = field(default_factory=lambda: np.zeros(0))

    def serialize(self) -> bytes:
        h = self.header
        return (struct.pack("<III", h.seq & 0xFFFFFFFF, h.secs & 0xFFFFFFFF, h.nsecs & 0xFFFFFFFF)
                + _string(h.frame_id) + _string_array(self.name) + _f64_array(self.position)
                + _f64_array(self.velocity) + _f64_array(self.effort))

    @classmethod
    def deserialize(cls, buf: bytes) -> "JointState":
        r = _Reader(buf)
        seq, secs, nsecs = r.u32(), r.u32(), r.u32()
        hdr = Header(seq, secs, nsecs, r.string())
        m = cls(hdr, r.string_array(), r.f64_array(), r.f64_array(), r.f64_array())
        r.done()
        return m


@dataclass
class MultiArrayDimension:
    label: str = ""
    size: int = 0
    stride: int = 0


@dataclass
class Float64MultiArray:
    """std_msgs/Float64MultiArray: MultiArrayLayout (dim[], data_offset) + float64[] data."""
    data: np.ndarray = field(default_factory=lambda: np.zeros(0))
    dim: List[MultiArrayDimension] = field(default_factory=list)
    data_offset: int = 0

    def serialize(self) -> bytes:
        out = [struct.pack("<I", len(self.dim))]
        for d in self.dim:
            out.append(_string(d.label) + struct.pack("<II", d.size, d.stride))
        out.append(struct.pack("<I", self.data_offset))
        out.append(_f64_array(self.data))
        return b"".join(out)

    @classmethod
    def deserialize(cls, buf: bytes) -> "Float64MultiArray":
        r = _Reader(buf)
        dims = []
        for _ in range(r.u32()):
            label = r.string()
            size, stride = r.u32(), r.u32()
            dims.append(MultiArrayDimension(label, size, stride))
        off = r.u32()
        m = cls(r.f64_array(), dims, off)
        r.done()
        return m


# ------------------------------------------------------ plugin-side layouts
def robot_states(position_xyz, quat_xyzw, lin_vel, ang_rate, robot_q=None, robot_qdot=None,
                 seq: int = 0) -> JointState:
    """The plugin's state message (``controller.cpp:305-333``): position[14], velocity[13].

    ``robot_q`` / ``robot_qdot`` (7,) are the manipulator joints; ``None`` leaves them 0,
    as the plugin does when ``manipulator_bool`` is false (``:327``).
    """
    pos = np.zeros(N_POSITION)
    vel = np.zeros(N_VELOCITY)
    pos[0:3] = np.asarray(position_xyz, np.float64).reshape(3)
    pos[3:7] = np.asarray(quat_xyzw, np.float64).reshape(4)
    vel[0:3] = np.asarray(lin_vel, np.float64).reshape(3)
    vel[3:6] = np.asarray(ang_rate, np.float64).reshape(3)
    if robot_q is not None:
        pos[7:14] = np.asarray(robot_q, np.float64).reshape(7)
    if robot_qdot is not None:
        vel[6:13] = np.asarray(robot_qdot, np.float64).reshape(7)
    return JointState(Header(seq=seq), [], pos, vel, np.zeros(0))


def robot_cmd(torque) -> JointState:
    """The arm node's command: ``msg.effort = [float(t) for t in torque[:7]]`` (``kinova.py:189-190``)."""
    t = np.asarray(torque, np.float64).reshape(-1)
    if t.size < N_EFFORT:
        raise WireError(f"robot_cmd needs {N_EFFORT} torques, got {t.size}")
    return JointState(effort=t[:N_EFFORT].copy())


def plugin_torques(msg: JointState) -> np.ndarray:
    """``control_callback`` (``controller.cpp:659-665``): kinova_torques(i) = effort[i], i < 7."""
    if msg.effort.size < N_EFFORT:
        raise WireError(f"robot_cmd carries {msg.effort.size} efforts, the plugin reads {N_EFFORT}")
    return msg.effort[:N_EFFORT].copy()


def drone_pose(xdes) -> Float64MultiArray:
    """``msg.data = xdes.to('cpu').tolist()`` (``drone.py:239-240``): the fp32 desired
    position widened to float64 element by element (empty layout)."""
    if hasattr(xdes, "detach"):
        xdes = xdes.detach().to("cpu").tolist()
    return Float64MultiArray(np.asarray(xdes, np.float64).reshape(-1))


def plugin_drone_target(msg: Float64MultiArray) -> Tuple[float, float, float]:
    """``drone_callback`` (``controller.cpp:667-672``): des_x, des_y, des_z = data[0:3]."""
    if msg.data.size < 3:
        raise WireError(f"drone_pose carries {msg.data.size} values, the plugin reads 3")
    return float(msg.data[0]), float(msg.data[1]), float(msg.data[2])


# ------------------------------------------------------------- node loops
def _quat_R(x, y, z, w):
    n = np.sqrt(x * x + y * y + z * z + w * w)
    x, y, z, w = x / n, y / n, z / n, w / n
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


class DroneNode:
    """The drone node's MPPI loop on wire payloads (``drone.py``).

    * ``on_robot_states(payload)`` = ``joint_state_callback`` (``drone.py:99-109``):
      q = position[:7], v = velocity[:6], v[:3] rotated by the base rotation
      (``pin.XYZQUATToSE3`` of q[:7], ``:107-109``).  The Pinocchio terms computed there
      are unused by the MPPI branch and are not evaluated.
    * ``tick()`` = one pass of ``main`` (``drone.py:160-241``): ``set_state(q[:3], v[:3])``,
      ``xdes, _ = compute_control_input()`` and the ``/drone_pose`` payload.
    """

    def __init__(self, mppi=None):
        if mppi is None:
            from .drone_mppi import MPPI
            mppi = MPPI()
        self.mppi = mppi
        self.q: Optional[np.ndarray] = None
        self.v: Optional[np.ndarray] = None
        self._lock = threading.Lock()

    def on_robot_states(self, payload: bytes):
        msg = JointState.deserialize(payload)
        if msg.position.size < 7 or msg.velocity.size < 6:
            raise WireError(f"robot_states needs position[7] and velocity[6], "
                            f"got {msg.position.size} / {msg.velocity.size}")
        q = np.array(msg.position[:7], np.float64)
        v = np.array(msg.velocity[:6], np.float64)
        v[:3] = _quat_R(*q[3:7]) @ v[:3]
        with self._lock:
            self.q, self.v = q, v

    def tick(self, noise=None) -> Optional[bytes]:
        with self._lock:
            if self.q is None:
                return None
            trans, vel = self.q[:3].copy(), self.v[:3].copy()
        self.mppi.set_state(trans, vel)
        xdes, _ = self.mppi.compute_control_input(noise)
        return drone_pose(xdes).serialize()


def arm_on_robot_states(node, payload: bytes):
    """``kinova.py:106-116`` on a ``/robot_states`` payload: feeds ``ArmTorqueNode.joint_state``."""
    msg = JointState.deserialize(payload)
    if msg.position.size < N_POSITION or msg.velocity.size < N_VELOCITY:
        raise WireError(f"robot_states needs position[{N_POSITION}] and velocity[{N_VELOCITY}], "
                        f"got {msg.position.size} / {msg.velocity.size}")
    node.joint_state(msg.position[:N_POSITION], msg.velocity[:N_VELOCITY])


def arm_tick_message(node, noise=None) -> Optional[bytes]:
    """One ``ArmTorqueNode.tick`` published as the ``/robot_cmd`` payload (``kinova.py:180-191``)."""
    out = node.tick(noise)
    if out is None:
        return None
    return robot_cmd(out[0]).serialize()
