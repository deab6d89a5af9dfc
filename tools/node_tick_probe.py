"""Latency of the arm node's tick (kinova.py:180-190): MPPI step + computed torque, and of
the host dynamics alone (computed_torque: one RNEA pass; compute_all_terms: M + nle).
   python tools/node_tick_probe.py [K]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from quadrotor_manipulator_mppi_amd.mppi_solver.arm_node import ArmTorqueNode
from quadrotor_manipulator_mppi_amd.mppi_solver.mppi import MPPI

K = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
node = ArmTorqueNode(MPPI(n_samples=K))
pos = np.array([0, 0, 1.0, 0, 0, 0, 1.0, 1.57, 1.7, 0, 4.4, 0, 4.71, 0.0])
vel = np.zeros(13)


def p50(fn, n):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return 1e6 * float(np.median(ts)), 1e6 * float(np.percentile(ts, 99))


node.joint_state(pos, vel)
for _ in range(50):
    node.tick()
tick = p50(lambda: (node.joint_state(pos, vel), node.tick()), 500)
qdes = pos[7:] + 0.01
ct = p50(lambda: node.dyn.computed_torque(node.q, node.v, qdes), 5000)
terms = p50(lambda: node.dyn.compute_all_terms(node.q, node.v), 2000)
print(f"arm node K={K}: joint_state+tick p50 {tick[0]:.1f} us p99 {tick[1]:.1f} us | computed_torque "
      f"p50 {ct[0]:.2f} us | compute_all_terms (M 13x13 + nle) p50 {terms[0]:.2f} us (Python call overhead incl.)")
