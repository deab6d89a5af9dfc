"""Test-only stand-in for ROS ``rospkg`` (not installed in this image).

Used ONLY by ``tests/golden/make_golden.py`` when it imports the reference
solver (``mppi_solver/mppi.py:79-81`` resolves the URDF through
``rospkg.RosPack().get_path("aerial_manipulation")``).  Never imported by the
product package, the GPU tests, ``smoke()`` or ``bench.py``.
"""
import os

_REF_SRC = os.environ.get("MPPI_REFERENCE_SRC", "/root/reference/src")


class RosPack:
    def get_path(self, name):
        path = os.path.join(_REF_SRC, name)
        if not os.path.isdir(path):
            raise KeyError(name)
        return path
