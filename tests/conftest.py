import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def load_golden(name):
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


@pytest.fixture(scope="session")
def kinova_chain():
    """The shipped joint table as oracle ``Joint`` objects."""
    from oracle.mppi_oracle import Joint
    from quadrotor_manipulator_mppi_amd.robot.urdf_chain import load_chain
    return [Joint(j["name"], j["type"], j["xyz"], j["rpy"], j["axis"], j["q_index"])
            for j in load_chain()]
