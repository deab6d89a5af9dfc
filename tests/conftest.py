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


REFERENCE = os.environ.get("MPPI_REFERENCE_ROOT", "/root/reference")


def load_golden_from(root, name):
    import numpy as np
    return dict(np.load(os.path.join(root, name), allow_pickle=False))


def load_golden(name):
    return load_golden_from(GOLDEN, name)


@pytest.fixture(scope="session")
def fresh_golden_dir(tmp_path_factory):
    """Fixtures regenerated from the reference on this host (``make_golden.py``, ~2 s),
    or None where /root/reference is absent (the GPU box)."""
    import subprocess
    if not os.path.isdir(os.path.join(REFERENCE, "src", "mav_mppi")):
        return None
    out = tmp_path_factory.mktemp("golden_fresh")
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, os.path.join(GOLDEN, "make_golden.py"), "--out", str(out)],
                       cwd=str(out), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return str(out)


@pytest.fixture(scope="session")
def kinova_chain():
    """The shipped joint table as oracle ``Joint`` objects."""
    from oracle.mppi_oracle import Joint
    from quadrotor_manipulator_mppi_amd.robot.urdf_chain import load_chain
    return [Joint(j["name"], j["type"], j["xyz"], j["rpy"], j["axis"], j["q_index"])
            for j in load_chain()]
