"""The committed fixtures are reproducible from the reference: ``tests/golden/make_golden.py``
re-run into a scratch directory (it imports the reference hot path read-only from
/root/reference, with the test-only shims) must give every array of every fixture
bit for bit -- same keys, dtypes, shapes and bytes.  Skipped where the reference is absent
(the GPU box)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN

REF = os.environ.get("MPPI_REFERENCE_ROOT", "/root/reference")


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src", "mav_mppi")), reason="reference not present")
def test_fixtures_regenerate_bit_identical(tmp_path):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, os.path.join(GOLDEN, "make_golden.py"), "--out", str(tmp_path)],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    committed = sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz"))
    assert sorted(f for f in os.listdir(tmp_path) if f.endswith(".npz")) == committed
    for name in committed:
        new = np.load(tmp_path / name, allow_pickle=False)
        old = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
        assert sorted(new.files) == sorted(old.files), name
        for k in old.files:
            a, b = new[k], old[k]
            assert a.dtype == b.dtype and a.shape == b.shape and a.tobytes() == b.tobytes(), f"{name}[{k}]"
