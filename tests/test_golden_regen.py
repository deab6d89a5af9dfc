"""The committed fixtures are reproducible from the reference: ``tests/golden/make_golden.py``
re-run into a scratch directory (it imports the reference hot path read-only from
/root/reference, with the test-only shims) must give every fixture with the same keys,
dtypes and shapes, integer/bool arrays bit for bit, and floating arrays bit for bit on
the host that made them or within the cross-host ulp budget elsewhere (torch's
vectorised libm and reductions differ across CPU microarchitectures; see
``test_oracle_golden.py``).  Skipped where the reference is absent (the GPU box)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from test_oracle_golden import CROSS_HOST_RTOL


def test_fixtures_regenerate(fresh_golden_dir):
    if fresh_golden_dir is None:
        pytest.skip("reference not present")
    committed = sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz"))
    assert sorted(f for f in os.listdir(fresh_golden_dir) if f.endswith(".npz")) == committed
    for name in committed:
        new = np.load(os.path.join(fresh_golden_dir, name), allow_pickle=False)
        old = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
        assert sorted(new.files) == sorted(old.files), name
        for k in old.files:
            a, b = new[k], old[k]
            assert a.dtype == b.dtype and a.shape == b.shape, f"{name}[{k}]"
            if a.tobytes() == b.tobytes():
                continue
            assert np.issubdtype(b.dtype, np.floating), f"{name}[{k}] (non-float arrays must be identical)"
            scale = np.abs(b.astype(np.float64)).max()
            d = np.abs(a.astype(np.float64) - b.astype(np.float64)).max()
            assert d <= CROSS_HOST_RTOL * scale, f"{name}[{k}] max|d|={d} scale={scale}"
