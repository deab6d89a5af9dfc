"""bench.py's CPU baseline (the oracle's control step, oracle/mppi_oracle.py) timed against the
reference itself (BASELINE.md §3 / SURVEY.md §8d: "timing within +-15%"), cell by cell: C1 drone
K=128 H=20, C2 drone K=4096 H=32, C3 arm K=4096 H=32 and the whole-body K=4096 H=64, at one thread
and at every thread of this container (tools/validate_cpu_baseline.py; its committed run is
profiles/r06/cpu_baseline_validation.json).

Slow (minutes) and host-noise sensitive, so it runs only when asked (MPPI_RUN_SLOW=1) and only
where the reference exists (the build container; never the GPU box).  The ratio is the median of
per-round oracle/reference ratios, the two steps run back to back in alternating order."""
import os

import pytest

from conftest import REFERENCE

pytestmark = [pytest.mark.slow,
              pytest.mark.skipif(not os.environ.get("MPPI_RUN_SLOW"), reason="slow: set MPPI_RUN_SLOW=1"),
              pytest.mark.skipif(not os.path.isdir(os.path.join(REFERENCE, "src", "mav_mppi")),
                                 reason="reference not present")]


def test_oracle_step_time_within_15_percent_of_the_reference(monkeypatch):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import validate_cpu_baseline as V
    monkeypatch.setattr(sys, "argv", ["validate_cpu_baseline.py", "--rounds", os.environ.get("MPPI_VAL_ROUNDS", "21")])
    res = V.main()
    bad = {f"{cell}/{t}": round(v["ratio"], 3) for cell, d in res["cells"].items() for t, v in d.items()
           if not 0.85 <= v["ratio"] <= 1.15}
    assert not bad, f"oracle/reference step time outside [0.85, 1.15]: {bad}"
