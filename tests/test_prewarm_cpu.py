"""The prewarm thread's cadence prediction (mppi_prewarm.cpp prewarm_plan, through the diagnostic
mppi_debug_prewarm_plan; host code only, no GPU): from the last call starts it predicts the next
call of a node that ticks at a fixed rate (kinova.py:101, rospy.Rate(100)) and opens a window of
+- window_us around it; no window for fewer than 4 calls, back-to-back calls or a cadence slower
than 1 s; one late or early tick does not move the prediction (median interval)."""
import ctypes as C

import numpy as np
import pytest

from quadrotor_manipulator_mppi_amd import _capi


@pytest.fixture(scope="module")
def plan():
    L = _capi.lib()
    f = L.mppi_debug_prewarm_plan
    f.restype = C.c_int32
    f.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]

    def run(starts_ns, window_us):
        t = np.ascontiguousarray(starts_ns, np.int64)
        s, e = C.c_int64(), C.c_int64()
        r = f(t.ctypes.data, len(t), window_us, C.byref(s), C.byref(e))
        return r, s.value, e.value
    return run


MS = 1_000_000


def test_steady_100hz(plan):
    t = 5 * MS + np.arange(8) * 10 * MS
    r, s, e = plan(t, 200)
    assert r == 1 and s == t[-1] + 10 * MS - 200_000 and e == t[-1] + 10 * MS + 200_000


def test_median_ignores_one_late_tick(plan):
    t = np.arange(8) * 10 * MS
    t[5:] += 3 * MS     # one 13 ms interval, the rest 10 ms
    r, s, _ = plan(t, 200)
    assert r == 1 and s == t[-1] + 10 * MS - 200_000


@pytest.mark.parametrize("m", [0, 1, 2, 3])
def test_too_few_calls(plan, m):
    assert plan(np.arange(m) * 10 * MS, 200)[0] == 0


def test_back_to_back_and_slow_cadences_get_no_window(plan):
    assert plan(np.arange(8) * 20_000, 200)[0] == 0            # 20 us apart: back to back
    assert plan(np.arange(8) * 799_000, 200)[0] == 0           # < 4 windows apart
    assert plan(np.arange(8) * 800_000, 200)[0] == 1           # = 4 windows
    assert plan(np.arange(8) * 2_000_000_000, 200)[0] == 0     # slower than 1 s


def test_bad_arguments(plan):
    assert plan(np.arange(9) * 10 * MS, 200)[0] < 0           # more than the ring's 8 starts
