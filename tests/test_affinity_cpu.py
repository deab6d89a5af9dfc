"""The launch path's CPU binding helper (quadrotor_manipulator_mppi_amd.affinity), without a
GPU: the sysfs cpulist parser, and that binding is a no-op that never widens the affinity
where the device's PCIe-local CPU list cannot be found."""
import os

from quadrotor_manipulator_mppi_amd import affinity


def test_parse_cpulist():
    assert affinity._parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert affinity._parse_cpulist("5") == [5]
    assert affinity._parse_cpulist("") == []


def test_bind_without_device_info_keeps_affinity(monkeypatch):
    before = os.sched_getaffinity(0)
    monkeypatch.setattr(affinity, "gpu_local_cpus", lambda device=0: None)
    info = affinity.bind_to_gpu_numa(0)
    assert not info["bound"] and os.sched_getaffinity(0) == before


def test_bind_intersects_never_widens(monkeypatch):
    before = sorted(os.sched_getaffinity(0))
    monkeypatch.setattr(affinity, "gpu_local_cpus", lambda device=0: before + [10 ** 6])
    info = affinity.bind_to_gpu_numa(0)
    assert not info["bound"] and info["reason"] == "affinity already local"
    assert sorted(os.sched_getaffinity(0)) == before
    if len(before) > 1:
        try:
            monkeypatch.setattr(affinity, "gpu_local_cpus", lambda device=0: before[:1])
            info = affinity.bind_to_gpu_numa(0)
            assert info["bound"] and sorted(os.sched_getaffinity(0)) == before[:1]
        finally:
            os.sched_setaffinity(0, before)
