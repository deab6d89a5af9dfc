"""Native dispatch, CPU side (csrc/mppi_aql.cpp): the build writes one gfx950 code object per
kernel unit next to the library, and the symbols the launchers name for native dispatch
(mppi_rollout.h rollout_symbol, the finalize and quadrotor launchers) are in them.  The GPU
side -- packets, parity with the HIP launches -- is tests/test_gpu_aql.py."""
import os
import struct

import pytest

from quadrotor_manipulator_mppi_amd import build as B

EM_AMDGPU = 224


def _code_objects():
    lib = B.LIB
    if not os.path.exists(lib):
        pytest.skip("library not built")
    return {u: B.code_object_path(lib, u) for u in B.KERNEL_UNITS}


def test_every_kernel_unit_has_a_gfx950_code_object():
    for unit, path in _code_objects().items():
        assert os.path.exists(path), f"{unit}: {path} missing (python -m quadrotor_manipulator_mppi_amd.build)"
        with open(path, "rb") as f:
            head = f.read(64)
        assert head[:4] == b"\x7fELF", path
        (e_machine,) = struct.unpack_from("<H", head, 18)
        assert e_machine == EM_AMDGPU, f"{path}: e_machine {e_machine}"
        (flags,) = struct.unpack_from("<I", head, 48)
        assert flags & 0xFF == 0x4F, f"{path}: not gfx950 (mach {flags & 0xFF:#x})"


def _rollout(model, na, nch, lseg, f64, vone, xc, oneg):
    return (f"_Z9k_rolloutILi{model}ELi{na}ELi{nch}ELi{lseg}ELb{int(f64)}ELb{int(vone)}ELb{int(xc)}ELb{int(oneg)}"
            "EEvjjjjiiiPKfPKN4mppi8JointDevENS2_9DevParamsE")


# the symbols the launchers name for the shapes the benchmarks and the drop-in classes run
EXPECTED = {
    "mppi_rollout_arm_h32.hip": [_rollout(1, 7, 1, 32, True, True, False, True)],    # arm C3, fp64 state
    "mppi_rollout_arm.hip": [_rollout(1, 7, 1, 64, True, True, False, True)],        # arm H = 64, fp64 state
    "mppi_rollout_arm32.hip": [_rollout(1, 7, 1, 32, False, True, False, True)],
    "mppi_rollout_wb.hip": [_rollout(2, 10, 1, 64, False, True, False, True),         # C4 shard
                            _rollout(2, 10, 1, 64, False, True, False, False)],       # K=65536
    "mppi_rollout_drone.hip": [_rollout(0, 3, 1, 32, False, True, False, True)],
    "mppi_rollout_quad.hip": ["_Z14k_rollout_quadILb1ELb0ELi1ELi512EEvjjjjiiPKfN4mppi9DevParamsE"],
    "mppi_finalize.hip": ["_Z10k_finalizeILi32ELi9ELi512EEvPKfS1_PKN4mppi7FinTailEjjiiiiijNS2_9FinParamsE",
                          "_Z10k_finalizeILi16ELi9ELi256EEvPKfS1_PKN4mppi7FinTailEjjiiiiijNS2_9FinParamsE"],
}


def test_native_dispatch_symbols_present():
    cos = _code_objects()
    for unit, names in EXPECTED.items():
        with open(cos[unit], "rb") as f:
            blob = f.read()
        for n in names:
            assert (n + ".kd").encode() in blob, f"{unit}: {n}.kd not in {cos[unit]}"
