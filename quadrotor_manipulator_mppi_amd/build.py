"""Build ``lib/libmppi_hip.so`` (gfx950) in-tree with hipcc.

    python -m quadrotor_manipulator_mppi_amd.build [--debug]

The shared library is the drop-in boundary (``include/mppi_hip.h``).  It is
git-ignored but travels to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIB_DIR, "libmppi_hip.so")
LIB_STAMPS = os.path.join(LIB_DIR, "libmppi_hip_stamps.so")   # diagnostic phase-stamp build
SOURCES = ["mppi_kernels.hip", "mppi_capi.cpp"]
HEADERS = ["mppi_dev.h", os.path.join("..", "..", "include", "mppi_hip.h")]
ARCH = os.environ.get("MPPI_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (set ROCM_PATH)")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, debug: bool = False, verbose: bool = False, stamps: bool = False) -> str:
    out = LIB_STAMPS if stamps else LIB
    if not force and not stamps and not _stale():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = out + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-shared",
           "-O1" if debug else "-O3", "-I", os.path.join(ROOT, "include"),
           "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
           "-o", tmp] + (["-DMPPI_STAMPS"] if stamps else []) + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd))
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed ({res.returncode}):\n{res.stdout}\n{res.stderr}")
    if verbose and res.stderr.strip():
        print(res.stderr)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--stamps", action="store_true", help="diagnostic build with per-phase s_memtime stamps")
    a = ap.parse_args()
    print(build(force=a.force or True, debug=a.debug, verbose=True, stamps=a.stamps))
    sys.exit(0)
