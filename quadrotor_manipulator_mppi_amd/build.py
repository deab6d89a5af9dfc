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
LIB_ASAN = os.path.join(LIB_DIR, "libmppi_hip_asan.so")       # host AddressSanitizer build (CPU tests only)
# AddressSanitizer on the HOST side of every translation unit only (-Xarch_host): the device
# code is unchanged, and the library runs the CPU tests with the runtime preloaded
# (scripts/asan_cpu_tests.sh).  GPU sanitizers are not available on the GPU pool.
_ASAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer", "-g"]
# (source, extra flags).  The rollout is built without the SLP vectorizer: its
# v_pk_* pairings cost more register moves than they save and raise the kernel
# from 110 to 184 VGPRs (2 instead of 4 waves per SIMD) -- DESIGN.md §kernels.
# The kernels' leading scalar arguments (rollout: Philox key/step, sample offset,
# noise mode, H, u_prev, joint table; finalize: record and tail pointers, sizes, sequence)
# are preloaded into SGPRs at wave launch.
_ROLL = ["-fno-slp-vectorize", "-mllvm", "-amdgpu-kernarg-preload-count=11"]
# the C3 unit (arm, fp64 state, H <= 32) and the 6-DoF quadrotor unit with the max-ilp scheduler:
# both kernels are one wave's dependent chain (profiles/r05/sched_maxilp: C3 -0.28 us, quadrotor
# K=4096 H=32 -0.25 us, K=65536 -0.8..-1.4 us; on the other units it measured mixed or slower)
_MAXILP = ["-mllvm", "-amdgpu-sched-strategy=" + os.environ.get("MPPI_C3_SCHED", "max-ilp")]   # (knob: experiments)
_FIN = ["-mllvm", "-amdgpu-kernarg-preload-count=14"]
# (experiments: MPPI_MAXILP_UNITS = extra units built with max-ilp, comma-separated)
_XI = [u for u in os.environ.get("MPPI_MAXILP_UNITS", "").split(",") if u]
SOURCES = [(u, f + (_MAXILP if u in _XI else [])) for u, f in
           [("mppi_rollout_drone.hip", _ROLL), ("mppi_rollout_arm.hip", _ROLL), ("mppi_rollout_arm32.hip", _ROLL),
            ("mppi_rollout_wb.hip", _ROLL), ("mppi_finalize.hip", _FIN)]] + \
          [("mppi_rollout_arm_h32.hip", _ROLL + _MAXILP + os.environ.get("MPPI_C3_EXTRA", "").split()), ("mppi_rollout_quad.hip", _ROLL + _MAXILP),
           ("mppi_host_math.cpp", []), ("mppi_engine.cpp", []), ("mppi_step.cpp", []), ("mppi_exchange.cpp", []),
           ("mppi_prewarm.cpp", []), ("mppi_dynamics.cpp", []), ("mppi_aql.cpp", [])]
HEADERS = ["mppi_dev.h", "mppi_device.h", "mppi_rollout.h", "mppi_aql.h", "mppi_engine.h",
           os.path.join("..", "..", "include", "mppi_hip.h")]
# Native dispatch (mppi_aql.cpp) loads each kernel unit's gfx950 code object from next to the
# library: <library stem>.<unit>.co, built from the same source with the same flags.
KERNEL_UNITS = [s for s, _ in SOURCES if s.endswith(".hip")]


def code_object_path(lib: str, unit: str) -> str:
    return os.path.splitext(lib)[0] + "." + os.path.splitext(unit)[0] + ".co"


ARCH = os.environ.get("MPPI_OFFLOAD_ARCH", "gfx950")
EXTRA = os.environ.get("MPPI_HIPCC_EXTRA", "").split()   # experiment flags (tools/), empty in production
# every environment knob that changes the flags of some unit (experiments only); BUILD_INFO.json records
# the ones set, and the production library refuses them (build one elsewhere with MPPI_BUILD_OUT)
KNOBS = ("MPPI_HIPCC_EXTRA", "MPPI_C3_SCHED", "MPPI_C3_EXTRA", "MPPI_MAXILP_UNITS", "MPPI_OFFLOAD_ARCH")


def knobs_set() -> dict:
    return {k: os.environ[k] for k in KNOBS if os.environ.get(k)}


def hipcc() -> str:
    for cand in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (set ROCM_PATH)")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    if not all(os.path.exists(code_object_path(LIB, u)) for u in KERNEL_UNITS):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s, _ in SOURCES] + [os.path.join(CSRC, h) for h in HEADERS] + \
        [os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, debug: bool = False, verbose: bool = False, stamps: bool = False,
          asan: bool = False) -> str:
    out = os.environ.get("MPPI_BUILD_OUT") or (LIB_STAMPS if stamps else LIB_ASAN if asan else LIB)
    if os.path.abspath(out) == os.path.abspath(LIB) and knobs_set():
        raise RuntimeError(f"experiment build knobs {sorted(knobs_set())} set for the production library "
                           f"{LIB}: unset them, or build elsewhere with MPPI_BUILD_OUT")
    if not force and not stamps and not asan and not _stale():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = out + ".tmp"
    base = [hipcc(), f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-O1" if debug else "-O3",
            "-I", os.path.join(ROOT, "include"), "-Wall", "-Wno-unused-function", "-Wno-unused-variable"] + \
        (["-DMPPI_STAMPS"] if stamps else []) + (_ASAN if asan else []) + EXTRA
    objdir = os.path.join(LIB_DIR, "obj" + ("_stamps" if stamps else "_asan" if asan else ""))
    os.makedirs(objdir, exist_ok=True)
    objs, procs, cos = [], [], []
    for src, flags in SOURCES:   # compile the translation units in parallel
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        cmd = base + flags + ["-c", "-o", obj, os.path.join(CSRC, src)]
        if verbose:
            print(" ".join(cmd))
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
        objs.append(obj)
        if src in KERNEL_UNITS and not asan:   # the same unit's device code alone, for native dispatch
            co = code_object_path(out, src)
            cmd = base + flags + ["--cuda-device-only", "-c", "--no-gpu-bundle-output", "-o", co + ".tmp",
                                  os.path.join(CSRC, src)]
            procs.append((src + " (code object)", subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                                                   text=True)))
            cos.append(co)
    for src, pr in procs:
        so, se = pr.communicate()
        if pr.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src} ({pr.returncode}):\n{so}\n{se}")
        if verbose and se.strip():
            print(se)
    for co in cos:
        os.replace(co + ".tmp", co)
    rocm_lib = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib")
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + \
        ["-L", rocm_lib, "-lhsa-runtime64"] + \
        (["-Xarch_host", "-fsanitize=address", "-shared-libsan"] if asan else [])
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc link failed ({res.returncode}):\n{res.stdout}\n{res.stderr}")
    os.replace(tmp, out)
    _write_build_info(out)
    return out


def _write_build_info(out: str) -> None:
    """lib/BUILD_INFO.json: which source state a library came from (bench.py reports it;
    the GPU box has no .git)."""
    import datetime
    import json
    head = None
    try:
        head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                              text=True, timeout=10).stdout.strip() or None
        dirty = subprocess.run(["git", "-C", ROOT, "status", "--porcelain", "--untracked-files=no", "--",
                                "quadrotor_manipulator_mppi_amd/csrc", "include"], capture_output=True, text=True,
                               timeout=10).stdout.strip()
        if head and dirty:
            head += "+dirty"
    except (OSError, subprocess.SubprocessError):
        pass
    info = {"library": os.path.basename(out), "git_head": head, "arch": ARCH, "extra_flags": EXTRA,
            "knobs": knobs_set(),
            "built_utc": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")}
    if out == LIB:
        with open(os.path.join(LIB_DIR, "BUILD_INFO.json"), "w") as f:
            json.dump(info, f, indent=1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--stamps", action="store_true", help="diagnostic build with per-phase s_memtime stamps")
    ap.add_argument("--asan", action="store_true", help="host AddressSanitizer build (lib/libmppi_hip_asan.so)")
    a = ap.parse_args()
    print(build(force=a.force, debug=a.debug, verbose=True, stamps=a.stamps, asan=a.asan))
    sys.exit(0)
