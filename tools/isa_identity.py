"""Do two builds of the library run the same GPU code?  (tools/, not shipped.)

    python tools/isa_identity.py <lib_a.so> <lib_b.so>

Disassembles every kernel unit's gfx950 code object next to each library
(<stem>.<unit>.co, the objects native dispatch loads; build.py KERNEL_UNITS) with llvm-objdump and
compares the instruction text.  Exit status 0 when every unit is identical.  Used in round 6 to
show that source edits which only add experiment knobs (off by default) leave the production
kernels bit for bit as the build the round's GPU evidence was taken on.
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quadrotor_manipulator_mppi_amd.build import KERNEL_UNITS, code_object_path  # noqa: E402

OBJDUMP = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin", "llvm-objdump")


def isa(co: str) -> list:
    out = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", co], capture_output=True, text=True, check=True).stdout
    return [ln for ln in out.splitlines()[3:]]   # (the first lines name the file)


def main() -> int:
    a, b = sys.argv[1], sys.argv[2]
    same = True
    for unit in KERNEL_UNITS:
        la, lb = isa(code_object_path(a, unit)), isa(code_object_path(b, unit))
        nd = sum(1 for x, y in zip(la, lb) if x != y) + abs(len(la) - len(lb))
        same &= nd == 0
        print(f"{unit:28s} {len(lb):7d} lines  {'identical' if nd == 0 else f'{nd} lines differ'}")
    print("identical GPU code" if same else "GPU code differs")
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
