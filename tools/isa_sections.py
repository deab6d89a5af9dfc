"""Per-section static instruction mix of one kernel in a hipcc -S listing of a -DMPPI_SECTIONS
build (tools/, not shipped): the rollout's SECTION() markers (mppi_rollout.h) split the kernel,
and each section is classified with tools/isa_count.py (VALU by issue class, SALU, LDS, VMEM).

    python tools/isa_sections.py listing.s <kernel-name-substring>

In a single-group (ONEG) kernel every section is straight-line code that runs once per wave, so
its static count is its dynamic count per wave (lane = one (rollout, t) pair: per lane-step).
"""
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from isa_count import classify, kernel_lines  # noqa: E402


def sections(lines):
    out, name, cur = [], "prologue_loads", []
    for ln in lines:
        m = re.search(r"MPPI_SECTION (\w+)", ln)
        if m:
            out.append((name, cur))
            name, cur = m.group(1), []
            continue
        cur.append(ln)
    out.append((name, cur))
    return out


if __name__ == "__main__":
    lines = kernel_lines(sys.argv[1], sys.argv[2])
    tot = {}
    rows = []
    for name, ls in sections(lines):
        c = classify(ls)
        rows.append((name, c))
        for k, v in c.items():
            tot[k] = tot.get(k, 0) + v
    print(f"{'section':24s} {'VALU':>6s} {'full':>6s} {'quarter':>7s} {'trans':>6s} {'dpp':>5s} {'cycles':>7s} "
          f"{'SALU':>6s} {'LDS':>5s} {'VMEMld':>6s} {'VMEMst':>6s}")
    for name, c in rows + [("TOTAL", tot)]:
        print(f"{name:24s} {c['valu']:6d} {c['full']:6d} {c['quarter']:7d} {c['trans']:6d} {c['dpp']:5d} "
              f"{c['valu_cycles']:7d} {c['salu']:6d} {c['lds']:5d} {c['vmem_ld']:6d} {c['vmem_st']:6d}")
