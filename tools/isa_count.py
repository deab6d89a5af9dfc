"""Static instruction mix of one kernel in a hipcc -S listing (tools/, not shipped).

    python tools/isa_count.py listing.s <kernel-name-substring>

Counts VALU by issue class (full-rate fp32/int, quarter-rate 64-bit/DPP/mul32,
transcendental), SALU, LDS, VMEM, and prints the weighted SIMD cycles per wave using
the gfx950 issue costs of profiles/r01/microbench_valu_issue.txt (2.4 / 4.2 / 8.2).
Static counts: a straight-line kernel (iters == 1) executes each once.
"""
import re
import sys

TRANS = re.compile(r"^v_(log|exp|sin|cos|sqrt|rsq|rcp)_f32")
QUARTER = re.compile(r"^v_(mad_u64_u32|mad_i64_i32|mul_lo_u32|mul_hi_u32|mul_hi_i32|lshl_add_u64|"
                     r"\w+_f64|cvt_f64_f32|cvt_f32_f64|pk_\w+|readlane_b32|writelane_b32|readfirstlane_b32)")


def kernel_lines(path, name):
    out, on = [], False
    for ln in open(path):
        if re.match(r"^_Z\w*:", ln):
            on = name in ln.split(":")[0]
            continue
        if on and ln.strip().startswith(".Lfunc_end"):
            on = False
        if on:
            out.append(ln.strip())
    return out


def classify(lines):
    c = dict(valu=0, full=0, quarter=0, trans=0, dpp=0, salu=0, lds=0, vmem_ld=0, vmem_st=0, other=0)
    for ln in lines:
        if not ln or ln.startswith((";", ".", "s_nop")) or ln.endswith(":"):
            continue
        op = ln.split()[0]
        if op.startswith("v_"):
            c["valu"] += 1
            if "dpp" in op or "row_" in ln or "quad_perm" in ln or "wave_shr" in ln:
                c["dpp"] += 1
            elif TRANS.match(op):
                c["trans"] += 1
            elif QUARTER.match(op):
                c["quarter"] += 1
            else:
                c["full"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("global_load", "buffer_load", "flat_load")):
            c["vmem_ld"] += 1
        elif op.startswith(("global_store", "buffer_store", "flat_store")):
            c["vmem_st"] += 1
        else:
            c["other"] += 1
    c["valu_cycles"] = round(2.4 * c["full"] + 4.2 * (c["quarter"] + c["dpp"]) + 8.2 * c["trans"])
    return c


if __name__ == "__main__":
    lines = kernel_lines(sys.argv[1], sys.argv[2])
    print(sys.argv[1], sys.argv[2], classify(lines))
