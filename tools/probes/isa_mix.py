"""Static instruction mix of the kernels in a gfx950 assembly listing.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude --cuda-device-only -S <file.hip> -o k.s
    python tools/probes/isa_mix.py k.s [name-substring ...]

Per kernel: static counts of VALU / MFMA / LDS / global / SALU / branch
instructions and the VGPR / spill figures the assembler reports.  Static
counts only (loops are counted once); the dynamic mix comes from the SQ
counters (tools/probes/pmc_sq.py).
"""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_pk_",)):
        return "valu_pk"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_load") or op.startswith("s_buffer"):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def parse(path):
    kern, out, meta = None, {}, {}
    for line in open(path):
        m = re.match(r"^(_Z\S+|k_\S+):\s*(;.*)?$", line)
        if m:
            kern = m.group(1)
            out[kern] = Counter()
            continue
        if kern is None:
            continue
        if line.startswith("\t.end_amdhsa_kernel") or re.match(r"^\.Lfunc_end", line):
            kern = None
            continue
        s = line.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        c = classify(op)
        out[kern][c] += 1
        if op in ("v_rcp_f32", "v_rcp_f64", "v_sqrt_f32", "v_sqrt_f64", "v_div_scale_f32", "v_div_fmas_f32"):
            out[kern][op] += 1
        if op.startswith("v_cndmask"):
            out[kern]["cndmask"] += 1
    for line in open(path):
        m = re.match(r"^\s*\.(\S+\.(vgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size)):\s*(\d+)", line)
        if m:
            pass
    return out


def main():
    path = sys.argv[1]
    subs = sys.argv[2:]
    mix = parse(path)
    keys = ["valu", "valu_pk", "mfma", "lds", "vmem", "smem", "salu", "branch", "wait", "cndmask"]
    print("%-70s " % "kernel" + " ".join("%7s" % k for k in keys))
    for k, c in mix.items():
        if subs and not any(s in k for s in subs):
            continue
        print("%-70s " % k[:70] + " ".join("%7d" % c[x] for x in keys))


if __name__ == "__main__":
    main()
