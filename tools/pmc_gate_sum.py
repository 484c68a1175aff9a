"""Summarise tools/pmc_gate.sh: SQ counters of k_gate_mfma per size class and phase."""
import csv, glob, os, re, sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
kre = sys.argv[2] if len(sys.argv) > 2 else r"k_gate_mfma<(\d+)"
tab = defaultdict(dict)   # (phase, class) -> counter -> value
for f in glob.glob(os.path.join(root, "ph*_*/run_counter_collection.csv")):
    ph = re.search(r"ph(\d+)_", f).group(1)
    for r in csv.DictReader(open(f)):
        m = re.search(kre, r["Kernel_Name"])
        if not m:
            continue
        key = (ph, int(m.group(1)) if m.groups() else 0)
        tab[key][r["Counter_Name"]] = tab[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
cols = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU",
        "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU", "SQ_VALU_MFMA_BUSY_CYCLES",
        "SQ_LDS_BANK_CONFLICT"]
print("phase class " + " ".join("%12s" % c.replace("SQ_", "")[:12] for c in cols))
for key in sorted(tab):
    d = tab[key]
    w = d.get("SQ_WAVES", 1.0) or 1.0
    print("%5s %5d " % key + " ".join("%12.0f" % (d.get(c, float("nan")) / (1 if c == "SQ_WAVES" else w)) for c in cols))
print("(per-wave values except SQ_WAVES; cycle counters in quad-cycles)")
