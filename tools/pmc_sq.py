"""Per-kernel SQ counter summary of one rocprofv3 --pmc pass (per-wave values)."""
import csv, re, sys
from collections import defaultdict

t = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("msckf::", "").replace("void ", "")
    k = re.sub(r"\(.*", "", k)
    t[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in sorted(t.items()):
    w = d.get("SQ_WAVES", 0.0) or 1.0
    print("%-34s waves=%8d " % (k[:34], w) + " ".join(
        "%s=%.0f" % (c.replace("SQ_", "").lower(), v if c in ("SQ_WAVES", "SQ_BUSY_CYCLES") else v / w)
        for c, v in sorted(d.items()) if c != "SQ_WAVES"))
