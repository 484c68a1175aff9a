"""Print the top kernels of a rocprofv3 kernel_stats.csv: python tools/kstats.py FILE [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    name = r["Name"].replace("msckf::", "").replace("(anonymous namespace)::", "").replace("void ", "")
    print("%-58s %5s %10.1f us" % (name[:58], r["Calls"], float(r["AverageNs"]) / 1e3))
