#!/bin/bash
# Print VGPR / AGPR / scratch / LDS / occupancy per kernel (hipcc resource remarks).
SRC="${1:-visual-inertial-odometry-msckf-stereo_amd/csrc/msckf_kernels.hip}"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -fno-slp-vectorize -c "$SRC" -o /tmp/_ru.o \
    -Rpass-analysis=kernel-resource-usage 2>&1 | grep remark | sed 's/.*remark: //; s/ \[-Rpass.*//' \
 | python3 -c '
import sys, subprocess, re
rows, cur = [], {}
for line in sys.stdin:
    line = line.strip()
    if line.startswith("Function Name:"):
        cur = {"name": line.split()[-1]}; rows.append(cur)
    elif ":" in line:
        k, v = line.rsplit(":", 1); cur[k.strip()] = v.strip()
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, n in zip(rows, names):
    n = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "")).replace("msckf::", "").replace("void ", "")
    print("%-26s vgpr=%-4s agpr=%-4s scratch=%-5s lds=%-6s occ=%s" % (n, r.get("VGPRs"), r.get("AGPRs"), r.get("ScratchSize [bytes/lane]"), r.get("LDS Size [bytes/block]"), r.get("Occupancy [waves/SIMD]")))
'
