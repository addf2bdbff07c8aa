#!/bin/bash
# Register / scratch / occupancy of every step-kernel instance (hipcc kernel-resource-usage remarks).
#   tools/res_usage.sh [out-file]
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R/lattice-boltzmann-method-gpu_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -c csrc/lbm_kernels.hip -o /tmp/lbm_res.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re, sys
cur = None
rows = {}
for ln in sys.stdin:
    m = re.search(r"Function Name: (\S+)", ln)
    if m: cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark: +(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", ln)
    if m and cur: rows[cur][m.group(1).split()[0]] = int(m.group(2))
for k in sorted(rows):
    if "k_step" in k:
        r = rows[k]; print("%-70s vgpr %s scratch %s occ %s" % (k, r.get("VGPRs"), r.get("ScratchSize"), r.get("Occupancy")))
' | tee ${1:-/dev/null}
