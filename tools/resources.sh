#!/bin/bash
# Per-kernel VGPR / SGPR spill / scratch / occupancy of libppfit for gfx950.
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -c \
  -Iinclude -Ipulseportraiture_amd/csrc pulseportraiture_amd/csrc/ppfit_lib.hip -o /tmp/ppfit_dev.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys, subprocess
pat = sys.argv[1] if len(sys.argv) > 1 else ""
cur = {}
rows = []
for ln in sys.stdin:
    m = re.search(r"remark:\s+(.*?):\s+(\S+) \[-Rpass", ln)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    else:
        cur[k] = v
for r in rows:
    if pat and not re.search(pat, r["name"]):
        continue
    print("%-44s vgpr %4s vspill %3s sspill %3s scratch %5s occ %s lds %s" % (r["name"][:44], r.get("VGPRs"), r.get("VGPRs Spill"),
          r.get("SGPRs Spill"), r.get("ScratchSize [bytes/lane]"), r.get("Occupancy [waves/SIMD]"),
          r.get("LDS Size [bytes/block]")))
' "$1"
