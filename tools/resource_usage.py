#!/usr/bin/env python3
"""Per-kernel register / LDS / scratch use of libppfit (hipcc
-Rpass-analysis=kernel-resource-usage on the unity source, no GPU).

  resource_usage.py [FILTER ...] [-- -DFLAG=V ...]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pulseportraiture_amd import build as B  # noqa: E402

args = sys.argv[1:]
flags = args[args.index("--") + 1:] if "--" in args else []
filt = args[:args.index("--")] if "--" in args else args
with tempfile.TemporaryDirectory() as d:
    cmd = [B.HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I" + os.path.join(ROOT, "include"), "-I" + B.CSRC] + flags + \
          [os.path.join(B.CSRC, B.SOURCES[0]), "-o", os.path.join(d, "x.so"),
           "-Rpass-analysis=kernel-resource-usage"]
    txt = subprocess.run(cmd, capture_output=True, text=True, check=True).stderr
rows, cur = [], None
for line in txt.splitlines():
    m = re.search(r"remark: (?:\s*)Function Name: (\S+)", line)
    if m:
        cur = {"name": subprocess.run(["c++filt", m.group(1)], capture_output=True,
                                      text=True).stdout.strip()}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\S+) \[-Rpass", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
for r in rows:
    if filt and not any(f in r["name"] for f in filt):
        continue
    print("%-48s VGPR %4s spill %3s scratch %4s LDS %6s occ %s" % (
        r["name"].replace("void ppf::", "").replace("(ppf::FitArgs)", "")[:48], r.get("VGPRs"),
        r.get("VGPRs Spill"), r.get("ScratchSize"), r.get("LDS Size"), r.get("Occupancy")))
