#!/usr/bin/env python3
"""Build an A/B variant of libppfit.so with extra -D flags into
pulseportraiture_amd/variants/libppfit_NAME.so (selected at run time with
PPF_LIB=...).  usage: build_variant.py NAME [-DFLAG=V ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pulseportraiture_amd import build as B  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
out = os.path.join(B.HERE, "variants", "libppfit_%s.so" % name)
os.makedirs(os.path.dirname(out), exist_ok=True)
cmd = [B.HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
       "-I" + os.path.join(ROOT, "include"), "-I" + B.CSRC] + flags + \
      [os.path.join(B.CSRC, B.SOURCES[0]), "-o", out]
print(" ".join(cmd))
subprocess.check_call(cmd)
