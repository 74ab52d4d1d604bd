#!/usr/bin/env python3
"""Run tools/probe_xspec.hip (built into tools/libprobe_xspec.so by
`probe_xspec.py build`, on CPU) at the headline shape and report each mode's
ms and HBM rate next to k_data_xspec<10>'s (one bench step's HIP-event
time of the data pass).  Diagnostic."""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tools", "libprobe_xspec.so")


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                           "-fPIC", "-shared", "-I" + os.path.join(ROOT, "include"),
                           "-I" + os.path.join(ROOT, "pulseportraiture_amd", "csrc"),
                           os.path.join(ROOT, "tools", "probe_xspec.hip"), "-o", LIB])


def run(nsub=10000, reps=6):
    import torch
    lib = ctypes.CDLL(LIB)
    dev = torch.device("cuda", 0)
    d = torch.randn(nsub, 64, 2048, dtype=torch.float64, device=dev)
    M = torch.randn(64, 1040, 2, dtype=torch.float64, device=dev)
    X = torch.empty(nsub, 64, 1040, 2, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    byts = nsub * (64 * 2048 * 8 + 64 * 1040 * 16)
    for mode in (0, 1, 2):
        ts = []
        for r in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            rc = lib.probe_xspec(mode, nsub, ctypes.c_void_p(d.data_ptr()),
                                 ctypes.c_void_p(M.data_ptr()), ctypes.c_void_p(X.data_ptr()),
                                 ctypes.c_void_p(st.cuda_stream))
            b.record(st)
            torch.cuda.synchronize()
            assert rc == 0
            if r:
                ts.append(a.elapsed_time(b))
        ms = sorted(ts)[len(ts) // 2]
        print("mode %d: %.3f ms  %.2f TB/s (%.3f of 8)" % (mode, ms, byts / ms / 1e9,
                                                         byts / ms / 1e9 / 8.0), flush=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["build"]:
        build()
    else:
        run(*(int(x) for x in sys.argv[1:]))
