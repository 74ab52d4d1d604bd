#!/usr/bin/env python3
"""Fit time at a generic nbin against the neighbouring power of two (same
subints x channels, phase + DM, guess): where the direct-sum data pass
(k_data_xspec_gen, O(nbin^2) per row) puts the generic-length path.

  generic_nbin_probe.py [NSUB] [NCHAN]
"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))))
from pulseportraiture_amd import synth  # noqa: E402
from pulseportraiture_amd.engine import Engine  # noqa: E402

nsub = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
nchan = int(sys.argv[2]) if len(sys.argv) > 2 else 64
eng = Engine(0)
eng.set_timing(True)
for nbin in (1024, 1000, 2048, 1536):
    w = synth.make_workload(1, nchan, nbin, seed=5)
    one = torch.as_tensor(synth.workload_data_host(w)[0], device="cuda")
    data = one.expand(nsub, nchan, nbin).contiguous()
    nu = float(np.mean(w.freqs))
    args = (data, w.model, w.freqs, w.P, [0.0, w.DM0, 0, 0, 0], [1, 1, 0, 0, 0])
    eng.fit_batch(*args, nu_fit=[nu] * 3, guess=True)
    torch.cuda.synchronize()
    eng.reset_kernel_times()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        eng.fit_batch(*args, nu_fit=[nu] * 3, guess=True)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    ks = {k: eng.kernel_time(k)[0] / reps for k in ("data_xspec", "guess", "fit_taylor", "post",
                                                     "model_fft")}
    print("nbin %5d  %8.2f ms per %d x %d fit  %s" % (
        nbin, ms, nsub, nchan, " ".join("%s %.2f" % kv for kv in ks.items())), flush=True)
