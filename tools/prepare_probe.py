"""Where GetTOAs._prepare's ~2 ms go on the device box: the template build
(gen_gaussian_portraits_device: H2D of the frequencies, the kernel, D2H of
the portrait) and a bare pageable H2D, each timed alone.  Diagnostic."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from pulseportraiture_amd import pplib, synth  # noqa: E402
from pulseportraiture_amd.engine import get_engine  # noqa: E402

eng = get_engine(0)
w = synth.make_workload(1, 64, 2048, seed=1)
name, code, nu_ref, ngauss, gparams, mflags, alpha, fit_alpha = pplib.read_model(
    synth.EXAMPLE_GMODEL, quiet=True)
f = np.ascontiguousarray(w.freqs[None])


def t(fn, n=30):
    ts = []
    for _ in range(n):
        torch.cuda.synchronize()
        a = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - a)
    return "%.3f ms (min %.3f)" % (np.median(ts) * 1e3, min(ts) * 1e3)


dev = eng.device
print("as_tensor 64 doubles:", t(lambda: torch.as_tensor(f, device=dev)))
print("as_tensor + sync:", t(lambda: (torch.as_tensor(f, device=dev), torch.cuda.synchronize())))
print("gaussian_portraits (device):", t(lambda: eng.gaussian_portraits(code, gparams, alpha, 2048,
                                                                         f, nu_ref)))
print("gen_gaussian_portraits_device (+ D2H):", t(lambda: pplib.gen_gaussian_portraits_device(
    code, gparams, alpha, 2048, f, nu_ref)))
print("read_model:", t(lambda: pplib.read_model(synth.EXAMPLE_GMODEL, quiet=True)))
