"""ppalign (config 5) under engine options / SPEC_CACHE settings, one process:
  python tools/ab_ppalign_opts.py [narch] [niter]
Prints per setting the faster of two timed align_archives calls (ms per
iteration) and the per-iteration kernel times (HIP events, a third call)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pulseportraiture_amd import archive, ppalign, synth  # noqa: E402
from pulseportraiture_amd.engine import get_engine  # noqa: E402

SETTINGS = [("cache", True, {}), ("cache, moments apart", True, {"fuse_moments": 0}),
            ("plain", False, {})]


def main():
    narch = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    niter = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    eng = get_engine(0)
    nchan, nbin = 256, 2048
    w = synth.make_workload(narch, nchan, nbin, seed=20240917 + 555)
    data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
    names = ["ab_pa_%d" % i for i in range(narch)]
    archive.register_archives(names, [dict(subints=data[i:i + 1, None], freqs=w.freqs, Ps=[w.P],
                                           epochs=[(57000 + i, 0, 0.0)], DM=w.DM0)
                                      for i in range(narch)])
    archive.register_archive("ab_pa_guess", dict(subints=w.model[None, None], freqs=w.freqs,
                                                 Ps=[w.P], epochs=[(57000, 0, 0.0)], DM=w.DM0,
                                                 dmc=1))
    ports = {}
    for label, cache, opts in SETTINGS:
        ppalign.SPEC_CACHE = cache
        saved = {k: eng.get_option(k) for k in opts}
        for k, v in opts.items():
            eng.set_option(k, v)
        try:
            ppalign.align_archives(names, "ab_pa_guess", fit_dm=True, niter=niter, quiet=True)
            calls = []
            for _ in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                port = ppalign.align_archives(names, "ab_pa_guess", fit_dm=True, niter=niter,
                                              quiet=True)
                torch.cuda.synchronize()
                calls.append(time.perf_counter() - t0)
            ports[label] = port
            eng.set_timing(True)
            eng.reset_kernel_times()
            ph = {}
            ppalign.align_archives(names, "ab_pa_guess", fit_dm=True, niter=niter, quiet=True,
                                   timings=ph)
            kt = {k: eng.kernel_time(k)[0] / niter for k in
                  ("data_xspec", "rot_accum", "guess", "moments", "fit_taylor", "post")}
            eng.set_timing(False)
        finally:
            for k, v in saved.items():
                eng.set_option(k, v)
        print("%-22s %.2f ms/iter  calls %s  phases %s\n%24s%s" % (
            label, min(calls) / niter * 1e3, [round(c * 1e3, 1) for c in calls],
            {k: round(v * 1e3, 2) for k, v in ph.items() if k != "start"}, "",
            " ".join("%s %.3f" % kv for kv in kt.items())), flush=True)
    ppalign.SPEC_CACHE = True
    ref = ports["plain"]
    for k, p in ports.items():
        print("%-22s max |port - plain| / max|plain| = %.3g" % (
            k, np.abs(p - ref).max() / np.abs(ref).max()))


if __name__ == "__main__":
    main()
