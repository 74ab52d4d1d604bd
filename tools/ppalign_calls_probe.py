"""Wall time of consecutive align_archives calls at config 5 (the bench
leg's set-up), each with its phase split: does a call's time depend on its
position after the warm-up?"""
import gc
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pulseportraiture_amd import archive, ppalign, synth  # noqa: E402
from pulseportraiture_amd.engine import get_engine  # noqa: E402


def main():
    eng = get_engine()
    narch = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    _, nchan, nbin, _, _, _, _, _ = bench.CONFIGS["ppalign"]
    w = synth.make_workload(narch, nchan, nbin, seed=555)
    data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
    torch.cuda.synchronize()
    names = ["pc_%d" % i for i in range(narch)]
    archive.register_archives(names, [dict(subints=data[i:i + 1, None], freqs=w.freqs, Ps=[w.P],
                                           epochs=[(57000 + i, 0, 0.0)], DM=w.DM0)
                                      for i in range(narch)])
    archive.register_archive("pc_guess", dict(subints=w.model[None, None], freqs=w.freqs,
                                              Ps=[w.P], epochs=[(57000, 0, 0.0)], DM=w.DM0, dmc=1))
    gct = {"n2": 0, "t2": 0.0, "t": 0.0}

    def cb(phase, info):  # full (generation 2) collections and their time
        if phase == "start":
            gct["t"] = time.perf_counter()
        elif info["generation"] == 2:
            gct["n2"] += 1
            gct["t2"] += time.perf_counter() - gct["t"]
    gc.callbacks.append(cb)
    for k in range(6):
        gct["n2"], gct["t2"] = 0, 0.0
        ph = {} if k >= 3 else None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ppalign.align_archives(names, "pc_guess", fit_dm=True, niter=3, quiet=True, timings=ph)
        torch.cuda.synchronize()
        print("call %d: %.1f ms (gen-2 collections %d, %.1f ms) %s" % (
            k, (time.perf_counter() - t0) * 1e3, gct["n2"], gct["t2"] * 1e3,
                                       "" if ph is None else
                                       {a: round(b * 1e3, 1) for a, b in ph.items()}), flush=True)


if __name__ == "__main__":
    main()
