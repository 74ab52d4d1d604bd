#!/usr/bin/env python3
"""Bitwise A/B of two libppfit builds on bench.py's synthetic batches.

  ab_bitwise.py run OUT.npz CONFIG NSUB [exact|tnc|ncg]   (GPU; library from PPF_LIB)
  ab_bitwise.py cmp A.npz B.npz

`run` fits the config's batch once (trust-ncg, or the exact-sweep / TNC /
Newton-CG paths) and saves every per-TOA output; `cmp` reports how many
entries differ and fails unless all are bitwise equal.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KEYS = ["params", "param_errs", "nu_out", "red_chi2", "snr", "status", "nfev"]


def run(out, config, nsub, variant):
    import torch
    import bench
    from pulseportraiture_amd.engine import Engine
    eng = Engine(0)
    w, data, kw, _ = bench.synth_inputs(eng, config, nsub, 20240917, 0)
    flags = bench.CONFIGS[config][3]
    log10_tau = bench.CONFIGS[config][5]
    extra = {}
    if variant == "exact":
        extra["exact"] = True
    elif variant == "tnc":
        extra["method"] = "TNC"
    elif variant == "ncg":
        extra["method"] = "Newton-CG"
    res = eng.fit_batch(data, kw["model"], kw["freqs"], kw["P"], kw["init"], flags,
                        nu_fit=kw["nu"], log10_tau=log10_tau, guess=True, guess_Ns=100,
                        guess_tau=kw["gtau"], **extra)
    torch.cuda.synchronize()
    np.savez(out, **{k: res[k].cpu().numpy() for k in KEYS})
    print("saved", out, "mean nfev %.3f" % res["nfev"].double().mean().item(), flush=True)


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in KEYS:
        x, y = A[k], B[k]
        same = (x.view(np.uint8) == y.view(np.uint8)).reshape(x.shape[0], -1).all(axis=1) \
            if x.dtype.kind == "f" else (x == y).reshape(x.shape[0], -1).all(axis=1)
        nd = int((~same).sum())
        bad += nd
        print("%-10s %d of %d rows differ" % (k, nd, len(same)))
    print("BITWISE_EQUAL" if bad == 0 else "DIFFER")
    return bad == 0


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5] if len(sys.argv) > 5 else "")
    else:
        sys.exit(0 if cmp(sys.argv[2], sys.argv[3]) else 1)
