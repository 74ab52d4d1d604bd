#!/usr/bin/env python3
"""The reference's headline fits (headline_2k.npz) under reordered sums.

TEST INFRASTRUCTURE ONLY -- run in the build container, never on the GPU box
and never by the product.  The reference is loaded through the SURVEY.md
§8(c) shim exactly as in make_golden.py; only numbers are written.

Each of the 2,000 subints of headline_2k.npz (64 x 2048, phase + DM, the
get_TOAs guess + trust-ncg, make_golden_r2.ref_subint) is fitted again from
the same start with its channels in NPERM seeded random orders -- data,
template, frequencies and noise permuted together, so only the order of the
reference's own channel sums changes.  With gtol = -1 the last steps of
trust-ncg are decided at the objective's rounding (pptoaslib.py:1002), so
these runs give the reference's own spread in phi, DM and nfev.

Fixture headline_2k_perm.npz: perm_phi, perm_DM, perm_nu_DM, perm_status,
perm_nfev [nsub, NPERM]; perm_seed = base + subint.

Usage:  python tests/golden/make_golden_hl_perm.py [NSUB] [NPERM]
"""
import contextlib
import io
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import make_golden as MG  # noqa: E402
import make_golden_r2 as R2  # noqa: E402
from pulseportraiture_amd import synth  # noqa: E402

PERM_BASE = 9000
FIELDS = ["phi", "DM", "nu_DM", "status", "nfev"]


def perm_subint(pplib, pptoaslib, i, model, nperm, z):
    w = synth.make_workload(1, 64, 2048, seed=R2.HEAD_SEED, sub0=i)
    port = synth.workload_data_host(w)[0]
    freqs = w.freqs
    errs = pplib.get_noise(port, chans=True)
    nu_fit = float(z["nu_fit"][i])
    init = [float(z["phi_guess"][i]), MG.DM0, 0.0, 0.0, 0.0]
    rng = np.random.default_rng(PERM_BASE + i)
    rows = []
    for _ in range(nperm):
        p = rng.permutation(64)
        with contextlib.redirect_stdout(io.StringIO()):
            r = pptoaslib.fit_portrait_full(port[p], model[p], list(init), w.P, freqs[p],
                                            [nu_fit] * 3, [None] * 3, errs[p], [1, 1, 0, 0, 0],
                                            None, False, option=0, sub_id=None,
                                            method="trust-ncg", is_toa=True, quiet=True)
        rows.append([r.phi, r.DM, r.nu_DM, r.return_code, r.nfeval])
    return i, rows


def _worker(args):
    subs, nperm = args
    import warnings
    warnings.simplefilter("ignore")
    import shutil
    tmp, pplib, pptoaslib, _, _ = MG.load_reference()
    try:
        z = np.load(os.path.join(HERE, "headline_2k.npz"))
        model = synth.make_workload(1, 64, 2048, seed=R2.HEAD_SEED).model
        return [perm_subint(pplib, pptoaslib, i, model, nperm, z) for i in subs]
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main(nsub=2000, nperm=4, nproc=8):
    from multiprocessing import Pool
    os.environ["OMP_NUM_THREADS"] = "1"
    chunks = [(list(range(k, nsub, nproc)), nperm) for k in range(nproc)]
    t0 = time.time()
    with Pool(nproc) as p:
        parts = p.map(_worker, chunks)
    got = dict(r for part in parts for r in part)
    arr = np.array([got[i] for i in range(nsub)], dtype=float)
    print("headline %d subints x %d channel orders: %.1f s" % (nsub, nperm, time.time() - t0))
    out = {"perm_" + f: arr[:, :, j] for j, f in enumerate(FIELDS)}
    out.update(nsub=np.array(nsub), nperm=np.array(nperm), perm_base=np.array(PERM_BASE))
    MG.save("headline_2k_perm.npz", **out)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
