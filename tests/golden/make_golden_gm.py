#!/usr/bin/env python3
"""The reference's get_TOAs fits at config 4's shape (gm_1k.npz).

TEST INFRASTRUCTURE ONLY -- run in the build container, never on the GPU box
and never by the product.  The reference is loaded through the SURVEY.md
§8(c) shim exactly as in make_golden.py; only numbers are written.

bench.py --config gm fits synthetic subints of 128 channels x 2048 bins for
phi, DM and GM (BASELINE config 4, 1M subints sharded over 8 GPUs).  For the
first NSUB of them (the same Philox seed and subint indices, regenerated on
the host) this runs get_TOAs' per-subint flow with the reference's own
functions (pptoas.py:383-488): load_data's noise, guess_fit_freq with SNRs
1, the phase guess (pptoas.py:420-456), then pptoaslib.fit_portrait_full
(trust-ncg, fit_flags [1,1,1,0,0], option 0: nu_zero from the GM cubic,
pptoaslib.py:779-812).  The reference's own spread is recorded with it:
restarts from the guess moved one ulp either way, and NPERM fits with the
channels in seeded random orders (only the order of the channel sums
changes).

Fixture gm_1k.npz: per subint phi, phi_err, DM, DM_err, GM, GM_err, nu_DM,
status, nfev, red_chi2, snr, the guess and nu_fit; alt_<field> [nsub, nalt]
for the restarts and channel orders.

Usage:  python tests/golden/make_golden_gm.py [NSUB] [NPERM]
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
from pulseportraiture_amd import synth  # noqa: E402

SEED = 20240917  # bench.py --seed default
NCHAN, NBIN, FLAGS = 128, 2048, [1, 1, 1, 0, 0]
PERM_BASE = 11000
MAIN = ["phi", "phi_err", "DM", "DM_err", "GM", "GM_err", "nu_DM", "status", "nfev",
        "red_chi2", "snr", "phi_guess", "nu_fit"]
ALT = ["phi", "DM", "GM", "nu_DM", "status", "nfev"]


def ref_subint(pplib, pptoaslib, i, model, nperm):
    w = synth.make_workload(1, NCHAN, NBIN, seed=SEED, sub0=i)
    port = synth.workload_data_host(w)[0]
    freqs = w.freqs
    errs = pplib.get_noise(port, chans=True)
    nu_fit = pplib.guess_fit_freq(freqs, np.ones(NCHAN))
    nu_mean = freqs.mean()
    rot = pplib.rotate_data(port, 0.0, MG.DM0, w.P, freqs, nu_mean)
    prof = np.average(rot, axis=0, weights=np.ones(NCHAN))
    phi_g = pplib.fit_phase_shift(prof, model.mean(axis=0), Ns=100).phase
    phi_g = pplib.phase_transform(phi_g, MG.DM0, nu_mean, nu_fit, w.P, mod=True)
    init = [phi_g, MG.DM0, 0.0, 0.0, 0.0]

    def fit(x0, p=None):
        if p is None:
            p = np.arange(NCHAN)
        with contextlib.redirect_stdout(io.StringIO()):
            return pptoaslib.fit_portrait_full(port[p], model[p], x0, w.P, freqs[p],
                                               [nu_fit] * 3, [None] * 3, errs[p], list(FLAGS),
                                               None, False, option=0, sub_id=None,
                                               method="trust-ncg", is_toa=True, quiet=True)
    r = fit(list(init))
    main = [r.phi, r.phi_err, r.DM, r.DM_err, r.GM, r.GM_err, r.nu_DM, r.return_code,
            r.nfeval, r.red_chi2, r.snr, phi_g, nu_fit]
    alts = []
    for d in (np.inf, -np.inf):
        x0 = list(init)
        x0[0] = np.nextafter(x0[0], d)
        q = fit(x0)
        alts.append([q.phi, q.DM, q.GM, q.nu_DM, q.return_code, q.nfeval])
    rng = np.random.default_rng(PERM_BASE + i)
    for _ in range(nperm):
        q = fit(list(init), rng.permutation(NCHAN))
        alts.append([q.phi, q.DM, q.GM, q.nu_DM, q.return_code, q.nfeval])
    return i, main, alts


def _worker(args):
    subs, nperm = args
    import warnings
    warnings.simplefilter("ignore")
    import shutil
    tmp, pplib, pptoaslib, _, _ = MG.load_reference()
    try:
        model = synth.make_workload(1, NCHAN, NBIN, seed=SEED).model
        return [ref_subint(pplib, pptoaslib, i, model, nperm) for i in subs]
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main(nsub=600, nperm=2, nproc=8):
    from multiprocessing import Pool
    os.environ["OMP_NUM_THREADS"] = "1"
    chunks = [(list(range(k, nsub, nproc)), nperm) for k in range(nproc)]
    t0 = time.time()
    with Pool(nproc) as p:
        parts = p.map(_worker, chunks)
    got = {i: (m, a) for part in parts for i, m, a in part}
    M = np.array([got[i][0] for i in range(nsub)], dtype=float)
    A = np.array([got[i][1] for i in range(nsub)], dtype=float)  # [nsub, nalt, field]
    print("gm %d subints: %.1f s" % (nsub, time.time() - t0))
    out = {c: M[:, j] for j, c in enumerate(MAIN)}
    out.update({"alt_" + c: A[:, :, j] for j, c in enumerate(ALT)})
    out.update(seed=np.array(SEED), nsub=np.array(nsub), nperm=np.array(nperm),
               perm_base=np.array(PERM_BASE))
    for name, sig in (("phi", "phi_err"), ("DM", "DM_err"), ("GM", "GM_err")):
        d = (np.abs(out["alt_" + name] - out[name][:, None]) / out[sig][:, None]).max(axis=1)
        print("%s: reference's own spread > 1e-3 sigma on %d (max %.3g)" % (
            name, np.sum(d > 1e-3), d.max()))
    MG.save("gm_1k.npz", **out)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
