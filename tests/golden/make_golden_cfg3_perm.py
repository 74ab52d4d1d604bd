#!/usr/bin/env python3
"""The reference's config-3 scattering fits under reordered sums.

TEST INFRASTRUCTURE ONLY -- run in the build container, never on the GPU box
and never by the product.  The reference is loaded through the SURVEY.md
§8(c) shim exactly as in make_golden.py; only numbers are written.

make_golden_cfg3.py records, per subint, the reference's end point and four
restarts one ulp away.  A one-ulp restart perturbs the start, not the
rounding of the objective's sums, and on these fits (trust-ncg with gtol = -1
stops at the first predicted reduction <= 0, pptoaslib.py:1002, scipy
_trustregion.py) that rounding decides where the fit stops.  This script
reruns each of the same subints with its channels in NPERM seeded random
orders: data, template, frequencies and noise permuted together, so every
per-channel term is the same number and only the order of the reference's
own channel sums changes (pptoaslib.py:525-643, 733-836).  Whatever end
points the reference reaches this way are its own answers on that input.

Fixture scattering_200_perm.npz: per subint and permutation, phi, DM, tau,
alpha (at the permuted fit's own nu_DM / nu_tau), nu_DM, nu_tau, status,
nfev and red_chi2 ([nsub, NPERM] each); perm_seed = base + subint.

Usage:  python tests/golden/make_golden_cfg3_perm.py [NSUB] [NPERM]
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
import make_golden_cfg3 as C3  # noqa: E402
from pulseportraiture_amd import synth  # noqa: E402

PERM_BASE = 7000
FIELDS = ["phi", "DM", "tau", "alpha", "nu_DM", "nu_tau", "status", "nfev", "red_chi2"]


def perm_subint(pplib, pptoaslib, i, model, nperm):
    w = synth.make_workload(1, C3.NCHAN, C3.NBIN, seed=C3.SEED, sub0=i, tau=C3.TAU)
    port = synth.workload_data_host(w)[0]
    freqs = w.freqs
    errs = pplib.get_noise(port, chans=True)
    # get_TOAs' guess exactly as make_golden_cfg3.ref_subint (channel order
    # as stored: the guess is not what is being perturbed)
    nu_fit = pplib.guess_fit_freq(freqs, np.ones(C3.NCHAN))
    nu_mean = freqs.mean()
    tau_g = C3.TAU * (nu_fit / w.nu_ref) ** w.alpha
    rot = pplib.rotate_data(port, 0.0, MG.DM0, w.P, freqs, nu_mean)
    prof = np.average(rot, axis=0, weights=np.ones(C3.NCHAN))
    prof_scat = np.fft.irfft(pplib.scattering_portrait_FT(
        np.array([pplib.scattering_times(tau_g, w.alpha, nu_fit, nu_fit)]), C3.NBIN)[0] *
        np.fft.rfft(model.mean(axis=0)))
    phi_g = pplib.fit_phase_shift(prof, prof_scat, Ns=100).phase
    phi_g = pplib.phase_transform(phi_g, MG.DM0, nu_mean, nu_fit, w.P, mod=True)
    init = [phi_g, MG.DM0, 0.0, np.log10(tau_g), w.alpha]
    rng = np.random.default_rng(PERM_BASE + i)
    rows = []
    for _ in range(nperm):
        p = rng.permutation(C3.NCHAN)
        with contextlib.redirect_stdout(io.StringIO()):
            r = pptoaslib.fit_portrait_full(port[p], model[p], list(init), w.P, freqs[p],
                                            [nu_fit] * 3, [None] * 3, errs[p], list(C3.FLAGS),
                                            None, True, option=0, sub_id=None,
                                            method="trust-ncg", is_toa=True, quiet=True)
        rows.append([r.phi, r.DM, r.tau, r.alpha, r.nu_DM, r.nu_tau, r.return_code, r.nfeval,
                     r.red_chi2])
    return i, rows


def _worker(args):
    subs, nperm = args
    import warnings
    warnings.simplefilter("ignore")
    import shutil
    tmp, pplib, pptoaslib, _, _ = MG.load_reference()
    try:
        model = synth.make_workload(1, C3.NCHAN, C3.NBIN, seed=C3.SEED, tau=C3.TAU).model
        return [perm_subint(pplib, pptoaslib, i, model, nperm) for i in subs]
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main(nsub=200, nperm=8, nproc=8):
    from multiprocessing import Pool
    os.environ["OMP_NUM_THREADS"] = "1"
    chunks = [(list(range(k, nsub, nproc)), nperm) for k in range(nproc)]
    t0 = time.time()
    with Pool(nproc) as p:
        parts = p.map(_worker, chunks)
    got = dict(r for part in parts for r in part)
    arr = np.array([got[i] for i in range(nsub)], dtype=float)  # [nsub, nperm, nfield]
    print("scattering %d subints x %d channel orders: %.1f s" % (nsub, nperm, time.time() - t0))
    out = {"perm_" + f: arr[:, :, j] for j, f in enumerate(FIELDS)}
    out.update(seed=np.array(C3.SEED), nsub=np.array(nsub), nperm=np.array(nperm),
               perm_base=np.array(PERM_BASE))
    MG.save("scattering_200_perm.npz", **out)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
