#!/usr/bin/env python3
"""Oracle vs reference wall time per BASELINE config (round 3).

TEST INFRASTRUCTURE ONLY -- run in the build container, never on the GPU box.
The reference is loaded through the SURVEY.md §8(c) shim (make_golden.py);
only timings are written, into tests/golden/timing_r3.json.  bench.py's
cpu_baseline leg times the oracle on the GPU box's host cores and divides by
the ratio measured here, so the reported rate can also be read as the
reference's own (target ratio 0.8-1.25, both reported if not).

Per config, one thread each (threadpoolctl), the same pre-generated subints
for both:
  headline   64 x 2048 phase+DM: get_TOAs guess + trust-ncg fit (pptoas.py:383-488)
  gm         128 x 2048 phase+DM+GM
  scattering 512 x 1024 phase+DM+tau+alpha, log10 tau, scattered guess template
  ppalign    256 x 2048 one align_archives unit: guess (Ns = nbin at nu_fit),
             phase+DM fit, rotate_data + weighted accumulate (ppalign.py:160-208)

Usage:  python tests/golden/make_timing_r3.py [n_headline]
"""
import json
import os
import sys
import time
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import make_golden as MG  # noqa: E402
from pulseportraiture_amd import synth  # noqa: E402

SEED = 20240917
CONFIGS = {
    # name: (nchan, nbin, flags, tau [rot at 1500 MHz], log10_tau, n)
    "headline": (64, 2048, (1, 1, 0, 0, 0), 0.0, False, 8),
    "gm": (128, 2048, (1, 1, 1, 0, 0), 0.0, False, 4),
    "scattering": (512, 1024, (1, 1, 0, 1, 1), 2e-3, True, 2),
    "ppalign": (256, 2048, (1, 1, 0, 0, 0), 0.0, False, 3),
}


def ref_toa(pplib, pptoaslib, port, model, freqs, P, flags, log10_tau, tau_g, alpha_g):
    """The reference's per-subint get_TOAs work, pptoas.py:383-488."""
    nchan, nbin = port.shape
    errs = pplib.get_noise(port, chans=True)
    nu_fit = pplib.guess_fit_freq(freqs, np.ones(nchan))
    nu_mean = freqs.mean()
    rot = pplib.rotate_data(port, 0.0, MG.DM0, P, freqs, nu_mean)
    prof = np.average(rot, axis=0, weights=np.ones(nchan))
    mprof = model.mean(axis=0)
    if flags[3]:
        mprof = np.fft.irfft(pplib.scattering_portrait_FT(np.array([
            pplib.scattering_times(tau_g, alpha_g, nu_fit, nu_fit)]), nbin)[0] *
            np.fft.rfft(mprof))
    phi = pplib.fit_phase_shift(prof, mprof, Ns=100).phase
    phi = pplib.phase_transform(phi, MG.DM0, nu_mean, nu_fit, P, mod=True)
    t0 = np.log10(tau_g) if log10_tau else tau_g
    init = [phi, MG.DM0, 0.0, t0 if flags[3] else 0.0, alpha_g if flags[3] else 0.0]
    return pptoaslib.fit_portrait_full(port, model, init, P, freqs, [nu_fit] * 3, [None] * 3,
                                       errs, list(flags), None, log10_tau, option=0, sub_id=None,
                                       method="trust-ncg", is_toa=True, quiet=True)


def ref_align_unit(pplib, pptoaslib, port, model, freqs, P):
    """One align_archives unit (ppalign.py:160-208)."""
    nchan, nbin = port.shape
    errs = pplib.get_noise(port, chans=True)
    nu_fit = pplib.guess_fit_freq(freqs, np.ones(nchan))
    rot = pplib.rotate_data(port, 0.0, MG.DM0, P, freqs, nu_fit)
    phase = pplib.fit_phase_shift(np.average(rot, axis=0, weights=np.ones(nchan)),
                                  model.mean(axis=0), Ns=nbin).phase
    r = pptoaslib.fit_portrait_full(port, model, [phase, MG.DM0, 0.0, 0.0, 0.0], P, freqs,
                                    [nu_fit] * 3, [None] * 3, errs, [1, 1, 0, 0, 0],
                                    log10_tau=False, quiet=True)
    w = np.outer(r.scales / errs ** 2, np.ones(nbin))
    return w * pplib.rotate_data(port, r.phi, r.DM, P, freqs, r.nu_DM)


def orc_toa(O, port, model, freqs, P, flags, log10_tau, tau_g, alpha_g):
    nchan = port.shape[0]
    errs = O.get_noise_PS(port, chans=True)
    return O.fit_subint_pptoas(port, model, freqs, np.ones(nchan), errs, np.ones(nchan), P,
                               MG.DM0, flags, log10_tau=log10_tau, tau_guess=tau_g,
                               alpha_guess=alpha_g)


def orc_align_unit(O, port, model, freqs, P):
    nchan, nbin = port.shape
    errs = O.get_noise_PS(port, chans=True)
    nu_fit = O.guess_fit_freq(freqs, np.ones(nchan))
    phase = O.pptoas_guess(port, model, freqs, np.ones(nchan), MG.DM0, P, nu_fit, Ns=nbin,
                           nu_rot=nu_fit, wrap=False)
    r = O.fit_portrait_full(port, model, [phase, MG.DM0, 0.0, 0.0, 0.0], P, freqs,
                            [nu_fit] * 3, [None] * 3, errs, [1, 1, 0, 0, 0], log10_tau=False)
    w = np.outer(r.scales / errs ** 2, np.ones(nbin))
    return w * O.rotate_data(port, r.phi, r.DM, P, freqs, r.nu_DM)


def main():
    warnings.simplefilter("ignore")
    np.seterr(all="ignore")
    from threadpoolctl import threadpool_limits
    from oracle import ppfit_oracle as O
    tmp, pplib, pptoaslib, _, _ = MG.load_reference()
    out = {"threads": 1, "note": "same pre-generated subints for both legs; one warm-up "
                                 "subint each, untimed"}
    try:
        with threadpool_limits(limits=1):
            for name, (nchan, nbin, flags, tau, log10_tau, n) in CONFIGS.items():
                w = synth.make_workload(n, nchan, nbin, seed=SEED, tau=tau)
                ports = synth.workload_data_host(w)
                nu_fit = O.guess_fit_freq(w.freqs, np.ones(nchan))
                tau_g = tau * (nu_fit / w.nu_ref) ** w.alpha if flags[3] else 0.0
                alpha_g = w.alpha if flags[3] else 0.0
                if name == "ppalign":
                    ref = lambda p: ref_align_unit(pplib, pptoaslib, p, w.model, w.freqs, w.P)
                    orc = lambda p: orc_align_unit(O, p, w.model, w.freqs, w.P)
                else:
                    ref = lambda p: ref_toa(pplib, pptoaslib, p, w.model, w.freqs, w.P, flags,
                                            log10_tau, tau_g, alpha_g)
                    orc = lambda p: orc_toa(O, p, w.model, w.freqs, w.P, flags, log10_tau,
                                            tau_g, alpha_g)
                ref(ports[0])
                orc(ports[0])
                t0 = time.perf_counter()
                for p in ports:
                    ref(p)
                t_ref = (time.perf_counter() - t0) / n
                t0 = time.perf_counter()
                for p in ports:
                    orc(p)
                t_orc = (time.perf_counter() - t0) / n
                out[name] = dict(shape="%dx%d" % (nchan, nbin), flags=list(flags), subints=n,
                                 reference_s_per_unit=t_ref, oracle_s_per_unit=t_orc,
                                 ratio_oracle_over_reference=t_orc / t_ref)
                print(name, out[name], flush=True)
    finally:
        import shutil
        shutil.rmtree(tmp, ignore_errors=True)
    with open(os.path.join(HERE, "timing_r3.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
