#!/usr/bin/env python3
"""Host-side cost of GetTOAs.get_TOAs with the device fit stubbed out.

Registers one archive of NSUB subints x 64 chan x NBIN bins (the data are
never read by the stub), replaces pptoas.fit_pipeline with a synchronous pipeline over a function
that returns result arrays of the right shapes at zero cost, and times
get_TOAs end to end (metadata, per-subint set-up, TOA records) plus the .tim
text of every TOA (write_TOAs' bulk writer, checked against the per-TOA
toa_line text).  usage: host_driver_bench.py [NSUB] [NBIN]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def stub_fit(data, model, init, P, freqs, nu_fits=None, nu_outs=None, errs=None,
             fit_flags=(1, 1, 0, 0, 0), chan_mask=None, **kw):
    n, nchan = np.shape(data)[:2]
    init = np.asarray(init, dtype=np.float64)
    cov = np.zeros((n, 5, 5))
    cov[:, 0, 0], cov[:, 1, 1], cov[:, 0, 1] = 1e-8, 4e-8, 1e-9
    return dict(params=init + 1e-4, param_errs=np.tile([1e-4, 2e-4, 0, 0, 0], (n, 1)),
                nu_out=np.asarray(nu_fits, dtype=np.float64).reshape(n, 3).copy(), cov=cov,
                scales=np.ones((n, nchan)), scale_errs=np.full((n, nchan), 0.1),
                channel_snrs=np.full((n, nchan), 10.0), chi2=np.full(n, 2048.0),
                red_chi2=np.ones(n), snr=np.full(n, 80.0), nfev=np.full(n, 5, np.int32),
                status=np.full(n, 2, np.int32))


def main():
    from pulseportraiture_amd import archive, pplib, pptoas, synth
    from pulseportraiture_amd.pptoaslib import SyncPipeline
    from pulseportraiture_amd.mjd import MJD
    nsub = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    nbin = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    nchan = 64
    w = synth.make_workload(1, nchan, nbin, seed=1)
    sub = np.zeros((nsub, 1, nchan, nbin))
    archive.register_archive("hostbench.fits", dict(
        subints=sub, freqs=w.freqs, Ps=np.full(nsub, w.P),
        epochs=[MJD(57000.0 + 1e-3 * k) for k in range(nsub)], DM=w.DM0))
    pptoas.fit_pipeline = lambda keys: SyncPipeline(stub_fit, keys)
    pptoas.gen_gaussian_portraits_device = lambda code, params, alpha, nb, freqs, nu_ref: \
        np.zeros((len(np.atleast_2d(freqs)), nchan, nb))
    # warm-up on the same archive: numpy / module first-use costs are per process
    pptoas.GetTOAs(["hostbench.fits"], synth.EXAMPLE_GMODEL, quiet=True).get_TOAs(quiet=True)
    gt = pptoas.GetTOAs(["hostbench.fits"], synth.EXAMPLE_GMODEL, quiet=True)
    t0 = time.perf_counter()
    gt.get_TOAs(quiet=True)
    t1 = time.perf_counter()
    pplib.write_TOAs(gt.TOA_list, outfile="/tmp/hostbench.tim", append=False)
    t2 = time.perf_counter()
    lines = open("/tmp/hostbench.tim").read().splitlines()
    assert len(lines) == nsub
    slow = [pplib.toa_line(t) for t in gt.TOA_list]  # TOA objects, one line each
    t3 = time.perf_counter()
    assert slow == lines, "bulk .tim text differs from the per-TOA text"
    print("per-TOA objects + toa_line: %.3f s" % (t3 - t2))
    print("nsub %d: get_TOAs %.3f s (%.0f TOAs/s), .tim text %.3f s (%.0f lines/s), "
          "together %.0f TOAs/s" % (nsub, t1 - t0, nsub / (t1 - t0), t2 - t1,
                                    nsub / (t2 - t1), nsub / (t2 - t0)))


if __name__ == "__main__":
    main()
