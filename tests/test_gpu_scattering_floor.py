"""Config 3 at its own shape against the reference: 200 of bench.py's
scattering subints (512 x 1024, phi + DM + log10 tau + alpha, get_TOAs' guess
and trust-ncg), fitted on the device and by the reference
(tests/golden/scattering_200.npz, make_golden_cfg3.py: the reference's
get_TOAs per-subint flow, pptoas.py:383-488, plus four restarts one ulp
away in phase and log10 tau).

What holds, and is asserted:
* the guess (init phase) and every status are the reference's;
* every device end point is as good a minimum as the reference's:
  |chi^2_device - chi^2_reference| <= 1e-3 (one sigma in one parameter
  moves chi^2 by 1);
* at least 85 % of the end points are within 1e-3 sigma of the reference's.
The rest are subints on which trust-ncg's stopping test (predicted
reduction <= 0, status 2) or the basin it settles in is decided by rounding:
the reference itself moves by > 1e-3 sigma under one-ulp restarts on 23 of
these 200 subints (up to 24 sigma), and the device ends within 2.2e-4 of the
reference's chi^2 wherever its parameters differ.  Every comparison prints.
"""
import os

import numpy as np
import pytest

from tests.conftest import GOLDEN
from tests.golden_consts import DM0

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pulseportraiture_amd.engine import get_engine
    return get_engine(0)


def test_scattering_200_subints_vs_reference(gpu):
    from pulseportraiture_amd import synth
    z = np.load(os.path.join(GOLDEN, "scattering_200.npz"))
    nsub, seed = int(z["nsub"]), int(z["seed"])
    nchan, nbin, tau = 512, 1024, 2e-3
    data = synth.workload_data_host_parallel(nsub, nchan, nbin, seed=seed,
                                             procs=min(16, os.cpu_count() or 1), tau=tau)
    w = synth.make_workload(1, nchan, nbin, seed=seed, tau=tau)
    nu = z["nu_fit"]
    tau_g = 10.0 ** z["init_tau"]
    init = np.stack([np.zeros(nsub), np.full(nsub, DM0), np.zeros(nsub), z["init_tau"],
                     z["init_alpha"]], 1)
    out = gpu.fit_batch(data, w.model, w.freqs, w.P, init, [1, 1, 0, 1, 1],
                        nu_fit=np.stack([nu] * 3, 1), log10_tau=True, guess=True, guess_Ns=100,
                        guess_tau=tau_g)
    r = {k: v.cpu().numpy() for k, v in out.items() if not k.startswith("_")}
    np.testing.assert_allclose(r["init_used"][:, 0], z["init_phi"], rtol=0, atol=1e-6)
    assert np.array_equal(r["status"], z["status"].astype(int)), np.where(
        r["status"] != z["status"])
    sig = np.stack([z["phi_err"], z["DM_err"], z["tau_err"], z["alpha_err"]], 1)
    ref = np.stack([z["phi"], z["DM"], z["tau"], z["alpha"]], 1)
    dev = r["params"][:, [0, 1, 3, 4]]
    dx = (np.abs(dev - ref) / sig).max(axis=1)
    floor = np.max([(np.abs(np.stack([z["r%d_%s" % (k, c)] for c in
                                      ["phi", "DM", "tau", "alpha"]], 1) - ref) / sig).max(axis=1)
                    for k in range(4)], axis=0)
    dof = nchan * nbin - (4 + nchan)
    dchi2 = (r["red_chi2"] - z["red_chi2"]) * dof
    near = dx <= 1e-3
    print("config 3, %d subints: %d within 1e-3 sigma of the reference (max %.3g); reference "
          "one-ulp floor > 1e-3 sigma on %d (max %.3g); |dchi2| max %.2e; nfev equal on %d" % (
              nsub, near.sum(), dx.max(), (floor > 1e-3).sum(), floor.max(),
              np.abs(dchi2).max(), (r["nfev"] == z["nfev"]).sum()))
    for i in np.where(~near)[0]:
        print("   subint %3d: |dx|/sigma %.3g, reference floor %.3g, nfev %d (reference %d), "
              "dchi2 %.2e" % (i, dx[i], floor[i], r["nfev"][i], z["nfev"][i], dchi2[i]))
    assert np.abs(dchi2).max() <= 1e-3
    assert near.mean() >= 0.85
