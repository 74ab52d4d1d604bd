"""Config 3 at its own shape against the reference: 200 of bench.py's
scattering subints (512 x 1024, phi + DM + log10 tau + alpha, get_TOAs' guess
and trust-ncg), fitted on the device and by the reference.

Fixtures (the reference's own get_TOAs per-subint flow, pptoas.py:383-488,
through the SURVEY §8(c) shim):
* scattering_200.npz (make_golden_cfg3.py): the reference's init, end point,
  errors, status, nfev, red chi2, and four restarts one ulp away in phase
  and log10 tau;
* scattering_200_perm.npz (make_golden_cfg3_perm.py): the same fits with the
  channels in 24 seeded random orders -- every per-channel term the same
  number, only the order of the reference's own channel sums changed.

trust-ncg with gtol = -1 (pptoaslib.py:1002) stops at the first predicted
reduction <= 0, i.e. when its trust radius has collapsed onto rounding; on
45 of these 200 subints the reference itself ends more than 1e-3 sigma away
from its own answer under a reordering of its sums (up to 46 sigma in phi: the
end points differ by ~1e-2 sigma in DM, tau, alpha, and the zero-covariance
frequency nu_DM the phase is reported at moves with them).  Those end points
are discrete: the device lands on them.

Asserted, per subint:
* the guess (init phase) and the status are the reference's;
* nfev (scipy's count: a proposal equal to the last evaluated point is not
  re-evaluated) is within 2 of the reference's;
* |chi^2_device - chi^2_reference| <= 1e-3;
* the end point is within 1e-3 sigma of the reference's, or of one of the
  reference's own end points under a one-ulp restart or a channel
  reordering -- no "between them" category: a device end point the
  reference never reaches fails;
* where the reference's own spread is below 1e-3 sigma, within 1e-3 sigma of
  the reference.
And over the set, a bar that does not move with the device's results:
* at most ON_ALT_MAX (24, the count at r05) subints are on an alternate end
  point of the reference's only;
* the alternate set is frozen at the 4 restarts + 24 reorderings committed
  in r04 (asserted: 24 orderings);
* the device agrees with the reference (within 1e-3 sigma) on at least as
  many subints as the reference agrees with itself under its *worst* channel
  ordering -- min over the 24 orderings of the fraction of subints whose
  reordered end point is within 1e-3 sigma of the unpermuted one (0.87 on
  this fixture).  The device is held to be no worse a summation order than
  any of the reference's own.
"""
import os

import numpy as np
import pytest

from tests.conftest import GOLDEN
from tests.golden_consts import DM0

pytestmark = pytest.mark.gpu

PARAMS = ["phi", "DM", "tau", "alpha"]
ON_ALT_MAX = 24  # subints on a reference end point other than its own (r05: 24 of 200)


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
    zp = np.load(os.path.join(GOLDEN, "scattering_200_perm.npz"))
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
    sig = np.stack([z[c + "_err"] for c in PARAMS], 1)
    ref = np.stack([z[c] for c in PARAMS], 1)
    dev = r["params"][:, [0, 1, 3, 4]]
    dx = (np.abs(dev - ref) / sig).max(axis=1)
    # the reference's own end points: one-ulp restarts and channel reorderings
    alts = [np.stack([z["r%d_%s" % (k, c)] for c in PARAMS], 1) for k in range(4)]
    alts += [np.stack([zp["perm_" + c][:, k] for c in PARAMS], 1)
             for k in range(int(zp["nperm"]))]
    alts = np.stack(alts, 1)  # [nsub, nalt, 4]
    spread = (np.abs(alts - ref[:, None]) / sig[:, None]).max(axis=2).max(axis=1)
    to_alt = (np.abs(alts - dev[:, None]) / sig[:, None]).max(axis=2).min(axis=1)
    dof = nchan * nbin - (4 + nchan)
    dchi2 = (r["red_chi2"] - z["red_chi2"]) * dof
    near = dx <= 1e-3
    on_alt = to_alt <= 1e-3
    dn = r["nfev"] - z["nfev"].astype(int)
    print("config 3, %d subints: %d within 1e-3 sigma of the reference (max %.3g), %d more on "
          "one of the reference's own end points, %d between them; reference's own spread > "
          "1e-3 sigma on %d (max %.3g); |dchi2| max %.2e; nfev equal on %d, max |dnfev| %d" % (
              nsub, near.sum(), dx.max(), (on_alt & ~near).sum(), (~near & ~on_alt).sum(),
              (spread > 1e-3).sum(), spread.max(), np.abs(dchi2).max(), (dn == 0).sum(),
              np.abs(dn).max()))
    for i in np.where(~near)[0]:
        print("   subint %3d: |dx|/sigma %.3g, to nearest reference end point %.3g, reference "
              "spread %.3g, nfev %d (reference %d), dchi2 %.2e" % (
                  i, dx[i], to_alt[i], spread[i], r["nfev"][i], z["nfev"][i], dchi2[i]))
    assert np.abs(dchi2).max() <= 1e-3
    assert np.abs(dn).max() <= 2, np.where(np.abs(dn) > 2)
    assert (near | on_alt).all(), np.where(~(near | on_alt))
    assert (on_alt & ~near).sum() <= ON_ALT_MAX, np.where(on_alt & ~near)
    stable = spread <= 1e-3
    assert near[stable].all(), np.where(stable & ~near)
    # the statistical bar: the reference's own agreement rate per ordering
    assert int(zp["nperm"]) == 24
    perm = np.stack([np.stack([zp["perm_" + c][:, k] for c in PARAMS], 1)
                     for k in range(int(zp["nperm"]))], 1)  # [nsub, 24, 4]
    self_rate = ((np.abs(perm - ref[:, None]) / sig[:, None]).max(axis=2) <= 1e-3).mean(axis=0)
    print("agreement within 1e-3 sigma: device %.3f; reference with itself per ordering: "
          "min %.3f, mean %.3f, max %.3f" % (near.mean(), self_rate.min(), self_rate.mean(),
                                             self_rate.max()))
    assert near.mean() >= self_rate.min(), (near.mean(), self_rate.min())
