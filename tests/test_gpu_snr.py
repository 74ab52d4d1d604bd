"""Per-profile S/N for load_data's SNRs (pplib.py:2762-2770: Profile::snr()),
which get_TOAs uses to weight guess_fit_freq (pptoas.py:401) -- and so the
frequency every TOA is referenced to.  PSRCHIVE is not in this image and the
reference ships no archives: the estimator is PSRCHIVE's default phase S/N
restated (include/ppfit.h ppf_profile_snr, oracle.profile_snr), PARITY
UNPINNED.  Held here: the device against the oracle restatement on the same
rows, and get_TOAs on a PSRFITS file weighting nu_fit with them."""
import os
import shutil

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pulseportraiture_amd.engine import get_engine
    return get_engine(0)


def _rows(n, nbin, seed):
    rng = np.random.default_rng(seed)
    ph = np.arange(nbin) / nbin
    amp = rng.uniform(0.0, 20.0, n)[:, None]
    loc = rng.uniform(0, 1, n)[:, None]
    wid = rng.uniform(0.01, 0.08, n)[:, None]
    d = np.angle(np.exp(2j * np.pi * (ph - loc))) / (2 * np.pi)
    return amp * np.exp(-0.5 * (d / wid) ** 2) + rng.normal(3.0, 1.0, (n, nbin))


@pytest.mark.parametrize("nbin", [64, 512, 2048])
def test_profile_snr_vs_oracle(gpu, nbin):
    from oracle import ppfit_oracle as O
    x = _rows(24, nbin, nbin)
    x[0] = 5.0  # constant: zero variance -> 0
    got = gpu.profile_snr(x).cpu().numpy()
    want = O.profile_snr(x)
    assert got[0] == 0.0 and want[0] == 0.0
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)
    assert (want[1:] > 0).mean() > 0.9


def test_get_toas_psrfits_snr_weighted_nu_fit(gpu, tmp_path):
    """A PSRFITS archive whose channels differ in S/N: get_TOAs' nu_fit is
    guess_fit_freq(freqs, SNRs) with the per-profile S/N of the loaded data
    (VERDICT r03 missing #1), not the unweighted mean."""
    from oracle import ppfit_oracle as O
    from pulseportraiture_amd import archive, pplib, pptoas, synth
    from tests.test_gpu_psrfits import _coherence_archive
    path = str(tmp_path / "snr.fits")
    _coherence_archive(path, nsub=3, nchan=32, nbin=512, seed=77)
    d = archive.load_data(path, pscrunch=True, rm_baseline=False)
    sub = np.asarray(d.subints)
    np.testing.assert_allclose(d.SNRs, O.profile_snr(sub), rtol=1e-12, atol=1e-12)
    shutil.copy(synth.EXAMPLE_GMODEL, str(tmp_path / "example.gmodel"))
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        gt = pptoas.GetTOAs([path], "example.gmodel", quiet=True)
        gt.get_TOAs(quiet=True)
    finally:
        os.chdir(cwd)
    for isub in gt.ok_isubs[0]:
        ok = d.ok_ichans[isub]
        want = pplib.guess_fit_freq(d.freqs[isub, ok], d.SNRs[isub, 0, ok])
        assert abs(gt.nu_fits[0][isub][0] - want) < 1e-9
        assert abs(want - pplib.guess_fit_freq(d.freqs[isub, ok])) > 1e-6  # S/N matters here
