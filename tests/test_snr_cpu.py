"""oracle.profile_snr (the restated PSRCHIVE phase S/N behind load_data's
SNRs, pplib.py:2762-2770; PARITY UNPINNED, PSRCHIVE absent) on the CPU:
properties the estimator has by construction."""
import numpy as np

from oracle import ppfit_oracle as O


def _pulse(nbin, amp, loc=0.3, wid=0.03, seed=0, sigma=1.0):
    rng = np.random.default_rng(seed)
    ph = np.arange(nbin) / nbin
    d = np.angle(np.exp(2j * np.pi * (ph - loc))) / (2 * np.pi)
    return amp * np.exp(-0.5 * (d / wid) ** 2) + rng.normal(0.0, sigma, nbin)


def test_affine_invariance_and_degenerate_rows():
    x = _pulse(256, 15.0)
    s = O.profile_snr(x)
    assert s > 5
    # an offset and a positive gain do not change it (window, edges, ratio)
    assert abs(O.profile_snr(3.0 * x + 7.0) - s) < 1e-9 * s
    assert O.profile_snr(np.full(128, 2.0)) == 0.0


def test_grows_with_amplitude_and_shape():
    s = [float(O.profile_snr(_pulse(512, a, seed=3))) for a in (2.0, 8.0, 32.0)]
    assert s[0] < s[1] < s[2]
    assert O.profile_snr(np.stack([_pulse(64, 5.0), _pulse(64, 9.0)])).shape == (2,)
