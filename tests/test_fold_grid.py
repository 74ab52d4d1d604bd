"""The folded brute-force grid of k_guess (ppfit_kernels.hpp guess_search).

On get_TOAs' grid linspace(-0.5, 0.5, Ns) the FFTFIT objective
f(phi) = Re sum_k rm_k e^{2 pi i k phi} (pplib.py:1244-1256) is an L-point DFT
(L = Ns - 1) of the spectrum folded mod L with alternating signs.  This checks
the identity and that the grid argmin it gives equals scipy.optimize.brute's
on the direct sums, with numpy only (no device).
"""
import numpy as np
import pytest


def _direct(rm, Ns):
    ph = np.linspace(-0.5, 0.5, Ns)
    k = np.arange(len(rm))
    return np.real(np.exp(2j * np.pi * np.outer(ph, k)) @ rm)


def _folded(rm, Ns):
    L = Ns - 1
    k = np.arange(len(rm))
    b = np.zeros(L, complex)
    np.add.at(b, k % L, rm * np.where(k % 2, -1.0, 1.0))
    g = np.arange(Ns)
    w = np.exp(2j * np.pi * (np.outer(g, np.arange(L)) % L) / L)  # table w_m, m = jg mod L
    return np.real(w @ b)


@pytest.mark.parametrize("nh,Ns", [(1025, 100), (513, 100), (257, 64), (1025, 129)])
def test_fold_matches_direct(nh, Ns):
    rng = np.random.default_rng(nh + Ns)
    rm = rng.normal(size=nh) + 1j * rng.normal(size=nh)
    rm[0] = 0.0
    d, f = _direct(rm, Ns), _folded(rm, Ns)
    np.testing.assert_allclose(f, d, rtol=0, atol=1e-10 * np.abs(rm).sum())
    assert f[0] == f[-1]  # phi = -0.5 and 0.5 share one folded value


def test_fold_argmin_matches_brute():
    rng = np.random.default_rng(5)
    for trial in range(20):
        nh, Ns = 1025, 100
        true = rng.uniform(-0.5, 0.5)
        k = np.arange(nh)
        amp = np.exp(-0.5 * (k / 40.0) ** 2)
        rm = amp * np.exp(-2j * np.pi * k * true) + 0.05 * (rng.normal(size=nh) + 1j * rng.normal(size=nh))
        rm[0] = 0.0
        assert np.argmin(-_folded(rm, Ns)) == np.argmin(-_direct(rm, Ns)), trial
