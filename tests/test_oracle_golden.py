"""Pin the CPU oracle (oracle/ppfit_oracle.py) to the reference's own outputs.

Golden vectors come from tests/golden/make_golden.py (reference source run
through the SURVEY.md §8(c) shim).  Tolerances: objective/gradient/Hessian
values 1e-9 relative (same numpy FFT, same formulas); fitted parameters
1e-6 x their reported errors (scipy's optimisers are deterministic here).
"""
import numpy as np
import pytest

from oracle import ppfit_oracle as O


def rel(a, b):
    a = np.asarray(a, float)
    b = np.asarray(b, float)
    scale = np.maximum(np.abs(b), 1e-300)
    both_nan = np.isnan(a) & np.isnan(b)
    r = np.where(both_nan, 0.0, np.abs(a - b) / scale)
    return np.nanmax(r) if r.size else 0.0


def test_utils(golden):
    u = golden("utils.npz")
    P = float(u["P"])
    np.testing.assert_allclose(O.get_noise_PS(u["noise_port"], chans=True),
                               u["noise_chans"], rtol=1e-13)
    np.testing.assert_allclose(O.get_noise_PS(u["noise_port"]), u["noise_ravel"],
                               rtol=1e-13)
    np.testing.assert_allclose(O.rotate_data(u["rot_prof"], 0.137),
                               u["rot_prof_out"], atol=1e-13)
    np.testing.assert_allclose(O.rotate_data(u["noise_port"], -0.21),
                               u["rot_port_out_dm0"], atol=1e-13)
    np.testing.assert_allclose(
        O.rotate_data(u["noise_port"], 0.05, 12.3, P, u["rot_freqs"], 1400.0),
        u["rot_port_out"], atol=1e-12)
    np.testing.assert_allclose(
        O.rotate_data(u["rot_sub4"], -0.02, 3.4, np.array([P, 1.01 * P]),
                      u["rot_freqs"], 1500.0), u["rot_sub4_out"], atol=1e-12)
    np.testing.assert_allclose(
        O.rotate_portrait_full(u["noise_port"], 0.05, 12.3, 3e-5, u["rot_freqs"],
                               1400.0, 1300.0, P), u["rot_full_out"], atol=1e-12)
    assert O.guess_fit_freq(u["rot_freqs"], u["gff_snrs"]) == pytest.approx(
        float(u["gff_out"]), rel=1e-15)
    assert O.guess_fit_freq(u["rot_freqs"]) == pytest.approx(
        float(u["gff_out_nosnr"]), rel=1e-15)
    for phi, DM, n1, n2, wrapped, raw in u["phase_transform"]:
        assert O.phase_transform(phi, DM, n1, n2, P, mod=True) == pytest.approx(
            wrapped, abs=1e-14)
        assert O.phase_transform(phi, DM, n1, n2, P) == pytest.approx(raw, abs=1e-14)


def test_phase_shift(golden):
    g = golden("phase_shift.npz")
    for i in range(int(g["ncase"])):
        noise = float(g["p%d_noise" % i])
        r = O.fit_phase_shift(g["p%d_data" % i], g["model"],
                              noise=None if np.isnan(noise) else noise,
                              Ns=int(g["p%d_Ns" % i]))
        for key in ["phase", "phase_err", "scale", "scale_err", "snr", "red_chi2"]:
            assert r[key] == pytest.approx(float(g["p%d_%s" % (i, key)]),
                                           rel=1e-9, abs=1e-12), (i, key)


def _objective_args(o, ic, flags, log10):
    data, model = o["c%d_data" % ic], o["c%d_model" % ic]
    nbin = data.shape[1]
    dFT = np.fft.rfft(data, axis=-1)
    dFT[:, 0] = 0
    mFT = np.fft.rfft(model, axis=-1)
    mFT[:, 0] = 0
    errs_FT = o["c%d_errs" % ic] * np.sqrt(nbin / 2.0)
    nu = o["c%d_nu_fit" % ic]
    from tests.golden_consts import P0
    return (dFT, mFT, errs_FT, P0, o["c%d_freqs" % ic], nu[0], nu[1], nu[2],
            [bool(f) for f in flags], log10)


@pytest.mark.parametrize("ic", [0, 1])
def test_objective_grad_hess(golden, ic):
    o = golden("objective.npz")
    for ip in range(int(o["c%d_ncase" % ic])):
        key = "c%d_p%d" % (ic, ip)
        p = o[key + "_params"]
        flags = list(o[key + "_flags"])
        log10 = bool(o[key + "_log10"])
        args = _objective_args(o, ic, flags, log10)
        assert rel(O.fit_function(p, *args), o[key + "_f"]) < 1e-9, key
        g = O.fit_function_deriv(p, *args)
        ref_g = o[key + "_g"]
        np.testing.assert_allclose(g, ref_g, rtol=1e-8,
                                   atol=1e-9 * np.abs(ref_g).max(), err_msg=key)
        H = O.fit_function_2deriv(p, *args)
        ref_H = o[key + "_H"]
        np.testing.assert_allclose(H, ref_H, rtol=1e-8,
                                   atol=1e-9 * np.abs(ref_H).max(), err_msg=key)
        Hn = O.fit_function_2deriv(p, *args, per_channel=True)
        np.testing.assert_allclose(Hn, o[key + "_Hn"], rtol=1e-8,
                                   atol=1e-9 * np.abs(o[key + "_Hn"]).max(),
                                   err_msg=key)
        if not np.isnan(o[key + "_Hs"]).all():
            Hs, cov, scales = O.hessian_with_scales(p, *args)
            np.testing.assert_allclose(Hs, o[key + "_Hs"], rtol=1e-8,
                                       atol=1e-9 * np.abs(o[key + "_Hs"]).max())
            np.testing.assert_allclose(scales, o[key + "_scales"], rtol=1e-9)
            np.testing.assert_allclose(np.diag(cov), np.diag(o[key + "_cov"]),
                                       rtol=1e-6)
        a = args
        ref_nz = o[key + "_nz"]
        if np.any((ref_nz < 1.0) | (ref_nz > 1e6)):
            # an unphysical root (e.g. 2e-5 MHz) comes from a polynomial whose
            # constant term is cancellation noise at these off-optimum params;
            # its sign -- and so the root -- is not reproducible.
            continue
        try:
            nz = O.get_nu_zeros(p, a[0], a[1], a[2], a[3], a[4], a[5], a[6],
                                a[7], flags, log10, 0)
        except (ValueError, IndexError):
            # the reference raised too (no positive real root): stored as NaN
            assert np.isnan(ref_nz).all(), key
            continue
        for x, y in zip(nz, ref_nz):
            if np.isnan(y):
                continue
            assert x == pytest.approx(y, rel=1e-8), (key, nz, ref_nz)


def assert_cov_close(cov, ref, tol):
    """|dC_ij| <= tol * sqrt(C_ii C_jj): off-diagonals vanish at nu_zero."""
    cov, ref = np.asarray(cov), np.asarray(ref)
    d = np.sqrt(np.abs(np.outer(np.diag(ref), np.diag(ref))))
    assert np.all(np.abs(cov - ref) <= tol * d), (cov, ref)


FIT_SCALARS = ["phi", "DM", "GM", "tau", "alpha", "nu_DM", "nu_GM", "nu_tau",
               "chi2", "red_chi2", "snr", "phi_err", "DM_err", "GM_err",
               "tau_err", "alpha_err"]


@pytest.mark.parametrize("ic", range(8))
def test_fit_portrait_full(golden, ic):
    f = golden("fit_full.npz")
    k = "f%d_" % ic
    nu = float(f[k + "nu_fit"])
    r = O.fit_portrait_full(f[k + "data"], f[k + "model"], list(f[k + "init"]),
                            float(f["P"]), f[k + "freqs"], [nu, nu, nu],
                            [None, None, None], f[k + "errs"],
                            list(f[k + "flags"]), log10_tau=bool(f[k + "log10"]))
    assert r.return_code == int(f[k + "return_code"])
    assert r.nfeval == int(f[k + "nfeval"])
    for key in FIT_SCALARS:
        assert r[key] == pytest.approx(float(f[k + key]), rel=1e-7, abs=1e-12), key
    np.testing.assert_allclose(r.scales, f[k + "scales"], rtol=1e-7)
    np.testing.assert_allclose(r.scale_errs, f[k + "scale_errs"], rtol=1e-7)
    np.testing.assert_allclose(r.channel_snrs, f[k + "channel_snrs"], rtol=1e-7)
    assert_cov_close(r.covariance_matrix, f[k + "covariance_matrix"], 1e-6)


@pytest.mark.parametrize("ic", [0, 1])
def test_legacy_fit_portrait(golden, ic):
    g = golden("legacy_fit_portrait.npz")
    k = "l%d_" % ic
    from tests.golden_consts import P0
    r = O.fit_portrait(g[k + "data"], g[k + "model"], g[k + "init"], P0,
                       g[k + "freqs"], float(g[k + "nu_fit"]), None, g[k + "errs"])
    assert r.return_code == int(g[k + "return_code"])
    assert r.nfeval == int(g[k + "nfeval"])
    for key in ["phase", "phase_err", "DM", "DM_err", "nu_ref", "covariance",
                "chi2", "red_chi2", "snr"]:
        assert r[key] == pytest.approx(float(g[k + key]), rel=1e-7), key
    np.testing.assert_allclose(r.scales, g[k + "scales"], rtol=1e-7)
