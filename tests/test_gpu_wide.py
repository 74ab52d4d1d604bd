"""Channel counts above PPF_LDS_NCHAN: the per-channel tables in HBM.

Up to PPF_LDS_NCHAN (2048) channels a fit workgroup keeps its subint's
per-channel tables (frequencies, 1/sigma^2, template power, dispersion
derivatives, the fitted-channel list; the data pass's guess phases and
flags) in LDS.  Above it the same kernels, instantiated with WIDE = true,
keep those tables in the workgroup's slice of an HBM workspace
(`chan_tables`, ppfit_kernels.hpp) and scattering fits take one workgroup
per subint.  The reference takes any channel count (pptoaslib.py:928-1096
works on whatever [nchan, nbin] it is given).

Two kinds of check:
- PPF_OPT_HBM_TABLES forces the HBM tables at any channel count, so every
  solver path is compared BITWISE with the LDS path on the same inputs (the
  same values and the same arithmetic; only where the tables live differs):
  phase-family Taylor fits with and without pipelined pieces and masked
  channels, GM, the exact sweeps, split scattering fits, TNC, Newton-CG and
  ppalign's data-spectrum cache.
- nchan = 2112, 4096, 2100 (at nbin 200, with the generic-length data pass,
  ppfit_generic.hip) and PPF_MAX_NCHAN = 16384 against the oracle, at the
  north_star tolerance (|dphi| <= 1e-3 sigma_phi, |dDM| <= 1e-3 sigma_DM)
  with identical solver status.
- get_TOAs end to end on a 2,304-channel archive whose last 256 channels
  are zapped: the same TOAs and .tim text as the 2,048-channel archive.
"""
import numpy as np
import pytest

from oracle import ppfit_oracle as O
from pulseportraiture_amd import synth

pytestmark = pytest.mark.gpu

KEYS = ["params", "param_errs", "nu_out", "cov", "scales", "scale_errs", "channel_snrs",
        "chi2", "red_chi2", "snr", "nfev", "status", "init_used", "errs"]


@pytest.fixture(scope="module")
def eng():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pulseportraiture_amd.engine import Engine
    return Engine(0)


def _fit(eng, w, data, flags, hbm, pieces=1, tau=None, **kw):
    eng.set_option("hbm_tables", int(hbm))
    eng.set_pipeline(pieces)
    try:
        nu = O.guess_fit_freq(w.freqs)
        n = data.shape[0]
        init = np.tile([0.0, w.DM0, 0.0, 0.0, 0.0], (n, 1))
        gt = None
        if tau is not None:
            init[:, 3], init[:, 4] = np.log10(tau), w.alpha
            gt = np.full(n, tau)
            kw.setdefault("log10_tau", True)
        out = eng.fit_batch(data, w.model, w.freqs, w.P, init, flags, nu_fit=[nu] * 3,
                            guess=True, guess_Ns=100, guess_tau=gt, **kw)
        return {k: out[k].cpu().numpy() for k in KEYS if k in out}
    finally:
        eng.set_option("hbm_tables", 0)
        eng.set_pipeline(0)


def _same(a, b):
    assert a.keys() == b.keys()
    for k in a:
        assert np.array_equal(a[k], b[k], equal_nan=True), k


def test_option_default_off(eng):
    assert eng.get_option("hbm_tables") == 0


@pytest.mark.parametrize("pieces", [1, 3])
def test_hbm_tables_bitwise_phase_dm(eng, pieces):
    w = synth.make_workload(40, 64, 2048, seed=611)
    data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
    flags = [1, 1, 0, 0, 0]
    _same(_fit(eng, w, data, flags, False, pieces), _fit(eng, w, data, flags, True, pieces))


def test_hbm_tables_bitwise_masked_gm(eng):
    w = synth.make_workload(12, 96, 512, seed=612, gm=2e-6)
    data = synth.workload_data_host(w)
    mask = np.ones((12, 96), np.uint8)
    mask[0, ::3] = 0
    mask[1, :90] = 0
    mask[2, 95] = 0
    mask[3] = 0  # fully zapped subint
    for flags in ([1, 1, 0, 0, 0], [1, 1, 1, 0, 0]):
        a = _fit(eng, w, data, flags, False, chan_mask=mask)
        _same(a, _fit(eng, w, data, flags, True, chan_mask=mask))
        assert np.all(a["scales"][mask == 0] == 0.0)


def test_hbm_tables_bitwise_exact_tnc_ncg(eng):
    w = synth.make_workload(6, 40, 256, seed=613)
    data = synth.workload_data_host(w)
    for kw in (dict(exact=True), dict(method="TNC"), dict(method="Newton-CG")):
        _same(_fit(eng, w, data, [1, 1, 0, 0, 0], False, **kw),
              _fit(eng, w, data, [1, 1, 0, 0, 0], True, **kw))


def test_hbm_tables_bitwise_scattering(eng):
    """The LDS path splits each evaluation over workgroups (k_scat_sweep);
    the HBM-table path fits each subint in one workgroup (k_solve<true>):
    bitwise the same, as PPF_OPT_SCAT_SPLIT = 0 is (test_gpu_options.py)."""
    w = synth.make_workload(16, 128, 512, seed=614, tau=2e-3)
    data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
    nu = O.guess_fit_freq(w.freqs)
    tg = 2e-3 * (nu / w.nu_ref) ** w.alpha
    flags = [1, 1, 0, 1, 1]
    a = _fit(eng, w, data, flags, False, tau=tg)
    assert (a["nfev"] > 4).all()
    _same(a, _fit(eng, w, data, flags, True, tau=tg))


def test_hbm_tables_bitwise_spec_cache(eng):
    """ppalign's refits: data spectra stored by the first fit, the data pass
    skipped by the second (PPF_SPEC_STORE / _USE)."""
    w = synth.make_workload(10, 48, 512, seed=615)
    data = synth.workload_data_host(w)
    outs = []
    for hbm in (False, True):
        cache = eng.spec_cache(10, 48, 512)
        first = _fit(eng, w, data, [1, 1, 0, 0, 0], hbm, spec_cache=cache)
        second = _fit(eng, w, data, [1, 1, 0, 0, 0], hbm, spec_cache=cache)
        _same(first, second)
        outs.append(first)
    _same(*outs)


def _vs_oracle(eng, nsub, nchan, nbin, seed, flags=(1, 1, 0, 0, 0), **kw):
    w = synth.make_workload(nsub, nchan, nbin, seed=seed, **kw)
    data = synth.workload_data_host(w)
    mask = np.ones((nsub, nchan), np.uint8)
    mask[0, 7::11] = 0  # a few zapped channels, ragged
    out = _fit(eng, w, data, list(flags), nchan <= 2048, chan_mask=mask)
    nu = O.guess_fit_freq(w.freqs)
    for i in range(nsub):
        ok = mask[i].astype(bool)
        errs = O.get_noise_PS(data[i], chans=True)
        init = list(out["init_used"][i])
        ref = O.fit_portrait_full(data[i][ok], w.model[ok], init, w.P, w.freqs[ok], [nu] * 3,
                                  [None] * 3, errs[ok], list(flags), log10_tau=False)
        assert int(out["status"][i]) == ref.return_code, i
        assert abs(out["params"][i][0] - ref.phi) <= 1e-3 * ref.phi_err, i
        assert abs(out["params"][i][1] - ref.DM) <= 1e-3 * ref.DM_err, i
        np.testing.assert_allclose(out["param_errs"][i][:2], [ref.phi_err, ref.DM_err],
                                   rtol=1e-6)
        np.testing.assert_allclose(out["red_chi2"][i], ref.red_chi2, rtol=1e-8)
        np.testing.assert_allclose(out["snr"][i], ref.snr, rtol=1e-8)
        np.testing.assert_array_equal(out["scales"][i][~ok], 0.0)
    return out


@pytest.mark.parametrize("nchan,nbin", [(2112, 256), (4096, 128), (2100, 200), (16384, 64)])
def test_wide_nchan_vs_oracle(eng, nchan, nbin):
    _vs_oracle(eng, 3, nchan, nbin, seed=620 + nchan)


def test_nchan_limit(eng):
    from pulseportraiture_amd.engine import PPFitError
    w = synth.make_workload(1, 16, 64, seed=1)
    data = np.zeros((1, 16385, 64))
    with pytest.raises(PPFitError, match="nchan"):
        eng.fit_batch(data, np.zeros((16385, 64)), np.linspace(1000, 2000, 16385), w.P,
                      np.zeros(5), [1, 1, 0, 0, 0])


def test_get_toas_zapped_extra_channels(tmp_path):
    """get_TOAs end to end above the LDS limit: an archive of 2,304 channels
    whose last 256 carry zero weight gives the TOAs, errors, scales and .tim
    text of the same archive cut to its 2,048 weighted channels (the
    reference fits ok_ichans only, pptoas.py:343-364) -- the first on the
    HBM-table kernels, the second on the LDS ones."""
    import os
    import re
    import shutil
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pulseportraiture_amd import archive, pplib, pptoas
    from tests.golden_consts import DM0
    nsub, nchan, extra, nbin = 4, 2048, 256, 256
    w = synth.make_workload(nsub, nchan, nbin, seed=630)
    data = synth.workload_data_host(w)
    rng = np.random.default_rng(631)
    df = w.freqs[1] - w.freqs[0]
    freqs_x = np.concatenate([w.freqs, w.freqs[-1] + df * np.arange(1, extra + 1)])
    data_x = np.concatenate([data, rng.standard_normal((nsub, extra, nbin))], axis=1)
    weights_x = np.ones((nsub, nchan + extra))
    weights_x[:, nchan:] = 0.0
    common = dict(Ps=np.full(nsub, w.P), epochs=[(57200 + k, 0, 0.0) for k in range(nsub)],
                  DM=DM0, nu0=1500.0, dmc=0)
    archive.register_archive("cut", dict(subints=data[:, None], freqs=w.freqs,
                                         weights=np.ones((nsub, nchan)), **common))
    archive.register_archive("wide", dict(subints=data_x[:, None], freqs=freqs_x,
                                          weights=weights_x, **common))
    shutil.copy(synth.EXAMPLE_GMODEL, str(tmp_path / "example.gmodel"))
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        gts, tims = [], []
        for name in ("cut", "wide"):
            gt = pptoas.GetTOAs([name], "example.gmodel", quiet=True)
            gt.get_TOAs(quiet=True)
            tim = str(tmp_path / (name + ".tim"))
            pplib.write_TOAs(gt.TOA_list, SNR_cutoff=0.0, outfile=tim, append=False)
            gts.append(gt)
            # -nch counts the zapped channels too (pptoas.py:633, nchan);
            # every other flag, -nchx and -bw included, is over ok channels
            txt = re.sub(r" -nch \d+", "", open(tim).read())
            tims.append(re.sub(r"(?m)^wide ", "cut ", txt))
    finally:
        os.chdir(cwd)
        archive.unregister_archive("cut")
        archive.unregister_archive("wide")
    cut, wide = gts
    for attr in ("phis", "phi_errs", "DMs", "DM_errs", "snrs", "red_chi2s", "covariances",
                 "nfevals", "rcs", "nu_refs", "TOA_errs"):
        a = np.asarray(getattr(cut, attr)[0], dtype=np.float64)
        b = np.asarray(getattr(wide, attr)[0], dtype=np.float64)
        assert np.array_equal(a, b, equal_nan=True), attr
    for attr in ("scales", "scale_errs", "channel_snrs"):
        a = np.asarray(getattr(cut, attr)[0])
        b = np.asarray(getattr(wide, attr)[0])
        assert b.shape[-1] == nchan + extra, attr
        assert np.array_equal(a, b[..., :nchan]), attr
        assert np.all(b[..., nchan:] == 0.0), attr
    assert tims[0] == tims[1]
