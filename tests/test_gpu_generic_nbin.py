"""nbin that are not powers of two (ppfit_generic.hip).

The reference transforms with numpy's rfft / irfft of any length
(pptoaslib.py:976-978, pplib.py:2338-2426); the library's FFT kernels are
built per power of two, and for every other nbin in [16, 8192] the fit entry
point, the template spectra, the row rotations and the Gaussian templates
take direct-sum kernels instead.  Checked here against the oracle (numpy):
- rotated / scattered rows and Gaussian templates to 1e-12 of the row scale;
- fit_portrait_full (trust-ncg Taylor path, the exact sweeps, TNC,
  Newton-CG, GM, scattering) at the north_star tolerance, every fitted
  parameter within 1e-3 sigma of the oracle's end point with the oracle's
  status, on even and odd nbin (odd: no Nyquist harmonic).  Where the
  oracle's own stop is decided by rounding (trust-ncg's status-2 stop, TNC's
  converged / line-search-failed pair) the bar is the one of the config-3 and
  TNC golden tests: within 1e-3 sigma of the oracle's end point or of one of
  its own end points under a channel reordering or a one-ulp restart, and
  TNC's FCONVERGED (1) and LSFAIL (4) taken as one converged status;
- get_noise_PS, irfft, fit_phase_shift, the zapping residual chi2 and
  ppalign's rotate-and-sum rows against numpy / the oracle;
- get_TOAs and ppalign.align_archives end to end on 1000-bin archives.
"""
import numpy as np
import pytest

from oracle import ppfit_oracle as O
from pulseportraiture_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pulseportraiture_amd.engine import Engine
    return Engine(0)


@pytest.mark.parametrize("nbin", [16, 33, 100, 1000, 999, 3000, 8191])
def test_rotate_rows_generic(eng, nbin):
    rng = np.random.default_rng(nbin)
    rows = rng.standard_normal((5, nbin))
    ph = rng.uniform(-0.5, 0.5, 5)
    tau = rng.uniform(0.0, 3.0, 5)
    got = eng.rotate_rows(rows, ph).cpu().numpy()
    ref = np.fft.irfft(np.fft.rfft(rows) * np.exp(2j * np.pi * np.outer(ph, np.arange(nbin // 2 + 1))),
                       n=nbin)
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12 * np.abs(ref).max())
    got = eng.scatter_rotate_rows(rows, ph, tau).cpu().numpy()
    k = np.arange(nbin // 2 + 1)
    spec = np.fft.rfft(rows) * np.exp(2j * np.pi * np.outer(ph, k)) / (1 + 2j * np.pi * np.outer(tau, k))
    ref = np.fft.irfft(spec, n=nbin)
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12 * np.abs(ref).max())


@pytest.mark.parametrize("nbin", [1000, 999])
@pytest.mark.parametrize("tau", [0.0, 4.0])
def test_gaussian_portraits_generic(eng, nbin, tau):
    """The .gmodel template on the device (k_gauss_port, and the scattering
    rotation through k_rotate_rows_gen) against gen_gaussian_portrait's numpy
    form, at 1e-12 of the row scale.  Odd nbin with scattering: the
    reference's irfft has no n= (pplib.py:921) and returns nbin - 1 bins, a
    template that no longer matches its data; the device keeps nbin bins,
    i.e. irfft(..., n=nbin), as the host gen_gaussian_portrait now does."""
    from pulseportraiture_amd import pplib
    m = pplib.read_model(synth.EXAMPLE_GMODEL, quiet=True)
    name, code, nu_ref, ngauss, params, fit_flags, alpha = m[:7]
    params = np.array(params, dtype=float)
    params[1] = tau
    freqs = synth.channel_freqs(24)
    got = eng.gaussian_portraits(code, params, alpha, nbin, freqs, nu_ref).cpu().numpy()
    ref = pplib.gen_gaussian_portrait(code, params, alpha, pplib.get_bin_centers(nbin), freqs,
                                      nu_ref)
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12 * np.abs(ref).max())


def _vs_oracle(eng, nsub, nchan, nbin, seed, flags, method="trust-ncg", exact=False, **kw):
    w = synth.make_workload(nsub, nchan, nbin, seed=seed, **kw)
    data = synth.workload_data_host(w)
    nu = O.guess_fit_freq(w.freqs)
    init = np.tile([0.0, w.DM0, 0.0, 0.0, 0.0], (nsub, 1))
    log10_tau = False
    gt = None
    if flags[3]:
        tg = 2e-3 * (nu / w.nu_ref) ** w.alpha
        init[:, 3], init[:, 4] = np.log10(tg), w.alpha
        gt = np.full(nsub, tg)
        log10_tau = True
    out = eng.fit_batch(data, w.model, w.freqs, w.P, init, flags, nu_fit=[nu] * 3, guess=True,
                        guess_tau=gt, log10_tau=log10_tau, method=method, exact=exact)
    out = {k: v.cpu().numpy() for k, v in out.items() if not k.startswith("_")}
    n_alt = 0
    for i in range(nsub):
        errs = O.get_noise_PS(data[i], chans=True)
        np.testing.assert_allclose(out["errs"][i], errs, rtol=1e-10)
        init = list(out["init_used"][i])

        def oracle(perm=None, init=init):
            p = np.arange(nchan) if perm is None else perm
            return O.fit_portrait_full(data[i][p], w.model[p], init, w.P, w.freqs[p], [nu] * 3,
                                       [None] * 3, errs[p], list(flags), log10_tau=log10_tau,
                                       method=method)

        ref = oracle()
        rc, p = int(out["status"][i]), out["params"][i]
        if _gap(p, ref, flags) > 1e-3 or not _same_status(rc, ref.return_code, method):
            # the oracle's own end points under a reordering of its channel
            # sums or a one-ulp restart
            rng = np.random.default_rng(seed + i)
            alts = [oracle(perm=rng.permutation(nchan)) for _ in range(8)]
            alts += [oracle(init=[np.nextafter(init[0], s)] + init[1:]) for s in (-1, 1)]
            ok = [a for a in alts if _gap(p, a, flags) <= 1e-3 and
                  _same_status(rc, a.return_code, method)]
            assert ok, (i, rc, ref.return_code, _gap(p, ref, flags),
                        [(_gap(p, a, flags), a.return_code) for a in alts])
            n_alt += 1
        np.testing.assert_allclose(out["param_errs"][i][0], ref.phi_err, rtol=1e-4)
        np.testing.assert_allclose(out["red_chi2"][i], ref.red_chi2, rtol=1e-6)
    assert n_alt <= max(1, nsub // 3), n_alt
    return out


def _gap(p, ref, flags):
    """Largest |device - oracle| / sigma over the fitted parameters."""
    g = abs(p[0] - ref.phi) / ref.phi_err
    for i, nm in enumerate(["DM", "GM", "tau", "alpha"], start=1):
        if flags[i]:
            g = max(g, abs(p[i] - getattr(ref, nm)) / getattr(ref, nm + "_err"))
    return g


def _same_status(rc, ref_rc, method):
    if method == "TNC" and {rc, ref_rc} <= {1, 4}:
        return True  # FCONVERGED / LSFAIL at the rounding floor (test_gpu_golden_r2.py)
    return rc == ref_rc


@pytest.mark.parametrize("nbin,nchan", [(1000, 32), (999, 32), (1536, 32), (96, 32), (8190, 8),
                                        (6001, 8), (32, 32), (48, 16)])
def test_fit_generic_nbin_phase_dm(eng, nbin, nchan):
    _vs_oracle(eng, 4, nchan, nbin, 700 + nbin, [1, 1, 0, 0, 0])


@pytest.mark.parametrize("kw", [dict(exact=True), dict(method="TNC"), dict(method="Newton-CG")])
def test_fit_generic_nbin_methods(eng, kw):
    _vs_oracle(eng, 3, 24, 1000, 710, [1, 1, 0, 0, 0], **kw)


def test_fit_generic_nbin_gm(eng):
    _vs_oracle(eng, 3, 32, 768, 711, [1, 1, 1, 0, 0], gm=2e-6)


def test_fit_generic_nbin_scattering(eng):
    _vs_oracle(eng, 3, 64, 1000, 712, [1, 1, 0, 1, 1], tau=2e-3)


def test_generic_nbin_limits(eng):
    from pulseportraiture_amd.engine import PPFitError
    with pytest.raises(PPFitError, match="nbin"):
        eng.spec_cache(2, 4, 8200)
    w = synth.make_workload(1, 4, 64, seed=1)
    with pytest.raises(PPFitError, match="nbin"):
        eng.fit_batch(np.zeros((1, 4, 8200)), np.zeros((4, 8200)), w.freqs, w.P, np.zeros(5),
                      [1, 1, 0, 0, 0])


def test_get_toas_generic_nbin(tmp_path):
    """get_TOAs on 1000-bin profiles runs end to end (Gaussian template from
    the .gmodel, guess, fit, TOA records) and lands on the injected DM; the
    fit itself is held to the oracle by the tests above."""
    import os
    import shutil
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pulseportraiture_amd import archive, pptoas
    from tests.golden_consts import DM0
    nsub, nchan, nbin = 3, 32, 1000
    w = synth.make_workload(nsub, nchan, nbin, seed=720)
    data = synth.workload_data_host(w)
    archive.register_archive("gen1000", dict(subints=data[:, None], freqs=w.freqs,
                                             weights=np.ones((nsub, nchan)),
                                             Ps=np.full(nsub, w.P),
                                             epochs=[(57300 + k, 0, 0.0) for k in range(nsub)],
                                             DM=DM0, nu0=1500.0, dmc=0))
    shutil.copy(synth.EXAMPLE_GMODEL, str(tmp_path / "example.gmodel"))
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        gt = pptoas.GetTOAs(["gen1000"], "example.gmodel", quiet=True)
        gt.get_TOAs(quiet=True)
    finally:
        os.chdir(cwd)
        archive.unregister_archive("gen1000")
    assert len(gt.TOA_list) == nsub
    phis, errs = np.asarray(gt.phis[0]), np.asarray(gt.phi_errs[0])
    assert np.all(np.isfinite(phis)) and np.all(errs > 0)
    assert np.all(np.asarray(gt.rcs[0]) >= 0)
    # the synthetic truth: within a few sigma of the injected phase / DM
    dms = np.asarray(gt.DMs[0])
    assert np.all(np.abs(dms - (w.DM0 + w.dDM)) < 6 * np.asarray(gt.DM_errs[0]))


@pytest.mark.parametrize("nbin", [1000, 999, 8191])
def test_row_entry_points_generic(eng, nbin):
    """get_noise_PS, irfft, fit_phase_shift (ppalign / pplib FFTFIT), the
    zapping residual chi2 and ppalign's rotate-and-sum at a generic nbin,
    against numpy / the oracle."""
    import torch
    w = synth.make_workload(1, 6, nbin, seed=730 + nbin)
    data = synth.workload_data_host(w)[0]
    np.testing.assert_allclose(eng.noise_rows(data).cpu().numpy(),
                               O.get_noise_PS(data, chans=True), rtol=1e-10)
    spec = np.fft.rfft(data, axis=-1)
    np.testing.assert_allclose(eng.irfft_rows(spec, nbin).cpu().numpy(),
                               np.fft.irfft(spec, n=nbin, axis=-1), rtol=0,
                               atol=1e-12 * np.abs(data).max())
    out = eng.phase_shift_batch(data, w.model, model_idx=np.arange(6)).cpu().numpy()
    for i in range(6):
        ref = O.fit_phase_shift(data[i], w.model[i])
        d = abs(out[i, 0] - ref.phase)
        assert min(d, 1.0 - d) <= 1e-3 * ref.phase_err, i
        np.testing.assert_allclose(out[i, 1:], [ref.phase_err, ref.scale, ref.scale_err, ref.snr,
                                                ref.red_chi2], rtol=1e-6)
    k = np.arange(nbin // 2 + 1)
    ph = np.linspace(-0.3, 0.4, 6)
    tau = np.linspace(0.0, 2e-3, 6)
    sc, errs = np.linspace(0.9, 1.1, 6), np.full(6, 1.5)
    got = eng.resid_chi2_rows(data, ph, w.model, sc, errs, 100.0, tau=tau).cpu().numpy()
    rot = np.fft.irfft(spec * np.exp(2j * np.pi * np.outer(ph, k)), n=nbin, axis=-1)
    msc = np.fft.irfft(np.fft.rfft(w.model, axis=-1) / (1 + 2j * np.pi * np.outer(tau, k)),
                       n=nbin, axis=-1)
    ref = np.sum((rot - sc[:, None] * msc) ** 2, axis=-1) / errs ** 2 / 100.0
    np.testing.assert_allclose(got, ref, rtol=1e-9)
    d3 = np.stack([data, 0.5 * data[::-1]])  # [nsub 2, nchan 6, nbin]
    phs = np.stack([ph, -ph])
    wts = np.array([[1.0] * 6, [0.5, 0.0, 1.0, 2.0, 1.0, 1.0]])
    acc = torch.zeros(6, nbin // 2 + 1, 2, dtype=torch.float64, device=eng.device)
    eng.rotate_accumulate(d3, phs, wts, acc)
    torch.cuda.synchronize()
    ref = np.sum(wts[..., None] * np.fft.rfft(d3, axis=-1) *
                 np.exp(2j * np.pi * phs[..., None] * k), axis=0)
    got = acc.cpu().numpy()
    np.testing.assert_allclose(got[..., 0] + 1j * got[..., 1], ref, rtol=0,
                               atol=1e-12 * np.abs(ref).max())


def test_align_archives_generic_nbin():
    """ppalign.align_archives on 1000-bin archives (no data-spectrum cache at
    this length): runs end to end, and the aligned portrait is the template
    up to noise (every channel correlates with it)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pulseportraiture_amd import archive, ppalign
    from tests.golden_consts import DM0
    nbin, nchan = 1000, 16
    names = []
    for i in range(3):
        w = synth.make_workload(2, nchan, nbin, seed=740 + i, sigma=0.3)
        archive.register_archive("gal_%d" % i, dict(
            subints=synth.workload_data_host(w)[:, None], freqs=w.freqs, Ps=np.full(2, w.P),
            epochs=[(57000 + i, 0, 0.0), (57000 + i, 60, 0.0)], DM=DM0, nu0=1500.0, dmc=0,
            weights=np.ones((2, nchan))))
        names.append("gal_%d" % i)
    archive.register_archive("gal_guess", dict(subints=w.model[None, None], freqs=w.freqs,
                                               Ps=[w.P], epochs=[(57000, 0, 0.0)], DM=DM0,
                                               nu0=1500.0, dmc=1))
    try:
        port = np.asarray(ppalign.align_archives(names, "gal_guess", niter=2, quiet=True))
    finally:
        for n in names + ["gal_guess"]:
            archive.unregister_archive(n)
    assert port.shape[-2:] == (nchan, nbin) and np.all(np.isfinite(port))
    p = port.reshape(-1, nchan, nbin)[0]
    for n in range(nchan):
        assert np.corrcoef(p[n], w.model[n])[0, 1] > 0.99, n


@pytest.mark.parametrize("nbin", [1000, 999])
def test_instrumental_response_generic(eng, nbin):
    """instrumental_response_port_FT (pptoaslib.py:145-179, the oracle's) and
    its convolution of rows, irfft(R rfft(rows), n = nbin)."""
    rng = np.random.default_rng(nbin)
    rows = rng.normal(size=(6, nbin))
    f = np.linspace(1200.0, 1800.0, 6)
    R = O.instrumental_response_port_FT(nbin, f, 1.0, 0.002, [0.01], ["gauss"])
    np.testing.assert_allclose(eng.response_table(nbin, f, 1.0, 0.002, [0.01], ["gauss"])
                               .cpu().numpy(), np.real(R), rtol=0, atol=1e-14)
    got = eng.instrumental_response_rows(rows, f, 1.0, 0.002, [0.01], ["gauss"]).cpu().numpy()
    ref = np.fft.irfft(np.real(R) * np.fft.rfft(rows, axis=-1), n=nbin, axis=-1)
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12 * np.abs(ref).max())


@pytest.mark.parametrize("nbin", [1000, 999, 3000])
def test_spline_portrait_resampled_generic(tmp_path, nbin):
    """gen_spline_portrait (pplib.py:932-956) resampled to a generic nbin:
    scipy.signal.resample of the native-length portrait, then
    rotate_portrait by 0.5 (1/nbin - 1/nbin_in) -- with irfft(n = nbin), where
    the reference's rotate_portrait (pplib.py:2449-2461) drops a bin at odd
    nbin."""
    import json
    import os
    import torch
    from scipy import signal as ss
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pulseportraiture_amd import pplib
    from tests.conftest import GOLDEN
    z = np.load(os.path.join(GOLDEN, "templates_r3.npz"))
    meta = json.load(open(os.path.join(GOLDEN, "templates_r3.json")))
    path = tmp_path / "m3.spl"
    path.write_bytes(bytes(z["spl_m3_file"]))
    tag = meta["m3"]["cases"][0]
    freqs = z["spl_m3_%s_freqs" % tag]
    mean_prof = pplib.read_spline_model(str(path), quiet=True)[3]
    nin = len(mean_prof)
    _, native = pplib.read_spline_model(str(path), freqs, nin, quiet=True)
    _, port = pplib.read_spline_model(str(path), freqs, nbin, quiet=True)
    shift = 0.5 * (1.0 / nbin - 1.0 / nin)
    rs = np.fft.rfft(ss.resample(np.asarray(native), nbin, axis=1), axis=1)
    ref = np.fft.irfft(rs * np.exp(2j * np.pi * shift * np.arange(rs.shape[1])), n=nbin, axis=1)
    port = np.asarray(port)
    assert port.shape == ref.shape
    assert np.max(np.abs(port - ref)) <= 1e-12 * np.max(np.abs(ref))


@pytest.mark.parametrize("nbin", [1000, 999])
def test_generic_nbin_spec_cache_bitwise(eng, nbin):
    """ppalign's data-spectrum cache at a generic nbin: the storing fit and
    the refit from the cache (the data pass skipped) give the fit without a
    cache, bitwise (the spectra are the same GEMM's, stored or in place)."""
    nsub, nchan = 9, 24
    w = synth.make_workload(nsub, nchan, nbin, seed=760 + nbin)
    data = synth.workload_data_host(w)
    nu = O.guess_fit_freq(w.freqs)
    mask = np.ones((nsub, nchan), np.uint8)
    mask[2, ::5] = 0
    args = (data, w.model, w.freqs, w.P, [0.0, w.DM0, 0, 0, 0], [1, 1, 0, 0, 0])
    keys = ["params", "param_errs", "nu_out", "cov", "scales", "red_chi2", "snr", "nfev",
            "status", "errs", "init_used"]

    def run(**kw):
        out = eng.fit_batch(*args, nu_fit=[nu] * 3, guess=True, chan_mask=mask, **kw)
        return {k: out[k].cpu().numpy() for k in keys}

    ref = run()
    cache = eng.spec_cache(nsub, nchan, nbin)
    for o in (run(spec_cache=cache), run(spec_cache=cache)):
        for k in keys:
            np.testing.assert_array_equal(o[k], ref[k], err_msg=k)


def test_generic_nbin_pieces_and_chunks_bitwise(eng):
    """The piece pipeline (two queues, ppf_set_pipeline) and a workspace
    small enough to split the batch into chunks run the generic data pass on
    shifted slices: bitwise the single-launch results."""
    nsub, nchan, nbin = 37, 16, 1000
    w = synth.make_workload(nsub, nchan, nbin, seed=750)
    data = synth.workload_data_host(w)
    nu = O.guess_fit_freq(w.freqs)
    args = (data, w.model, w.freqs, w.P, [0.0, w.DM0, 0, 0, 0], [1, 1, 0, 0, 0])
    keys = ["params", "param_errs", "nu_out", "cov", "scales", "red_chi2", "snr", "nfev",
            "status", "errs"]

    def run():
        out = eng.fit_batch(*args, nu_fit=[nu] * 3, guess=True)
        return {k: out[k].cpu().numpy() for k in keys}

    try:
        eng.set_pipeline(1)
        ref = run()
        eng.set_pipeline(3)
        piped = run()
        eng.set_pipeline(1)
        eng.set_workspace_limit(12 * nchan * 1008 * 16 + (1 << 20))  # chunks of ~10 subints
        chunked = run()
    finally:
        eng.set_pipeline(0)
        eng.set_workspace_limit(32 << 30)
    for o in (piped, chunked):
        for k in keys:
            np.testing.assert_array_equal(o[k], ref[k], err_msg=k)


@pytest.mark.parametrize("nbin", [1000, 999])
def test_synth_generic(eng, nbin):
    """The synthetic-portrait generator (k_synth's Philox noise layout) at a
    generic nbin against its numpy twin, synth.synth_portraits_host."""
    nchan, nsub = 8, 3
    model = np.random.default_rng(3).normal(0, 1, (nchan, nbin))
    ph = np.random.default_rng(4).uniform(-2, 2, (nsub, nchan))
    got = eng.synth(model, ph, 1.5, 12345, sub0=7).cpu().numpy()
    ref = synth.synth_portraits_host(model, ph, 1.5, 12345, sub0=7)
    np.testing.assert_allclose(got, ref, atol=1e-11)
