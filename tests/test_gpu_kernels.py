"""GPU parity of the libppfit kernels against the oracle and the golden vectors.

Tolerances (north_star, BASELINE.json): |dphi| <= 1e-3 sigma_phi,
|dDM| <= 1e-3 sigma_DM, identical solver status; transforms agree with
numpy.fft to 1e-12 relative (different fp64 FFT factorisation).
"""
import numpy as np
import pytest

from oracle import ppfit_oracle as O
from tests.golden_consts import P0

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pulseportraiture_amd.engine import Engine
    return Engine(0)


NBINS = [64, 128, 256, 512, 1024, 2048, 4096, 8192]


def test_cross_lane_selftest(eng):
    """DPP / permlane16,32 swap / readlane semantics the reductions rely on."""
    assert eng.selftest() == [0] * 10


@pytest.mark.parametrize("nbin", NBINS)
def test_noise_rows(eng, nbin):
    rng = np.random.default_rng(nbin)
    rows = rng.normal(0, 1, (5, nbin)) + np.sin(np.arange(nbin) * 0.3)
    got = eng.noise_rows(rows).cpu().numpy()
    np.testing.assert_allclose(got, O.get_noise_PS(rows, chans=True), rtol=1e-12)


@pytest.mark.parametrize("nbin", NBINS)
def test_rotate_and_irfft_rows(eng, nbin):
    rng = np.random.default_rng(nbin + 1)
    rows = rng.normal(0, 1, (7, nbin))
    ph = rng.uniform(-3, 3, 7)
    got = eng.rotate_rows(rows, ph).cpu().numpy()
    ref = np.array([O.rotate_data(r, p) for r, p in zip(rows, ph)])
    np.testing.assert_allclose(got, ref, atol=1e-12 * np.abs(ref).max())
    spec = np.fft.rfft(rows, axis=-1) * (1 + 0.1j)
    got = eng.irfft_rows(spec, nbin).cpu().numpy()
    np.testing.assert_allclose(got, np.fft.irfft(spec, axis=-1), atol=1e-12 * np.abs(rows).max())


def test_phase_shift_golden(eng, golden):
    g = golden("phase_shift.npz")
    for i in range(int(g["ncase"])):
        noise = float(g["p%d_noise" % i])
        out = eng.phase_shift_batch(g["p%d_data" % i], g["model"],
                                    noise=None if np.isnan(noise) else noise,
                                    Ns=int(g["p%d_Ns" % i])).cpu().numpy()[0]
        ph, ph_err, scale, scale_err, snr, rc2 = out
        assert abs(ph - float(g["p%d_phase" % i])) <= 1e-3 * float(g["p%d_phase_err" % i]), i
        assert ph_err == pytest.approx(float(g["p%d_phase_err" % i]), rel=1e-6)
        assert scale == pytest.approx(float(g["p%d_scale" % i]), rel=1e-8)
        assert scale_err == pytest.approx(float(g["p%d_scale_err" % i]), rel=1e-10)
        assert snr == pytest.approx(float(g["p%d_snr" % i]), rel=1e-8)
        assert rc2 == pytest.approx(float(g["p%d_red_chi2" % i]), rel=1e-8)


def fit_case(eng, f, ic):
    k = "f%d_" % ic
    nu = float(f[k + "nu_fit"])
    out = eng.fit_batch(f[k + "data"], f[k + "model"], f[k + "freqs"], float(f["P"]),
                        f[k + "init"], list(f[k + "flags"]), nu_fit=[nu, nu, nu],
                        errs=f[k + "errs"], log10_tau=bool(f[k + "log10"]))
    return {kk: v.cpu().numpy() for kk, v in out.items() if not kk.startswith("_")}


@pytest.mark.parametrize("ic", range(8))
def test_fit_portrait_full_golden(eng, golden, ic):
    f = golden("fit_full.npz")
    k = "f%d_" % ic
    r = fit_case(eng, f, ic)
    flags = list(f[k + "flags"])
    assert int(r["status"][0]) == int(f[k + "return_code"])
    params, errs = r["params"][0], r["param_errs"][0]
    names = ["phi", "DM", "GM", "tau", "alpha"]
    for i, nm in enumerate(names):
        ref = float(f[k + nm])
        sig = float(f[k + nm + "_err"])
        if flags[i]:
            assert abs(params[i] - ref) <= 1e-3 * sig, (nm, params[i], ref, sig)
            assert errs[i] == pytest.approx(sig, rel=1e-5), nm
        else:
            assert params[i] == pytest.approx(ref, rel=1e-9, abs=1e-12), nm
    for i, nm in enumerate(["nu_DM", "nu_GM", "nu_tau"]):
        assert r["nu_out"][0][i] == pytest.approx(float(f[k + nm]), rel=1e-6), nm
    assert r["red_chi2"][0] == pytest.approx(float(f[k + "red_chi2"]), rel=1e-8)
    assert r["snr"][0] == pytest.approx(float(f[k + "snr"]), rel=1e-6)
    np.testing.assert_allclose(r["scales"][0], f[k + "scales"], rtol=1e-5)
    np.testing.assert_allclose(r["scale_errs"][0], f[k + "scale_errs"], rtol=1e-5)
    nf = int(np.sum(flags))
    cov = r["cov"][0][:nf, :nf]
    ref = f[k + "covariance_matrix"]
    d = np.sqrt(np.abs(np.outer(np.diag(ref), np.diag(ref))))
    assert np.all(np.abs(cov - ref) <= 1e-4 * d)
    assert abs(int(r["nfev"][0]) - int(f[k + "nfeval"])) <= 2


def test_fit_batch_matches_single(eng, golden):
    """Subints are independent: a batch equals its members fitted alone."""
    f = golden("fit_full.npz")
    k = "f7_"
    nu = float(f[k + "nu_fit"])
    data = np.stack([f[k + "data"], f[k + "data"][:, ::-1].copy(), f[k + "data"]])
    out = eng.fit_batch(data, f[k + "model"], f[k + "freqs"], float(f["P"]), f[k + "init"],
                        [1, 1, 0, 0, 0], nu_fit=[nu, nu, nu], errs=f[k + "errs"])
    p = out["params"].cpu().numpy()
    np.testing.assert_array_equal(p[0], p[2])
    single = fit_case(eng, f, 7)
    np.testing.assert_array_equal(p[0], single["params"][0])


def test_guess_matches_oracle(eng, golden):
    """In-kernel get_TOAs initial guess vs the oracle's pptoas_guess."""
    f = golden("fit_full.npz")
    for ic in [1, 2, 7]:
        k = "f%d_" % ic
        data, model, freqs = f[k + "data"], f[k + "model"], f[k + "freqs"]
        nu = float(f[k + "nu_fit"])
        ref = O.pptoas_guess(data, model, freqs, np.ones(len(freqs)), 34.56789, P0, nu)
        out = eng.fit_batch(data, model, freqs, P0, [0.0, 34.56789, 0, 0, 0], [1, 1, 0, 0, 0],
                            nu_fit=[nu, nu, nu], guess=True, guess_Ns=100)
        got = float(out["init_used"].cpu().numpy()[0, 0])
        assert abs(got - ref) < 1e-6, (ic, got, ref)


def test_synth_matches_numpy(eng):
    from pulseportraiture_amd import synth
    nchan, nbin, nsub = 8, 256, 3
    model = np.random.default_rng(3).normal(0, 1, (nchan, nbin))
    ph = np.random.default_rng(4).uniform(-2, 2, (nsub, nchan))
    got = eng.synth(model, ph, 1.5, 12345, sub0=7).cpu().numpy()
    ref = synth.synth_portraits_host(model, ph, 1.5, 12345, sub0=7)
    np.testing.assert_allclose(got, ref, atol=1e-11)


@pytest.mark.parametrize("nsub,nchan,nbin", [(5, 6, 128), (37, 10, 2048), (3, 3, 2048),
                                              (45, 300, 2048)])
def test_rotate_accumulate(eng, nsub, nchan, nbin):
    """Fourier-domain rotate-and-sum of ppalign (ppalign.py:202-208); nbin 2048
    takes the one-wave-per-row register-FFT kernel (k_rot_accum_w), including
    slices shorter than a group of four rows (3 x 3, 37 x 10) and slices of
    seven rows: a full group and a ragged one (45 x 300, 7 slices)."""
    import torch
    rng = np.random.default_rng(9)
    data = rng.normal(0, 1, (nsub, nchan, nbin))
    ph = rng.uniform(-1, 1, (nsub, nchan))
    w = rng.uniform(0, 2, (nsub, nchan))
    w[min(2, nsub - 1), min(3, nchan - 1)] = 0.0
    acc = torch.zeros(nchan, nbin // 2 + 1, 2, dtype=torch.float64, device=eng.device)
    eng.rotate_accumulate(data, ph, w, acc)
    got = torch.view_as_complex(acc).cpu().numpy()
    k = np.arange(nbin // 2 + 1)
    ref = np.sum(w[..., None] * np.fft.rfft(data, axis=-1) *
                 np.exp(2j * np.pi * ph[..., None] * k), axis=0)
    np.testing.assert_allclose(got, ref, atol=1e-11 * np.abs(ref).max())


def test_engine_on_side_stream_keeps_its_temporaries(eng):
    """An engine bound to a side stream (a second context generating data
    beside the fits, bench --config gm_shard) allocates its temporaries for
    that stream: host arguments dropped right after the call cannot be
    reused by other work while its kernel still reads them.  The default
    stream is kept busy meanwhile; every chunk must equal the same synth on
    the default stream."""
    import torch
    from pulseportraiture_amd import synth
    from pulseportraiture_amd.engine import Engine
    w = synth.make_workload(64, 32, 1024, seed=77)
    side = torch.cuda.Stream(eng.device)
    geng = Engine(eng.device.index)
    geng.bind_stream(side)
    try:
        ref = [eng.synth(w.template, w.phase * (1 + i), w.sigma, 5, sub0=64 * i) for i in range(4)]
        torch.cuda.synchronize()
        outs = [torch.empty_like(ref[0]) for _ in range(4)]
        busy = torch.randn(4096, 4096, dtype=torch.float64, device=eng.device)
        for i in range(4):
            for _ in range(3):  # the default stream is busy (and allocates)
                busy = busy @ busy.T / 4096.0
            geng.synth(w.template, w.phase * (1 + i), w.sigma, 5, sub0=64 * i, out=outs[i])
            scratch = torch.full((1 << 20,), float(i), device=eng.device)  # reuse bait
            del scratch
        torch.cuda.synchronize()
        for r, o in zip(ref, outs):
            assert torch.equal(r, o)
    finally:
        geng.close()
