"""Data-spectrum cache (ppfit.h PPF_SPEC_*, Engine.spec_cache): ppalign's
refits of the same subints against each new template (ppalign.py:160-213).

The claim is bit-for-bit: a fit that stores the spectra (STORE: the Taylor
moment passes form X = D conj(M) from the stored D instead of reading X) and
a later fit from the cache (USE: no data pass for Taylor-path subints) give
exactly the fits of a plain call, for the same template and for a new one --
with masked channels, non-unit weights, estimated noise (NaN errs), two
templates, subints that recentre their Taylor expansion, subints the Taylor
path does not take (scattering at the start: they keep their X), and the
two-queue piece schedule.  rotate_accumulate_spec (the rotate-and-sum from
the cached spectra) agrees with rotate_accumulate (which transforms the rows
itself, with other twiddles) to rounding."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEYS = ["params", "param_errs", "nu_out", "cov", "scales", "scale_errs", "channel_snrs",
        "red_chi2", "snr", "nfev", "status", "init_used", "errs"]


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pulseportraiture_amd.engine import get_engine
    return get_engine(0)


def _case(gpu, nsub, nchan, nbin, seed, scat_rows=()):
    from pulseportraiture_amd import pplib, synth
    w = synth.make_workload(nsub, nchan, nbin, seed=seed)
    data = gpu.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
    rng = np.random.default_rng(seed)
    mask = (rng.random((nsub, nchan)) > 0.1).astype(np.uint8)
    mask[:, 0] = 1
    wts = rng.uniform(0.5, 2.0, (nsub, nchan))
    errs = np.where(rng.random((nsub, nchan)) < 0.5, np.nan, w.sigma)
    nu = pplib.guess_fit_freq(w.freqs)
    init = np.tile([0.0, w.DM0, 0.0, 0.0, 0.0], (nsub, 1))
    init[list(scat_rows), 3] = 1e-3  # tau at the start, not fitted: not the Taylor path
    model2 = np.roll(w.model, 3, axis=-1) * 1.01
    midx = (np.arange(nsub) % 2).astype(np.int32)
    models = np.stack([w.model, model2])
    return dict(w=w, data=data, mask=mask, wts=wts, errs=errs, nu=nu, init=init,
                models=models, midx=midx)


def _fit(gpu, c, model, spec=None, guess=True, init=None, midx=None):
    w = c["w"]
    out = gpu.fit_batch(c["data"], model, w.freqs, w.P, c["init"] if init is None else init,
                        [1, 1, 0, 0, 0], nu_fit=[c["nu"]] * 3, errs=c["errs"],
                        chan_mask=c["mask"], weights=c["wts"], model_idx=midx, guess=guess,
                        guess_Ns=w.nbin, guess_wrap=False, guess_nu=c["nu"], spec_cache=spec)
    return {k: out[k].cpu().numpy() for k in KEYS}


def _same(a, b):
    for k in KEYS:
        assert np.array_equal(a[k], b[k], equal_nan=True), k


@pytest.mark.parametrize("nbin", [512, 2048])
def test_store_use_bitwise(gpu, nbin):
    c = _case(gpu, 40, 64, nbin, 515 + nbin, scat_rows=(5, 17))
    w = c["w"]
    m1, m2 = c["models"][0], c["models"][1]
    base1, base2 = _fit(gpu, c, m1), _fit(gpu, c, m2)
    sc = gpu.spec_cache(*c["data"].shape)
    _same(base1, _fit(gpu, c, m1, spec=sc))           # STORE
    assert sc.stored
    _same(base2, _fit(gpu, c, m2, spec=sc))           # USE, a new template
    _same(base1, _fit(gpu, c, m1, spec=sc))           # USE, the first again
    # two templates by model_idx
    basei = _fit(gpu, c, c["models"], midx=c["midx"])
    _same(basei, _fit(gpu, c, c["models"], spec=sc, midx=c["midx"]))
    assert (base1["status"][[5, 17]] >= 0).all()


def test_recentring_bitwise(gpu):
    """No guess and a start a quarter turn out: the Taylor fits recentre
    (moment_tile8's path) -- counted by the phase profile."""
    c = _case(gpu, 24, 64, 1024, 777)
    init = c["init"].copy()
    init[:, 0] = 0.25  # the injected phases are within 0.1 of 0
    gpu.phase_profile(True)
    base = _fit(gpu, c, c["models"][0], guess=False, init=init)
    sc = gpu.spec_cache(*c["data"].shape)
    _same(base, _fit(gpu, c, c["models"][0], spec=sc, guess=False, init=init))
    _same(base, _fit(gpu, c, c["models"][0], spec=sc, guess=False, init=init))
    counts = gpu.phase_profile(False)
    assert counts[8] > 0, "no recentre exercised"


def test_pieces_schedule_bitwise(gpu):
    """The two-queue piece schedule (ppf_set_pipeline), with and without the
    cache, and with subints the Taylor path does not take among the pieces
    (their scattering solve and post-fit run per piece as on one queue)."""
    c = _case(gpu, 48, 64, 2048, 9191, scat_rows=(3, 30))
    base = _fit(gpu, c, c["models"][0])
    assert (base["status"][[3, 30]] >= 0).all() and (base["nfev"][[3, 30]] > 0).all()
    gpu.set_pipeline(3)
    try:
        _same(base, _fit(gpu, c, c["models"][0]))
        sc = gpu.spec_cache(*c["data"].shape)
        _same(base, _fit(gpu, c, c["models"][0], spec=sc))
        _same(base, _fit(gpu, c, c["models"][0], spec=sc))
    finally:
        gpu.set_pipeline(0)


@pytest.mark.parametrize("nbin", [256, 2048, 4096])
def test_rotate_accumulate_spec(gpu, nbin):
    import torch
    c = _case(gpu, 20, 32, nbin, 31 + nbin)
    sc = gpu.spec_cache(*c["data"].shape)
    _fit(gpu, c, c["models"][0], spec=sc)
    rng = np.random.default_rng(5)
    ph = rng.uniform(-0.5, 0.5, (20, 32))
    wt = rng.uniform(0.0, 2.0, (20, 32))
    wt[3] = 0.0
    wt[c["mask"] == 0] = 0.0  # masked rows: no spectrum stored (zeros), weight 0 as in ppalign
    nh = nbin // 2 + 1
    a0 = torch.zeros(32, nh, 2, dtype=torch.float64, device=gpu.device)
    a1 = torch.zeros_like(a0)
    gpu.rotate_accumulate(c["data"], ph, wt, a0)
    gpu.rotate_accumulate_spec(sc, ph, wt, a1)
    a0, a1 = a0.cpu().numpy(), a1.cpu().numpy()
    scale = np.abs(a0).max()
    assert np.abs(a1 - a0).max() <= 1e-12 * scale
    # and against numpy: sum_s w rfft(row) e^{2 pi i k ph}
    d = c["data"].cpu().numpy()
    ref = np.einsum("sn,snk->nk", wt, np.fft.rfft(d, axis=-1) *
                    np.exp(2j * np.pi * np.arange(nh)[None, None] * ph[..., None]))
    assert np.abs(a1[..., 0] + 1j * a1[..., 1] - ref).max() <= 1e-10 * np.abs(ref).max()


def test_spec_cache_rejects(gpu):
    from pulseportraiture_amd.engine import PPFitError
    c = _case(gpu, 4, 16, 256, 3)
    w = c["w"]
    sc = gpu.spec_cache(*c["data"].shape)
    with pytest.raises(PPFitError, match="phase-family"):
        gpu.fit_batch(c["data"], w.model, w.freqs, w.P, c["init"], [1, 1, 0, 1, 0],
                      spec_cache=sc)
    with pytest.raises(PPFitError, match="phase-family"):
        gpu.fit_batch(c["data"], w.model, w.freqs, w.P, c["init"], [1, 1, 0, 0, 0],
                      exact=True, spec_cache=sc)
    with pytest.raises(PPFitError):
        gpu.rotate_accumulate_spec(sc, np.zeros((4, 16)), np.ones((4, 16)), None)
    with pytest.raises(PPFitError, match="spec_cache is for"):
        gpu.fit_batch(c["data"][:2], w.model, w.freqs, w.P, c["init"][:2], [1, 1, 0, 0, 0],
                      spec_cache=sc)
