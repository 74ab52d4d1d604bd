"""Launch-schedule options (ppf_set_option) change no result.

Each option of include/ppfit.h selects another launch schedule of the same
kernels -- the split scattering solve's hipGraph groups, its split over
workgroups or the one-workgroup k_solve, the tail split, the fused or
separate first moment pass, the single-wave guess -- and every one of them
is claimed to give bitwise the same fits.  These run one batch per setting
in this process, on one context, and compare params, errors, nfev and status
bitwise (the graph / non-graph equality was only checked by an
A/B script)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEYS = ["params", "param_errs", "nu_out", "red_chi2", "snr", "nfev", "status", "init_used"]


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pulseportraiture_amd.engine import get_engine
    return get_engine(0)


def _fit(eng, w, data, flags, log10_tau, **opts):
    from pulseportraiture_amd import pplib
    saved = {k: eng.get_option(k) for k in opts}
    for k, v in opts.items():
        eng.set_option(k, v)
    try:
        nu = pplib.guess_fit_freq(w.freqs)
        n = data.shape[0]
        init = np.tile([0.0, w.DM0, 0.0, 0.0, 0.0], (n, 1))
        gt = None
        if flags[3]:
            tg = 2e-3 * (nu / w.nu_ref) ** w.alpha
            init[:, 3], init[:, 4] = np.log10(tg), w.alpha
            gt = np.full(n, tg)
        out = eng.fit_batch(data, w.model, w.freqs, w.P, init, flags, nu_fit=[nu] * 3,
                            log10_tau=log10_tau, guess=True, guess_Ns=100, guess_tau=gt)
        return {k: out[k].cpu().numpy() for k in KEYS}
    finally:
        for k, v in saved.items():
            eng.set_option(k, v)


def _same(a, b):
    for k in KEYS:
        assert np.array_equal(a[k], b[k], equal_nan=True), k


def test_option_roundtrip(gpu):
    assert gpu.get_option("scat_graph") == 1 and gpu.get_option("scat_tail") == 512
    gpu.set_option("scat_tail", 7)
    assert gpu.get_option("scat_tail") == 7
    gpu.set_option("scat_tail", 512)
    from pulseportraiture_amd.engine import PPFitError
    with pytest.raises(PPFitError):
        gpu.set_option("scat_graph", 2)


def test_scattering_schedules_bitwise(gpu):
    from pulseportraiture_amd import synth
    w = synth.make_workload(48, 128, 512, seed=4242, tau=2e-3)
    data = gpu.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
    flags = [1, 1, 0, 1, 1]
    base = _fit(gpu, w, data, flags, True)
    assert (base["nfev"] > 8).all()  # past the first graph group (iteration 4)
    _same(base, _fit(gpu, w, data, flags, True, scat_graph=0))
    _same(base, _fit(gpu, w, data, flags, True, scat_tail=0))
    _same(base, _fit(gpu, w, data, flags, True, scat_tail=100000))
    _same(base, _fit(gpu, w, data, flags, True, scat_tail=100000, scat_graph=0))
    _same(base, _fit(gpu, w, data, flags, True, scat_split=0))


def test_phase_family_schedules_bitwise(gpu):
    from pulseportraiture_amd import synth
    w = synth.make_workload(96, 64, 2048, seed=4343)
    data = gpu.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
    flags = [1, 1, 0, 0, 0]
    base = _fit(gpu, w, data, flags, False)
    _same(base, _fit(gpu, w, data, flags, False, fuse_moments=0))
    _same(base, _fit(gpu, w, data, flags, False, guess_wave=0))
