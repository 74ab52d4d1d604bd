"""Edges of the device path: every supported nbin (64 ... 8192, including the
one-wave-per-workgroup data pass above nbin 2048), an empty batch, a subint
whose channels are all masked, a one-channel phase-only fit, and a batch
whose subints run different templates.  Each is held to the oracle (the
numpy/scipy restatement pinned to the reference's fixtures) at north_star's
1e-3 sigma with identical status."""
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


def _oracle_fit(O, d, model, init, P, freqs, nu, errs, flags):
    return O.fit_portrait_full(d, model, list(init), P, freqs, [nu] * 3, [None] * 3, errs,
                               list(flags), log10_tau=False)


def _check(O, res, i, d, model, P, freqs, nu, errs, flags):
    ref = _oracle_fit(O, d, model, res["init_used"][i], P, freqs, nu, errs, flags)
    assert int(res["status"][i]) == ref.return_code, (i, res["status"][i], ref.return_code)
    assert abs(res["params"][i][0] - ref.phi) <= 1e-3 * ref.phi_err, (i, "phi")
    if flags[1]:
        assert abs(res["params"][i][1] - ref.DM) <= 1e-3 * ref.DM_err, (i, "DM")
    return ref


@pytest.mark.parametrize("nbin", [64, 128, 4096, 8192])
def test_nbin_range_vs_oracle(gpu, nbin):
    from oracle import ppfit_oracle as O
    from pulseportraiture_amd import pptoaslib, synth
    nsub, nchan = 3, 8
    w = synth.make_workload(nsub, nchan, nbin, seed=200 + nbin)
    data = synth.workload_data_host(w)
    errs = np.array([O.get_noise_PS(d, chans=True) for d in data])
    nu = O.guess_fit_freq(w.freqs)
    init = np.array([[0.0, w.DM0, 0.0, 0.0, 0.0]] * nsub)
    res = pptoaslib.fit_portraits_batch(data, w.model, init, w.P, w.freqs,
                                        nu_fits=np.full((nsub, 3), nu), errs=errs,
                                        fit_flags=[1, 1, 0, 0, 0], guess=True)
    for i in range(nsub):
        _check(O, res, i, data[i], w.model, w.P, w.freqs, nu, errs[i], [1, 1, 0, 0, 0])
    # the device's own noise estimate (errs=None) is get_noise_PS's
    r2 = pptoaslib.fit_portraits_batch(data, w.model, init, w.P, w.freqs,
                                       nu_fits=np.full((nsub, 3), nu), errs=None,
                                       fit_flags=[1, 1, 0, 0, 0], guess=True)
    np.testing.assert_allclose(r2["params"], res["params"], rtol=0,
                               atol=1e-9 * np.abs(res["params"]).max())


def test_empty_batch(gpu):
    from pulseportraiture_amd import pptoaslib, synth
    w = synth.make_workload(1, 8, 256, seed=5)
    res = pptoaslib.fit_portraits_batch(np.zeros((0, 8, 256)), w.model, np.zeros((0, 5)), w.P,
                                        np.zeros((0, 8)), nu_fits=np.zeros((0, 3)),
                                        fit_flags=[1, 1, 0, 0, 0], guess=True)
    assert res["params"].shape == (0, 5) and res["status"].shape == (0,)


def test_all_masked_subint_and_neighbours(gpu):
    """A subint with no fitted channel reports status -1 and NaN parameters
    (the drivers never send one: get_TOAs skips it via ok_isubs,
    pplib.py:2757-2758); its neighbours in the batch are unaffected."""
    from oracle import ppfit_oracle as O
    from pulseportraiture_amd import pptoaslib, synth
    nsub, nchan, nbin = 4, 16, 512
    w = synth.make_workload(nsub, nchan, nbin, seed=77)
    data = synth.workload_data_host(w)
    mask = np.ones((nsub, nchan), dtype=np.uint8)
    mask[2] = 0
    mask[1, 3:6] = 0
    errs = np.array([O.get_noise_PS(d, chans=True) for d in data])
    nu = O.guess_fit_freq(w.freqs)
    init = np.array([[0.0, w.DM0, 0.0, 0.0, 0.0]] * nsub)
    res = pptoaslib.fit_portraits_batch(data, w.model, init, w.P, w.freqs,
                                        nu_fits=np.full((nsub, 3), nu), errs=errs,
                                        fit_flags=[1, 1, 0, 0, 0], chan_mask=mask, guess=True)
    assert int(res["status"][2]) == -1 and np.isnan(res["params"][2]).all()
    for i in (0, 3):
        _check(O, res, i, data[i], w.model, w.P, w.freqs, nu, errs[i], [1, 1, 0, 0, 0])
    # subint 1 with three channels masked: the oracle on its fitted rows
    ok = mask[1].astype(bool)
    _check(O, res, 1, data[1][ok], w.model[ok], w.P, w.freqs[ok], nu, errs[1][ok],
           [1, 1, 0, 0, 0])


def test_single_channel_phase_only(gpu):
    """One channel, phase only (get_TOAs' flags for a 1-channel subint,
    pptoas.py:474-476)."""
    from oracle import ppfit_oracle as O
    from pulseportraiture_amd import pptoaslib, synth
    nsub, nbin = 3, 1024
    w = synth.make_workload(nsub, 1, nbin, seed=91)
    data = synth.workload_data_host(w)
    errs = np.array([O.get_noise_PS(d, chans=True) for d in data])
    nu = float(w.freqs[0])
    init = np.array([[0.0, w.DM0, 0.0, 0.0, 0.0]] * nsub)
    res = pptoaslib.fit_portraits_batch(data, w.model, init, w.P, w.freqs,
                                        nu_fits=np.full((nsub, 3), nu), errs=errs,
                                        fit_flags=[1, 0, 0, 0, 0], guess=True)
    for i in range(nsub):
        _check(O, res, i, data[i], w.model, w.P, w.freqs, nu, errs[i], [1, 0, 0, 0, 0])


def test_mixed_templates_in_one_batch(gpu):
    """model_idx: subints of one batch fitted against different templates
    (get_TOAs builds one template per distinct frequency row / response)
    equal to fitting each subint alone."""
    from pulseportraiture_amd import pptoaslib, synth
    nchan, nbin = 16, 512
    wa = synth.make_workload(2, nchan, nbin, seed=301)
    wb = synth.make_workload(2, nchan, nbin, seed=302, tau=1e-3)
    data = np.concatenate([synth.workload_data_host(wa), synth.workload_data_host(wb)])
    models = np.stack([wa.model, wb.model])
    midx = np.array([0, 1, 0, 1], dtype=np.int32)
    nu = float(np.mean(wa.freqs))
    init = np.array([[0.0, wa.DM0, 0.0, 0.0, 0.0]] * 4)
    res = pptoaslib.fit_portraits_batch(data, models, init, wa.P, wa.freqs,
                                        nu_fits=np.full((4, 3), nu), fit_flags=[1, 1, 0, 0, 0],
                                        model_idx=midx, guess=True)
    for i in range(4):
        one = pptoaslib.fit_portraits_batch(data[i:i + 1], models[midx[i]], init[:1], wa.P,
                                            wa.freqs, nu_fits=np.full((1, 3), nu),
                                            fit_flags=[1, 1, 0, 0, 0], guess=True)
        np.testing.assert_array_equal(res["params"][i], one["params"][0])
        assert res["status"][i] == one["status"][0]
