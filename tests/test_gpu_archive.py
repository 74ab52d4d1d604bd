"""load_data's processing on the device (archive.py): dedisperse /
dededisperse (pplib.py:2686-2687: rotate_data by the stored DM about the
archive centre frequency, pplib.py:2338-2426, held to the oracle's
rotate_data), remove_baseline (pplib.py:2691; PSRCHIVE's default estimator
restated in the oracle -- parity with PSRCHIVE itself is unpinned), the
dmc = 1 reload of get_TOAs (pptoas.py:255-264), ppalign's dedispersed initial
guess (ppalign.py:103-106), rm_baseline on a PSRFITS file with a DAT_OFFS
baseline through get_channels_to_zap (pptoas.py:1201-1278), and the
meta-first, per-range loading the sharded drivers use."""
import os
import shutil

import numpy as np
import pytest

from tests.golden_consts import DM0
from tests.psrfits_writer import quantize, write_psrfits

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pulseportraiture_amd.engine import get_engine
    return get_engine(0)


def _no_nyquist(x):
    """x without its Nyquist harmonic: a rotation keeps only Re X_N (irfft
    drops Im X_N), so only Nyquist-free rows survive a dedispersion round trip
    exactly -- and these fits move by hundreds of sigma with X_N alone."""
    f = np.fft.rfft(x, axis=-1)
    f[..., -1] = 0.0
    return np.fft.irfft(f, n=x.shape[-1], axis=-1)


def _bunch(nsub=3, nchan=16, nbin=256, seed=5, offsets=0.0, nyquist=True, **kw):
    from pulseportraiture_amd import synth
    w = synth.make_workload(nsub, nchan, nbin, seed=seed)
    data = synth.workload_data_host(w)
    data = (data if nyquist else _no_nyquist(data)) + offsets
    b = dict(subints=data[:, None], freqs=w.freqs, Ps=np.full(nsub, w.P),
             epochs=[(57100 + k, 0, 0.0) for k in range(nsub)], DM=DM0, nu0=1500.0,
             weights=np.ones((nsub, nchan)))
    b.update(kw)
    return w, b


def test_dedisperse_and_dededisperse_vs_oracle(gpu):
    from oracle import ppfit_oracle as O
    from pulseportraiture_amd import archive
    w, b = _bunch(dmc=0)
    archive.register_archive("dd_raw", b)
    d = archive.load_data("dd_raw", dedisperse=True, rm_baseline=False, quiet=True)
    ref = O.rotate_data(b["subints"], 0.0, DM0, b["Ps"], b["freqs"], 1500.0)
    assert d.dmc == 1
    np.testing.assert_allclose(d.subints, ref, rtol=0, atol=1e-12 * np.abs(ref).max())
    # dedisperse on a dedispersed archive is a no-op; dededisperse undoes it
    b2 = dict(b, subints=ref, dmc=1)
    archive.register_archive("dd_done", b2)
    same = archive.load_data("dd_done", dedisperse=True, rm_baseline=False, quiet=True)
    np.testing.assert_array_equal(same.subints, ref)
    back = archive.load_data("dd_done", dededisperse=True, rm_baseline=False, quiet=True)
    assert back.dmc == 0
    ref2 = O.rotate_data(ref, 0.0, -DM0, b["Ps"], b["freqs"], 1500.0)
    np.testing.assert_allclose(back.subints, ref2, rtol=0, atol=1e-12 * np.abs(ref2).max())
    # a rotation loses Im X_N (irfft drops it), so the round trip restores every
    # harmonic but the Nyquist one
    x0, x2 = (np.fft.rfft(np.asarray(v), axis=-1)[..., :-1] for v in (b["subints"], back.subints))
    np.testing.assert_allclose(x2, x0, rtol=0, atol=1e-10 * np.abs(x0).max())


def test_remove_baseline_vs_oracle(gpu):
    from oracle import ppfit_oracle as O
    from pulseportraiture_amd import archive
    rng = np.random.default_rng(3)
    offs = rng.uniform(-20, 40, size=(3, 16, 1))
    w, b = _bunch(offsets=offs, baseline_removed=False)
    b["weights"][1, 4] = 0.0
    archive.register_archive("bl_raw", b)
    d = archive.load_data("bl_raw", rm_baseline=True, quiet=True)
    ref, starts = O.remove_baseline(b["subints"], b["weights"])
    assert d.baseline_removed
    np.testing.assert_allclose(d.subints, ref, rtol=0, atol=1e-11 * np.abs(b["subints"]).max())
    # the window is the same on the device (its start is returned by the ABI)
    import torch
    t = torch.as_tensor(b["subints"], device=gpu.device).contiguous()
    win = gpu.remove_baseline(t, b["weights"]).cpu().numpy()
    np.testing.assert_array_equal(win, starts)
    # a second removal changes nothing beyond rounding (the window's mean is 0)
    again, _ = O.remove_baseline(ref, b["weights"])
    np.testing.assert_allclose(again, ref, rtol=0, atol=1e-11 * np.abs(ref).max())


def test_get_toas_dmc1_reloads_dededispersed(gpu, tmp_path):
    """A dedispersed archive (dmc = 1) is reloaded with dededisperse=True
    (pptoas.py:255-264): its TOAs equal those of the raw archive."""
    from oracle import ppfit_oracle as O
    from pulseportraiture_amd import archive, pptoas, synth
    w, b = _bunch(nsub=3, nchan=32, nbin=512, seed=9, dmc=0, nyquist=False)
    archive.register_archive("g_raw", b)
    ded = O.rotate_data(b["subints"], 0.0, DM0, b["Ps"], b["freqs"], 1500.0)
    archive.register_archive("g_ded", dict(b, subints=ded, dmc=1))
    shutil.copy(synth.EXAMPLE_GMODEL, str(tmp_path / "example.gmodel"))
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        out = []
        for name in ["g_raw", "g_ded"]:
            gt = pptoas.GetTOAs([name], "example.gmodel", quiet=True)
            gt.get_TOAs(quiet=True)
            out.append(gt)
    finally:
        os.chdir(cwd)
    a, c = out
    assert np.array_equal(a.rcs[0], c.rcs[0])
    for attr, err in [("phis", "phi_errs"), ("DMs", "DM_errs")]:
        e = np.asarray(getattr(a, err)[0])
        d = np.abs(np.asarray(getattr(a, attr)[0]) - np.asarray(getattr(c, attr)[0]))
        print(attr, "max |delta| / sigma", (d / e).max())
        assert np.all(d <= 1e-4 * e)


def test_align_initial_guess_is_dedispersed(gpu):
    """ppalign loads its initial guess with dedisperse=True (ppalign.py:103-106):
    a dispersed (dmc = 0) guess gives the same template as its dedispersed copy."""
    from oracle import ppfit_oracle as O
    from pulseportraiture_amd import archive, ppalign, synth
    names = []
    for i in range(3):
        w, b = _bunch(nsub=1, nchan=16, nbin=256, seed=40 + i)
        archive.register_archive("al_%d" % i, b)
        names.append("al_%d" % i)
    w = synth.make_workload(1, 16, 256, seed=40)
    w.model = _no_nyquist(w.model)
    disp = O.rotate_data(w.model[None, None], 0.0, -DM0, [w.P], w.freqs[None], 1500.0)
    archive.register_archive("guess_disp", dict(subints=disp, freqs=w.freqs, Ps=[w.P],
                                                epochs=[(57000, 0, 0.0)], DM=DM0, nu0=1500.0,
                                                dmc=0))
    archive.register_archive("guess_ded", dict(subints=w.model[None, None], freqs=w.freqs,
                                               Ps=[w.P], epochs=[(57000, 0, 0.0)], DM=DM0,
                                               nu0=1500.0, dmc=1))
    p1 = ppalign.align_archives(names, "guess_disp", niter=1, quiet=True)
    p2 = ppalign.align_archives(names, "guess_ded", niter=1, quiet=True)
    np.testing.assert_allclose(p1, p2, rtol=0, atol=1e-8 * np.abs(p2).max())


def test_psrfits_rm_baseline_zap_equals_offset_free(gpu, tmp_path):
    """show_fit / get_channels_to_zap load with rm_baseline=True
    (pptoas.py:1301, 1332): a PSRFITS file whose profiles carry a large
    DAT_OFFS baseline zaps the same channels, with the same per-channel
    reduced chi2, as the same samples without the offsets."""
    from pulseportraiture_amd import archive, pptoas, synth
    nsub, nchan, nbin = 2, 32, 512
    w = synth.make_workload(nsub, nchan, nbin, seed=61)
    I = synth.workload_data_host(w)
    I[0, 7] += 6.0 * np.sin(np.arange(nbin) * 0.3)  # a channel the zapper flags
    raw, scl, offs = quantize(I[:, None])
    big = np.full_like(offs, 75.0)
    path = str(tmp_path / "b.fits")
    wts = np.ones((nsub, nchan), np.float32)
    write_psrfits(path, raw, scl, offs + big, np.tile(w.freqs, (nsub, 1)), wts,
                  tsubint=[30.0] * nsub, offs_sub=15.0 + 30.0 * np.arange(nsub),
                  period=[w.P] * nsub, par_ang=np.zeros(nsub), pol_type="AA+BB")
    phys = raw.astype(np.float64) * scl[..., None] + offs[..., None]
    d = archive.load_data(path, pscrunch=True, rm_baseline=False, quiet=True)
    reg = {k: d[k] for k in ["freqs", "weights", "Ps", "epochs", "DM", "dmc", "backend",
                             "frontend", "backend_delay", "telescope", "telescope_code", "bw",
                             "nu0", "subtimes", "source", "state"]}
    reg.update(subints=phys, baseline_removed=False)
    archive.register_archive("zap_free", reg)
    shutil.copy(synth.EXAMPLE_GMODEL, str(tmp_path / "example.gmodel"))
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        res = []
        for name in [path, "zap_free"]:
            gt = pptoas.GetTOAs([name], "example.gmodel", quiet=True)
            gt.get_TOAs(quiet=True)
            gt.get_channels_to_zap(SNR_threshold=0.0, rchi2_threshold=1.3)
            res.append(gt)
    finally:
        os.chdir(cwd)
    a, b = res
    assert a.zap_channels == b.zap_channels and any(len(z) for z in a.zap_channels[0])
    for ra, rb in zip(a.channel_red_chi2s[0], b.channel_red_chi2s[0]):
        np.testing.assert_allclose(ra, rb, rtol=1e-6)


def test_open_archive_reads_ranges(gpu):
    """open_archive: metadata without DATA, then any subint range -- the
    per-rank read of the sharded drivers -- equals the same rows of a whole
    load (registered numpy, registered device tensor)."""
    import torch
    from pulseportraiture_amd import archive
    w, b = _bunch(nsub=6, baseline_removed=False)
    archive.register_archive("rng_np", b)
    archive.register_archive("rng_dev", dict(b, subints=torch.as_tensor(b["subints"],
                                                                        device=gpu.device)))
    whole = archive.load_data("rng_np", rm_baseline=True, quiet=True).subints
    for name in ["rng_np", "rng_dev"]:
        a = archive.open_archive(name, rm_baseline=True)
        assert "subints" not in a.meta and a.meta.nsub == 6
        part = archive.host_array(a.read(2, 5))
        np.testing.assert_allclose(part, whole[2:5], rtol=0, atol=1e-13 * np.abs(whole).max())
    # the registered device tensor itself is never modified
    assert np.array_equal(archive._registry["rng_dev"].subints.cpu().numpy(), b["subints"])


@pytest.mark.parametrize("sparse", [False, True])
def test_get_toas_pieces_equal_one_piece(gpu, tmp_path, sparse):
    """Device-resident subints fitted in pipeline pieces (pipeline_fracs: the
    pieces' columns concatenated by _finish) give the per-archive columns and
    .tim text of one piece; sparse: one subint with no weight, so ok_isubs
    skips it (the spread into nsub rows)."""
    import torch
    from pulseportraiture_amd import archive, pplib, pptoas, synth
    w, b = _bunch(nsub=40, nchan=16, nbin=256, seed=21)
    if sparse:
        b["weights"][7] = 0.0
    b["subints"] = torch.as_tensor(b["subints"], device="cuda")
    archive.register_archive("pieces", b)
    shutil.copy(synth.EXAMPLE_GMODEL, str(tmp_path / "example.gmodel"))
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        out, tims = [], []
        for mins in (1 << 30, 8):
            gt = pptoas.GetTOAs(["pieces"], "example.gmodel", quiet=True)
            gt.pipeline_min_subints = mins
            gt.get_TOAs(quiet=True)
            tim = str(tmp_path / ("p%d.tim" % mins))
            pplib.write_TOAs(gt.TOA_list, SNR_cutoff=0.0, outfile=tim, append=False)
            out.append(gt)
            tims.append(open(tim).read())
    finally:
        os.chdir(cwd)
        archive.unregister_archive("pieces")
    one, two = out
    assert len(two.shard_blocks) == 2  # really two pieces
    assert len(one.ok_isubs[0]) == (39 if sparse else 40)
    for attr in ("phis", "phi_errs", "DMs", "DM_errs", "scales", "scale_errs", "channel_snrs",
                 "snrs", "red_chi2s", "covariances", "nfevals", "rcs", "nu_refs", "TOA_errs"):
        a, c = np.asarray(getattr(one, attr)[0]), np.asarray(getattr(two, attr)[0])
        assert a.shape == c.shape, attr
        assert np.array_equal(a.astype(np.float64), c.astype(np.float64), equal_nan=True), attr
    assert tims[0] == tims[1]
