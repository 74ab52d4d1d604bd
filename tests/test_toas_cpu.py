"""The column-built TOA records (pulseportraiture_amd/toas.py) and the native
.tim writer (libpptim.so, include/pptim.h) on CPU.

- The writer's numbers are Python's %-formatting, digit for digit, over
  random values of every magnitude, the special values and the rounding ties
  (pplib.py:3471-3503 formats with Python-2 %).
- get_TOAs (device fit replaced by tests/test_dist_drivers_cpu.fake_fit)
  under every flag variant: write_TOAs' bulk text of the never-built records
  equals toa_line over the TOA objects, which are the reference's records
  (the .tim goldens hold those on the GPU, test_gpu_drivers /
  test_gpu_configs).
- TOA_list behaves as the reference's list: indexing, iteration, slicing,
  mutation; a record modified by the caller is written as modified.
- TOAs[iarch] (MJDArray) indexes like the reference's object array.
"""
import os
import tempfile

import numpy as np
import pytest

from tests.test_dist_drivers_cpu import DM0, fake_fit
from pulseportraiture_amd.pptoaslib import SyncPipeline  # noqa: E402


# ---------------------------------------------------------------------------
# the writer's number formatting
# ---------------------------------------------------------------------------
def _fmt(kind, prec, x):
    from pulseportraiture_amd import toas as T
    return str(T.format_rows(len(x), [(kind, prec, x, None, None)])).split("\n")[:-1]


def test_fixed_digits_equal_python_formatting():
    from pulseportraiture_amd import toas as T
    rng = np.random.default_rng(5)
    n = 40000
    x = np.concatenate([
        rng.standard_normal(n) * 10.0 ** rng.integers(-20, 17, n),
        rng.random(n),
        (rng.integers(0, 10 ** 6, n) + 0.5) / 10.0 ** rng.integers(0, 8, n),  # decimal ties
        [0.0, -0.0, 1e-300, 5e-324, -5e-324, 0.5, 1.5, 2.5, -0.5, 9.9999995, 2.0 ** 53 - 1,
         2.0 ** 62, 2.0 ** 63, 2.0 ** 64 + 2048, 1e300, -1e300, np.inf, -np.inf, np.nan, -np.nan,
         0.0005, 0.00049999999999999999, 1234.5678, 0.9999999999999999]])
    for p in (0, 1, 3, 5, 7, 8, 15, 17):
        got = _fmt(T.PPT_F64_FIXED, p, x)
        ref = ["%.*f" % (p, v) for v in x]
        bad = [(a, b) for a, b in zip(ref, got) if a != b]
        assert not bad, (p, bad[:5])
    assert _fmt(T.PPT_F64_FRAC, 15, x) == [("%.15f" % v)[1:] for v in x]
    assert _fmt(T.PPT_F64_EXP, 1, x) == ["%.1e" % v for v in x]
    i = np.concatenate([rng.integers(-2 ** 62, 2 ** 62, 1000), [0, -1, 2 ** 63 - 1, -2 ** 63]])
    assert _fmt(T.PPT_I64, 0, i) == ["%d" % v for v in i]


def test_writer_fields_presence_and_threads():
    """Presence masks leave a field out per row; keep drops rows; the text
    does not depend on the thread count."""
    from pulseportraiture_amd import toas as T
    n = 9000
    x = np.arange(n) * 0.25
    pres = (np.arange(n) % 3 != 0).astype(np.uint8)
    strs = ["s%d" % k if k % 2 else "" for k in range(n)]
    fields = [(T.PPT_TEXT, 0, b"a ", None, None), (T.PPT_F64_FIXED, 2, x, None, None),
              (T.PPT_TEXT, 0, b" -p ", None, pres), (T.PPT_I64, 0, np.arange(n), None, pres),
              T._strs_field(strs)]
    ref = ["a %.2f%s%s" % (x[k], " -p %d" % k if pres[k] else "", strs[k]) for k in range(n)]
    keep = np.arange(n) % 5 != 1
    outs = []
    for nt in (1, 3, 8):
        T._host_threads, old = (lambda: nt), T._host_threads
        try:
            outs.append(str(T.format_rows(n, fields)).split("\n")[:-1])
            kept = str(T.format_rows(n, fields, keep)).split("\n")[:-1]
        finally:
            T._host_threads = old
        assert kept == [r for r, k in zip(ref, keep) if k]
    assert outs[0] == ref and outs[1] == ref and outs[2] == ref


# ---------------------------------------------------------------------------
# get_TOAs records: bulk text == per-object text
# ---------------------------------------------------------------------------
def _archives(one_chan=True, gaps=True):
    from pulseportraiture_amd import archive, synth
    from pulseportraiture_amd.mjd import MJD
    names = []
    for i, (nsub, nchan) in enumerate([(6, 8), (4, 8)]):
        w = synth.make_workload(nsub, nchan, 64, seed=70 + i)
        data = synth.workload_data_host(w)
        wts = np.ones((nsub, nchan))
        wts[1, 2] = 0.0
        if one_chan and i == 0:
            wts[3, 1:] = 0.0  # a 1-channel subint: phase only, no DM (pptoas.py:474-484)
        if gaps and i == 1:
            wts[2] = 0.0  # a subint with no channel: not an ok subint
        name = "toas_cpu%d.npz" % i
        archive.register_archive(name, dict(
            subints=data[:, None], freqs=w.freqs, Ps=np.full(nsub, w.P), weights=wts,
            noise_stds=np.full((nsub, 1, nchan), 1.5),
            epochs=[MJD(57000.0 + 0.37 * k) for k in range(nsub)], DM=DM0, backend="be",
            frontend="fe", telescope="GBT", telescope_code="1",
            parallactic_angles=np.linspace(-30, 40, nsub), subtimes=[59.5 + k for k in range(nsub)]))
        names.append(name)
    return names


def _get_toas(names, fit=fake_fit, **kw):
    from pulseportraiture_amd import pplib, pptoas, synth
    pptoas.fit_pipeline = lambda keys: SyncPipeline(fit, keys)
    pptoas.gen_gaussian_portraits_device = lambda code, params, alpha, nbin, freqs, nu_ref: \
        np.array([pplib.gen_gaussian_portrait(code, params, alpha, pplib.get_bin_centers(nbin), f,
                                              nu_ref) for f in np.atleast_2d(freqs)])
    gt = pptoas.GetTOAs(names, synth.EXAMPLE_GMODEL, quiet=True)
    gt.get_TOAs(quiet=True, **kw)
    return gt


def _bulk(gt, **kw):
    from pulseportraiture_amd import pplib
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "x.tim")
        pplib.write_TOAs(gt.TOA_list, outfile=path, append=False, **kw)
        return open(path).read().splitlines()


def _per_toa(gt, inf_is_zero=True, SNR_cutoff=0.0):
    from pulseportraiture_amd import pplib
    toas = pplib.filter_TOAs(list(gt.TOA_list), "snr", SNR_cutoff, ">=", pass_unflagged=False)
    return [pplib.toa_line(t, inf_is_zero) for t in toas]


VARIANTS = [
    dict(),
    dict(print_phase=True, print_flux=True, print_parangle=True),
    dict(addtnl_toa_flags={"pta": "NANOGrav", "snr": 1.0, "ver": 3, "none": None,
                           "DM_mean": True, "gm": 0.5}),
    dict(fit_GM=True, nu_refs=(1400.0, 1500.0)),
    dict(fit_DM=False, bary=False),
    dict(fit_scat=True, log10_tau=True, print_phase=True),
    dict(fit_scat=True, log10_tau=False, fix_alpha=True),
]


@pytest.mark.parametrize("kw", VARIANTS, ids=[",".join(sorted(v)) or "default" for v in VARIANTS])
def test_bulk_text_equals_per_toa_text(kw):
    gt = _get_toas(_archives(), **kw)
    bulk = _bulk(gt)
    assert len(bulk) == len(gt.TOA_list) == 9  # 6 + 4 subints, one without channels
    assert bulk == _per_toa(gt)


def test_zapped_first_subint_shared_rows():
    """Subint 0 fully zapped and every other subint sharing one weights row:
    the one row handed to the fits is an ok subint's, not subint
    0's all-zero row (nor its frequencies) -- every fitted channel keeps its
    scale, and the ok subints' results equal those of the same archive
    without subint 0."""
    from pulseportraiture_amd import archive, synth
    from pulseportraiture_amd.mjd import MJD
    nsub, nchan = 5, 8
    w = synth.make_workload(nsub, nchan, 64, seed=91)
    data = synth.workload_data_host(w)
    out = []
    for name, s0 in (("zap0.npz", 0), ("zap0_dropped.npz", 1)):
        wts = np.ones((nsub, nchan))
        wts[:, 5] = 0.25
        wts[0] = 0.0
        freqs = np.tile(w.freqs, (nsub, 1))
        freqs[0] += 1.0  # subint 0's own row differs too
        archive.register_archive(name, dict(
            subints=data[s0:, None], freqs=freqs[s0:], Ps=np.full(nsub - s0, w.P),
            weights=wts[s0:], noise_stds=np.full((nsub - s0, 1, nchan), 1.5),
            epochs=[MJD(57000.0 + 0.37 * k) for k in range(s0, nsub)], DM=DM0, backend="be",
            frontend="fe", telescope="GBT", telescope_code="1",
            parallactic_angles=np.zeros(nsub - s0), subtimes=[60.0] * (nsub - s0)))
        try:
            out.append(_get_toas([name]))
        finally:
            archive.unregister_archive(name)
    a, b = out
    assert list(a.ok_isubs[0]) == [1, 2, 3, 4] and list(b.ok_isubs[0]) == [0, 1, 2, 3]
    sc = np.asarray(a.scales[0])
    assert (sc[1:] > 0).all() and not sc[0].any()
    for attr in ("phis", "DMs", "scales", "channel_snrs", "nu_refs", "snrs"):
        assert np.array_equal(np.asarray(getattr(a, attr)[0], float)[1:],
                              np.asarray(getattr(b, attr)[0], float), equal_nan=True), attr


def test_flag_maps_and_types():
    """TOA objects built from the columns carry the reference's flag order and
    Python types (ints %d, floats, strings; None kept in the dict)."""
    gt = _get_toas(_archives(), addtnl_toa_flags={"pta": "X", "none": None, "gm": 0.5})
    t0 = gt.TOA_list[0]
    keys = list(t0.flags)
    assert keys[:2] == ["be", "fe"]  # no GM fit: "gm" is an added flag, last
    assert keys[-3:] == ["pta", "none", "gm"]
    assert type(t0.flags["nbin"]) is int and type(t0.flags["subint"]) is int
    assert type(t0.flags["snr"]) is float and type(t0.flags["tobs"]) is float
    assert t0.flags["none"] is None and t0.snr == t0.flags["snr"]
    one = gt.TOA_list[3]  # archive 0's 1-channel subint: phase only
    assert one.DM is None and one.DM_error is None and "phi_DM_cov" not in one.flags


def test_snr_cutoff_and_inf_frequency():
    def fit_inf(*a, **k):
        r = fake_fit(*a, **k)
        r["nu_out"][0, 0] = np.inf
        return r
    gt = _get_toas(_archives(), fit=fit_inf)
    snr = sorted(t.snr for t in list(gt.TOA_list))
    cut = snr[len(snr) // 2]
    gt2 = _get_toas(_archives(), fit=fit_inf)
    for kw in (dict(SNR_cutoff=cut), dict(inf_is_zero=False), dict(SNR_cutoff=1e300)):
        assert _bulk(gt2, **kw) == _per_toa(gt, **kw)
    assert " 0.00000000 " in _bulk(gt2)[0] and " inf " in _bulk(gt2, inf_is_zero=False)[0]


def test_toa_list_sequence_semantics():
    from pulseportraiture_amd import pplib
    from pulseportraiture_amd.toas import TOA, TOAList
    gt = _get_toas(_archives())
    ref = _bulk(gt)
    L = gt.TOA_list
    assert isinstance(L, TOAList) and len(L) == len(ref)
    # a record modified through indexing is written as modified (pptoas.py:1593-1602)
    t = L[4]
    assert L[4] is t and L[-1] is L[len(L) - 1]
    t.DM = 1.25
    t.flags["DM_mean"] = True
    got = _bulk(gt)
    exp = list(ref)
    exp[4] = pplib.toa_line(t)
    assert got == exp and "-DM_mean 1" in got[4] and "-pp_dm 1.2500000" in got[4]
    # list operations
    sl = L[2:5]
    assert isinstance(sl, list) and sl[2] is t
    extra = TOA("x.ar", 1400.0, t.MJD, 1.0, "GBT", "1", None, None, {"snr": 5.0})
    L.append(extra)
    assert L[-1] is extra and len(L) == len(ref) + 1
    assert _bulk(gt)[-1] == pplib.toa_line(extra)
    objs = [x for x in L]
    assert objs[4] is t and objs[-1] is extra
    del L[0]
    assert L[0] is objs[1] and len(L) == len(ref)
    L.insert(0, objs[0])
    assert [x for x in L] == objs
    L2 = TOAList(L)
    assert L2 == objs and (L + [extra])[-1] is extra


def test_mjd_array_matches_records():
    gt = _get_toas(_archives())
    for ia, arr in enumerate(gt.TOAs):
        ok = set(int(i) for i in gt.ok_isubs[ia])
        assert len(arr) == len(gt.phis[ia])
        for isub in range(len(arr)):
            if isub not in ok:
                assert arr[isub] == 0
    recs = [x for x in gt.TOA_list]
    okl = [(ia, int(i)) for ia in range(len(gt.TOAs)) for i in gt.ok_isubs[ia]]
    for t, (ia, isub) in zip(recs, okl):
        m = gt.TOAs[ia][isub]
        assert (m.days, m.secs, m.fracsec) == (t.MJD.days, t.MJD.secs, t.MJD.fracsec)
    a = np.asarray(gt.TOAs[0])
    assert a.dtype == object and a.shape == (6,)
    sub = gt.TOAs[0][gt.ok_isubs[0]]
    assert len(sub) == len(gt.ok_isubs[0]) and all(x != 0 for x in sub)


def test_pipeline_pieces_equal_one_piece(monkeypatch):
    """get_TOAs fitted in many pipeline pieces (each turned into its own
    column shard as it completes) gives the one-piece records and arrays."""
    from pulseportraiture_amd import pptoaslib
    ref = _get_toas(_archives(), print_phase=True)
    monkeypatch.setattr(pptoaslib, "STREAM_CHUNK_BYTES", 2 * 8 * 8 * 64)  # 2 subints a piece
    got = _get_toas(_archives(), print_phase=True)
    assert len(got.shard_blocks) > len(ref.shard_blocks) >= 2
    assert _bulk(got) == _bulk(ref) == _per_toa(got)
    for k in ("phis", "DMs", "scales", "covariances", "nu_refs", "rcs"):
        for a, b in zip(getattr(got, k), getattr(ref, k)):
            np.testing.assert_array_equal(np.asarray(a), np.asarray(b))
    assert got.DeltaDM_means == ref.DeltaDM_means
