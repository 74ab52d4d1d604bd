"""Host PSRFITS reader (include/ppfits.h, libppfits.so) on files written by
tests/psrfits_writer.py: headers, SUBINT metadata, raw samples of every
supported type, POLYCO periods, HISTORY dedispersion, error paths.
Parity unpinned against PSRCHIVE (absent here; the reference ships no
archives): these are round trips of the PSRFITS layout."""
import os

import numpy as np
import pytest

from tests.psrfits_writer import quantize, write_psrfits


@pytest.fixture(scope="module")
def lib():
    from pulseportraiture_amd import build
    build.build_fits()
    from pulseportraiture_amd import psrfits
    return psrfits


def _arch(rng, nsub=3, npol=4, nchan=8, nbin=64):
    data = rng.normal(size=(nsub, npol, nchan, nbin)) * 3.0 + 10.0
    raw, scl, offs = quantize(data)
    freqs = np.tile(np.linspace(1100.0, 1900.0, nchan), (nsub, 1)) + 0.125
    wts = np.ones((nsub, nchan), dtype=np.float32)
    wts[1, 3] = 0.0
    return raw, scl, offs, freqs, wts


def test_int16_roundtrip(lib, tmp_path):
    rng = np.random.default_rng(1)
    raw, scl, offs, freqs, wts = _arch(rng)
    path = str(tmp_path / "a.fits")
    write_psrfits(path, raw, scl, offs, freqs, wts, tsubint=[10.0, 10.0, 9.5],
                  offs_sub=[5.0, 15.0, 24.75], period=[0.003, 0.0030001, 0.0030002],
                  par_ang=[10.5, 11.0, 11.5], pol_type="AABBCRCI", dedisp=[0, 1])
    f = lib.PSRFITSFile(path)
    I = f.info
    assert (f.nsub, f.npol, f.nchan, f.nbin) == raw.shape
    assert I.raw_type == 2 and I.has_period and I.has_par_ang and I.dedispersed == 1
    assert f.text("telescope") == "GBT" and f.text("backend") == "GUPPI"
    assert f.text("pol_type") == "AABBCRCI" and f.text("source") == "J1234+5678"
    assert I.stt_imjd == 57300 and I.stt_smjd == 43200 and I.stt_offs == 0.25
    assert I.be_delay == 2e-6 and I.dm == 34.56789 and np.isnan(I.chan_dm)
    m = f.meta()
    np.testing.assert_array_equal(m["freqs"], freqs)
    np.testing.assert_array_equal(m["weights"], wts)
    np.testing.assert_array_equal(m["scl"], scl.astype(np.float64))
    np.testing.assert_array_equal(m["offs"], offs.astype(np.float64))
    np.testing.assert_array_equal(m["period"], [0.003, 0.0030001, 0.0030002])
    np.testing.assert_array_equal(m["par_ang"], np.float32([10.5, 11.0, 11.5]))
    np.testing.assert_array_equal(f.raw(), raw)
    np.testing.assert_array_equal(f.raw(1, 2), raw[1:3])
    assert f.polyco() is None
    with pytest.raises(lib.PSRFITSError):
        f.raw(2, 5)
    f.close()


@pytest.mark.parametrize("dtype", [np.uint8, np.float32])
def test_other_raw_types(lib, tmp_path, dtype):
    rng = np.random.default_rng(2)
    raw = (rng.integers(0, 255, size=(2, 1, 4, 32)) if dtype == np.uint8
           else rng.normal(size=(2, 1, 4, 32))).astype(dtype)
    scl = np.full((2, 1, 4), 0.5, np.float32)
    offs = np.full((2, 1, 4), -1.0, np.float32)
    path = str(tmp_path / "b.fits")
    write_psrfits(path, raw, scl, offs, np.tile([1400.0, 1450, 1500, 1550], (2, 1)),
                  np.ones((2, 4), np.float32), tsubint=[1.0, 1.0], offs_sub=[0.5, 1.5],
                  period=[0.1, 0.1])
    f = lib.PSRFITSFile(path)
    assert f.info.raw_type == {np.uint8: 1, np.float32: 3}[dtype]
    assert not f.info.has_par_ang and f.info.dedispersed == 0
    np.testing.assert_array_equal(f.raw(), raw)
    assert np.all(np.isnan(f.meta()["par_ang"]))


def test_polyco_period(lib, tmp_path):
    rng = np.random.default_rng(3)
    raw, scl, offs, freqs, wts = _arch(rng, nsub=2, npol=1)
    pc = dict(ref_mjd=[57300.49, 57300.51], ref_f0=[345.678901, 345.678902],
              ref_phs=[0.1, 0.2], nspan=[60, 60],
              coeff=[[0.0, 1e-3, 2e-7, 0.0], [0.0, -2e-3, 1e-7, 3e-9]])
    path = str(tmp_path / "c.fits")
    write_psrfits(path, raw, scl, offs, freqs, wts, tsubint=[10.0, 10.0],
                  offs_sub=[5.0, 2000.0], polyco=pc)
    f = lib.PSRFITSFile(path)
    assert not f.info.has_period and f.info.npolyco == 2 and f.info.ncoef == 4
    got = f.polyco()
    for k in ["ref_mjd", "ref_f0", "ref_phs", "nspan", "coeff"]:
        np.testing.assert_array_equal(got[k], np.asarray(pc[k], float))
    mjd = 57300.495
    dt = (mjd - 57300.49) * 1440.0  # nearest row: the first
    f_exp = 345.678901 + (1e-3 + 2 * 2e-7 * dt) / 60.0
    assert lib.polyco_period(got, mjd) == pytest.approx(1.0 / f_exp, rel=1e-15)


def test_bad_files(lib, tmp_path):
    p = tmp_path / "x.fits"
    p.write_bytes(b"not a fits file" * 300)
    with pytest.raises(lib.PSRFITSError):
        lib.PSRFITSFile(str(p))
    with pytest.raises(lib.PSRFITSError):
        lib.PSRFITSFile(str(tmp_path / "missing.fits"))
    # a FITS file without a SUBINT table
    from tests.psrfits_writer import _card, _header
    p2 = tmp_path / "y.fits"
    p2.write_bytes(_header([_card("SIMPLE", True), _card("BITPIX", 8), _card("NAXIS", 0)]))
    with pytest.raises(lib.PSRFITSError, match="SUBINT"):
        lib.PSRFITSFile(str(p2))


def test_pscrunch_mode(lib):
    assert lib.pscrunch_mode(1, "AA+BB") == 0
    assert lib.pscrunch_mode(4, "AABBCRCI") == 1
    assert lib.pscrunch_mode(2, "AABB") == 1
    assert lib.pscrunch_mode(4, "IQUV") == 2
