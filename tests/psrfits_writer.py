"""A minimal fold-mode PSRFITS writer for the loader tests (numpy only).

Writes what a PSRCHIVE-written archive holds for load_data: the primary
header (TELESCOP, FRONTEND, BACKEND, SRC_NAME, STT_*, OBSFREQ, OBSBW,
CHAN_DM, BE_DELAY), the SUBINT binary table (TSUBINT, OFFS_SUB, PERIOD or
not, PAR_ANG, DAT_FREQ, DAT_WTS, DAT_OFFS, DAT_SCL, DATA with TDIM
(NBIN,NCHAN,NPOL), big-endian) and optionally POLYCO and HISTORY tables.
Test infrastructure: the loader under test is include/ppfits.h.
"""
import numpy as np

BLOCK = 2880


def _card(key, value=None, comment=""):
    if value is None:
        s = key.ljust(80)
    else:
        if isinstance(value, bool):
            v = ("T" if value else "F").rjust(20)
        elif isinstance(value, str):
            v = ("'" + value.replace("'", "''").ljust(8) + "'").ljust(20)
        elif isinstance(value, (int, np.integer)):
            v = str(int(value)).rjust(20)
        else:
            v = "%.17G" % float(value)
            if "E" not in v and "." not in v:
                v += ".0"
            if key == "BE_DELAY":  # Fortran-style exponent, as some writers emit
                v = v.replace("E", "D")
            v = v.rjust(20)
        s = (key.ljust(8) + "= " + v + (" / " + comment if comment else "")).ljust(80)
    assert len(s) == 80, s
    return s


def _header(cards):
    txt = "".join(cards) + "END".ljust(80)
    pad = (-len(txt)) % BLOCK
    return (txt + " " * pad).encode("ascii")


def _pad(b):
    return b + b"\0" * ((-len(b)) % BLOCK)


FORM = {np.dtype(">u1"): "B", np.dtype(">i2"): "I", np.dtype(">i4"): "J",
        np.dtype(">f4"): "E", np.dtype(">f8"): "D", np.dtype("S1"): "A"}


def _bintable(extname, columns, extra_cards=(), tdims=None):
    """columns: list of (name, big-endian dtype, per-row shape, values [nrow, ...])."""
    nrow = len(columns[0][3])
    fields = [(name, dt, shape) for name, dt, shape, _ in columns]
    rec = np.zeros(nrow, dtype=[(n, d, s) if s else (n, d) for n, d, s in fields])
    for name, dt, shape, vals in columns:
        rec[name] = np.asarray(vals).reshape((nrow,) + tuple(shape))
    cards = [_card("XTENSION", "BINTABLE"), _card("BITPIX", 8), _card("NAXIS", 2),
             _card("NAXIS1", rec.dtype.itemsize), _card("NAXIS2", nrow), _card("PCOUNT", 0),
             _card("GCOUNT", 1), _card("TFIELDS", len(columns))]
    for i, (name, dt, shape, _) in enumerate(columns, 1):
        rep = int(np.prod(shape)) if shape else 1
        cards.append(_card("TTYPE%d" % i, name))
        cards.append(_card("TFORM%d" % i, "%d%s" % (rep, FORM[np.dtype(dt)])))
        if tdims and name in tdims:
            cards.append(_card("TDIM%d" % i, tdims[name]))
    cards.append(_card("EXTNAME", extname))
    cards.extend(extra_cards)
    return _header(cards) + _pad(rec.tobytes())


def write_psrfits(path, raw, scl, offs, freqs, wts, *, tsubint, offs_sub, period=None,
                  par_ang=None, pol_type="AA+BB", telescope="GBT", frontend="Rcvr1_2",
                  backend="GUPPI", source="J1234+5678", stt_imjd=57300, stt_smjd=43200,
                  stt_offs=0.25, obsfreq=1500.0, obsbw=800.0, dm=34.56789, chan_dm=None,
                  be_delay=2e-6, polyco=None, dedisp=None):
    """raw [nsub][npol][nchan][nbin] (uint8 / int16 / float32), scl/offs
    [nsub][npol][nchan], freqs/wts [nsub][nchan]; polyco: dict of ref_mjd,
    ref_f0, ref_phs, nspan, coeff [k][ncoef]; dedisp: HISTORY DEDISP values."""
    raw = np.asarray(raw)
    nsub, npol, nchan, nbin = raw.shape
    big = {np.dtype(np.uint8): ">u1", np.dtype(np.int16): ">i2",
           np.dtype(np.float32): ">f4"}[raw.dtype]
    prim = [_card("SIMPLE", True), _card("BITPIX", 8), _card("NAXIS", 0),
            _card("EXTEND", True), _card("FITSTYPE", "PSRFITS"), _card("OBS_MODE", "PSR"),
            _card("TELESCOP", telescope), _card("FRONTEND", frontend), _card("BACKEND", backend),
            _card("SRC_NAME", source), _card("OBSFREQ", obsfreq), _card("OBSBW", obsbw),
            _card("OBSNCHAN", nchan), _card("STT_IMJD", stt_imjd), _card("STT_SMJD", stt_smjd),
            _card("STT_OFFS", stt_offs), _card("BE_DELAY", be_delay)]
    if chan_dm is not None:
        prim.append(_card("CHAN_DM", chan_dm))
    out = _header(prim)
    cols = [("TSUBINT", ">f8", (), tsubint), ("OFFS_SUB", ">f8", (), offs_sub)]
    if period is not None:
        cols.append(("PERIOD", ">f8", (), period))
    if par_ang is not None:
        cols.append(("PAR_ANG", ">f4", (), par_ang))
    cols += [("DAT_FREQ", ">f8", (nchan,), freqs), ("DAT_WTS", ">f4", (nchan,), wts),
             ("DAT_OFFS", ">f4", (npol * nchan,), np.asarray(offs).reshape(nsub, -1)),
             ("DAT_SCL", ">f4", (npol * nchan,), np.asarray(scl).reshape(nsub, -1)),
             ("DATA", big, (npol * nchan * nbin,), raw.reshape(nsub, -1))]
    extra = [_card("NPOL", npol), _card("POL_TYPE", pol_type), _card("NBIN", nbin),
             _card("NCHAN", nchan), _card("CHAN_BW", obsbw / nchan), _card("DM", dm),
             _card("NSBLK", 1)]
    out += _bintable("SUBINT", cols, extra, tdims={"DATA": "(%d,%d,%d)" % (nbin, nchan, npol)})
    if polyco is not None:
        k = len(polyco["ref_mjd"])
        nc = np.asarray(polyco["coeff"]).shape[1]
        out += _bintable("POLYCO", [("NSPAN", ">i2", (), polyco["nspan"]),
                                    ("NCOEF", ">i2", (), [nc] * k),
                                    ("REF_MJD", ">f8", (), polyco["ref_mjd"]),
                                    ("REF_PHS", ">f8", (), polyco["ref_phs"]),
                                    ("REF_F0", ">f8", (), polyco["ref_f0"]),
                                    ("COEFF", ">f8", (nc,), polyco["coeff"])])
    if dedisp is not None:
        out += _bintable("HISTORY", [("NSUB", ">i4", (), [nsub] * len(dedisp)),
                                     ("DEDISP", ">i2", (), dedisp)])
    with open(path, "wb") as fh:
        fh.write(out)
    return path


def quantize(data, nbits=16):
    """int16 samples plus per-(subint, pol, chan) scale/offset, as PSRCHIVE
    writes them: offs = mean, scl = max|x - offs| / 32767 (float32)."""
    data = np.asarray(data, dtype=np.float64)
    offs = data.mean(axis=-1).astype(np.float32)
    span = np.abs(data - offs[..., None].astype(np.float64)).max(axis=-1)
    scl = (np.where(span > 0, span, 1.0) / 32767.0).astype(np.float32)
    raw = np.rint((data - offs[..., None]) / scl[..., None].astype(np.float64)).astype(np.int16)
    return raw, scl, offs
