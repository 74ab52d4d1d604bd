"""PSRFITS archives for load_data.

``PSRFITSSource`` is the archive.Archive source for a fold-mode PSRFITS
file: the host reader ``libppfits.so`` (include/ppfits.h, plain C++) parses
the headers and tables and returns the raw DATA column of any subint range;
the GPU turns the 8/16-bit samples into physical values and sums the
polarisations (``ppf_unpack_subints``).  load_data's processing
(dedisperse / dededisperse, remove_baseline, tscrunch) then runs on the device
in archive.py, and the per-channel noise is get_noise_PS on the device, as
load_data's ``noise_stds`` (pplib.py:2740-2748).

What PSRCHIVE computes from resources this build does not have is set as
follows, and documented in DESIGN.md: Doppler factors 1 (PSRCHIVE derives
them from the ephemeris and observatory), channel S/N 1 (Profile.snr()
weights only guess_fit_freq's reference frequency).  The folding period is
the SUBINT PERIOD column when present, else the POLYCO predictor's frequency
at the subint epoch; the DEDISP flag of the last HISTORY row is ``dmc``.
"""
import ctypes
import os

import numpy as np

from .mjd import MJD

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libppfits.so")

RAW_DTYPE = {1: np.uint8, 2: np.int16, 3: np.float32}

# tempo2 observatory short codes for the telescopes PSRFITS headers name
# (load_data's telescope_code, pplib.py:2675-2677; TEMPO2's observatories.dat
# when $TEMPO2 is set)
TELESCOPE_CODES = {"ARECIBO": "ao", "AO": "ao", "GBT": "gb", "GREENBANK": "gb",
                   "PARKES": "pks", "PKS": "pks", "JODRELL": "jb", "JB": "jb",
                   "LOVELL": "jb", "EFFELSBERG": "eff", "EFF": "eff", "NANCAY": "ncy",
                   "NCY": "ncy", "NUPPI": "ncy", "WSRT": "wsrt", "GMRT": "gmrt",
                   "VLA": "vla", "LOFAR": "lofar", "MEERKAT": "meerkat", "FAST": "fast",
                   "CHIME": "chime", "SRT": "srt", "LWA1": "lwa1", "MWA": "mwa"}


class PSRFITSError(RuntimeError):
    """Unreadable archive: load_data's callers skip it like a failed Archive_load."""


class _Info(ctypes.Structure):
    _fields_ = [("nsub", ctypes.c_int32), ("npol", ctypes.c_int32), ("nchan", ctypes.c_int32),
                ("nbin", ctypes.c_int32), ("raw_type", ctypes.c_int32),
                ("has_period", ctypes.c_int32), ("has_par_ang", ctypes.c_int32),
                ("npolyco", ctypes.c_int32), ("ncoef", ctypes.c_int32),
                ("dedispersed", ctypes.c_int32), ("stt_imjd", ctypes.c_int32),
                ("stt_smjd", ctypes.c_double), ("stt_offs", ctypes.c_double),
                ("obsfreq", ctypes.c_double), ("obsbw", ctypes.c_double),
                ("chan_dm", ctypes.c_double), ("dm", ctypes.c_double),
                ("be_delay", ctypes.c_double), ("chan_bw", ctypes.c_double),
                ("telescope", ctypes.c_char * 32), ("frontend", ctypes.c_char * 32),
                ("backend", ctypes.c_char * 32), ("source", ctypes.c_char * 32),
                ("pol_type", ctypes.c_char * 16), ("obs_mode", ctypes.c_char * 16)]


_lib = None


def load_library():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libppfits.so not found at %s: build it with "
                           "`python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    vp, dp = ctypes.c_void_p, ctypes.c_void_p
    lib.ppfits_open.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp)]
    lib.ppfits_open.restype = ctypes.c_int
    lib.ppfits_close.argtypes = [vp]
    lib.ppfits_close.restype = None
    lib.ppfits_error.argtypes = [vp]
    lib.ppfits_error.restype = ctypes.c_char_p
    lib.ppfits_get_info.argtypes = [vp, ctypes.POINTER(_Info)]
    lib.ppfits_get_info.restype = ctypes.c_int
    lib.ppfits_read_meta.argtypes = [vp] + [dp] * 8
    lib.ppfits_read_meta.restype = ctypes.c_int
    lib.ppfits_read_raw.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, dp]
    lib.ppfits_read_raw.restype = ctypes.c_int
    lib.ppfits_read_polyco.argtypes = [vp] + [dp] * 5
    lib.ppfits_read_polyco.restype = ctypes.c_int
    _lib = lib
    return lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class PSRFITSFile:
    """An open PSRFITS archive (host side: headers, tables, raw samples)."""

    def __init__(self, path):
        self.lib = load_library()
        self.path = path
        self.h = ctypes.c_void_p()
        rc = self.lib.ppfits_open(path.encode(), ctypes.byref(self.h))
        if rc != 0:
            msg = self.lib.ppfits_error(self.h).decode() if self.h else "open failed"
            self.close()
            raise PSRFITSError("%s: %s" % (path, msg))
        info = _Info()
        self._chk(self.lib.ppfits_get_info(self.h, ctypes.byref(info)))
        self.info = info
        self.nsub, self.npol, self.nchan, self.nbin = info.nsub, info.npol, info.nchan, info.nbin

    def _chk(self, rc):
        if rc != 0:
            raise PSRFITSError("%s: %s" % (self.path, self.lib.ppfits_error(self.h).decode()))

    def text(self, name):
        return getattr(self.info, name).decode(errors="replace")

    def meta(self):
        n, c, p = self.nsub, self.nchan, self.npol
        out = dict(freqs=np.empty((n, c)), weights=np.empty((n, c)), offs=np.empty((n, p, c)),
                   scl=np.empty((n, p, c)), tsubint=np.empty(n), offs_sub=np.empty(n),
                   period=np.empty(n), par_ang=np.empty(n))
        self._chk(self.lib.ppfits_read_meta(self.h, *[_p(out[k]) for k in
                                                      ["freqs", "weights", "offs", "scl",
                                                       "tsubint", "offs_sub", "period",
                                                       "par_ang"]]))
        return out

    def raw(self, isub0=0, n=None):
        n = self.nsub - isub0 if n is None else n
        out = np.empty((n, self.npol, self.nchan, self.nbin), dtype=RAW_DTYPE[self.info.raw_type])
        self._chk(self.lib.ppfits_read_raw(self.h, int(isub0), int(n), _p(out)))
        return out

    def polyco(self):
        k, nc = self.info.npolyco, self.info.ncoef
        if not k:
            return None
        out = dict(ref_mjd=np.empty(k), ref_f0=np.empty(k), ref_phs=np.empty(k),
                   nspan=np.empty(k), coeff=np.empty((k, nc)))
        self._chk(self.lib.ppfits_read_polyco(self.h, *[_p(out[x]) for x in
                                                        ["ref_mjd", "ref_f0", "ref_phs",
                                                         "nspan", "coeff"]]))
        return out

    def close(self):
        if getattr(self, "h", None):
            self.lib.ppfits_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def polyco_period(pc, mjd):
    """Folding period [s] at mjd from tempo polycos: the row whose REF_MJD is
    nearest, f = REF_F0 + (1/60) sum_i i c_i dt^(i-1), dt = 1440 (mjd -
    REF_MJD) minutes (tempo's polyco definition)."""
    i = int(np.argmin(np.abs(pc["ref_mjd"] - mjd)))
    dt = (mjd - pc["ref_mjd"][i]) * 1440.0
    c = pc["coeff"][i]
    df = sum(j * c[j] * dt ** (j - 1) for j in range(1, len(c)))
    return 1.0 / (pc["ref_f0"][i] + df / 60.0)


def pscrunch_mode(npol, pol_type):
    """ppf_unpack_subints pmode of pscrunch for a PSRFITS POL_TYPE: coherence
    (AABBCRCI) and 2-pol (AABB) sum AA + BB; Stokes (IQUV) keep I."""
    if npol == 1:
        return 0
    pt = pol_type.upper()
    if pt.startswith("IQUV") or pt == "STOKE":
        return 2
    return 1


class PSRFITSSource:
    """A fold-mode PSRFITS archive as an archive.Archive source: the metadata
    load_data returns (pplib.py:2670-2735, 2809-2819) without touching DATA,
    and ``read(lo, hi)`` = subints lo:hi, raw samples read on the host
    (ppfits_read_raw) and unpacked + pscrunched on the device
    (ppf_unpack_subints) -- only the 8/16-bit samples cross PCIe."""
    eager_noise = True  # load_data computes noise_stds (pplib.py:2740-2748)
    owns_reads = True   # read() returns a fresh device tensor

    def __init__(self, path, pscrunch=True):
        self.f = PSRFITSFile(path)
        f, I = self.f, self.f.info
        if f.nsub == 0:
            f.close()
            raise PSRFITSError("%s: no subintegrations" % path)
        self.path = path
        self.m = f.meta()
        self.pc = f.polyco() if not I.has_period else None
        self.pmode = pscrunch_mode(f.npol, f.text("pol_type")) if pscrunch else 0
        self.npo = 1 if self.pmode else f.npol
        self.period_at = None if self.pc is None else (lambda mjd: polyco_period(self.pc, mjd))

    def meta(self):
        from .archive import normalize
        f, I, m = self.f, self.f.info, self.m
        nsub = f.nsub
        # epochs: STT_IMJD + (STT_SMJD + STT_OFFS + OFFS_SUB) / 86400
        start = MJD(I.stt_imjd, int(I.stt_smjd), float(I.stt_offs) + (I.stt_smjd - int(I.stt_smjd)))
        epochs = [start + float(m["offs_sub"][i]) for i in range(nsub)]
        if I.has_period:
            Ps = m["period"].copy()
        elif self.pc is not None:
            Ps = np.array([polyco_period(self.pc, e.in_days()) for e in epochs])
        else:
            raise PSRFITSError("%s: no PERIOD column and no POLYCO table" % self.path)
        tel = f.text("telescope")
        DM = I.dm if np.isfinite(I.dm) else (I.chan_dm if np.isfinite(I.chan_dm) else 0.0)
        par = m["par_ang"] if I.has_par_ang else np.zeros(nsub)
        state = "Intensity" if (self.pmode or f.npol == 1) else f.text("pol_type")
        b = dict(nsub=nsub, npol=self.npo, nchan=f.nchan, nbin=f.nbin, freqs=m["freqs"],
                 weights=m["weights"], Ps=Ps, epochs=epochs, noise_stds=None,
                 SNRs=np.ones((nsub, self.npo, f.nchan)), snr_deferred=True,
                 doppler_factors=np.ones(nsub),
                 parallactic_angles=np.asarray(par, float), DM=float(DM),
                 dmc=int(I.dedispersed), baseline_removed=False, backend=f.text("backend"),
                 frontend=f.text("frontend"), backend_delay=float(I.be_delay), telescope=tel,
                 telescope_code=TELESCOPE_CODES.get(tel.upper(), tel), bw=float(I.obsbw),
                 nu0=float(I.obsfreq), subtimes=list(m["tsubint"]),
                 source=f.text("source") or "noname", state=state, filename=self.path)
        return normalize(b, self.path, subints=False)

    def read(self, lo, hi, engine=None):
        from .engine import get_engine
        import torch
        f, I = self.f, self.f.info
        n = hi - lo
        raw = f.raw(lo, n)
        eng = engine or get_engine()
        dev = eng.device
        rd = torch.from_numpy(raw).to(dev)
        scl = torch.from_numpy(np.ascontiguousarray(self.m["scl"][lo:hi])).to(dev)
        offs = torch.from_numpy(np.ascontiguousarray(self.m["offs"][lo:hi])).to(dev)
        sub = torch.empty((n, self.npo, f.nchan, f.nbin), dtype=torch.float64, device=dev)
        eng._chk(eng.lib.ppf_unpack_subints(eng.ctx, n, f.npol, f.nchan, f.nbin, I.raw_type,
                                            ctypes.c_void_p(rd.data_ptr()),
                                            ctypes.c_void_p(scl.data_ptr()),
                                            ctypes.c_void_p(offs.data_ptr()), self.pmode,
                                            ctypes.c_void_p(sub.data_ptr())))
        sub._keep = (rd, scl, offs)
        return sub

    def close(self):
        self.f.close()


def load_psrfits(path, pscrunch=True, dedisperse=False, dededisperse=False, tscrunch=False,
                 rm_baseline=False, quiet=True):
    """pplib.load_data (pplib.py:2650-2820) for a fold-mode PSRFITS archive."""
    from .archive import load_data
    return load_data(path, pscrunch=pscrunch, dedisperse=dedisperse, dededisperse=dededisperse,
                     tscrunch=tscrunch, rm_baseline=rm_baseline, quiet=quiet)
