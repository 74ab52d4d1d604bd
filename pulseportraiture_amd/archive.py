"""Archive access for the drivers (pplib.load_data, pplib.py:2650-2820).

PSRCHIVE is not part of this build.  Archives reach the
drivers as fold-mode PSRFITS files (psrfits.py: the native reader of
include/ppfits.h plus device unpacking, §8(f) next #1), as in-memory
DataBunches with the keys of pplib.py:2809-2819 registered under a name, or
as ``.npz`` archives written by ``save_archive``.  Anything else raises
RuntimeError, which the drivers treat exactly like a failed PSRCHIVE load
(skip the archive, pptoas.py:271).

Loading is split in two so a rank reads only the subints it fits
(pptoas.py:246,343 sharded): ``open_archive`` returns the metadata (every
load_data key but ``subints``) and a reader of subint ranges; ``load_data``
is the two together.  The processing load_data asks PSRCHIVE for runs on the
device in the reference's order (pplib.py:2686-2700): ``dedisperse`` /
``dededisperse`` (per-channel rotation by the stored DM about the archive
centre frequency, ppf_rotate_rows), ``rm_baseline`` (ppf_remove_baseline),
then ``tscrunch`` (ppf_tscrunch).  A registered bunch or .npz is a load_data
result: its ``dmc`` says whether it is dedispersed and its baseline counts as
removed unless it says ``baseline_removed=False``.
"""
import os

import numpy as np

from .mjd import MJD, epoch_parts
from .pplib import DataBunch, Dconst, get_bin_centers

_registry = {}

REQUIRED = ["subints", "freqs", "Ps", "epochs"]
DUTY_CYCLE = 0.15  # PSRCHIVE's default baseline duty cycle (Profile::default_duty_cycle)


def _is_tensor(x):
    try:
        import torch
    except ImportError:  # pragma: no cover
        return False
    return isinstance(x, torch.Tensor)


def register_archive(name, bunch):
    """Make an in-memory archive loadable under ``name``.  ``subints`` may be
    a numpy array or a float64 device tensor (kept on the device)."""
    _registry[name] = normalize(bunch, name)
    return name


class _Stack:
    """Archives registered together (register_archives) with one subints
    shape [nsub, npol, nchan, nbin]: their metadata arrays stacked on a
    leading archive axis -- freqs / weights [narch, nsub, nchan], snrs /
    noise (SNRs / noise_stds [narch, nsub, npol, nchan]; noise NaN for the
    archives without, has_noise [narch], None when none has them) and their
    polarisation-0 views snrs0 / noise0, Ps [narch, nsub], DM [narch] --
    each archive's bunch holding views of its own row, and ``rows`` one
    [narch, nsub, npol, nchan, nbin] view of their subints when those are
    equally spaced views of one tensor (else None).  allok: every archive's
    ok_isubs is every subint and every ok_ichans every channel.  names /
    bunches: the archives in registration order; views(): one read-only
    _RegisteredView per archive, made once."""
    _views = None

    def views(self):
        if self._views is None:
            self._views = [_RegisteredView(b) for b in self.bunches]
        return self._views


def _stacked_view(subs):
    """One [narch, *shape] view of equally spaced tensors of one storage with
    the same shape and strides, or None."""
    t0 = subs[0]
    if not _is_tensor(t0) or not t0.is_contiguous():
        return None
    shape, st0 = t0.shape, t0.stride()
    base0 = t0._base
    if base0 is None or not all(_is_tensor(t) and t._base is base0 and t.shape == shape and
                                t.stride() == st0 for t in subs):
        return None
    q = np.fromiter((t.data_ptr() for t in subs), dtype=np.int64, count=len(subs))
    es = t0.element_size()
    d = int(q[1] - q[0]) if len(subs) > 1 else t0.numel() * es
    if d < t0.numel() * es or d % es or (len(subs) > 2 and (np.diff(q) != d).any()):
        return None
    return t0.as_strided((len(subs),) + tuple(shape), (d // es,) + tuple(st0),
                         t0.storage_offset())


def register_archives(names, bunches):
    """register_archive for many archives at once (a driver's whole data set
    kept in memory, e.g. every archive ppalign aligns).  Each archive stays
    loadable under its own name exactly as if registered alone; when they all
    have one subints shape their metadata arrays are also stacked (_Stack), so
    a driver that opens every one of them indexes one array per key instead
    of visiting each archive (ppalign's unit set-up).

    The stacked keys (freqs, weights, Ps, SNRs, noise_stds) of each archive's
    bunch are views of its stack row: change them in place.  Registered
    bunches are otherwise frozen: a key *reassigned* after registration (or
    a new DM) reaches the per-archive path only -- register the archives
    again after such a change."""
    bs = [normalize(b, nm) for nm, b in zip(names, bunches)]
    for nm, b in zip(names, bs):
        _registry[nm] = b
    if len(bs) < 2:
        return list(names)
    shape = tuple(bs[0].subints.shape)
    if any(tuple(b.subints.shape) != shape for b in bs):
        return list(names)
    nsub, npol, nchan, nbin = shape
    stk = _Stack()
    stk.nsub, stk.npol, stk.nchan, stk.nbin = shape
    stk.names, stk.bunches = tuple(names), bs
    try:
        stk.freqs = np.stack([b.freqs for b in bs])
        stk.weights = np.stack([b.weights for b in bs])
        stk.snrs = np.stack([np.asarray(b.SNRs, dtype=np.float64) for b in bs])
        stk.snrs0 = stk.snrs[:, :, 0]
        stk.Ps = np.stack([b.Ps for b in bs])
        stk.DM = np.array([float(b.DM) for b in bs])
        stk.has_noise = np.array([b.noise_stds is not None for b in bs])
        nan = np.full((nsub, npol, nchan), np.nan)
        stk.noise = np.stack([np.asarray(b.noise_stds, dtype=np.float64)
                              if b.noise_stds is not None else nan for b in bs]) \
            if stk.has_noise.any() else None
        stk.noise0 = None if stk.noise is None else stk.noise[:, :, 0]
    except (ValueError, IndexError, TypeError):
        return list(names)
    if stk.freqs.shape != (len(bs), nsub, nchan) or stk.weights.shape != stk.freqs.shape or \
            stk.snrs0.shape != stk.freqs.shape or stk.Ps.shape != (len(bs), nsub) or \
            (stk.noise is not None and stk.noise.shape != stk.snrs.shape):
        return list(names)
    full = np.arange(nsub)
    stk.allok = all(len(b.ok_isubs) == nsub and np.array_equal(b.ok_isubs, full) and
                    all(len(oi) == nchan for oi in b.ok_ichans) for b in bs)
    stk.rows = _stacked_view([b.subints for b in bs])
    for i, b in enumerate(bs):
        # the bunch's own arrays become views of its stack row (equal values),
        # so an in-place change reaches both the per-archive and the stacked
        # paths
        b.freqs, b.weights, b.Ps = stk.freqs[i], stk.weights[i], stk.Ps[i]
        b.SNRs = stk.snrs[i]
        if b.noise_stds is not None:
            b.noise_stds = stk.noise[i]
        b["_stack"] = (stk, i)
    return list(names)


def unregister_archive(name):
    _registry.pop(name, None)


def _ok_ichans(wn):
    """[np.compress(wn[i], range(nchan)) for i] (pplib.py:2757-2758): rows with
    every channel on share one index array."""
    nsub, nchan = wn.shape
    full = np.arange(nchan)
    allok = wn.all(axis=1)
    return [full if a else np.flatnonzero(r) for a, r in zip(allok.tolist(), wn)]


def normalize(b, name="archive", subints=True):
    """Fill the load_data keys the drivers use from the minimal set.

    masks (pplib.py:2759-2761) is a read-only broadcast view of the
    per-channel weight flags, not an [nsub, npol, nchan, nbin] array."""
    b = DataBunch(**dict(b))
    if subints:
        sub = b["subints"]
        if _is_tensor(sub):
            import torch
            sub = sub.to(torch.float64)
            if sub.dim() == 3:
                sub = sub.unsqueeze(1)
            sub = sub.contiguous()
        else:
            sub = np.asarray(sub, dtype=np.float64)
            if sub.ndim == 3:
                sub = sub[:, None]
        b.subints = sub
        nsub, npol, nchan, nbin = tuple(sub.shape)
    else:
        nsub, npol, nchan, nbin = b.nsub, b.npol, b.nchan, b.nbin
    b.setdefault("filename", name)
    b.nsub, b.npol, b.nchan, b.nbin = nsub, npol, nchan, nbin
    freqs = np.asarray(b["freqs"], dtype=np.float64)
    b.freqs = np.tile(freqs, (nsub, 1)) if freqs.ndim == 1 else freqs
    b.Ps = np.asarray(b["Ps"], dtype=np.float64) * np.ones(nsub)
    ep = b["epochs"]
    b.epochs = [e if isinstance(e, MJD) else MJD(*e) if np.ndim(e) else MJD(e) for e in ep]
    b.epoch_parts = epoch_parts(b.epochs)  # (days, secs, fracsec) arrays of the epochs
    w = np.asarray(b.get("weights", np.ones((nsub, nchan))), dtype=np.float64)
    b.weights = w
    wn = w != 0.0
    b.setdefault("ok_isubs", np.flatnonzero(wn.any(axis=1)))
    b.setdefault("ok_ichans", _ok_ichans(wn))
    if "masks" not in b:
        b.masks = np.broadcast_to(wn.astype(np.float64)[:, None, :, None],
                                  (nsub, npol, nchan, nbin))
    b.setdefault("phases", get_bin_centers(nbin))
    b.setdefault("SNRs", np.ones((nsub, npol, nchan)))
    b.setdefault("doppler_factors", np.ones(nsub))
    b.setdefault("parallactic_angles", np.zeros(nsub))
    b.setdefault("DM", 0.0)
    b.setdefault("dmc", 0)
    b.setdefault("baseline_removed", True)
    b.setdefault("backend", "unknown")
    b.setdefault("frontend", "unknown")
    b.setdefault("backend_delay", 0.0)
    b.setdefault("telescope", "unknown")
    b.setdefault("telescope_code", b.get("telescope", "unknown"))
    b.setdefault("bw", float(np.ptp(b.freqs[0]) * nchan / max(nchan - 1, 1)))
    b.setdefault("nu0", float(b.freqs[0].mean()))
    b.setdefault("subtimes", [60.0] * nsub)
    b.setdefault("integration_length", float(np.sum(b.subtimes)))
    b.setdefault("source", "noname")
    b.setdefault("state", "Intensity")
    b.setdefault("prof_SNR", np.inf)
    b.setdefault("arch", None)
    if "noise_stds" not in b:
        b.noise_stds = None  # filled on the GPU by the drivers (use_get_noise)
    return b


# ---------------------------------------------------------------------------
# sources: metadata + a reader of raw subint ranges
# ---------------------------------------------------------------------------
class _Registered:
    owns_reads = False  # read() returns views of the caller's registered array

    def __init__(self, name):
        self.base = _registry[name]

    def meta(self):
        b = DataBunch()
        b.update(self.base)  # shallow copy (C-level), then drop the data
        b.pop("subints", None)
        b.pop("_stack", None)  # register_archives' stack: registered views only
        return b

    def read(self, lo, hi):
        return self.base.subints[lo:hi]

    def close(self):
        pass


def _npy_member(path, member):
    """(dtype, shape, fortran_order, data offset or None) of an .npz member
    from its .npy header alone.  The offset is the member's array data in the
    .npz file itself when the member is stored uncompressed (np.savez), so
    subint ranges can be memory-mapped; None for a compressed member."""
    import zipfile
    with zipfile.ZipFile(path) as zf:
        info = zf.getinfo(member)
        with zf.open(info) as f:
            ver = np.lib.format.read_magic(f)
            rd = np.lib.format.read_array_header_1_0 if ver == (1, 0) else \
                np.lib.format.read_array_header_2_0
            shape, fortran, dtype = rd(f)
            hdr = f.tell()
    off = None
    if info.compress_type == zipfile.ZIP_STORED:
        with open(path, "rb") as raw:
            raw.seek(info.header_offset)
            lh = raw.read(30)  # local file header: name / extra lengths at 26 / 28
            n, m = int.from_bytes(lh[26:28], "little"), int.from_bytes(lh[28:30], "little")
            off = info.header_offset + 30 + n + m + hdr
    return dtype, tuple(shape), fortran, off


class _Npz:
    """An .npz archive (save_archive).  The metadata comes from the small
    members and the subints' .npy header (no DATA read); read(lo, hi) maps
    only rows lo:hi of a stored member (a compressed one is loaded once)."""
    owns_reads = True

    def __init__(self, path):
        self.z = np.load(path, allow_pickle=False)
        self.path = path
        self._full = None

    def meta(self):
        z = self.z
        b = {k: z[k] for k in z.files if k not in ("subints", "epochs") and
             not k.startswith("meta_")}
        b["epochs"] = [MJD(int(d), int(s), f) for d, s, f in z["epochs"]]
        for k in z.files:
            if k.startswith("meta_"):
                v = z[k]
                b[k[5:]] = v.item() if v.ndim == 0 else v
        if "dmc" in b:
            b["dmc"] = int(b["dmc"])
        _, sh, _, _ = _npy_member(self.path, "subints.npy")
        sh = sh if len(sh) == 4 else (sh[0], 1) + tuple(sh[1:])
        b.update(nsub=sh[0], npol=sh[1], nchan=sh[2], nbin=sh[3])
        return normalize(b, self.path, subints=False)

    def read(self, lo, hi):
        dtype, sh, fortran, off = _npy_member(self.path, "subints.npy")
        if off is not None and not fortran:
            mm = np.memmap(self.path, dtype=dtype, mode="r", offset=off, shape=sh)
            s = np.array(mm[lo:hi])  # only these rows are read
            del mm
        else:
            if self._full is None:
                self._full = self.z["subints"]
            s = self._full[lo:hi]
        return s if s.ndim == 4 else s[:, None]

    def close(self):
        self._full = None
        self.z.close()


def _source(filename, pscrunch):
    if filename in _registry:
        return _Registered(filename)
    if isinstance(filename, str) and is_fits(filename):
        from .psrfits import PSRFITSSource
        return PSRFITSSource(filename, pscrunch=pscrunch)
    if isinstance(filename, str) and os.path.exists(filename) and filename.endswith(".npz"):
        return _Npz(filename)
    raise RuntimeError("Cannot load_data(%s): not a registered, .npz or PSRFITS archive "
                       "(other PSRCHIVE formats need PSRCHIVE)" % filename)


def _tscrunch_meta(b, period_at=None):
    """Metadata of arch.tscrunch() (pplib.py:2700): one subint, weights summed
    per channel; epoch the duration-weighted mean epoch (the middle of the
    span for contiguous equal subints); duration the sum; period period_at
    (epoch in days) when the archive has a predictor (PSRFITS POLYCO), else the
    duration-weighted mean; Doppler factor, parallactic angle: the
    (duration-weighted) means; SNRs added in quadrature.  PSRCHIVE recomputes
    some of these from the ephemeris and its own estimators, which this build
    does not have: parity with PSRCHIVE is unpinned."""
    dur = np.asarray(b.subtimes, dtype=np.float64)
    wt = dur / dur.sum() if dur.sum() > 0 else np.full(b.nsub, 1.0 / b.nsub)
    e0 = b.epochs[0]
    offs = np.array([(e.days - e0.days) * 86400.0 + (e.secs - e0.secs) +
                     (e.fracsec - e0.fracsec) for e in b.epochs])
    epoch = e0 + float(np.sum(wt * offs))
    out = DataBunch(**{k: v for k, v in b.items()
                       if k not in ("ok_isubs", "ok_ichans", "masks", "epoch_parts")})
    out.weights = np.asarray(b.weights).sum(axis=0)[None]
    out.nsub = 1
    out.epochs = [epoch]
    out.subtimes = [float(dur.sum())]
    out.Ps = np.array([period_at(epoch.in_days()) if period_at is not None
                       else float(np.sum(wt * b.Ps))])
    out.freqs = b.freqs[:1]
    out.doppler_factors = np.array([float(np.sum(wt * np.asarray(b.doppler_factors)))])
    out.parallactic_angles = np.array([float(np.sum(wt * np.asarray(b.parallactic_angles)))])
    out.SNRs = np.sqrt(np.sum(np.asarray(b.SNRs) ** 2, axis=0))[None]
    out.noise_stds = None  # re-estimated from the averaged profiles (use_get_noise)
    return normalize(out, b.filename, subints=False)


def dedispersion_phases(freqs, Ps, DM, nu_ref):
    """Per-(subint, channel) rotation [rot] of arch.dedisperse() about nu_ref:
    rotate_data(port, 0.0, DM, P, freqs, nu_ref) (pplib.py:2338-2426, the
    reference's own convention: positive DM moves freqs < nu_ref earlier).
    PSRCHIVE's dispersion constant is the reference's Dconst = 1/2.41e-4."""
    f = np.asarray(freqs, dtype=np.float64)
    return Dconst * DM * (f ** -2.0 - nu_ref ** -2.0) / np.asarray(Ps, dtype=np.float64)[:, None]


class Archive:
    """An opened archive: ``meta`` holds every load_data key but ``subints``
    (after the requested processing); ``read(lo, hi)`` returns processed
    subints [hi - lo, npol, nchan, nbin] -- a numpy array when nothing had to
    run on the device, else a float64 device tensor.

    An Archive holds no open file: the source is opened for the metadata
    and closed again, and every read() reopens it for just that range, so a
    driver may keep one Archive per datafile for any number of datafiles."""

    def __init__(self, filename, dedisperse=False, dededisperse=False, tscrunch=False,
                 pscrunch=False, rm_baseline=True, quiet=True):
        self._src_args = (filename, pscrunch)
        src = _source(filename, pscrunch)
        try:
            raw = src.meta()
            period_at = getattr(src, "period_at", None)
            self.eager_noise = bool(getattr(src, "eager_noise", False))
            self.owns_reads = bool(getattr(src, "owns_reads", True))
        finally:
            src.close()
        # a registered source holds no file: keep it for the reads
        self._reg = src if isinstance(src, _Registered) else None
        if not isinstance(filename, str):
            filename = raw.get("filename", "archive")
        raw.setdefault("filename", filename)
        self.raw = raw
        dmc = int(raw.get("dmc", 0))
        self.rot_sign = 0.0
        if dedisperse and not dmc:  # arch.dedisperse() (pplib.py:2686)
            self.rot_sign, dmc = 1.0, 1
        elif dededisperse and dmc:  # arch.dededisperse() (pplib.py:2687)
            self.rot_sign, dmc = -1.0, 0
        self.rm_base = bool(rm_baseline) and not raw.get("baseline_removed", True)
        self.tscrunch = bool(tscrunch) and raw.nsub > 1
        m = DataBunch()
        m.update(raw)
        m.dmc = dmc
        m.baseline_removed = bool(raw.get("baseline_removed", True) or rm_baseline)
        if self.tscrunch:
            m = _tscrunch_meta(m, period_at)
        self.meta = m
        if not quiet:
            print("\nReading data from %s on source %s..." % (filename, m.get("source", "")))

    @property
    def nsub(self):
        return self.meta.nsub

    def _read_src(self, lo, hi):
        if self._reg is not None:
            return self._reg.read(lo, hi)
        src = _source(*self._src_args)
        try:
            return src.read(lo, hi)
        finally:
            src.close()

    def _process(self, sub, lo, hi):
        """dedisperse / dededisperse, then remove_baseline, on subints lo:hi."""
        if not self.rot_sign and not self.rm_base:
            return sub
        import torch
        from .engine import get_engine
        eng = get_engine()
        r = self.raw
        if _is_tensor(sub) and sub.device == eng.device:
            d = sub.to(torch.float64).contiguous()
            if not self.owns_reads and d.data_ptr() == sub.data_ptr():
                d = d.clone()  # never modify a caller's registered tensor
        else:
            d = torch.as_tensor(np.ascontiguousarray(sub, dtype=np.float64), device=eng.device)
        n, npol, nchan, nbin = d.shape
        if self.rot_sign:
            ph = self.rot_sign * dedispersion_phases(r.freqs[lo:hi], r.Ps[lo:hi], r.DM, r.nu0)
            eng.rotate_rows(d, np.repeat(ph[:, None, :], npol, axis=1), inplace=True)
        if self.rm_base:
            ntot = 2 if (npol >= 2 and str(r.get("state", "")).upper().startswith("COH")) else 1
            eng.remove_baseline(d, r.weights[lo:hi], ntot=ntot, duty=DUTY_CYCLE)
        return d

    @staticmethod
    def snrs(sub):
        """load_data's SNRs of processed subints [n, npol, nchan, nbin]
        (Profile::snr() per profile, pplib.py:2762-2770; ppf_profile_snr,
        PSRCHIVE's default estimator restated, parity unpinned) as numpy
        [n, npol, nchan].  Sources with snr_deferred metadata (PSRFITS) fill
        SNRs this way from the data they read."""
        from .engine import get_engine
        return get_engine().profile_snr(sub).cpu().numpy()

    def registered_rows(self):
        """The registered subints tensor itself (every subint, nothing to
        process), or None: a reader of a few rows of it can index it directly
        instead of slicing read(lo, hi)."""
        if self._reg is None or self.tscrunch or self.rot_sign or self.rm_base:
            return None
        sub = self._reg.base.subints
        return sub if _is_tensor(sub) else None

    def read(self, lo=0, hi=None):
        if self.tscrunch:  # the one averaged subint needs every raw subint
            from .engine import get_engine
            r = self.raw
            sub = self._process(self._read_src(0, r.nsub), 0, r.nsub)
            out, _ = get_engine().tscrunch(sub, r.weights)
            return out
        hi = self.meta.nsub if hi is None else hi
        return self._process(self._read_src(lo, hi), lo, hi)


class _RegisteredView:
    """A registered archive opened for reading only, when the request has
    nothing to process (Archive would copy its metadata unchanged): the
    metadata IS the registered bunch (callers must not modify it), reads are
    views of its subints.  Used by drivers that open many archives at once
    (ppalign) to skip the per-archive copies."""
    owns_reads = False
    eager_noise = False
    tscrunch = False
    rot_sign = 0.0
    rm_base = False
    snrs = staticmethod(Archive.snrs)

    def __init__(self, base):
        self.meta = self.raw = base

    @property
    def nsub(self):
        return self.meta.nsub

    def registered_rows(self):
        sub = self.meta.subints
        return sub if _is_tensor(sub) else None

    def read(self, lo=0, hi=None):
        return self.meta.subints[lo:(self.meta.nsub if hi is None else hi)]


def registered_view(filename, dedisperse=False, dededisperse=False, tscrunch=False,
                    rm_baseline=True):
    """A read-only _RegisteredView of a registered archive when opening it
    with these options would process nothing, else None (use open_archive)."""
    b = _registry.get(filename) if isinstance(filename, str) else None
    if b is None:
        return None
    if dedisperse or dededisperse:  # would arch.dedisperse() / dededisperse() rotate?
        dmc = int(b.get("dmc", 0))
        if (dedisperse and not dmc) or (dededisperse and dmc):
            return None
    if (tscrunch and b.nsub > 1) or (rm_baseline and not b.get("baseline_removed", True)):
        return None
    return _RegisteredView(b)


def open_archive(filename, dedisperse=False, dededisperse=False, tscrunch=False, pscrunch=False,
                 rm_baseline=True, quiet=True):
    """Metadata now, subints on demand (see Archive)."""
    return Archive(filename, dedisperse=dedisperse, dededisperse=dededisperse,
                   tscrunch=tscrunch, pscrunch=pscrunch, rm_baseline=rm_baseline, quiet=quiet)


def host_array(x):
    """numpy view/copy of subints that may live on the device."""
    if _is_tensor(x):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def load_data(filename, state=None, dedisperse=False, dededisperse=False, tscrunch=False,
              pscrunch=False, fscrunch=False, rm_baseline=True, flux_prof=False,
              refresh_arch=True, return_arch=True, quiet=False, get_SNRs=True, host=True):
    """pplib.load_data (pplib.py:2650-2820) for a registered bunch, an .npz or
    a fold-mode PSRFITS file.  host=False leaves device-resident subints on the
    device.  noise_stds is get_noise_PS per profile (pplib.py:2740-2748), on the
    device, unless the archive already holds it."""
    if isinstance(filename, dict):
        return normalize(filename)
    if fscrunch:
        raise NotImplementedError("load_data(fscrunch=True) is not on the fitting path")
    a = open_archive(filename, dedisperse=dedisperse, dededisperse=dededisperse,
                     tscrunch=tscrunch, pscrunch=pscrunch, rm_baseline=rm_baseline, quiet=quiet)
    b = DataBunch(**dict(a.meta))
    sub = a.read()
    if b.get("noise_stds") is None and a.eager_noise:
        from .engine import get_engine
        n, npol, nchan, nbin = tuple(sub.shape)
        b.noise_stds = get_engine().noise_rows(sub.reshape(-1, nbin)).reshape(
            n, npol, nchan).cpu().numpy()
    if b.get("snr_deferred"):
        if get_SNRs:
            b.SNRs = a.snrs(sub)
        else:
            b.SNRs = np.zeros_like(np.asarray(b.SNRs))  # pplib.py:2762 (get_SNRs=False)
        b.snr_deferred = False
    b.subints = host_array(sub) if host else sub
    for k in ("ok_isubs", "ok_ichans", "masks"):
        b.pop(k, None)
    return normalize(b, b.get("filename", filename))


def tscrunch(b, period_at=None):
    """load_data(tscrunch=True) of an already loaded bunch (ppf_tscrunch)."""
    from .engine import get_engine
    b = normalize(b, b.get("filename", "archive"))
    if b.nsub == 1:
        return b
    m = _tscrunch_meta(b, period_at)
    sub, _ = get_engine().tscrunch(b.subints, b.weights)
    out = DataBunch(**dict(m))
    out.subints = sub.cpu().numpy()
    for k in ("ok_isubs", "ok_ichans", "masks"):
        out.pop(k, None)
    return normalize(out, b.filename)


ARRAY_KEYS = ["subints", "freqs", "weights", "Ps", "SNRs", "doppler_factors",
              "parallactic_angles", "noise_stds", "subtimes"]
SCALAR_KEYS = ["DM", "dmc", "backend", "frontend", "backend_delay", "telescope",
               "telescope_code", "bw", "nu0", "source", "state", "prof_SNR"]


def save_archive(path, bunch):
    """Write a normalised archive as .npz (numbers and strings only)."""
    b = normalize(bunch, os.path.basename(path))
    arrs = {k: host_array(b[k]) for k in ARRAY_KEYS if b.get(k) is not None}
    arrs["epochs"] = np.array([e.as_tuple() for e in b.epochs], dtype=np.float64)
    for k in SCALAR_KEYS:
        arrs["meta_" + k] = np.asarray(b[k])
    np.savez(path, **arrs)
    return path


def is_fits(filename):
    """A FITS file on disk (the 'SIMPLE  =' card that opens every FITS file)."""
    try:
        with open(filename, "rb") as f:
            return f.read(9) == b"SIMPLE  ="
    except (OSError, TypeError):
        return False


def file_is_type(filename, filetype="ASCII"):
    """Stand-in for pplib.file_is_type (pplib.py:3021-3037) without `file -L`."""
    if filetype == "ASCII":
        if not isinstance(filename, str) or filename in _registry or \
                not os.path.isfile(filename) or filename.endswith(".npz") or is_fits(filename):
            return False
        try:
            with open(filename) as f:
                f.read(4096)
            return True
        except (UnicodeDecodeError, OSError):
            return False
    if filetype == "FITS":
        return isinstance(filename, str) and (filename in _registry or filename.endswith(".npz")
                                              or is_fits(filename))
    return False
