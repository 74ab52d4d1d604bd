"""Archive access for the drivers (pplib.load_data, pplib.py:2650-2820).

PSRCHIVE is not part of this build.  Archives reach the
drivers as fold-mode PSRFITS files (psrfits.py: the native reader of
include/ppfits.h plus device unpacking, §8(f) next #1), as in-memory
DataBunches with the keys of pplib.py:2809-2819 registered under a name, or
as ``.npz`` archives written by ``save_archive``.  Anything else raises
RuntimeError, which the drivers treat exactly like a failed PSRCHIVE load
(skip the archive, pptoas.py:271).
"""
import os

import numpy as np

from .mjd import MJD
from .pplib import DataBunch, get_bin_centers

_registry = {}

REQUIRED = ["subints", "freqs", "Ps", "epochs"]


def register_archive(name, bunch):
    """Make an in-memory archive loadable under ``name``."""
    _registry[name] = normalize(bunch, name)
    return name


def unregister_archive(name):
    _registry.pop(name, None)


def normalize(b, name="archive"):
    """Fill the load_data keys the drivers use from the minimal set."""
    b = DataBunch(**dict(b))
    subints = np.asarray(b["subints"], dtype=np.float64)
    if subints.ndim == 3:
        subints = subints[:, None]
    nsub, npol, nchan, nbin = subints.shape
    b.subints = subints
    b.setdefault("filename", name)
    b.setdefault("nsub", nsub)
    b.setdefault("npol", npol)
    b.setdefault("nchan", nchan)
    b.setdefault("nbin", nbin)
    freqs = np.asarray(b["freqs"], dtype=np.float64)
    b.freqs = np.tile(freqs, (nsub, 1)) if freqs.ndim == 1 else freqs
    b.Ps = np.asarray(b["Ps"], dtype=np.float64) * np.ones(nsub)
    ep = b["epochs"]
    b.epochs = [e if isinstance(e, MJD) else MJD(*e) if np.ndim(e) else MJD(e) for e in ep]
    w = np.asarray(b.get("weights", np.ones((nsub, nchan))), dtype=np.float64)
    b.weights = w
    wn = np.where(w == 0.0, 0.0, 1.0)
    b.setdefault("ok_isubs", np.compress(wn.mean(axis=1), range(nsub)))
    b.setdefault("ok_ichans", [np.compress(wn[i], range(nchan)) for i in range(nsub)])
    b.setdefault("masks", np.einsum("j,ikl", np.ones(npol), np.einsum("ij,k", wn, np.ones(nbin))))
    b.setdefault("phases", get_bin_centers(nbin))
    b.setdefault("SNRs", np.ones((nsub, npol, nchan)))
    b.setdefault("doppler_factors", np.ones(nsub))
    b.setdefault("parallactic_angles", np.zeros(nsub))
    b.setdefault("DM", 0.0)
    b.setdefault("dmc", 0)
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


def tscrunch(b, period_at=None):
    """arch.tscrunch() as load_data applies it (pplib.py:2700) to a normalised
    archive: one subint whose profiles are the weight-averaged profiles of
    all subints (fold-mode subints share the predictor's phase, so they add
    without rotation), weights summed per channel (ppf_tscrunch, on the
    device).  Epoch: the duration-weighted mean epoch (the middle of the span
    for contiguous equal subints); duration: the sum; period: period_at(epoch
    in days) when the archive has a predictor (PSRFITS POLYCO), else the
    duration-weighted mean; Doppler factor, parallactic angle and SNRs: the
    (duration-weighted) means.  PSRCHIVE recomputes some of these from the
    ephemeris and its own estimators, which this build does not have: parity
    with PSRCHIVE is unpinned."""
    from .engine import get_engine
    b = normalize(b, b.get("filename", "archive"))
    if b.nsub == 1:
        return b
    sub, ws = get_engine().tscrunch(b.subints, b.weights)
    dur = np.asarray(b.subtimes, dtype=np.float64)
    wt = dur / dur.sum() if dur.sum() > 0 else np.full(b.nsub, 1.0 / b.nsub)
    e0 = b.epochs[0]
    offs = np.array([(e.days - e0.days) * 86400.0 + (e.secs - e0.secs) +
                     (e.fracsec - e0.fracsec) for e in b.epochs])
    epoch = e0 + float(np.sum(wt * offs))
    out = DataBunch(**dict(b))
    out.subints = sub.cpu().numpy()
    out.weights = ws.cpu().numpy()
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
    for k in ["ok_isubs", "ok_ichans", "masks"]:
        out.pop(k, None)
    return normalize(out, b.filename)


ARRAY_KEYS = ["subints", "freqs", "weights", "Ps", "SNRs", "doppler_factors",
              "parallactic_angles", "noise_stds", "subtimes"]
SCALAR_KEYS = ["DM", "dmc", "backend", "frontend", "backend_delay", "telescope",
               "telescope_code", "bw", "nu0", "source", "state", "prof_SNR"]


def save_archive(path, bunch):
    """Write a normalised archive as .npz (numbers and strings only)."""
    b = normalize(bunch, os.path.basename(path))
    arrs = {k: np.asarray(b[k]) for k in ARRAY_KEYS if b.get(k) is not None}
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


def load_data(filename, **kw):
    """Archive by name: registered bunch, an .npz written by save_archive, or a
    fold-mode PSRFITS file (psrfits.load_psrfits: host reader + device unpack)."""
    if isinstance(filename, dict):
        return normalize(filename)
    if filename in _registry:
        b = _registry[filename]
        return tscrunch(b) if kw.get("tscrunch") else b
    if isinstance(filename, str) and is_fits(filename):
        from .psrfits import load_psrfits
        return normalize(load_psrfits(filename, pscrunch=kw.get("pscrunch", False),
                                      dededisperse=kw.get("dededisperse", False),
                                      tscrunch=kw.get("tscrunch", False),
                                      quiet=kw.get("quiet", True)), filename)
    if isinstance(filename, str) and os.path.exists(filename) and filename.endswith(".npz"):
        z = np.load(filename, allow_pickle=False)
        b = {k: z[k] for k in z.files if not k.startswith("meta_") and k != "epochs"}
        b["epochs"] = [MJD(int(d), int(s), f) for d, s, f in z["epochs"]]
        for k in z.files:
            if k.startswith("meta_"):
                v = z[k]
                b[k[5:]] = v.item() if v.ndim == 0 else v
        for k in ["dmc"]:
            if k in b:
                b[k] = int(b[k])
        b = normalize(b, filename)
        return tscrunch(b) if kw.get("tscrunch") else b
    raise RuntimeError("Cannot load_data(%s): not a registered, .npz or PSRFITS archive "
                       "(other PSRCHIVE formats need PSRCHIVE)" % filename)


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
