"""pplib drop-in: constants, templates, TOA output and the GPU-backed utilities.

Hot-path numerics (rfft/irfft, noise, rotation, FFTFIT search, portrait fits)
run in libppfit.so via ``engine``; this module keeps the reference's call
signatures (pplib.py) and its host-side producers/consumers:
Gaussian-component templates (read_model / gen_gaussian_portrait,
pplib.py:752-1046, 2834-2959) and the .tim writer (pplib.py:3386-3509).
"""
import pickle
import sys
import time

import numpy as np

# pplib.py:44-119 --------------------------------------------------------------
Dconst_exact = 4.148808e3
Dconst_trad = 0.000241 ** -1
Dconst = Dconst_trad
scattering_alpha = -4.0
use_get_noise = True
default_noise_method = "PS"
F0_fact = 0
wid_max = 0.25
default_model = "000"
binshift = 1.0
RCSTRINGS = {"-1": "INFEASIBLE: Infeasible (low > up).",
             "0": "LOCALMINIMUM: Local minima reach (|pg| ~= 0).",
             "1": "FCONVERGED: Converged (|f_n-f_(n-1)| ~= 0.)",
             "2": "XCONVERGED: Converged (|x_n-x_(n-1)| ~= 0.)",
             "3": "MAXFUN: Max. number of function evaluations reach.",
             "4": "LSFAIL: Linear search failed.",
             "5": "CONSTANT: All lower bounds are equal to the upper bounds.",
             "6": "NOPROGRESS: Unable to progress.",
             "7": "USERABORT: User requested end of minimization."}


class DataBunch(dict):
    """dict with attribute access (pplib.py:125-136)."""

    def __init__(self, **kwds):
        dict.__init__(self, kwds)
        self.__dict__ = self


def _engine():
    from .engine import get_engine
    return get_engine()


# ---------------------------------------------------------------------------
# Gaussian-component templates (host-side input producer)
# ---------------------------------------------------------------------------
def get_bin_centers(nbin, lo=0.0, hi=1.0):
    """pplib.py:671-684."""
    lo, hi = np.double(lo), np.double(hi)
    d = hi - lo
    return np.double(np.linspace(lo + d / (nbin * 2), hi - d / (nbin * 2), nbin))


def gaussian_profile(nbin, loc, wid, norm=False, abs_wid=False, zeroout=True):
    """Peak-1 Gaussian on bin centres, pplib.py:770-825."""
    if abs_wid:
        wid = abs(wid)
    if not wid > 0.0:
        if wid == 0.0 or (wid < 0.0 and zeroout):
            return np.zeros(nbin, "d")
        if not wid < 0.0:
            return 0
    sigma = wid / (2 * np.sqrt(2 * np.log(2)))
    mean = loc % 1.0
    x = get_bin_centers(nbin)
    if mean < 0.5:
        x = np.where(x > mean + 0.5, x - 1.0, x)
    else:
        x = np.where(x < mean - 0.5, x + 1.0, x)
    zs = (x - mean) / sigma
    out = np.zeros(nbin, "d")
    ok = np.fabs(zs) < 20.0
    out[ok] = np.exp(-0.5 * zs[ok] ** 2.0) / (sigma * np.sqrt(2 * np.pi))
    if norm or np.max(abs(out)) == 0.0:
        return out
    i = out.argmax()
    z = (x[i] - loc) / sigma
    return np.exp(-0.5 * z ** 2.0) / out[i] * out


def scattering_times(tau, alpha, freqs, nu_tau):
    """pplib.py:4055-4059."""
    return tau * (freqs / nu_tau) ** alpha


def scattering_profile_FT(tau, nbin, binshift=binshift):
    """(1 + 2 pi i k tau)^-1, pplib.py:4061-4084."""
    nharm = nbin // 2 + 1
    if tau == 0.0:
        return np.ones(nharm)
    return (1.0 + 2 * np.pi * 1.0j * np.arange(nharm) * tau) ** -1


def scattering_portrait_FT(taus, nbin, binshift=binshift):
    """pplib.py:4086-4101."""
    taus = np.atleast_1d(taus)
    nharm = nbin // 2 + 1
    if not np.any(taus):
        return np.ones([len(taus), nharm])
    return np.array([scattering_profile_FT(t, nbin) for t in taus])


def gen_gaussian_profile(params, nbin):
    """DC + sum of Gaussians, optionally scattered; pplib.py:827-851."""
    ngauss = (len(params) - 2) // 3
    model = np.zeros(nbin, dtype="d") + params[0]
    for ig in range(ngauss):
        loc, wid, amp = params[2 + ig * 3:5 + ig * 3]
        model += amp * gaussian_profile(nbin, loc, wid)
    if params[1] != 0.0:
        # n=nbin: the reference's irfft (pplib.py:850) drops a bin at odd
        # nbin; the same for even nbin
        model = np.fft.irfft(scattering_profile_FT(float(params[1]) / nbin, nbin)
                             * np.fft.rfft(model), n=nbin)
    return model


def power_law_evolution(freqs, nu_ref, parameter, index):
    """pplib.py:996-1011."""
    return np.exp(np.outer(np.log(freqs) - np.log(nu_ref), index) +
                  np.outer(np.ones(len(freqs)), np.log(parameter)))


def linear_evolution(freqs, nu_ref, parameter, slope):
    """pplib.py:1013-1028."""
    return np.outer(freqs - nu_ref, slope) + np.outer(np.ones(len(freqs)), parameter)


def evolve_parameter(freqs, nu_ref, parameter, evol_parameter, code):
    """pplib.py:1030-1046."""
    fn = {"0": power_law_evolution, "1": linear_evolution}[code]
    return fn(freqs, nu_ref, parameter, evol_parameter)


def gen_gaussian_portrait(model_code, params, scattering_index, phases, freqs, nu_ref,
                          join_ichans=[], P=None):
    """Frequency-evolving Gaussian portrait, pplib.py:853-930."""
    if len(join_ichans):
        raise NotImplementedError("join_ichans is ppgauss-only (out of scope)")
    params = np.asarray(params, dtype=float)
    ref = np.array([params[0], params[1] * 0.0] + list(params[2::2]))
    tau = params[1]
    nbin, nchan = len(phases), len(freqs)
    gp = np.empty([nchan, len(ref)])
    gp[:, 0] = ref[0]
    gp[:, 1] = ref[1]
    gp[:, 2::3] = evolve_parameter(freqs, nu_ref, ref[2::3], params[3::6], model_code[0])
    gp[:, 3::3] = evolve_parameter(freqs, nu_ref, ref[3::3], params[5::6], model_code[1])
    gp[:, 4::3] = evolve_parameter(freqs, nu_ref, ref[4::3], params[7::6], model_code[2])
    port = np.array([gen_gaussian_profile(gp[i], nbin) for i in range(nchan)])
    if tau != 0.0:
        taus = scattering_times(float(tau) / nbin, scattering_index, freqs, nu_ref)
        # n=nbin as the device's k_rotate_rows_gen (pplib.py:921 has no n=
        # and returns nbin - 1 bins at odd nbin); the same for even nbin
        port = np.fft.irfft(scattering_portrait_FT(taus, nbin) *
                            np.fft.rfft(port, axis=-1), n=nbin, axis=-1)
    return port


def read_model(modelfile, phases=None, freqs=None, P=None, quiet=False):
    """Read a .gmodel (and build the portrait when phases/freqs given), pplib.py:2873-2959."""
    read_only = phases is None and freqs is None
    comps = []
    name = code = None
    nu_ref = dc = tau = alpha = 0.0
    fit_dc = fit_tau = fit_alpha = 0
    with open(modelfile, "rb") as fh:  # a pickled spline model is not UTF-8 text
        lines = fh.read().decode("latin-1").splitlines()
    for line in lines:
        info = line.split()
        if not info:
            continue
        key = info[0]
        try:
            if key == "MODEL":
                name = info[1]
            elif key == "CODE":
                code = info[1]
            elif key == "FREQ":
                nu_ref = np.float64(info[1])
            elif key == "DC":
                dc, fit_dc = np.float64(info[1]), int(info[2])
            elif key == "TAU":
                tau, fit_tau = np.float64(info[1]), int(info[2])
            elif key == "ALPHA":
                alpha, fit_alpha = np.float64(info[1]), int(info[2])
            elif key[:4] == "COMP":
                comps.append(line)
        except IndexError:
            pass
    if name is None or code is None:
        # what the reference's read_model raises on a non-.gmodel file (its
        # unassigned locals), which get_TOAs takes as "spline model"
        # (pptoas.py:375-378)
        raise UnboundLocalError("%s is not a .gmodel file" % modelfile)
    ngauss = len(comps)
    params = np.zeros(ngauss * 6 + 2)
    flags = np.zeros(len(params))
    params[0], params[1] = dc, tau
    flags[0], flags[1] = fit_dc, fit_tau
    for ig, comp in enumerate(comps):
        f = comp.split()
        params[2 + ig * 6:8 + ig * 6] = [np.float64(v) for v in f[1::2]]
        flags[2 + ig * 6:8 + ig * 6] = [int(v) for v in f[2::2]]
    if read_only:
        return (name, code, nu_ref, ngauss, params, flags, alpha, fit_alpha)
    nbin = len(phases)
    if params[1] != 0:
        if P is None:
            print("Need period P for non-zero scattering value TAU.")
            return 0
        params[1] *= nbin / P
    model = gen_gaussian_portrait(code, params, alpha, phases, freqs, nu_ref)
    return (name, ngauss, model)


def gen_gaussian_portraits_device(model_code, params, scattering_index, nbin, freqs, nu_ref):
    """gen_gaussian_portrait (pplib.py:853-930) for rows of frequencies
    ([..., nchan]) in one device call (ppf_gaussian_portraits); returns a
    numpy array [..., nchan, nbin].  params[1] (TAU) in bins, as there."""
    from .engine import get_engine
    return get_engine().gaussian_portraits(model_code, params, scattering_index, nbin, freqs,
                                           nu_ref).cpu().numpy()


def read_model_device(modelfile, nbin, freqs, P=None, quiet=False):
    """read_model(modelfile, phases, freqs, P) (pplib.py:2873-2959) with the
    portrait built on the device for every row of freqs ([..., nchan]): the
    .gmodel parse, TAU *= nbin / P, then gen_gaussian_portraits_device.
    Returns (name, ngauss, model [..., nchan, nbin])."""
    name, code, nu_ref, ngauss, params, flags, alpha, fit_alpha = read_model(modelfile,
                                                                             quiet=True)
    params = np.array(params, dtype=float)
    if params[1] != 0:
        if P is None:
            print("Need period P for non-zero scattering value TAU.")
            return 0
        params[1] *= nbin / P
    return name, ngauss, gen_gaussian_portraits_device(code, params, alpha, nbin, freqs, nu_ref)


# ---------------------------------------------------------------------------
# B-spline (PCA) templates: ppspline.py models (host reader, device builder)
# ---------------------------------------------------------------------------
class _SplineUnpickler(pickle.Unpickler):
    """Unpickler for ppspline model files (ppspline.py:206-228: a list of
    name, source, datafile, mean_prof, eigvec and tck) that resolves only
    numpy's array reconstruction: any other global in the file raises
    UnpicklingError, so loading a model executes nothing it names."""

    _ALLOWED = {("numpy.core.multiarray", "_reconstruct"),
                ("numpy._core.multiarray", "_reconstruct"),
                ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
                ("numpy", "ndarray"), ("numpy", "dtype"),
                ("_codecs", "encode"),  # protocol-2 bytes from Python 3
                ("__builtin__", "bytes"), ("builtins", "bytes")}  # ... and empty ones

    def find_class(self, module, name):
        if (module, name) not in self._ALLOWED:
            raise pickle.UnpicklingError("spline model: global %s.%s is not allowed"
                                         % (module, name))
        if name in ("ndarray", "dtype"):
            return getattr(np, name)
        if module == "_codecs":
            import codecs
            return codecs.encode
        if name == "bytes":
            return bytes
        try:
            from numpy._core import multiarray
        except ImportError:  # numpy 1.x
            from numpy.core import multiarray
        return getattr(multiarray, name)


def load_spline_model_file(modelfile):
    """(modelname, source, datafile, mean_prof, eigvec, tck) of a ppspline
    model: its Python-2 (or 3) pickle through _SplineUnpickler (latin-1 for
    Python-2 strings), or an .npz holding the same fields."""
    if str(modelfile).endswith(".npz"):
        z = np.load(modelfile, allow_pickle=False)
        tck = [z["t"], list(z["c"]), int(z["k"])]
        return (str(z["modelname"]), str(z["source"]), str(z["datafile"]), z["mean_prof"],
                z["eigvec"], tck)
    with open(modelfile, "rb") as fh:
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", DeprecationWarning)
            obj = _SplineUnpickler(fh, encoding="latin1").load()
    modelname, source, datafile, mean_prof, eigvec, tck = obj
    return modelname, source, datafile, np.asarray(mean_prof), np.asarray(eigvec), tck


def gen_spline_portrait(mean_prof, freqs, eigvec, tck, nbin=None):
    """gen_spline_portrait (pplib.py:932-956) on the device: FITPACK splev of
    the projections at freqs, eigvec . proj + mean_prof, and the resample +
    rotate when nbin != len(mean_prof) (ppf_spline_portraits).  Returns a
    numpy array [nchan, nbin]."""
    from .engine import get_engine
    eigvec = np.asarray(eigvec)
    return get_engine().spline_portraits(mean_prof, eigvec, tck, np.atleast_1d(freqs),
                                         nbin).cpu().numpy()


def read_spline_model(modelfile, freqs=None, nbin=None, quiet=False):
    """read_spline_model (pplib.py:2961-2993): the model tuple, or (name,
    portrait at freqs) built on the device."""
    if not quiet:
        print("Reading model from %s..." % modelfile)
    modelname, source, datafile, mean_prof, eigvec, tck = load_spline_model_file(modelfile)
    if freqs is None:
        return modelname, source, datafile, mean_prof, eigvec, tck
    return modelname, gen_spline_portrait(mean_prof, freqs, eigvec, tck, nbin)


def write_model(filename, name, model_code, nu_ref, model_params, fit_flags, alpha,
                fit_alpha, append=False, quiet=False):
    """pplib.py:2834-2871 (same text layout)."""
    with open(filename, "a" if append else "w") as out:
        out.write("MODEL   %s\n" % name)
        out.write("CODE    %s\n" % model_code)
        out.write("FREQ    %.5f\n" % nu_ref)
        out.write("DC     % .8f %d\n" % (model_params[0], fit_flags[0]))
        out.write("TAU    % .8f %d\n" % (model_params[1], fit_flags[1]))
        out.write("ALPHA  % .3f      %d\n" % (alpha, fit_alpha))
        for ig in range((len(model_params) - 2) // 6):
            comp = model_params[2 + ig * 6:8 + ig * 6]
            fc = fit_flags[2 + ig * 6:8 + ig * 6]
            line = (ig + 1,) + tuple(np.array(list(zip(comp, fc))).ravel())
            out.write("COMP%02d % .8f %d  % .8f %d  % .8f %d  % .8f %d  % .8f %d  % .8f %d\n"
                      % line)
    if not quiet:
        print("%s written." % filename)


# ---------------------------------------------------------------------------
# Scalar helpers (host)
# ---------------------------------------------------------------------------
def phase_transform(phi, DM, nu_ref1=np.inf, nu_ref2=np.inf, P=None, mod=False):
    """pplib.py:2592-2616."""
    if P is None:
        P, mod = 1.0, False
    out = phi + (Dconst * DM * P ** -1 * (nu_ref2 ** -2.0 - nu_ref1 ** -2.0))
    if mod:
        out = np.where(abs(out) >= 0.5, out % 1, out)
        out = np.where(out >= 0.5, out - 1.0, out)
        if not out.shape:
            out = np.float64(out)
    return out


def guess_fit_freq(freqs, SNRs=None):
    """pplib.py:2618-2632."""
    freqs = np.asarray(freqs, dtype=float)
    nu0 = (freqs.min() + freqs.max()) * 0.5
    if SNRs is None:
        SNRs = np.ones(len(freqs))
    return nu0 + np.sum((freqs - nu0) * SNRs * freqs ** -2) / np.sum(SNRs * freqs ** -2)


def DM_delay(DM, freq, freq_ref=np.inf, P=None):
    """pplib.py:2577-2590."""
    d = Dconst * DM * (freq ** -2.0 - freq_ref ** -2.0)
    return d / P if P else d


def weighted_mean(data, errs=1.0):
    """pplib.py:696-709."""
    if hasattr(errs, "is_integer"):
        errs = np.ones(len(data))
    i = np.where(errs > 0.0)[0]
    w = errs[i] ** -2.0
    return (data[i] * w).sum() / w.sum(), w.sum() ** -0.5


# ---------------------------------------------------------------------------
# GPU-backed utilities (libppfit)
# ---------------------------------------------------------------------------
def get_noise(data, method=default_noise_method, **kwargs):
    """pplib.py:2206-2225 (PS method on the GPU)."""
    if method != "PS":
        raise NotImplementedError("get_noise method %r: only 'PS' is on the hot path" % method)
    return get_noise_PS(data, **kwargs)


def get_noise_PS(data, frac=4, chans=False):
    """Noise from the top quarter of the power spectrum, pplib.py:2227-2253."""
    if frac != 4:
        raise NotImplementedError("frac != 4")
    data = np.asarray(data, dtype=np.float64)
    rows = data if chans else data.ravel()[None]
    out = _engine().noise_rows(rows).cpu().numpy()
    return out if chans else float(out[0])


def _rot_phases(shape, phase, DM, Ps, freqs, nu_ref):
    """Per-row rotation [rot] implied by rotate_data's arguments (pplib.py:2358-2415)."""
    ndim = len(shape)
    if DM == 0.0:
        nrow = int(np.prod(shape[:-1])) if ndim > 1 else 1
        return np.full(nrow, float(phase))
    d4 = (1,) * (4 - ndim) + tuple(shape)
    nsub, npol, nchan, _ = d4
    D = Dconst * DM / (np.ones(nsub) * Ps)
    f = np.asarray(freqs, dtype=float)
    if f.ndim == 0:
        f = np.ones(nchan) * float(f)
    fterm = (np.tile(f, nsub).reshape(nsub, nchan) if f.ndim == 1 else f) ** -2.0 - \
        nu_ref ** -2.0
    ph = phase + np.array([D[i] * fterm[i] for i in range(nsub)])
    return np.broadcast_to(ph[:, None, :], (nsub, npol, nchan)).ravel()


def rotate_data(data, phase=0.0, DM=0.0, Ps=None, freqs=None, nu_ref=np.inf):
    """Rotate/dedisperse 1-, 2- or 4-D data on the GPU, pplib.py:2338-2426."""
    data = np.asarray(data, dtype=np.float64)
    ph = _rot_phases(data.shape, phase, DM, Ps, freqs, nu_ref)
    rows = data.reshape(-1, data.shape[-1])
    out = _engine().rotate_rows(rows, ph).cpu().numpy()
    if DM == 0.0 or data.ndim in (1, 2, 4):
        return out.reshape(data.shape)
    return out


def rotate_portrait(port, phase=0.0, DM=None, P=None, freqs=None, nu_ref=np.inf):
    """pplib.py:2428-2460."""
    port = np.asarray(port, dtype=np.float64)
    if DM is None and freqs is None:
        ph = np.full(len(port), float(phase))
    else:
        ph = phase + Dconst * DM / P * (np.asarray(freqs) ** -2.0 - nu_ref ** -2.0)
    return _engine().rotate_rows(port, ph).cpu().numpy()


def rotate_profile(profile, phase=0.0):
    """pplib.py:2548-2559."""
    return rotate_data(profile, phase)


def fit_phase_shift(data, model, noise=None, bounds=[-0.5, 0.5], Ns=100):
    """FFTFIT: brute force + Nelder-Mead on the GPU, pplib.py:2054-2100."""
    t0 = time.time()
    out = _engine().phase_shift_batch(np.asarray(data, dtype=np.float64),
                                      np.asarray(model, dtype=np.float64), noise=noise,
                                      Ns=Ns, bounds=bounds).cpu().numpy()[0]
    return DataBunch(phase=out[0], phase_err=out[1], scale=out[2], scale_err=out[3],
                     snr=out[4], red_chi2=out[5], duration=time.time() - t0)


def fit_portrait(data, model, init_params, P, freqs, nu_fit=None, nu_out=None, errs=None,
                 bounds=[(None, None), (None, None)], id=None, quiet=True):
    """Legacy phase + DM fit (pplib.py:2102-2204) on the GPU.

    As the reference, scipy TNC (jac, bounds, xtol 1e-10; pplib.py:2144-2148)
    over (phase, DM) -- the device TNC (ppfit_tnc.hip) in its 2-parameter
    form -- then the legacy outputs: phase/DM errors from the 2x2 curvature
    matrix without amplitude covariance (pplib.py:2184-2190) and scale_errs
    = (p_n / errs^2)^-1/2 (pplib.py:2197).  return_code and nfeval are TNC's
    (RCSTRINGS, pplib.py:111-119).
    """
    from . import pptoaslib
    freqs = np.asarray(freqs, dtype=float)
    if nu_fit is None:
        nu_fit = freqs.mean()
    b = list(bounds) if bounds is not None else [(None, None)] * 2
    res = pptoaslib._fit_batch_host(
        np.asarray(data, float)[None], np.asarray(model, float)[None], [init_params[0],
        init_params[1], 0.0, 0.0, 0.0], P, freqs, [nu_fit, nu_fit, nu_fit],
        [nu_out, nu_out, nu_out], errs, [1, 1, 0, 0, 0], log10_tau=False, legacy=True,
        method="TNC-legacy", bounds=b + [(None, None)] * 3)
    r = {k: v[0] for k, v in res.items() if k != "legacy"}
    leg = {k: v[0] for k, v in res["legacy"].items()}
    return DataBunch(phase=r["params"][0], phase_err=leg["phase_err"], DM=r["params"][1],
                     DM_err=leg["DM_err"], scales=r["scales"], scale_errs=leg["scale_errs"],
                     nu_ref=r["nu_out"][0], covariance=leg["covariance"], chi2=r["chi2"],
                     red_chi2=r["red_chi2"], snr=r["snr"], duration=r["duration"],
                     nfeval=int(r["nfev"]), return_code=int(r["status"]))


# ---------------------------------------------------------------------------
# TOA output (pplib.py:3386-3509)
# ---------------------------------------------------------------------------
def filter_TOAs(TOAs, flag, cutoff, criterion=">=", pass_unflagged=False,
                return_culled=False):
    """pplib.py:3386-3413."""
    import operator
    op = {">=": operator.ge, ">": operator.gt, "<=": operator.le, "<": operator.lt,
          "==": operator.eq, "!=": operator.ne}[criterion]
    keep, cull = [], []
    for toa in TOAs:
        if hasattr(toa, flag):
            (keep if op(getattr(toa, flag), cutoff) else cull).append(toa)
        elif pass_unflagged:
            keep.append(toa)
        else:
            cull.append(toa)
    if return_culled:
        return keep, return_culled
    return keep


def _flag_fmt(flag, vtype):
    """Format of one flag in write_TOAs' Python-2 formatting (pplib.py:3486-3503)
    for a value of type vtype: str %s, int %d, '_cov' %.1e, 'phs' %.8f, 'flux'
    %.5f, else %.3f."""
    f = flag.replace("%", "%%")
    if hasattr(vtype, "lower"):
        return " -%s %%s" % f
    # Python-2 ints -- bool included (True.bit_length() exists, so
    # pptoas.py:1602's DM_mean=True prints "1") -- take %d; numpy's bool_ has
    # no bit_length and takes the float formats
    if issubclass(vtype, (int, np.integer)) and not issubclass(vtype, np.bool_):
        return " -%s %%d" % f
    if flag.find("_cov") >= 0:
        return " -%s %%.1e" % f
    if flag.find("phs") >= 0:
        return " -%s %%.8f" % f
    if flag.find("flux") >= 0:
        return " -%s %%.5f" % f
    return " -%s %%.3f" % f


def _flag_text(flag, value):
    """One flag as write_TOAs prints it (pplib.py:3486-3503)."""
    return _flag_fmt(flag, type(value)) % value


_LINE_FMTS = {}  # (flag names, value types) of a TOA's flags -> their joined format
_NoneType = type(None)


def toa_line(toa, inf_is_zero=True):
    """One loosely-IPTA .tim line, pplib.py:3471-3503.  The flags of every TOA
    with the same (flag, value type) signature share one format string; a
    None value is left out, as write_TOAs skips it."""
    freq = 0.0 if (toa.frequency == np.inf and inf_is_zero) else toa.frequency
    m = toa.MJD
    s = "%s %.8f %d" % (toa.archive, freq, m.intday()) + \
        ("%.15f   %.3f  %s" % (m.fracday(), toa.TOA_error, toa.telescope_code))[1:]
    if toa.DM is not None:
        s += " -pp_dm %.7f" % toa.DM
    if toa.DM_error is not None:
        s += " -pp_dme %.7f" % toa.DM_error
    fl = toa.flags
    vals = tuple(fl.values())
    types = tuple(map(type, vals))
    key = (tuple(fl), types)
    fmt = _LINE_FMTS.get(key)
    if fmt is None:
        fmt = "".join([_flag_fmt(k, t) for k, t in zip(key[0], types) if t is not _NoneType])
        if len(_LINE_FMTS) < 4096:
            _LINE_FMTS[key] = fmt
    if _NoneType in types:
        vals = tuple([v for v in vals if v is not None])
    return s + fmt % vals


def write_TOAs(TOAs, inf_is_zero=True, SNR_cutoff=0.0, outfile=None, append=True):
    """pplib.py:3451-3509.  A get_TOAs TOA_list (toas.TOAList) is written
    through its column blocks (native .tim writer, include/pptim.h, straight
    from its buffers to the file); any other sequence of TOAs one line at a
    time.  Returns None, as the reference does."""
    from .toas import TOAList, write_pieces
    if isinstance(TOAs, TOAList):
        pieces = TOAs.tim_chunks(inf_is_zero, SNR_cutoff)
        if outfile is None:
            sys.stdout.flush()
            write_pieces(sys.stdout.buffer, pieces)
            sys.stdout.buffer.flush()
        else:
            with open(outfile, "ab" if append else "wb") as f:
                write_pieces(f, pieces)
        return None
    toas = TOAs if hasattr(TOAs, "__len__") else [TOAs]
    toas = filter_TOAs(toas, "snr", SNR_cutoff, ">=", pass_unflagged=False)
    lines = [toa_line(t, inf_is_zero) for t in toas]
    if outfile is None:
        for ln in lines:
            print(ln)
    else:
        with open(outfile, "a" if append else "w") as f:
            for ln in lines:
                f.write(ln + "\n")
