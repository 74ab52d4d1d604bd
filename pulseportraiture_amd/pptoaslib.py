"""pptoaslib drop-in: fit_portrait_full on the GPU (pptoaslib.py:928-1096).

``fit_portrait_full`` keeps the reference signature and DataBunch keys; the
FFTs, objective passes, trust-region solve, zero-covariance frequencies and
the Woodbury covariance all run in libppfit (one workgroup per subint).
``fit_portraits_batch`` is the batched form the drivers (get_TOAs, ppalign)
use: one device call for many subints.
"""
import sys
import time

import numpy as np

from .pplib import (DataBunch, Dconst, RCSTRINGS, scattering_times,
                    scattering_portrait_FT)

__all__ = ["fit_portrait_full", "fit_portraits_batch", "instrumental_response_FT",
           "instrumental_response_port_FT", "phase_shifts",
           "phase_shifts_deriv", "rotate_portrait_full", "scattering_times",
           "scattering_portrait_FT"]


def phase_shifts(phi, DM, GM, freqs, nu_DM=np.inf, nu_GM=np.inf, P=None, mod=False):
    """Per-channel delay [rot], pptoaslib.py:181-214."""
    if P is None:
        P, mod = 1.0, False
    d = phi + Dconst * DM * (freqs ** -2 - nu_DM ** -2) / P + \
        Dconst ** 2 * GM * (freqs ** -4 - nu_GM ** -4) / P
    if mod:
        d = np.where(abs(d) >= 0.5, d % 1, d)
        d = np.where(d >= 0.5, d - 1.0, d)
        if not np.shape(d):
            d = np.float64(d)
    return d


def phase_shifts_deriv(freqs, nu_DM=np.inf, nu_GM=np.inf, P=None):
    """pptoaslib.py:216-225."""
    if P is None:
        P = 1.0
    dphi = np.ones(len(freqs)) if hasattr(freqs, "shape") else 1.0
    return np.array([dphi, Dconst * (freqs ** -2 - nu_DM ** -2) / P,
                     Dconst ** 2 * (freqs ** -4 - nu_GM ** -4) / P])


def rotate_portrait_full(port, phi, DM, GM, freqs, nu_DM=np.inf, nu_GM=np.inf, P=None):
    """Rotate/dedisperse a portrait on the GPU, pptoaslib.py:52-81."""
    from .engine import get_engine
    if P is None:
        P = 1.0
    ph = phase_shifts(phi, DM, GM, np.asarray(freqs, dtype=float), nu_DM, nu_GM, P)
    return get_engine().rotate_rows(np.asarray(port, dtype=float), ph).cpu().numpy()


def instrumental_response_port_FT(nbin, freqs, DM=0.0, P=1.0, wids=[], irf_types=[]):
    """pptoaslib.py:145-179 on the device: the [nchan, nharm] product of the
    responses ('rect' np.sinc(k wid), 'gauss' the normalised Gaussian FT of
    FWHM wid) and, for DM != 0, the rect smearing of width 8.3e-6 chan_bw /
    (freq / 1e3)^3 / P (the reference's formula, where DM only switches it
    on).  Returned real (the reference's imaginary parts are zero)."""
    from .engine import get_engine
    freqs = np.atleast_1d(np.asarray(freqs, dtype=np.float64))
    if DM == len(wids) == 0.0:
        return np.ones([len(freqs), nbin // 2 + 1])
    return get_engine().response_table(nbin, freqs, DM, P, wids, irf_types).cpu().numpy()


def instrumental_response_FT(nbin, wid=0.0, irf_type="rect"):
    """pptoaslib.py:112-143: one response row (wid 0 -> ones)."""
    if wid == 0.0:
        return np.ones(nbin // 2 + 1)
    return instrumental_response_port_FT(nbin, [1.0], 0.0, 1.0, [wid], [irf_type])[0]


# host inputs above STREAM_BYTES are fitted in chunks of STREAM_CHUNK_BYTES
# with the host -> device copies overlapped (fit_portraits_batch)
STREAM_BYTES = 1 << 30
STREAM_CHUNK_BYTES = 1 << 29


def _nan(v):
    return np.nan if v is None else float(v)


def fit_portraits_batch(data, model, init, P, freqs, nu_fits=None, nu_outs=None,
                        errs=None, fit_flags=(1, 1, 0, 0, 0), log10_tau=False, option=0,
                        is_toa=True, chan_mask=None, weights=None, model_idx=None,
                        guess=False, guess_Ns=100, guess_wrap=True, guess_nu=None,
                        guess_tau=None, method="trust-ncg", bounds=None, device=None,
                        to_host=True, host_keys=None, spec_cache=None):
    """Batched fit_portrait_full over subints; returns arrays keyed like its DataBunch.

    method selects the device solver as minimize(method=...) does in the
    reference (pptoaslib.py:995-1014); bounds are applied by TNC only.
    host_keys: the result keys to copy to the host (None: all) -- one
    packed D2H (engine.results_to_host).  spec_cache: Engine.fit_batch's
    data-spectrum cache (device-resident data only)."""
    if method not in ("trust-ncg", "TNC", "Newton-CG", "TNC-legacy"):
        print("Method '%s' is not implemented." % method)
        sys.exit()
    from .engine import get_engine
    import torch
    eng = get_engine(device)
    t0 = time.time()
    kw = dict(nu_fit=nu_fits, nu_out=nu_outs, errs=errs, chan_mask=chan_mask, weights=weights,
              model_idx=model_idx, log10_tau=log10_tau, option=option, is_toa=is_toa,
              guess=guess, guess_Ns=guess_Ns, guess_wrap=guess_wrap, guess_nu=guess_nu,
              guess_tau=guess_tau, method=method,
              bounds=bounds if method.startswith("TNC") else None)
    host = not isinstance(data, torch.Tensor) or data.device.type == "cpu"
    nbytes = int(np.prod(np.shape(data))) * 8
    if host and np.ndim(data) == 3 and nbytes > STREAM_BYTES:
        # host-resident subints: chunks staged through pinned buffers and
        # copied to the device on a second stream while the previous chunk is
        # fitted (Engine.fit_batch_streamed)
        if spec_cache is not None:
            raise ValueError("spec_cache: device-resident data only")
        per = int(np.prod(np.shape(data)[1:])) * 8
        out = eng.fit_batch_streamed(data, model, freqs, P, init, fit_flags,
                                     chunk=max(1, STREAM_CHUNK_BYTES // per), **kw)
    else:
        if spec_cache is not None:
            kw["spec_cache"] = spec_cache
        out = eng.fit_batch(data, model, freqs, P, init, fit_flags, **kw)
    if not to_host:
        return out
    from .engine import results_to_host
    res = results_to_host(out, host_keys, eng.stream)
    n = int(out["status"].shape[0])
    res["duration"] = np.full(n, (time.time() - t0) / max(n, 1))
    return res


class SyncPipeline:
    """engine.FitPipeline's interface over a fit_portraits_batch-style
    function, run at submit (the CPU tests' stand-in for the device)."""

    def __init__(self, fit_fn, keys=None):
        self.fit_fn, self.keys, self.pending = fit_fn, keys, []

    def __len__(self):
        return len(self.pending)

    def submit(self, tag, data, model, freqs, P, init, fit_flags, nu_fit=None, nu_out=None,
               **kw):
        res = self.fit_fn(data, model, init, P, freqs, nu_fits=nu_fit, nu_outs=nu_out,
                          fit_flags=fit_flags, **kw)
        self.pending.append((tag, {k: np.asarray(v) for k, v in res.items()
                                   if self.keys is None or k in self.keys}))

    def collect(self):
        return self.pending.pop(0)


def _fit_batch_host(data, model, init, P, freqs, nu_fits, nu_outs, errs, fit_flags,
                    log10_tau, legacy=False, **kw):
    res = fit_portraits_batch(data, model, init, P, freqs,
                              nu_fits=[_nan(v) for v in nu_fits],
                              nu_outs=[_nan(v) for v in nu_outs], errs=errs,
                              fit_flags=fit_flags, log10_tau=log10_tau, **kw)
    if legacy:
        cn = res["cov_nosc"]
        S = (res["channel_snrs"] / res["scales"]) ** 2
        res["legacy"] = dict(phase_err=cn[:, 0, 0] ** 0.5, DM_err=cn[:, 1, 1] ** 0.5,
                             covariance=cn[:, 0, 1], scale_errs=S ** -0.5)
    return res


def result_bunch(res, i, fit_flags, duration=None):
    """DataBunch of subint i in the layout of pptoaslib.py:1086-1095."""
    ifit = np.where(fit_flags)[0]
    nfit = len(ifit)
    p = res["params"][i]
    e = res["param_errs"][i]
    cov = res["cov"][i][:nfit, :nfit]
    return DataBunch(params=list(p), param_errs=e.copy(), phi=p[0], phi_err=e[0],
                     DM=p[1], DM_err=e[1], GM=p[2], GM_err=e[2], tau=p[3],
                     tau_err=e[3], alpha=p[4], alpha_err=e[4],
                     scales=res["scales"][i], scale_errs=res["scale_errs"][i],
                     nu_DM=res["nu_out"][i][0], nu_GM=res["nu_out"][i][1],
                     nu_tau=res["nu_out"][i][2], covariance_matrix=cov,
                     chi2=res["chi2"][i], red_chi2=res["red_chi2"][i], snr=res["snr"][i],
                     channel_snrs=res["channel_snrs"][i],
                     duration=res["duration"][i] if duration is None else duration,
                     nfeval=int(res["nfev"][i]), return_code=int(res["status"][i]))


def report_failure(status, sub_id=None, stream=sys.stderr):
    """The reference's stderr note for a 'failed' fit, pptoaslib.py:1022-1033."""
    success = status == 0
    if success or status in (1, 2, 4):
        return
    rc = RCSTRINGS.get(str(status), "")
    if sub_id is not None:
        ii = sub_id[::-1].index("_")
        stream.write("Fit 'failed' with return code %d: %s -- %s subint %s\n"
                     % (status, rc, sub_id[:-ii - 1], sub_id[-ii:]))
    else:
        stream.write("Fit 'failed' with return code %d -- %s" % (status, rc))


def fit_portrait_full(data_port, model_port, init_params, P, freqs,
                      nu_fits=[None, None, None], nu_outs=[None, None, None], errs=None,
                      fit_flags=[1, 1, 1, 1, 1],
                      bounds=[(None, None), (None, None), (None, None), (None, None),
                              (None, None)],
                      log10_tau=True, option=0, sub_id=None, method="trust-ncg",
                      is_toa=True, quiet=True):
    """Fit phase, DM, GM, tau, alpha between data and model portraits (pptoaslib.py:928)."""
    if method not in ("trust-ncg", "TNC", "Newton-CG", "TNC-legacy"):
        print("Method '%s' is not implemented." % method)
        sys.exit()
    data_port = np.asarray(data_port, dtype=float)
    freqs = np.asarray(freqs, dtype=float)
    res = _fit_batch_host(data_port[None], np.asarray(model_port, dtype=float)[None],
                          list(init_params), P, freqs, nu_fits, nu_outs,
                          None if errs is None else np.asarray(errs, dtype=float),
                          fit_flags, log10_tau, option=option, is_toa=is_toa,
                          method=method, bounds=bounds)
    report_failure(int(res["status"][0]), sub_id)
    return result_bunch(res, 0, fit_flags)
