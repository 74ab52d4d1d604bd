"""CPU oracle for the wideband FFTFIT hot path -- TEST INFRASTRUCTURE ONLY.

This module is a clean-room numpy/scipy restatement of the reference
algorithm (kmjc/PulsePortraiture, Python 2).  It is the *checker* and the
box-side CPU baseline ("kind": "port"); the product never imports it.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may use it.

Parity pinning: the restatement is checked against golden vectors produced
from the reference source itself (``tests/golden/make_golden.py``, SURVEY.md
§8(c) shim) by ``tests/test_oracle_golden.py``.

Third-party algorithms used here exactly as the reference uses them:
numpy.fft (pocketfft) rfft/irfft, scipy.optimize.minimize(method='trust-ncg'
| 'TNC' | 'Newton-CG'), scipy.optimize.brute + fmin (Nelder-Mead); scipy
1.15.3 / numpy 2.2.6 in this image.

Every function cites the reference file:line it restates.
"""
import time
import warnings

import numpy as np
import scipy.optimize as opt

# pplib.py:44-66
DCONST = 0.000241 ** -1          # "traditional" dispersion constant, Dconst
F0_FACT = 0.0                    # DC harmonic ignored in Fourier fits
SCATTERING_ALPHA = -4.0


class Bunch(dict):
    """dict with attribute access (pplib.py:125-136 DataBunch)."""

    def __init__(self, **kw):
        dict.__init__(self, kw)
        self.__dict__ = self


# ---------------------------------------------------------------------------
# L1 signal utilities
# ---------------------------------------------------------------------------
def get_bin_centers(nbin, lo=0.0, hi=1.0):
    """pplib.py:671-684."""
    d = float(hi) - float(lo)
    return np.linspace(lo + d / (nbin * 2), hi - d / (nbin * 2), nbin)


def get_noise_PS(data, frac=4, chans=False):
    """Noise from the top 1/frac of the power spectrum, pplib.py:2227-2253."""
    data = np.asarray(data, dtype=float)

    def one(prof):
        spec = np.fft.rfft(prof)
        pows = (spec.real ** 2 + spec.imag ** 2) / len(prof)
        kc = int((1 - 1.0 / frac) * len(pows))
        return np.sqrt(np.mean(pows[kc:]))

    if chans:
        return np.array([one(row) for row in data])
    return one(data.ravel())


def phase_transform(phi, DM, nu_ref1=np.inf, nu_ref2=np.inf, P=None, mod=False):
    """Move a delay between reference frequencies, pplib.py:2592-2616."""
    if P is None:
        P, mod = 1.0, False
    out = phi + DCONST * DM / P * (nu_ref2 ** -2.0 - nu_ref1 ** -2.0)
    if mod:
        out = np.where(np.abs(out) >= 0.5, out % 1, out)
        out = np.where(out >= 0.5, out - 1.0, out)
        if not np.shape(out):
            out = np.float64(out)
    return out


def guess_fit_freq(freqs, SNRs=None):
    """SNR*nu^-2 weighted centre of the band, pplib.py:2618-2632."""
    freqs = np.asarray(freqs, dtype=float)
    nu0 = 0.5 * (freqs.min() + freqs.max())
    w = (np.ones(len(freqs)) if SNRs is None else np.asarray(SNRs)) * freqs ** -2
    return nu0 + np.sum((freqs - nu0) * w) / np.sum(w)


def rotate_data(data, phase=0.0, DM=0.0, Ps=None, freqs=None, nu_ref=np.inf):
    """Fourier-domain rotation/dedispersion, pplib.py:2338-2426.

    Positive phase/DM rotate to earlier phase.  DM == 0 rotates along the last
    axis only; otherwise the data are promoted to [nsub, npol, nchan, nbin].
    """
    data = np.asarray(data, dtype=float)
    if DM == 0.0:
        spec = np.fft.rfft(data, axis=-1)
        k = np.arange(spec.shape[-1])
        return np.fft.irfft(spec * np.exp(2.0j * np.pi * phase * k), axis=-1)
    ndim = data.ndim
    d4 = data.reshape((1,) * (4 - ndim) + data.shape)
    nsub, npol, nchan, nbin = d4.shape
    spec = np.fft.rfft(d4, axis=-1)
    k = np.arange(spec.shape[-1])
    D = DCONST * DM / (np.ones(nsub) * Ps)
    f = np.asarray(freqs, dtype=float)
    if f.ndim == 0:
        f = np.ones(nchan) * float(f)
    fterm = (np.tile(f, nsub).reshape(nsub, nchan) if f.ndim == 1 else f) ** -2.0 \
        - nu_ref ** -2.0
    ph = phase + D[:, None] * fterm                       # [nsub, nchan]
    rot = np.exp(2.0j * np.pi * ph[:, None, :, None] * k)  # broadcast over pol
    out = np.fft.irfft(spec * rot, axis=-1)
    return out.reshape(data.shape) if ndim in (1, 2) else out


def remove_baseline(subints, weights, ntot=1, duty=0.15):
    """arch.remove_baseline() as load_data calls it (pplib.py:2691), restated
    from PSRCHIVE's documented default (Integration::remove_baseline with the
    BaselineWindow estimator, duty cycle 0.15): per subint, the off-pulse
    window is the circular run of floor(duty * nbin) bins with the smallest
    sum of the total-intensity profile (weighted frequency sum of the first
    ntot polarisations; first window on ties), and every profile has its mean
    over that window subtracted.  PARITY UNPINNED: PSRCHIVE is not in this
    image and the reference ships no archives.  Returns (out, window starts)."""
    d = np.array(subints, dtype=float)
    nsub, npol, nchan, nbin = d.shape
    width = max(1, int(duty * nbin))
    w = np.asarray(weights, dtype=float)
    starts = np.zeros(nsub, dtype=int)
    for s in range(nsub):
        on = w[s] != 0.0
        t = np.einsum("n,nj->j", w[s][on], d[s, :ntot][:, on].sum(axis=0))
        box = np.array([t[(j + np.arange(width)) % nbin].sum() for j in range(nbin)])
        j0 = int(np.argmin(box))
        idx = (j0 + np.arange(width)) % nbin
        d[s] -= d[s][..., idx].mean(axis=-1)[..., None]
        starts[s] = j0
    return d, starts


def profile_snr(rows, duty=0.15, threshold=0.1):
    """Profile::snr() as load_data fills SNRs (pplib.py:2762-2770), restated
    from PSRCHIVE's default "phase" S/N estimator: off-pulse window = the
    circular run of floor(duty nbin) bins of smallest sum (first on ties),
    its mean m and sample variance v; the on-pulse edges from the running
    power of y = row - m read from the bin after the window (the first bins
    where it reaches threshold and 1 - threshold of the total C); snr =
    sum(y[rise..fall]) / sqrt(fall - rise + 1) / sqrt(v) (0 if C <= 0 or
    v <= 0).  PARITY UNPINNED: PSRCHIVE is not in this image and the
    reference ships no archives.  The sums run in the order ppf_profile_snr
    forms them (window sums bin by bin from the start; the running power in
    64 contiguous segments, then the segment totals in order), so discrete
    choices (window, edges) are the device's on the same rows."""
    shape = np.shape(rows)[:-1]
    x = np.asarray(rows, dtype=float).reshape(-1, np.shape(rows)[-1])
    nrow, nbin = x.shape
    width = max(1, int(duty * nbin))
    out = np.zeros(nrow)
    per = (nbin + 63) // 64
    for r in range(nrow):
        row = x[r]
        box = np.zeros(nbin)
        for i in range(width):  # sequential per window start, as the device
            box = box + row[(np.arange(nbin) + i) % nbin]
        j0 = int(np.argmin(box))
        win = row[(j0 + np.arange(width)) % nbin]
        m = 0.0
        for v_ in win:
            m += v_
        m /= width
        v = 0.0
        for v_ in win:
            v += (v_ - m) * (v_ - m)
        v = v / (width - 1) if width > 1 else 0.0
        y = row[(j0 + width + np.arange(nbin)) % nbin] - m
        segs = [(min(nbin, q * per), min(nbin, q * per + per)) for q in range(64)]
        tot = []
        for i0, i1 in segs:  # each segment summed in sequence
            t = 0.0
            for i in range(i0, i1):
                t += y[i]
            tot.append(t)
        pre, C = [], 0.0
        for t in tot:  # exclusive prefix of the totals, in order
            pre.append(C)
            C += t
        rise = fall = None
        for (i0, i1), cc in zip(segs, pre):
            for i in range(i0, i1):
                cc += y[i]
                if rise is None and cc >= threshold * C:
                    rise, crise, yrise = i, cc, y[i]
                if fall is None and cc >= (1.0 - threshold) * C:
                    fall, cfall = i, cc
        if C > 0 and v > 0 and rise is not None and fall is not None and fall >= rise:
            out[r] = (cfall - crise + yrise) / np.sqrt(fall - rise + 1) / np.sqrt(v)
    return out.reshape(shape)


def phase_shifts(phi, DM, GM, freqs, nu_DM=np.inf, nu_GM=np.inf, P=None):
    """Per-channel delay [rot], pptoaslib.py:181-214 (mod=False)."""
    if P is None:
        P = 1.0
    return phi + DCONST * DM * (freqs ** -2 - nu_DM ** -2) / P + \
        DCONST ** 2 * GM * (freqs ** -4 - nu_GM ** -4) / P


def phase_shift_jacobian(freqs, nu_DM, nu_GM, P):
    """d phi_n / d(phi, DM, GM), pptoaslib.py:216-225 (second derivs are 0)."""
    return np.array([np.ones(len(freqs)),
                     DCONST * (freqs ** -2 - nu_DM ** -2) / P,
                     DCONST ** 2 * (freqs ** -4 - nu_GM ** -4) / P])


def rotate_portrait_full(port, phi, DM, GM, freqs, nu_DM=np.inf, nu_GM=np.inf,
                         P=None):
    """pptoaslib.py:52-81."""
    if P is None:
        P = 1.0
    spec = np.fft.rfft(port, axis=-1)
    k = np.arange(spec.shape[-1])
    ph = phase_shifts(phi, DM, GM, np.asarray(freqs), nu_DM, nu_GM, P)
    return np.fft.irfft(spec * np.exp(2.0j * np.pi * np.outer(ph, k)))


# ---------------------------------------------------------------------------
# Scattering (pplib.py:4055-4101, pptoaslib.py:246-356)
# ---------------------------------------------------------------------------
def scattering_times(tau, alpha, freqs, nu_tau):
    """pplib.py:4055-4059."""
    return tau * (freqs / nu_tau) ** alpha


def scattering_portrait_FT(taus, nbin):
    """B_nk = 1/(1 + 2 pi i k tau_n), pplib.py:4061-4101."""
    nharm = nbin // 2 + 1
    taus = np.atleast_1d(taus)
    if not np.any(taus):
        return np.ones((len(taus), nharm))
    return 1.0 / (1.0 + 2.0j * np.pi * np.outer(taus, np.arange(nharm)))


def _tau_jacobians(tau, freqs, nu_tau, log10_tau, taus):
    """d tau_n/d(tau, alpha) and second derivatives, pptoaslib.py:246-274."""
    has = bool(taus.sum())
    if not log10_tau:
        dtau = taus / tau if has else np.zeros(len(freqs))
        d2tau = np.zeros(len(freqs))
        dalpha = np.log(freqs / nu_tau) * taus
        dtaudalpha = dalpha / tau if has else np.zeros(len(freqs))
    else:
        dtau = np.log(10.0) * taus
        dalpha = np.log(freqs / nu_tau) * taus
        d2tau = np.log(10.0) * dtau
        dtaudalpha = np.log(10.0) * dalpha
    d2alpha = np.log(freqs / nu_tau) * dalpha
    return (np.array([dtau, dalpha]),
            np.array([[d2tau, dtaudalpha], [dtaudalpha, d2alpha]]))


def _scat_FT_derivs(taus, dts, d2ts, B):
    """dB/d(tau,alpha) and the 2x2 second derivatives, pptoaslib.py:318-356."""
    nchan, nharm = B.shape
    dB = np.zeros((2, nchan, nharm), complex)
    d2B = np.zeros((2, 2, nchan, nharm), complex)
    if not taus.sum():
        return dB, d2B
    base = B * (B - 1.0)
    f = base / taus[:, None]
    dB[0] = f * dts[0][:, None]
    dB[1] = f * dts[1][:, None]
    H = base / (taus ** 2)[:, None]
    # diagonal blocks: the bracket is applied only when the jacobian sums != 0
    for j in range(2):
        h = H * (dts[j] ** 2)[:, None]
        if dts[j].sum():
            h = h * (2 * (B - 1.0) + (d2ts[j, j] * taus / dts[j] ** 2)[:, None])
        d2B[j, j] = h
    h = H * (dts[0] * dts[1])[:, None]
    if dts[1].sum() and dts[0].sum():
        h = h * (2 * (B - 1.0) + (d2ts[0, 1] * taus / (dts[0] * dts[1]))[:, None])
    d2B[0, 1] = d2B[1, 0] = h
    return dB, d2B


# ---------------------------------------------------------------------------
# L2 objective: per-channel terms and their assembly
# ---------------------------------------------------------------------------
def channel_terms(params, dFT, mFT, errs_FT, P, freqs, nu_DM, nu_GM, nu_tau,
                  log10_tau):
    """Per-channel C_n, dC, d2C, S_n, dS, d2S (all divided by errs_FT^2).

    Restates Sbp / Sbp_deriv / Sbp_2deriv / Cdbp / Cdbp_deriv / Cdbp_2deriv and
    the phasor/scattering helpers, pptoaslib.py:233-523.
    """
    phi, DM, GM, tau, alpha = params
    if log10_tau:
        tau = 10 ** tau
    nchan, nharm = dFT.shape
    nbin = 2 * (nharm - 1)
    k = np.arange(nharm)
    ph = phase_shifts(phi, DM, GM, freqs, nu_DM, nu_GM, P)
    dph = phase_shift_jacobian(freqs, nu_DM, nu_GM, P)
    taus = scattering_times(tau, alpha, freqs, nu_tau)
    W = dFT * np.conj(mFT) * np.exp(2.0j * np.pi * np.outer(ph, k))
    m2 = np.abs(mFT) ** 2
    w2 = errs_FT ** 2
    tpk = 2.0j * np.pi * k
    if not taus.sum():
        # tau = 0: B = 1 and every tau/alpha derivative of B vanishes
        # (pptoaslib.py:318-356 return zeros), so only the phase family is left
        C = np.real(W.sum(-1))
        C1 = np.real((tpk * W).sum(-1))
        C2 = np.real((tpk ** 2 * W).sum(-1))
        S = m2.sum(-1)
        dC = np.zeros((5, nchan))
        dC[:3] = C1 * dph
        d2C = np.zeros((5, 5, nchan))
        d2C[:3, :3] = C2 * dph[:, None] * dph[None]
        z5 = np.zeros((5, nchan))
        return Bunch(C=C / w2, dC=dC / w2, d2C=d2C / w2, S=S / w2, dS=z5,
                     d2S=np.zeros((5, 5, nchan)), taus=taus)
    dts, d2ts = _tau_jacobians(tau, freqs, nu_tau, log10_tau, taus)
    B = scattering_portrait_FT(taus, nbin)
    dB, d2B = _scat_FT_derivs(taus, dts, d2ts, B)
    C = np.real(np.sum(W * np.conj(B), -1))
    C1 = np.real(np.sum(tpk * W * np.conj(B), -1))
    C2 = np.real(np.sum(tpk ** 2 * W * np.conj(B), -1))
    S = np.sum(np.abs(B) ** 2 * m2, -1)
    dC = np.zeros((5, nchan))
    dC[:3] = C1 * dph
    dC[3:] = np.real(np.sum(W[None] * np.conj(dB), -1))
    d2C = np.zeros((5, 5, nchan))
    d2C[:3, :3] = C2 * dph[:, None] * dph[None]
    d2C[3:, 3:] = np.real(np.sum(W[None, None] * np.conj(d2B), -1))
    cross = np.real(np.sum(tpk * W[None] * np.conj(dB), -1))      # [2, nchan]
    d2C[:3, 3:] = dph[:, None] * cross[None]
    d2C[3:, :3] = np.transpose(d2C[:3, 3:], (1, 0, 2))
    dS = np.zeros((5, nchan))
    dS[3:] = np.sum(2 * np.real(B[None] * np.conj(dB)) * m2, -1)
    d2S = np.zeros((5, 5, nchan))
    abs2 = np.zeros((2, 2, nchan, nharm))
    for i in range(2):
        for j in range(2):
            abs2[i, j] = 2 * np.real(dB[i] * np.conj(dB[j]) + B * np.conj(d2B[i, j]))
    d2S[3:, 3:] = np.sum(abs2 * m2, -1)
    return Bunch(C=C / w2, dC=dC / w2, d2C=d2C / w2, S=S / w2, dS=dS / w2,
                 d2S=d2S / w2, taus=taus)


def _split(args):
    (dFT, mFT, errs_FT, P, freqs, nu_DM, nu_GM, nu_tau, fit_flags, log10_tau) = args
    return (dFT, mFT, errs_FT, P, freqs, nu_DM, nu_GM, nu_tau, log10_tau), \
        np.array([bool(f) for f in fit_flags], dtype=float)


def fit_function(params, *args):
    """pptoaslib.py:525-542 (argument order of fit_portrait_full's other_args)."""
    a, _ = _split(args)
    t = channel_terms(params, *a)
    return -np.sum(t.C ** 2 / t.S)


def fit_function_deriv(params, *args):
    """pptoaslib.py:544-574."""
    a, flags = _split(args)
    t = channel_terms(params, *a)
    g = -np.sum((t.C ** 2 / t.S) * (2 * t.dC / t.C - t.dS / t.S), -1)
    return g * flags


def hessian_per_channel(t, flags):
    """H_ij,n of pptoaslib.py:619-630."""
    C, S, dC, dS, d2C, d2S = t.C, t.S, t.dC, t.dS, t.d2C, t.d2S
    H = -2 * (C ** 2 / S) * (d2C / C - 0.5 * d2S / S
                             + dC[:, None] * dC[None] / C ** 2
                             + dS[:, None] * dS[None] / S ** 2
                             - (dC[:, None] * dS[None] + dS[:, None] * dC[None]) / (C * S))
    return H * (flags[:, None] * flags[None])[..., None]


def fit_function_2deriv(params, *args, per_channel=False):
    """pptoaslib.py:576-643 (hessian only)."""
    a, flags = _split(args)
    t = channel_terms(params, *a)
    H = hessian_per_channel(t, flags)
    return H if per_channel else H.sum(-1)


def hessian_with_scales(params, *args):
    """Joint Hessian with amplitudes and its Woodbury inverse, pptoaslib.py:645-731.

    Returns (H[5+nchan,5+nchan], covariance[(nfit+nchan)^2], scales[nchan]).
    """
    a, flags = _split(args)
    t = channel_terms(params, *a)
    nchan = len(t.C)
    scales = t.C / t.S
    Hij = -2 * ((t.C ** 2 / t.S) * (t.d2C / t.C - 0.5 * t.d2S / t.S))
    Hij = Hij * (flags[:, None] * flags[None])[..., None]
    cross = -2 * (t.dC - scales * t.dS)                       # [5, nchan]
    H = np.zeros((5 + nchan, 5 + nchan))
    H[:5, :5] = Hij.sum(-1)
    H[5 + np.arange(nchan), 5 + np.arange(nchan)] = 2 * t.S
    H[5:, :5] = (cross * flags[:, None]).T
    H[:5, 5:] = cross * flags[:, None]
    ifit = np.where(flags)[0]
    A = H[:5, :5][np.ix_(ifit, ifit)]
    Cinv = 1.0 / (2 * t.S)
    U = cross[ifit]
    Xinv = np.linalg.inv(A - (U * Cinv) @ U.T)
    UR = -(Xinv @ U) * Cinv
    LL = -(Cinv[:, None] * U.T) @ Xinv
    LR = -(LL @ U) * Cinv + np.diag(Cinv)
    cov = 2.0 * np.block([[Xinv, UR], [LL, LR]])
    return H, cov, scales


def get_nu_zeros(params, dFT, mFT, errs_FT, P, freqs, nu_DM, nu_GM, nu_tau,
                 fit_flags, log10_tau, option=0):
    """Zero-covariance reference frequencies per flag set, pptoaslib.py:733-906."""
    phi, DM, GM, tau, alpha = params
    if log10_tau:
        tau = 10 ** tau
    flags = np.array([bool(f) for f in fit_flags], dtype=float)
    t = channel_terms(params, dFT, mFT, errs_FT, P, freqs, nu_DM, nu_GM, nu_tau,
                      log10_tau)
    Hn = hessian_per_channel(t, flags)
    dph = phase_shift_jacobian(freqs, nu_DM, nu_GM, P)
    taus = scattering_times(tau, alpha, freqs, nu_tau)
    dts, _ = _tau_jacobians(tau, freqs, nu_tau, log10_tau, taus)
    f2, f4, lnf = freqs ** -2, freqs ** -4, np.log(freqs)
    ff = list(int(bool(f)) for f in fit_flags)
    nz = [nu_DM, nu_GM, nu_tau]

    def closest_root(coeffs, sq):
        r = np.roots(coeffs)
        r = np.real(r[np.where(np.imag(r) == 0.0)[0]])
        r = r[np.where(r > 0.0)[0]]
        if sq:
            r = r ** 0.5
        return r[np.argmin(abs(freqs.mean() - r))]

    if ff == [1, 1, 0, 0, 0]:
        h = Hn[0, 1] / dph[1]
        nz[0] = (np.sum(f2 * h) / np.sum(h)) ** -0.5
    elif ff == [1, 0, 1, 0, 0]:
        h = Hn[0, 2] / dph[2]
        nz[1] = (np.sum(f4 * h) / np.sum(h)) ** -0.25
    elif ff == [0, 0, 0, 1, 1]:
        h = Hn[3, 4] / (dts[1] / taus)
        nz[2] = np.exp(np.sum(lnf * h) / np.sum(h))
    elif ff == [1, 1, 0, 1, 0]:
        H21, H23 = Hn[1, 0] / dph[1], Hn[1, 3] / dph[1]
        Hs = Hn.sum(-1)
        H13, H33 = Hs[3, 0], Hs[3, 3]
        num = H13 * np.sum(f2 * H23) - H33 * np.sum(f2 * H21)
        den = H13 * np.sum(H23) - H33 * np.sum(H21)
        nz[0] = (num / den) ** -0.5
    elif ff == [1, 1, 1, 0, 0]:
        if option in (0, 1):
            if option == 0:
                H21, H23 = Hn[1, 0] / dph[1], Hn[1, 2] / dph[1]
                H31, H33 = Hn[2, 0] / dph[2], Hn[2, 2] / dph[2]
                A, B = np.sum(H31 * f4), np.sum(H31)
                C, D = np.sum(H23 * f2), np.sum(H23)
                E, F = np.sum(H33 * f4), np.sum(H33)
                G, H = np.sum(H21 * f2), np.sum(H21)
            else:
                H21, H22 = Hn[1, 0] / dph[1], Hn[1, 1] / dph[1]
                H31, H32 = Hn[2, 0] / dph[2], Hn[2, 1] / dph[2]
                A, B = np.sum(H21 * f4), np.sum(H21)
                C, D = np.sum(H32 * f2), np.sum(H32)
                E, F = np.sum(H22 * f4), np.sum(H22)
                G, H = np.sum(H31 * f2), np.sum(H31)
            coeffs = [A * C - E * G, 0.0, E * H - A * D, 0.0, F * G - B * C, 0.0,
                      B * D - F * H]
            nz[0] = nz[1] = closest_root(coeffs, False)
    elif ff == [1, 1, 0, 1, 1]:
        # delete the GM row/column, pptoaslib.py:813-836
        keep = [0, 1, 3, 4]
        Hk = Hn[np.ix_(keep, keep)]
        H21, H23, H24 = (Hk[1, [0, 2, 3]] / dph[1])
        H41, H42, H43 = (Hk[3, [0, 1, 2]] / (dts[1] / taus))
        Hs = Hk.sum(-1)
        H11, H22, H33, H44 = np.diag(Hs)
        H12, H13, H14 = Hs[0, 1:]
        H23s, H24s = Hs[1, 2:]
        H34 = Hs[2, 3]
        a1 = H34 * H34 - H33 * H44
        a2 = H13 * H44 - H14 * H34
        a3 = H14 * H33 - H13 * H34
        num = a1 * np.sum(f2 * H21) + a2 * np.sum(f2 * H23) + a3 * np.sum(f2 * H24)
        den = a1 * np.sum(H21) + a2 * np.sum(H23) + a3 * np.sum(H24)
        nz[0] = (num / den) ** -0.5
        b1 = H13 * H22 - H12 * H23s
        b2 = H11 * H23s - H12 * H13
        b3 = H12 * H12 - H11 * H22
        num = b1 * np.sum(lnf * H41) + b2 * np.sum(lnf * H42) + b3 * np.sum(lnf * H43)
        den = b1 * np.sum(H41) + b2 * np.sum(H42) + b3 * np.sum(H43)
        nz[2] = np.exp(num / den)
    elif ff == [1, 1, 1, 1, 0]:
        if option in (0, 1):
            Hk = Hn[:4, :4]
            Hs = Hk.sum(-1)
            g2 = freqs ** -2 - nu_DM ** -2
            g4 = freqs ** -4 - nu_GM ** -4
            H14, H44 = Hs[3, 0], Hs[3, 3]
            if option == 0:
                H21, H23, H24 = Hk[1, [0, 2, 3]] / g2
                H31, H33, H34 = Hk[2, [0, 2, 3]] / g4
                A, a = np.sum(f4 * H34), np.sum(H34)
                B, b = np.sum(f2 * H21), np.sum(H21)
                C, c = np.sum(f4 * H31), np.sum(H31)
                D, d = np.sum(f2 * H23), np.sum(H23)
                E, e = np.sum(f4 * H33), np.sum(H33)
                F, f = np.sum(f2 * H24), np.sum(H24)
                coeffs = [A * A * B + H44 * C * D + H14 * E * F - H44 * B * E - A * C * F - H14 * A * D,
                          -A * A * b - H44 * C * d - H14 * E * f + H44 * b * E + A * C * f + H14 * A * d,
                          -2 * A * a * B - H44 * c * D - H14 * e * F + H44 * B * e + (A * c + a * C) * F + H14 * a * D,
                          2 * A * a * b + H44 * c * d + H14 * e * f - H44 * b * e - (A * c + a * C) * f - H14 * a * d,
                          a * a * B - a * c * F,
                          -a * a * b + a * c * f]
            else:
                H21, H22, H24 = Hk[1, [0, 1, 3]] / g2
                H31, H32, H34 = Hk[2, [0, 1, 3]] / g4
                A, a = np.sum(f2 * H24), np.sum(H24)
                B, b = np.sum(f4 * H31), np.sum(H31)
                C, c = np.sum(f2 * H21), np.sum(H21)
                D, d = np.sum(f4 * H32), np.sum(H32)
                E, e = np.sum(f2 * H22), np.sum(H22)
                F, f = np.sum(f4 * H34), np.sum(H34)
                coeffs = [A * A * B + H44 * C * D + H14 * E * F - H44 * B * E - A * C * F - H14 * A * D,
                          -2 * A * a * B - H44 * c * D - H14 * e * F + H44 * B * e + (A * c + a * C) * F + H14 * a * D,
                          -(A * A * b - a * a * B) - H44 * C * d - H14 * E * f + H44 * b * E + (A * C * f - a * c * F) + H14 * A * d,
                          2 * A * a * b + H44 * c * d + H14 * e * f - H44 * b * e - (A * c + a * C) * f - H14 * a * d,
                          -a * a * b + a * c * f]
            nz[0] = nz[1] = closest_root(coeffs, True)
    elif ff == [1, 1, 1, 1, 1]:
        return get_nu_zeros(params, dFT, mFT, errs_FT, P, freqs, nu_DM, nu_GM,
                            nu_tau, [1, 1, 0, 1, 1], log10_tau, option)
    return nz


# ---------------------------------------------------------------------------
# L3 fit API
# ---------------------------------------------------------------------------
TRUST_NCG_OPTIONS = {"gtol": -1}


def fit_portrait_full(data_port, model_port, init_params, P, freqs,
                      nu_fits=(None, None, None), nu_outs=(None, None, None),
                      errs=None, fit_flags=(1, 1, 1, 1, 1), bounds=None,
                      log10_tau=True, option=0, method="trust-ncg"):
    """Restatement of pptoaslib.fit_portrait_full, pptoaslib.py:928-1096."""
    freqs = np.asarray(freqs, dtype=float)
    fit_flags = list(fit_flags)
    ifit = np.where(fit_flags)[0]
    nfit = len(ifit)
    nbin = data_port.shape[-1]
    dof = data_port.size - (nfit + len(freqs))
    dFT = np.fft.rfft(data_port, axis=-1)
    dFT[:, 0] *= F0_FACT
    mFT = np.fft.rfft(model_port, axis=-1)
    mFT[:, 0] *= F0_FACT
    if errs is None:
        errs = get_noise_PS(data_port, chans=True)
    errs_FT = np.asarray(errs) * np.sqrt(nbin / 2.0)
    Sd = np.sum((np.abs(dFT) ** 2).T / errs_FT ** 2.0)
    nu_fit = [f if f is not None else freqs.mean() for f in nu_fits]
    other = (dFT, mFT, errs_FT, P, freqs, nu_fit[0], nu_fit[1], nu_fit[2],
             [bool(f) for f in fit_flags], log10_tau)
    if method == "trust-ncg":
        kw = dict(hess=fit_function_2deriv, options={"gtol": -1})
    elif method == "Newton-CG":
        kw = dict(hess=fit_function_2deriv,
                  options={"maxiter": 2000, "disp": False, "xtol": -1})
    elif method == "TNC":
        kw = dict(bounds=bounds, options={"maxiter": 2000, "disp": False,
                                          "xtol": 1e-10, "minfev": dof - Sd})
    else:
        raise ValueError("Method '%s' is not implemented." % method)
    t0 = time.time()
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", opt.OptimizeWarning)
        res = opt.minimize(fit_function, init_params, args=other, method=method,
                           jac=fit_function_deriv, **kw)
    duration = time.time() - t0
    phi_f, DM_f, GM_f, tau_f, alpha_f = res.x
    nu_out = list(nu_outs)
    if not bool(np.all(nu_outs)):
        nz = get_nu_zeros(res.x, dFT, mFT, errs_FT, P, freqs, nu_fit[0],
                          nu_fit[1], nu_fit[2], fit_flags, log10_tau, option)
        nu_out = [nz[i] if nu_out[i] is None else nu_out[i] for i in range(3)]
    if fit_flags[1]:
        nu_out[1] = nu_out[0]
    elif fit_flags[2]:
        nu_out[0] = nu_out[1]
    phi_inf = phase_shifts(phi_f, DM_f, GM_f, np.inf, nu_fit[0], nu_fit[1], P)
    phi_out = phi_inf + DCONST / P * DM_f * nu_out[0] ** -2 + \
        DCONST ** 2 / P * GM_f * nu_out[1] ** -4
    if abs(phi_out) >= 0.5:
        phi_out %= 1
    if phi_out >= 0.5:
        phi_out -= 1.0
    tau_lin = 10 ** tau_f if log10_tau else tau_f
    tau_out = scattering_times(tau_lin, alpha_f, nu_out[2], nu_fit[2])
    taus = scattering_times(tau_out, alpha_f, freqs, nu_out[2])
    if log10_tau:
        tau_out = np.log10(tau_out)
    params = [phi_out, DM_f, GM_f, tau_out, alpha_f]
    param_errs = np.zeros(5)
    H, cov, scales = hessian_with_scales(
        params, dFT, mFT, errs_FT, P, freqs, nu_out[0], nu_out[1], nu_out[2],
        fit_flags, log10_tau)
    all_errs = np.diag(cov) ** 0.5
    param_errs[ifit] = all_errs[:nfit]
    scale_errs = all_errs[nfit:]
    B = scattering_portrait_FT(taus, nbin)
    S = np.sum(np.abs(B) ** 2 * np.abs(mFT) ** 2, -1) / errs_FT ** 2
    channel_snrs = scales * np.sqrt(S)
    chi2 = Sd + res.fun
    return Bunch(params=params, param_errs=param_errs, phi=phi_out,
                 phi_err=param_errs[0], DM=DM_f, DM_err=param_errs[1], GM=GM_f,
                 GM_err=param_errs[2], tau=tau_out, tau_err=param_errs[3],
                 alpha=alpha_f, alpha_err=param_errs[4], scales=scales,
                 scale_errs=scale_errs, nu_DM=nu_out[0], nu_GM=nu_out[1],
                 nu_tau=nu_out[2], covariance_matrix=cov[:nfit, :nfit],
                 chi2=chi2, red_chi2=chi2 / dof,
                 snr=np.sqrt(np.sum(channel_snrs ** 2)),
                 channel_snrs=channel_snrs, duration=duration,
                 nfeval=res.nfev, return_code=res.status)


def _phase_shift_fn(phase, model, data, err):
    """pplib.py:1244-1256."""
    k = np.arange(len(model))
    return -np.real(np.sum(data * np.conj(model) * np.exp(2.0j * np.pi * k * phase))) / err ** 2


def _phase_shift_2deriv(phase, model, data, err):
    """pplib.py:1270-1280."""
    k = np.arange(len(model))
    return -np.real(np.sum(-4.0 * np.pi ** 2 * k ** 2 * data * np.conj(model)
                           * np.exp(2.0j * np.pi * k * phase))) / err ** 2


def fit_phase_shift(data, model, noise=None, bounds=(-0.5, 0.5), Ns=100):
    """Brute-force FFTFIT + Nelder-Mead polish, pplib.py:2054-2100."""
    data = np.asarray(data, dtype=float)
    nbin = len(data)
    dFT = np.fft.rfft(data)
    dFT[0] *= F0_FACT
    mFT = np.fft.rfft(model)
    mFT[0] *= F0_FACT
    if noise is None:
        err = get_noise_PS(data) * np.sqrt(nbin / 2.0)
    else:
        err = noise * np.sqrt(nbin / 2.0)
    d = np.real(np.sum(dFT * np.conj(dFT))) / err ** 2
    p = np.real(np.sum(mFT * np.conj(mFT))) / err ** 2
    t0 = time.time()
    res = opt.brute(_phase_shift_fn, [tuple(bounds)], args=(mFT, dFT, err),
                    Ns=Ns, full_output=True)
    duration = time.time() - t0
    phase = res[0][0]
    fmin = res[1]
    scale = -fmin / p
    return Bunch(phase=phase,
                 phase_err=(scale * _phase_shift_2deriv(phase, mFT, dFT, err)) ** -0.5,
                 scale=scale, scale_err=p ** -0.5, snr=(scale ** 2 * p) ** 0.5,
                 red_chi2=(d - fmin ** 2 / p) / (nbin - 2), duration=duration)


# Legacy phase+DM TNC fit, pplib.py:1282-1391 and 2102-2204 --------------------
def _legacy_terms(params, model, p_n, data, errs, P, freqs, nu_ref):
    phase, DM = params
    D = DCONST * DM / P
    k = np.arange(model.shape[1])
    ph = phase + D * (freqs ** -2.0 - nu_ref ** -2.0)
    W = data * np.conj(model) * np.exp(2.0j * np.pi * np.outer(ph, k))
    C = np.real(W).sum(-1)
    C1 = np.real(2.0j * np.pi * k * W).sum(-1)
    C2 = np.real((2.0j * np.pi * k) ** 2 * W).sum(-1)
    dDM = (freqs ** -2.0 - nu_ref ** -2.0) * (DCONST / P)
    return C, C1, C2, dDM, errs ** 2 * p_n


def legacy_function(params, model, p_n, data, errs, P, freqs, nu_ref):
    C, _, _, _, w = _legacy_terms(params, model, p_n, data, errs, P, freqs, nu_ref)
    return -np.sum(C ** 2 / w)


def legacy_deriv(params, model, p_n, data, errs, P, freqs, nu_ref):
    C, C1, _, dDM, w = _legacy_terms(params, model, p_n, data, errs, P, freqs, nu_ref)
    return np.array([np.sum(-2 * C * C1 / w), np.sum(-2 * C * C1 * dDM / w)])


def legacy_2deriv(params, model, p_n, data, errs, P, freqs, nu_ref):
    C, C1, C2, dDM, w = _legacy_terms(params, model, p_n, data, errs, P, freqs, nu_ref)
    Wn = (C1 ** 2 + C * C2) / w
    d2 = np.array([np.sum(-2 * Wn), np.sum(-2 * Wn * dDM ** 2), np.sum(-2 * Wn * dDM)])
    return d2, (Wn.sum() / np.sum(Wn * freqs ** -2)) ** 0.5


def fit_portrait(data, model, init_params, P, freqs, nu_fit=None, nu_out=None,
                 errs=None, bounds=((None, None), (None, None))):
    """pplib.py:2102-2204 (scipy TNC)."""
    freqs = np.asarray(freqs, dtype=float)
    dFT = np.fft.rfft(data, axis=1)
    dFT[:, 0] *= F0_FACT
    mFT = np.fft.rfft(model, axis=1)
    mFT[:, 0] *= F0_FACT
    if errs is None:
        errs = get_noise_PS(data, chans=True) * np.sqrt(len(data[0]) / 2.0)
    else:
        errs = np.copy(errs) * np.sqrt(len(data[0]) / 2.0)
    d = np.real(np.sum((errs ** -2.0 * (dFT * np.conj(dFT)).T).T))
    p_n = np.real(np.sum(mFT * np.conj(mFT), axis=1))
    if nu_fit is None:
        nu_fit = freqs.mean()
    args = (mFT, p_n, dFT, errs, P, freqs, nu_fit)
    t0 = time.time()
    with warnings.catch_warnings():
        # the reference passes 'maxiter', which scipy's TNC ignores (it warns
        # and keeps its default maxfun); pass the same options verbatim.
        warnings.simplefilter("ignore", opt.OptimizeWarning)
        res = opt.minimize(legacy_function, init_params, args=args,
                           method="TNC", jac=legacy_deriv, bounds=bounds,
                           options={"maxiter": 1000, "disp": False,
                                    "xtol": 1e-10})
    duration = time.time() - t0
    phi, DM = res.x
    nu_zero = legacy_2deriv(np.array([phi, DM]), *args)[1]
    if nu_out is None:
        nu_out = nu_zero
    phi_out = phase_transform(phi, DM, nu_fit, nu_out, P, mod=True)
    h = legacy_2deriv(np.array([phi_out, DM]), mFT, p_n, dFT, errs, P, freqs, nu_out)[0]
    cov = np.linalg.inv(0.5 * np.array([[h[0], h[2]], [h[2], h[1]]]))
    dof = data.size - (len(freqs) + 2)
    chi2 = d + res.fun
    k = np.arange(mFT.shape[1])
    ph = phi + DCONST * DM / P * (freqs ** -2.0 - nu_fit ** -2.0)
    scales = np.real(np.sum(dFT * np.conj(mFT) * np.exp(2.0j * np.pi * np.outer(ph, k)),
                            axis=1)) / p_n
    return Bunch(phase=phi_out, phase_err=cov[0, 0] ** 0.5, DM=DM,
                 DM_err=cov[1, 1] ** 0.5, scales=scales,
                 scale_errs=(p_n / errs ** 2.0) ** -0.5, nu_ref=nu_out,
                 covariance=cov[0, 1], chi2=chi2, red_chi2=chi2 / dof,
                 snr=np.sum(scales ** 2.0 * p_n / errs ** 2.0) ** 0.5,
                 duration=duration, nfeval=res.nfev, return_code=res.status)


# ---------------------------------------------------------------------------
# L4 per-subint driver steps (pptoas.py:383-530, ppalign.py:160-208)
# ---------------------------------------------------------------------------
def pptoas_guess(portx, modelx, freqsx, weightsx, DM_guess, P, nu_fit_DM,
                 Ns=100, nu_rot=None, wrap=True, model_prof=None, tau_guess=0.0):
    """Initial phase guess of get_TOAs, pptoas.py:420-456.

    Dedisperse at nu_rot (default: mean frequency), average with channel
    weights, brute-force FFTFIT against the mean model profile (scattered by
    tau_guess [rot] when fitting scattering, pptoas.py:441-444), then move
    the phase to nu_fit_DM.
    """
    nu_mean = freqsx.mean() if nu_rot is None else nu_rot
    rot = rotate_data(portx, 0.0, DM_guess, P, freqsx, nu_mean)
    prof = np.average(rot, axis=0, weights=weightsx)
    mp = modelx.mean(axis=0) if model_prof is None else model_prof
    if tau_guess:
        nbin = len(mp)
        mp = np.fft.irfft(scattering_portrait_FT(np.array([tau_guess]), nbin)[0] *
                          np.fft.rfft(mp))
    phi = fit_phase_shift(prof, mp, Ns=Ns).phase
    if not wrap:
        return phi
    return phase_transform(phi, DM_guess, nu_mean, nu_fit_DM, P, mod=True)


def fit_subint_pptoas(portx, modelx, freqsx, weightsx, errs, SNRsx, P, DM_stored,
                      fit_flags=(1, 1, 0, 0, 0), Ns=100, log10_tau=False,
                      tau_guess=0.0, alpha_guess=0.0):
    """One TOA of get_TOAs (guess + fit), pptoas.py:383-488.  For scattering
    fits tau_guess [rot] at nu_fit scatters the guess template and starts the
    fit (log10 of it with log10_tau; 1/nbin when 0, pptoas.py:441-450)."""
    nu_fit = guess_fit_freq(freqsx, SNRsx)
    phi_guess = pptoas_guess(portx, modelx, freqsx, weightsx, DM_stored, P,
                             nu_fit, Ns, tau_guess=tau_guess)
    tau0 = tau_guess
    if log10_tau:
        tau0 = np.log10(tau0 if tau0 else 1.0 / portx.shape[-1])
    init = [phi_guess, DM_stored, 0.0, tau0, alpha_guess]
    res = fit_portrait_full(portx, modelx, init, P, freqsx,
                            [nu_fit, nu_fit, nu_fit], [None, None, None], errs,
                            list(fit_flags), log10_tau=log10_tau, option=0)
    res.init = init
    res.nu_fit = nu_fit
    return res


# ---------------------------------------------------------------------------
# Template producers (SURVEY §8(f) #2 and pptoas.py:387-393)
# ---------------------------------------------------------------------------
def gen_spline_portrait(mean_prof, freqs, eigvec, tck, nbin=None):
    """pplib.py:932-956: FITPACK splev (ext=0) of the B-spline curve at the
    frequencies, projected back through the eigenvectors, plus the mean
    profile; scipy.signal.resample and rotate_portrait (pplib.py:2428-2460)
    when nbin differs from len(mean_prof)."""
    import scipy.interpolate as si
    import scipy.signal as ss
    freqs = np.atleast_1d(freqs)
    if not eigvec.shape[1]:
        port = np.tile(mean_prof, len(freqs)).reshape(len(freqs), len(mean_prof))
    else:
        proj_port = np.array(si.splev(freqs, tck, der=0, ext=0)).T
        port = np.dot(proj_port, eigvec.T) + mean_prof
    if nbin is not None and len(mean_prof) != nbin:
        shift = 0.5 * (nbin ** -1 - len(mean_prof) ** -1)
        port = ss.resample(port, nbin, axis=1)
        pFFT = np.fft.rfft(port, axis=1)
        pFFT *= np.exp(np.arange(pFFT.shape[1]) * 2.0j * np.pi * shift)
        port = np.fft.irfft(pFFT, axis=1)
    return port


def instrumental_response_FT(nbin, wid=0.0, irf_type="rect"):
    """pptoaslib.py:112-143 (with gaussian_profile_FT, pptoaslib.py:14-50)."""
    from scipy.special import erf
    nharm = nbin // 2 + 1
    if wid == 0.0:
        return np.ones(nharm)
    if irf_type == "rect":
        return np.sinc(np.arange(nharm) * wid)
    sigma = wid / (2 * np.sqrt(2 * np.log(2)))
    amp = (2 * np.pi * sigma ** 2) ** 0.5
    sigma = 1 / (sigma * 2 * np.pi)
    harmind = np.arange(nharm)
    a = sigma / ((1.0 / np.pi) * 2 ** 0.5)
    b = harmind / (sigma * 2 ** 0.5)
    gp = np.nan_to_num(np.exp(-b ** 2) * (erf(a - b * 1j) + erf(a + b * 1j)) / 2 * amp * nbin)
    return gp / gp[0]


def instrumental_response_port_FT(nbin, freqs, DM=0.0, P=1.0, wids=(), irf_types=()):
    """pptoaslib.py:145-179: product of the responses; DM switches on a rect
    smearing response of width 8.3e-6 chan_bw / (freq / 1e3)^3 / P."""
    nharm = nbin // 2 + 1
    nchan = len(freqs)
    if DM == len(wids) == 0.0:
        return np.ones([nchan, nharm])
    R = np.ones([nchan, nharm], dtype=complex)
    for wid, t in zip(wids, irf_types):
        R *= np.tile(instrumental_response_FT(nbin, wid, t), nchan).reshape(nchan, nharm)
    if DM:
        chan_bw = abs(freqs[1] - freqs[0])
        for ichan, freq in enumerate(freqs):
            wid = 8.3e-6 * chan_bw / (freq / 1e3) ** 3 / P
            R[ichan] *= instrumental_response_FT(nbin, wid, "rect")
    return R
