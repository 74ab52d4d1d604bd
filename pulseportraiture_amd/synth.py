"""Synthetic wideband archives (SURVEY.md §8(d) recipe).

Template from a Gaussian-component model (examples/example.gmodel layout),
P = 1/345.67890123456789 s, nu0 = 1500 MHz, bw = 800 MHz, injected
phi ~ U(-0.1, 0.1) rot and dDM ~ N(3e-4, 2e-4) (examples/example.py:28-31),
white noise sigma = 1.5.  Every random number comes from a counter-based
Philox4x32-10 stream keyed by (seed; bin pair, channel, subint), so the GPU
(ppf_synth_portraits) and this host version regenerate the same portraits
(to fp64 rounding) for any subint without replaying a sequential RNG.
"""
import os

import numpy as np

from . import pplib

HERE = os.path.dirname(os.path.abspath(__file__))
EXAMPLE_GMODEL = os.path.join(HERE, "data", "example.gmodel")
P_EXAMPLE = 1.0 / 345.67890123456789   # examples/example.par:4
DM_EXAMPLE = 34.56789                   # examples/example.par:8

_M0, _M1 = 0xD2511F53, 0xCD9E8D57
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_MASK = 0xFFFFFFFF


def philox4x32_10(c0, c1, c2, c3, seed):
    """Vectorised Philox4x32-10 (uint64 arrays holding 32-bit words)."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & _MASK for c in (c0, c1, c2, c3))
    k0 = np.uint64(seed & _MASK)
    k1 = np.uint64((seed >> 32) & _MASK)
    for _ in range(10):
        p0 = np.uint64(_M0) * c0
        p1 = np.uint64(_M1) * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(_MASK)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(_MASK)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + np.uint64(_W0)) & np.uint64(_MASK)
        k1 = (k1 + np.uint64(_W1)) & np.uint64(_MASK)
    return c0, c1, c2, c3


def philox_normal2(c0, c1, c2, c3, seed):
    """Two N(0,1) deviates per counter (Box-Muller on 53-bit uniforms)."""
    x0, x1, x2, x3 = philox4x32_10(c0, c1, c2, c3, seed)
    s53 = 2.0 ** -53
    u1 = ((x0 >> np.uint64(5)).astype(np.float64) * 67108864.0 +
          (x1 >> np.uint64(6)).astype(np.float64) + 0.5) * s53
    u2 = ((x2 >> np.uint64(5)).astype(np.float64) * 67108864.0 +
          (x3 >> np.uint64(6)).astype(np.float64)) * s53
    r = np.sqrt(-2.0 * np.log(u1))
    return r * np.cos(2.0 * np.pi * u2), r * np.sin(2.0 * np.pi * u2)


def noise_block(nsub, nchan, nbin, sigma, seed, sub0=0):
    """sigma * N(0,1) for subints sub0 .. sub0+nsub-1 (device layout)."""
    s = np.arange(nsub, dtype=np.uint64)[:, None, None] + np.uint64(sub0)
    n = np.arange(nchan, dtype=np.uint64)[None, :, None]
    nh = (nbin + 1) // 2  # odd nbin: the last pair's second value unused
    j = np.arange(nh, dtype=np.uint64)[None, None, :]
    shape = (nsub, nchan, nh)
    z0, z1 = philox_normal2(np.broadcast_to(j, shape), np.broadcast_to(n, shape),
                            np.broadcast_to(s & np.uint64(_MASK), shape),
                            np.broadcast_to(s >> np.uint64(32), shape), seed)
    out = np.empty((nsub, nchan, nbin))
    out[..., 0::2] = z0
    out[..., 1::2] = z1[..., :nbin // 2]
    return sigma * out


def synth_portraits_host(model, phase, sigma, seed, sub0=0):
    """Host twin of ppf_synth_portraits: irfft(rfft(model) e^{2 pi i k phase}) + noise."""
    model = np.asarray(model, dtype=np.float64)
    nchan, nbin = model.shape
    phase = np.asarray(phase, dtype=np.float64).reshape(-1, nchan)
    k = np.arange(nbin // 2 + 1)
    spec = np.fft.rfft(model, axis=-1)
    rot = np.fft.irfft(spec[None] * np.exp(2j * np.pi * phase[..., None] * k), nbin, axis=-1)
    if sigma:
        rot = rot + noise_block(phase.shape[0], nchan, nbin, sigma, seed, sub0)
    return rot


def injected_params(nsub, seed, sub0=0):
    """phi ~ U(-0.1, 0.1), dDM ~ N(3e-4, 2e-4) per subint (examples/example.py:29-31).

    Drawn from the same Philox stream with channel index 0xFFFFFFFF, so every
    subint's injection is independent of how the batch is split.
    """
    s = np.arange(nsub, dtype=np.uint64) + np.uint64(sub0)
    x0, x1, x2, x3 = philox4x32_10(np.zeros(nsub, np.uint64), np.full(nsub, _MASK, np.uint64),
                                   s & np.uint64(_MASK), s >> np.uint64(32), seed)
    u = ((x0 >> np.uint64(5)).astype(np.float64) * 67108864.0 +
         (x1 >> np.uint64(6)).astype(np.float64)) * 2.0 ** -53
    z0, _ = philox_normal2(np.ones(nsub, np.uint64), np.full(nsub, _MASK, np.uint64),
                           s & np.uint64(_MASK), s >> np.uint64(32), seed)
    return -0.1 + 0.2 * u, 3e-4 + 2e-4 * z0


def channel_freqs(nchan, nu0=1500.0, bw=800.0):
    """Channel centres, pplib.py:3242-3246."""
    cw = bw / nchan
    lo = nu0 - bw / 2.0
    return np.linspace(lo + cw / 2.0, lo + bw - cw / 2.0, nchan)


class Workload(pplib.DataBunch):
    pass


def make_workload(nsub, nchan, nbin, seed=20240917, sub0=0, sigma=1.5, tau=0.0,
                  alpha=-4.0, gm=0.0, nu_ref=1500.0, modelfile=None, P=P_EXAMPLE,
                  DM0=DM_EXAMPLE):
    """Inputs of one synthetic batch (no data yet): template, freqs, phases.

    phase[s, n] = -(phi_s + Dconst (DM0 + dDM_s)(nu_n^-2 - nu_ref^-2)/P
                    + Dconst^2 GM (nu_n^-4 - nu_ref^-4)/P)
    i.e. the template dispersed the way rotate_portrait_full(model, -phi,
    -DM, -GM, ...) does (pptoaslib.py:52-81), plus optional scattering of the
    template at nu_ref (tau in rot, pplib.py:4055-4101).
    """
    freqs = channel_freqs(nchan)
    phases = pplib.get_bin_centers(nbin)
    _, _, model = pplib.read_model(modelfile or EXAMPLE_GMODEL, phases, freqs, P, quiet=True)
    template = model
    if tau:
        taus = pplib.scattering_times(tau, alpha, freqs, nu_ref)
        template = np.fft.irfft(pplib.scattering_portrait_FT(taus, nbin) *
                                np.fft.rfft(model, axis=-1), nbin, axis=-1)
    phi, dDM = injected_params(nsub, seed, sub0)
    D = pplib.Dconst
    rot = -(phi[:, None] + D * (DM0 + dDM)[:, None] * (freqs ** -2 - nu_ref ** -2) / P
            + D ** 2 * gm * (freqs ** -4 - nu_ref ** -4) / P)
    return Workload(nsub=nsub, nchan=nchan, nbin=nbin, seed=seed, sub0=sub0, sigma=sigma,
                    freqs=freqs, model=model, template=template, phase=rot, phi=phi, dDM=dDM,
                    P=P, DM0=DM0, nu_ref=nu_ref, tau=tau, alpha=alpha, gm=gm)


def workload_data_host(w):
    return synth_portraits_host(w.template, w.phase, w.sigma, w.seed, w.sub0)


def _data_chunk(args):
    nsub, nchan, nbin, seed, sub0, kw = args
    return np.stack([workload_data_host(make_workload(1, nchan, nbin, seed=seed, sub0=sub0 + i,
                                                      **kw))[0] for i in range(nsub)])


def workload_data_host_parallel(nsub, nchan, nbin, seed=20240917, sub0=0, procs=8, chunk=64,
                                **kw):
    """Subints sub0 .. sub0 + nsub - 1, each generated alone (bitwise what
    workload_data_host(make_workload(1, ..., sub0=i)) gives; a batched irfft
    can differ in the last bit), in `procs` spawned worker processes (no
    fork: the caller may own a GPU context)."""
    import multiprocessing as mp
    jobs = [(min(chunk, nsub - lo), nchan, nbin, seed, sub0 + lo, kw)
            for lo in range(0, nsub, chunk)]
    out = np.empty((nsub, nchan, nbin))
    with mp.get_context("spawn").Pool(procs) as pool:
        for j, part in zip(range(0, nsub, chunk), pool.imap(_data_chunk, jobs)):
            out[j:j + len(part)] = part
    return out
