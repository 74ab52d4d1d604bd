#!/usr/bin/env python3
"""Generate golden fixtures from the reference PulsePortraiture source.

TEST INFRASTRUCTURE ONLY.  Run in the build container (where /root/reference
exists); never on the GPU box and never by the product.  The reference is
Python 2, so it is loaded through the scratch shim recipe of SURVEY.md §8(c):

  1. copy /root/reference/{pplib,pptoaslib,pptoas,ppalign,telescope_codes}.py
     into a temporary directory OUTSIDE the repository;
  2. python -m lib2to3 -w -n on those copies;
  3. mechanical Python-3 fixes: integer '/' -> '//' where the code needs ints
     (pplib.py:839,2572,2864,4075,4090; pptoaslib.py:34,130,164), numpy-2
     dtype 'complex_' -> 'complex128' (pplib.py:4094, pptoaslib.py:169), the
     exec-unpack loop at pptoas.py:277-278 replaced by explicit assignments and
     the exec flag-append in write_TOAs (pplib.py:3486-3503) by direct '+=';
  4. an in-process 'psrchive' module exposing only MJD (the hot path never
     calls PSRCHIVE; MJD arithmetic is needed to turn phases into TOAs);
  5. MPLBACKEND=Agg.

Only numbers (inputs and outputs) are written into tests/golden/; no reference
source, bytecode or shim text is kept.  Seeds are fixed, so rerunning this
script reproduces the fixtures (numpy 2.2.6 / scipy 1.15.3 in this image).

Usage:  python tests/golden/make_golden.py
"""
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
REF_FILES = ["pplib.py", "pptoaslib.py", "pptoas.py", "ppalign.py",
             "telescope_codes.py"]

# Keys of the load_data DataBunch (pplib.py:2809-2819).
LOAD_DATA_KEYS = ["arch", "backend", "backend_delay", "bw", "doppler_factors",
                  "DM", "dmc", "epochs", "filename", "flux_prof", "freqs",
                  "frontend", "integration_length", "masks", "nbin", "nchan",
                  "noise_stds", "npol", "nsub", "nu0", "ok_ichans", "ok_isubs",
                  "parallactic_angles", "phases", "prof", "prof_noise",
                  "prof_SNR", "Ps", "SNRs", "source", "state", "subints",
                  "subtimes", "telescope", "telescope_code", "weights"]


# --------------------------------------------------------------------------
# psrchive stand-in: only the MJD value type (days, secs, fracsec) is needed.
# --------------------------------------------------------------------------
class MJD(object):
    def __init__(self, *args):
        if len(args) == 0:
            self.days, self.secs, self.fracsec = 0, 0, 0.0
        elif len(args) == 1:
            dd = float(args[0])
            days = int(dd)
            fdays = dd - days
            secs = int(fdays * 86400.0)
            self.days, self.secs, self.fracsec = days, secs, fdays * 86400.0 - secs
        else:
            self.days, self.secs, self.fracsec = int(args[0]), int(args[1]), float(args[2])
        self._settle()

    def _settle(self):
        isec = int(np.floor(self.fracsec))
        self.secs += isec
        self.fracsec -= isec
        iday = self.secs // 86400
        self.days += iday
        self.secs -= iday * 86400

    def __add__(self, other):
        if not isinstance(other, MJD):
            other = MJD(0, 0, float(other))  # PSRCHIVE: MJD + double adds seconds
        return MJD(self.days + other.days, self.secs + other.secs,
                   self.fracsec + other.fracsec)

    __radd__ = __add__

    def __iadd__(self, other):
        return self.__add__(other)

    def in_days(self):
        return self.days + (self.secs + self.fracsec) / 86400.0

    def intday(self):
        return self.days

    def fracday(self):
        return (self.secs + self.fracsec) / 86400.0


def _psrchive_module():
    mod = types.ModuleType("psrchive")
    mod.MJD = MJD

    def Archive_load(fname):
        raise RuntimeError("psrchive is not available in this container")
    mod.Archive_load = Archive_load
    return mod


def build_shim():
    tmp = tempfile.mkdtemp(prefix="ppref_shim_")
    for f in REF_FILES:
        shutil.copy(os.path.join(REF, f), tmp)
    subprocess.check_call([sys.executable, "-m", "lib2to3", "-w", "-n"]
                          + REF_FILES, cwd=tmp, stdout=subprocess.DEVNULL,
                          stderr=subprocess.DEVNULL)

    def sub(fname, pattern, repl, count_min=1):
        p = os.path.join(tmp, fname)
        txt = open(p).read()
        new, n = re.subn(pattern, repl, txt)
        assert n >= count_min, (fname, pattern)
        open(p, "w").write(new)

    for f in ["pplib.py", "pptoaslib.py"]:
        sub(f, r"nbin/2 \+ 1", "nbin//2 + 1")
        sub(f, r"'complex_'", "'complex128'")
    sub("pplib.py", r"\(len\((\w+)\) - 2\) / (\d)", r"(len(\1) - 2) // \2", 3)
    sub("pplib.py", r"arr\.size/2", "arr.size//2")
    # pptoas.py:277-278: exec-unpack of the load_data bunch into locals.
    assign = "\n".join("                %s = data['%s']" % (k, k)
                       for k in LOAD_DATA_KEYS)
    sub("pptoas.py",
        r"            for key in list\(data\.keys\(\)\):\n                exec\(key \+ \" = data\['\" \+ key \+ \"'\]\"\)",
        "            if True:\n" + assign, 1)
    # pplib.py:3486-3503: exec-based string append in write_TOAs.
    sub("pplib.py", r"exec\(\"toa_string \+= '( -%s %[^']+)'\"%\(flag, value\)\)",
        r"toa_string += '\1'%(flag, value)", 2)
    sub("pplib.py", r"exec\(\"toa_string \+= '( -%s %[^']+)'\"%\(flag,\s*\n\s*toa\.flags\[flag\]\)\)",
        r"toa_string += '\1'%(flag, toa.flags[flag])", 4)
    return tmp


def load_reference():
    os.environ.setdefault("MPLBACKEND", "Agg")
    import matplotlib
    matplotlib.use("Agg")
    sys.modules["psrchive"] = _psrchive_module()
    tmp = build_shim()
    sys.path.insert(0, tmp)
    import io
    import contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        import pplib
        import pptoaslib
        import pptoas
        import ppalign
    return tmp, pplib, pptoaslib, pptoas, ppalign


# --------------------------------------------------------------------------
# Synthetic inputs (numbers only; the recipe mirrors SURVEY.md §8(d)).
# --------------------------------------------------------------------------
GMODEL = os.path.join(REF, "examples", "example.gmodel")
P0 = 1.0 / 345.67890123456789  # examples/example.par:4
DM0 = 34.56789                  # examples/example.par:8


def channel_freqs(nchan, nu0=1500.0, bw=800.0):
    # pplib.py:3242-3246
    cw = bw / nchan
    lo = nu0 - bw / 2.0
    return np.linspace(lo + cw / 2.0, lo + bw - cw / 2.0, nchan)


def make_portrait(ref, rng, nchan, nbin, phi, dDM, noise, tau=0.0, alpha=-4.0,
                  nu_ref=1500.0, gmodel=GMODEL):
    pplib, pptoaslib = ref
    freqs = channel_freqs(nchan)
    phases = pplib.get_bin_centers(nbin)
    _, _, model = pplib.read_model(gmodel, phases, freqs, P0, quiet=True)
    m = model
    if tau:
        taus = pplib.scattering_times(tau, alpha, freqs, nu_ref)
        m = np.fft.irfft(pplib.scattering_portrait_FT(taus, nbin)
                         * np.fft.rfft(m, axis=-1), axis=-1)
    data = pptoaslib.rotate_portrait_full(m, -phi, -(DM0 + dDM), 0.0, freqs,
                                          nu_ref, np.inf, P0)
    data = data + rng.normal(0.0, noise, data.shape)
    return freqs, model, data


def save(name, **arrs):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrs)
    print("wrote", path, os.path.getsize(path), "bytes")


FLAG_SETS = [[1, 0, 0, 0, 0], [1, 1, 0, 0, 0], [1, 0, 1, 0, 0], [1, 1, 1, 0, 0],
             [1, 1, 0, 1, 1], [1, 1, 0, 1, 0], [0, 0, 0, 1, 1], [1, 1, 1, 1, 0],
             [1, 1, 1, 1, 1]]


def gen_models(pplib):
    out = {}
    for (nchan, nbin) in [(8, 64), (16, 256), (64, 512)]:
        freqs = channel_freqs(nchan)
        phases = pplib.get_bin_centers(nbin)
        _, _, model = pplib.read_model(GMODEL, phases, freqs, P0, quiet=True)
        out["freqs_%dx%d" % (nchan, nbin)] = freqs
        out["phases_%dx%d" % (nchan, nbin)] = phases
        out["model_%dx%d" % (nchan, nbin)] = model
    # scattered template: TAU != 0 in the model file exercises read_model's
    # TAU*nbin/P conversion and gen_gaussian_portrait's scattering branch.
    tmpg = os.path.join(tempfile.mkdtemp(), "scat.gmodel")
    txt = open(GMODEL).read().replace("TAU     0.00000000 1",
                                      "TAU     0.00020000 1")
    open(tmpg, "w").write(txt)
    freqs = channel_freqs(16)
    phases = pplib.get_bin_centers(256)
    _, _, model = pplib.read_model(tmpg, phases, freqs, P0, quiet=True)
    out["model_scat_16x256"] = model
    out["freqs_scat_16x256"] = freqs
    out["phases_scat_16x256"] = phases
    save("models.npz", **out)


def gen_objective(pplib, pptoaslib):
    rng = np.random.default_rng(1234)
    out = {}
    cases = [dict(nchan=8, nbin=64, tau=0.0), dict(nchan=12, nbin=128, tau=3e-3)]
    for ic, c in enumerate(cases):
        freqs, model, data = make_portrait((pplib, pptoaslib), rng, c["nchan"],
                                           c["nbin"], 0.013, 2.5e-4, 0.5,
                                           tau=c["tau"])
        dFT = np.fft.rfft(data, axis=-1)
        dFT[:, 0] *= pplib.F0_fact
        mFT = np.fft.rfft(model, axis=-1)
        mFT[:, 0] *= pplib.F0_fact
        errs = pplib.get_noise(data, chans=True)
        errs_FT = errs * np.sqrt(c["nbin"] / 2.0)
        nu_fit = np.array([1480.0, 1490.0, 1470.0])
        out["c%d_data" % ic] = data
        out["c%d_model" % ic] = model
        out["c%d_freqs" % ic] = freqs
        out["c%d_errs" % ic] = errs
        out["c%d_nu_fit" % ic] = nu_fit
        ip = 0
        for log10_tau in [False, True]:
            for params in ([0.011, DM0 + 2.4e-4, 1.0e-6, 2.0e-3, -3.9],
                           [0.02, DM0 - 1e-4, 0.0, 0.0, -4.0],
                           [-0.2, DM0, 3e-6, 5e-4, -4.4]):
                p = list(params)
                if log10_tau:
                    if p[3] == 0.0:
                        continue
                    p[3] = np.log10(p[3])
                for flags in FLAG_SETS:
                    args = (dFT, mFT, errs_FT, P0, freqs, nu_fit[0], nu_fit[1],
                            nu_fit[2], flags, log10_tau)
                    key = "c%d_p%d" % (ic, ip)
                    f = pptoaslib.fit_portrait_full_function(p, *args)
                    g = pptoaslib.fit_portrait_full_function_deriv(p, *args)
                    H = pptoaslib.fit_portrait_full_function_2deriv(p, *args)
                    Hn = pptoaslib.fit_portrait_full_function_2deriv(
                        p, *args, per_channel=True)
                    try:
                        Hs, cov, scales = \
                            pptoaslib.fit_portrait_full_function_2deriv_with_scales(
                                p, *args, per_channel=False,
                                return_covariance_matrix=True, return_scales=True)
                    except np.linalg.LinAlgError:
                        Hs = cov = scales = np.array([np.nan])
                    import io
                    import contextlib
                    with contextlib.redirect_stdout(io.StringIO()):
                        try:
                            nz = pptoaslib.get_nu_zeros(p, dFT, mFT, errs_FT, P0,
                                                        freqs, nu_fit[0],
                                                        nu_fit[1], nu_fit[2],
                                                        flags, log10_tau, 0)
                        except (ValueError, IndexError):
                            nz = [np.nan] * 3
                    out[key + "_params"] = np.array(p)
                    out[key + "_flags"] = np.array(flags)
                    out[key + "_log10"] = np.array(log10_tau)
                    out[key + "_f"] = np.array(f)
                    out[key + "_g"] = np.array(g)
                    out[key + "_H"] = H
                    out[key + "_Hn"] = Hn
                    out[key + "_Hs"] = Hs
                    out[key + "_cov"] = cov
                    out[key + "_scales"] = scales
                    out[key + "_nz"] = np.array(nz, dtype=float)
                    ip += 1
        out["c%d_ncase" % ic] = np.array(ip)
    save("objective.npz", **out)


def gen_fit_full(pplib, pptoaslib):
    rng = np.random.default_rng(4321)
    out = {}
    cases = [
        # (nchan, nbin, tau_inj, flags, log10_tau, init tau, init alpha)
        (16, 256, 0.0, [1, 0, 0, 0, 0], False, 0.0, 0.0),
        (16, 256, 0.0, [1, 1, 0, 0, 0], False, 0.0, 0.0),
        (32, 256, 0.0, [1, 1, 0, 0, 0], False, 0.0, 0.0),
        (32, 512, 0.0, [1, 1, 1, 0, 0], False, 0.0, 0.0),
        (16, 256, 4e-3, [1, 1, 0, 1, 1], True, 3e-3, -4.0),
        (16, 256, 4e-3, [1, 1, 0, 1, 0], True, 3e-3, -4.0),
        (16, 256, 4e-3, [1, 1, 0, 1, 0], False, 3e-3, -4.0),
        (64, 512, 0.0, [1, 1, 0, 0, 0], False, 0.0, 0.0),
    ]
    import io
    import contextlib
    for ic, (nchan, nbin, tau, flags, log10_tau, t0, a0) in enumerate(cases):
        phi = rng.uniform(-0.1, 0.1)
        dDM = rng.normal(3e-4, 2e-4)
        freqs, model, data = make_portrait((pplib, pptoaslib), rng, nchan, nbin,
                                           phi, dDM, 1.5 if nbin > 256 else 0.4,
                                           tau=tau)
        errs = pplib.get_noise(data, chans=True)
        nu_fit = pplib.guess_fit_freq(freqs)
        # phi was injected at 1500 MHz; reference it to nu_fit as pptoas does
        # (pptoas.py:455-456) so every case starts in the right basin.
        phi0 = float(pplib.phase_transform(phi + 0.003, DM0 + dDM, 1500.0,
                                           nu_fit, P0, mod=True))
        init = [phi0, DM0, 0.0, np.log10(t0) if (log10_tau and t0) else t0,
                a0]
        with contextlib.redirect_stdout(io.StringIO()):
            res = pptoaslib.fit_portrait_full(
                data, model, init, P0, freqs, [nu_fit, nu_fit, nu_fit],
                [None, None, None], errs, flags, log10_tau=log10_tau, option=0)
        key = "f%d" % ic
        out[key + "_data"] = data
        out[key + "_model"] = model
        out[key + "_freqs"] = freqs
        out[key + "_errs"] = errs
        out[key + "_init"] = np.array(init)
        out[key + "_nu_fit"] = np.array(nu_fit)
        out[key + "_flags"] = np.array(flags)
        out[key + "_log10"] = np.array(log10_tau)
        for k in ["params", "param_errs", "scales", "scale_errs",
                  "covariance_matrix", "channel_snrs"]:
            out[key + "_" + k] = np.asarray(res[k], dtype=float)
        for k in ["phi", "phi_err", "DM", "DM_err", "GM", "GM_err", "tau",
                  "tau_err", "alpha", "alpha_err", "nu_DM", "nu_GM", "nu_tau",
                  "chi2", "red_chi2", "snr"]:
            out[key + "_" + k] = np.array(float(res[k]))
        out[key + "_nfeval"] = np.array(int(res["nfeval"]))
        out[key + "_return_code"] = np.array(int(res["return_code"]))
    out["ncase"] = np.array(len(cases))
    out["P"] = np.array(P0)
    save("fit_full.npz", **out)


def gen_phase_shift(pplib):
    rng = np.random.default_rng(99)
    out = {}
    nbin = 256
    phases = pplib.get_bin_centers(nbin)
    freqs = channel_freqs(4)
    _, _, model = pplib.read_model(GMODEL, phases, freqs, P0, quiet=True)
    mprof = model.mean(axis=0)
    k = 0
    for shift in [0.0, 0.123, -0.31, 0.49]:
        for Ns in [100, nbin]:
            for noise in [None, 0.3]:
                data = pplib.rotate_data(mprof, -shift) * 1.7 + \
                    rng.normal(0.0, 0.3, nbin)
                res = pplib.fit_phase_shift(data, mprof, noise=noise, Ns=Ns)
                out["p%d_data" % k] = data
                out["p%d_Ns" % k] = np.array(Ns)
                out["p%d_noise" % k] = np.array(np.nan if noise is None else noise)
                for key in ["phase", "phase_err", "scale", "scale_err", "snr",
                            "red_chi2"]:
                    out["p%d_%s" % (k, key)] = np.array(float(res[key]))
                k += 1
    out["model"] = mprof
    out["ncase"] = np.array(k)
    save("phase_shift.npz", **out)


def gen_utils(pplib, pptoaslib):
    rng = np.random.default_rng(7)
    out = {}
    port = rng.normal(0, 1, (6, 128))
    out["noise_port"] = port
    out["noise_chans"] = pplib.get_noise_PS(port, chans=True)
    out["noise_ravel"] = np.array(pplib.get_noise_PS(port))
    prof = rng.normal(0, 1, 128)
    out["rot_prof"] = prof
    out["rot_prof_out"] = pplib.rotate_data(prof, 0.137)
    freqs = channel_freqs(6)
    out["rot_freqs"] = freqs
    out["rot_port_out_dm0"] = pplib.rotate_data(port, -0.21)
    out["rot_port_out"] = pplib.rotate_data(port, 0.05, 12.3, P0, freqs, 1400.0)
    sub4 = rng.normal(0, 1, (2, 1, 6, 128))
    out["rot_sub4"] = sub4
    out["rot_sub4_out"] = pplib.rotate_data(sub4, -0.02, 3.4,
                                            np.array([P0, 1.01 * P0]), freqs, 1500.0)
    out["rot_full_out"] = pptoaslib.rotate_portrait_full(port, 0.05, 12.3, 3e-5,
                                                         freqs, 1400.0, 1300.0, P0)
    snrs = rng.uniform(1, 10, 6)
    out["gff_snrs"] = snrs
    out["gff_out"] = np.array(pplib.guess_fit_freq(freqs, snrs))
    out["gff_out_nosnr"] = np.array(pplib.guess_fit_freq(freqs))
    pt = []
    for (phi, DM, n1, n2) in [(0.3, 10.0, 1400.0, 1500.0), (-0.45, 34.5, 1100.0, 1900.0),
                              (0.9, 1.0, np.inf, 1500.0), (2.7, 0.0, 1400.0, 1400.0)]:
        pt.append([phi, DM, n1, n2,
                   float(pplib.phase_transform(phi, DM, n1, n2, P0, mod=True)),
                   float(pplib.phase_transform(phi, DM, n1, n2, P0, mod=False))])
    out["phase_transform"] = np.array(pt)
    out["P"] = np.array(P0)
    save("utils.npz", **out)


def gen_legacy_fit_portrait(pplib, pptoaslib):
    rng = np.random.default_rng(555)
    out = {}
    for ic, (nchan, nbin) in enumerate([(16, 256), (32, 512)]):
        phi = rng.uniform(-0.1, 0.1)
        dDM = rng.normal(3e-4, 2e-4)
        freqs, model, data = make_portrait((pplib, pptoaslib), rng, nchan, nbin,
                                           phi, dDM, 0.5)
        errs = pplib.get_noise(data, chans=True)
        nu_fit = pplib.guess_fit_freq(freqs)
        init = np.array([float(pplib.phase_transform(phi + 0.002, DM0 + dDM,
                                                     1500.0, nu_fit, P0,
                                                     mod=True)), DM0])
        res = pplib.fit_portrait(data, model, init, P0, freqs, nu_fit, None, errs)
        key = "l%d" % ic
        out[key + "_data"] = data
        out[key + "_model"] = model
        out[key + "_freqs"] = freqs
        out[key + "_errs"] = errs
        out[key + "_init"] = init
        out[key + "_nu_fit"] = np.array(nu_fit)
        for k in ["phase", "phase_err", "DM", "DM_err", "nu_ref", "covariance",
                  "chi2", "red_chi2", "snr"]:
            out[key + "_" + k] = np.array(float(res[k]))
        out[key + "_scales"] = np.asarray(res.scales)
        out[key + "_scale_errs"] = np.asarray(res.scale_errs)
        out[key + "_nfeval"] = np.array(int(res.nfeval))
        out[key + "_return_code"] = np.array(int(res.return_code))
    out["ncase"] = np.array(2)
    save("legacy_fit_portrait.npz", **out)


def fake_archive(pplib, pptoaslib, rng, name, nsub, nchan, nbin, mask=None,
                 dopp=1.0, tau=0.0):
    """An in-memory load_data() DataBunch (pplib.py:2809-2819)."""
    freqs1 = channel_freqs(nchan)
    phases = pplib.get_bin_centers(nbin)
    subints = np.zeros((nsub, 1, nchan, nbin))
    inj = []
    for isub in range(nsub):
        phi = rng.uniform(-0.1, 0.1)
        dDM = rng.normal(3e-4, 2e-4)
        _, _, data = make_portrait((pplib, pptoaslib), rng, nchan, nbin, phi, dDM,
                                   0.8, tau=tau)
        subints[isub, 0] = data
        inj.append((phi, dDM))
    weights = np.ones((nsub, nchan)) if mask is None else mask.astype(float)
    weights_norm = np.where(weights == 0.0, 0.0, 1.0)
    ok_isubs = np.compress(weights_norm.mean(axis=1), range(nsub))
    ok_ichans = [np.compress(weights_norm[isub], range(nchan))
                 for isub in range(nsub)]
    noise_stds = np.zeros((nsub, 1, nchan))
    for isub in range(nsub):
        noise_stds[isub, 0] = pplib.get_noise(subints[isub, 0], chans=True)
    SNRs = rng.uniform(5.0, 50.0, (nsub, 1, nchan))
    epochs = [MJD(57202.0 + 0.0001 * isub) + 30.0 for isub in range(nsub)]
    masks = np.einsum("ij,k", weights_norm, np.ones(nbin))
    masks = np.einsum("j,ikl", np.ones(1), masks)
    db = pplib.DataBunch(
        arch=None, backend="fake_be", backend_delay=1.5e-6, bw=800.0,
        doppler_factors=np.full(nsub, dopp), DM=DM0, dmc=0, epochs=epochs,
        filename=name, flux_prof=np.array([]),
        freqs=np.tile(freqs1, (nsub, 1)), frontend="fake_rx",
        integration_length=60.0 * nsub, masks=masks, nbin=nbin, nchan=nchan,
        noise_stds=noise_stds, npol=1, nsub=nsub, nu0=1500.0,
        ok_ichans=ok_ichans, ok_isubs=ok_isubs,
        parallactic_angles=np.zeros(nsub), phases=phases,
        prof=subints.mean(axis=(0, 1, 2)), prof_noise=1.0, prof_SNR=100.0,
        Ps=np.full(nsub, P0), SNRs=SNRs, source="J1234-5678",
        state="Intensity", subints=subints, subtimes=[60.0] * nsub,
        telescope="GBT", telescope_code="1", weights=weights)
    return db, inj


def archive_to_arrays(db, prefix, out):
    out[prefix + "subints"] = db.subints
    out[prefix + "freqs"] = db.freqs
    out[prefix + "weights"] = db.weights
    out[prefix + "noise_stds"] = db.noise_stds
    out[prefix + "SNRs"] = db.SNRs
    out[prefix + "Ps"] = db.Ps
    out[prefix + "doppler_factors"] = db.doppler_factors
    out[prefix + "epochs"] = np.array([[e.days, e.secs, e.fracsec] for e in db.epochs])


def gen_get_toas(pplib, pptoaslib, pptoas):
    import io
    import contextlib
    rng = np.random.default_rng(2024)
    nchan, nbin = 16, 256
    mask = np.ones((3, nchan), dtype=int)
    mask[1, :3] = 0
    mask[2, 5] = 0
    archives = {}
    archives["synthA.fits"], _ = fake_archive(pplib, pptoaslib, rng, "synthA.fits",
                                              3, nchan, nbin, mask=mask,
                                              dopp=1.0001)
    archives["synthB.fits"], _ = fake_archive(pplib, pptoaslib, rng, "synthB.fits",
                                              2, nchan, nbin)

    def fake_load_data(filename, **kw):
        return archives[filename]

    pptoas.load_data = fake_load_data
    pptoas.file_is_type = lambda f, t: False
    modelfile = os.path.join(tempfile.mkdtemp(), "example.gmodel")
    shutil.copy(GMODEL, modelfile)
    cwd = os.getcwd()
    os.chdir(os.path.dirname(modelfile))
    out = {}
    meta = {}
    try:
        for tag, kwargs in [("default", {}),
                            ("nodm_nobary", dict(fit_DM=False, bary=False)),
                            ("gm", dict(fit_GM=True)),
                            ("phs_flags", dict(print_phase=True,
                                               addtnl_toa_flags={"pta": "TEST",
                                                                 "ver": 2}))]:
            with contextlib.redirect_stdout(io.StringIO()):
                gt = pptoas.GetTOAs("synthA.fits", "example.gmodel", quiet=True)
                gt.datafiles = ["synthA.fits", "synthB.fits"]
                gt.get_TOAs(quiet=True, **kwargs)
            lines = []
            for toa in gt.TOA_list:
                buf = io.StringIO()
                with contextlib.redirect_stdout(buf):
                    pplib.write_TOAs(toa, outfile=None)
                lines.append(buf.getvalue().strip())
            meta[tag] = dict(kwargs={k: v for k, v in kwargs.items()}, tim=lines)
            for ia in range(len(gt.phis)):
                p = "%s_a%d_" % (tag, ia)
                out[p + "phis"] = gt.phis[ia]
                out[p + "phi_errs"] = gt.phi_errs[ia]
                out[p + "DMs"] = gt.DMs[ia]
                out[p + "DM_errs"] = gt.DM_errs[ia]
                out[p + "GMs"] = gt.GMs[ia]
                out[p + "GM_errs"] = gt.GM_errs[ia]
                out[p + "snrs"] = gt.snrs[ia]
                out[p + "red_chi2s"] = gt.red_chi2s[ia]
                out[p + "rcs"] = gt.rcs[ia]
                out[p + "nfevals"] = gt.nfevals[ia]
                out[p + "scales"] = gt.scales[ia]
                out[p + "nu_refs"] = np.array(gt.nu_refs[ia], dtype=float)
                out[p + "nu_fits"] = np.array(gt.nu_fits[ia], dtype=float)
                out[p + "covariances"] = gt.covariances[ia]
                out[p + "DeltaDM"] = np.array([gt.DeltaDM_means[ia],
                                               gt.DeltaDM_errs[ia]])
                out[p + "TOAs"] = np.array([[t.days, t.secs, t.fracsec]
                                            for t in gt.TOAs[ia][gt.ok_isubs[ia]]])
    finally:
        os.chdir(cwd)
    for name, db in archives.items():
        archive_to_arrays(db, name.split(".")[0] + "_", out)
    meta["archives"] = sorted(archives)
    meta["backend_delay"] = 1.5e-6
    meta["telescope_code"] = "1"
    meta["modelfile"] = "example.gmodel"
    save("get_toas.npz", **out)
    with open(os.path.join(HERE, "get_toas_tim.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote get_toas_tim.json")


class _Prof(object):
    def __init__(self, store, ipol, ichan):
        self.store, self.ipol, self.ichan = store, ipol, ichan

    def get_amps(self):
        return self.store[self.ipol, self.ichan]


class _Sub(object):
    def __init__(self, store, weights):
        self.store, self.weights = store, weights

    def get_Profile(self, ipol, ichan):
        return _Prof(self.store, ipol, ichan)

    def set_weight(self, ichan, w):
        self.weights[ichan] = w


class _Arch(object):
    """Captures what align_archives writes into the output archive."""
    def __init__(self, npol, nchan, nbin):
        self.store = np.zeros((npol, nchan, nbin))
        self.weights = np.ones(nchan)
        self.npol, self.nchan = npol, nchan

    def tscrunch(self):
        pass

    def pscrunch(self):
        pass

    def convert_state(self, s):
        pass

    def set_dispersion_measure(self, dm):
        self.dm = dm

    def __iter__(self):
        return iter([_Sub(self.store, self.weights)])

    def get_npol(self):
        return self.npol

    def get_nchan(self):
        return self.nchan

    def unload(self, fname):
        pass


def gen_align(pplib, pptoaslib, ppalign):
    import io
    import contextlib
    rng = np.random.default_rng(31415)
    nchan, nbin = 16, 128
    archives = {}
    names = ["al%d.fits" % i for i in range(4)]
    for i, n in enumerate(names):
        archives[n], _ = fake_archive(pplib, pptoaslib, rng, n, 1, nchan, nbin)
    freqs = channel_freqs(nchan)
    phases = pplib.get_bin_centers(nbin)
    _, _, model = pplib.read_model(GMODEL, phases, freqs, P0, quiet=True)
    guess = pplib.rotate_data(model, 0.01)  # a slightly mis-phased template
    arch = _Arch(1, nchan, nbin)
    model_db = pplib.DataBunch(**dict(archives[names[0]]))
    model_db["subints"] = guess[None, None]
    model_db["arch"] = arch
    model_db["freqs"] = freqs[None]
    model_db["ok_ichans"] = [np.arange(nchan)]
    model_db["masks"] = np.ones((1, 1, nchan, nbin))

    def fake_load_data(filename, **kw):
        if filename == "guess.fits":
            return model_db
        return archives[filename]

    class _Popen(object):
        def __init__(self, *a, **k):
            self.stdout = io.StringIO("filename nchan nbin\nguess.fits %d %d\n"
                                      % (nchan, nbin))

    fake_sub = types.SimpleNamespace(Popen=_Popen, PIPE=None)
    ppalign.load_data = fake_load_data
    ppalign.sub = fake_sub
    out = {}
    for niter in [1, 2]:
        arch.store[:] = 0.0
        with contextlib.redirect_stdout(io.StringIO()):
            ppalign.align_archives(list(names), "guess.fits", fit_dm=True,
                                   niter=niter, quiet=True, outfile="x.fits")
        out["aligned_niter%d" % niter] = arch.store.copy()
    out["guess"] = guess
    out["freqs"] = freqs
    out["P"] = np.array(P0)
    for n in names:
        archive_to_arrays(archives[n], n.split(".")[0] + "_", out)
    out["names"] = np.array(names)
    save("align.npz", **out)


def main():
    tmp, pplib, pptoaslib, pptoas, ppalign = load_reference()
    try:
        np.seterr(all="ignore")
        gen_models(pplib)
        gen_utils(pplib, pptoaslib)
        gen_phase_shift(pplib)
        gen_objective(pplib, pptoaslib)
        gen_fit_full(pplib, pptoaslib)
        gen_legacy_fit_portrait(pplib, pptoaslib)
        gen_get_toas(pplib, pptoaslib, pptoas)
        gen_align(pplib, pptoaslib, ppalign)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
