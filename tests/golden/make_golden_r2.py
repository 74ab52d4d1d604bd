#!/usr/bin/env python3
"""Round-2 golden fixtures from the reference PulsePortraiture source.

TEST INFRASTRUCTURE ONLY -- run in the build container, never on the GPU box
and never by the product.  The reference is loaded through the SURVEY.md
§8(c) shim exactly as in make_golden.py (imported from there); only numbers
are written into tests/golden/.  Inputs that are too large to commit are
regenerated from Philox seeds by ``pulseportraiture_amd.synth`` (the same
numpy code on the GPU box), so each fixture stores its seeds and shapes and
the reference's outputs.

Fixtures:
  fit_full_r2.npz    fit_portrait_full for the get_nu_zeros branches not in
                     fit_full.npz ([1,0,1,0,0], [0,0,0,1,1], [1,1,1,1,0]
                     option 0/1, [1,1,1,1,1], [1,1,1,0,0] option 1) and the
                     TNC / Newton-CG methods (pptoaslib.py:995-1014)
  configs_r2.npz     GetTOAs.get_TOAs on synthetic archives at BASELINE
  configs_r2.json    configs 3 (512x1024, phase+DM+tau+alpha, log10 tau) and
                     4 (128x2048, phase+DM+GM): per-subint outputs, .tim lines
  align5.npz         ppalign.align_archives at config 5's shape (256 x 2048,
                     Ns = nbin guess), 6 archives, niter 1 and 2
  headline_2k.npz    2000 subints of the bench workload (64 x 2048, seed
                     20240917): the get_TOAs guess + trust-ncg fit per subint,
                     and the reference's own floor -- the same fit restarted
                     from the guess moved by one ulp either way
  timing_r2.json     oracle vs reference wall time per TOA (BASELINE.md:47)
  tnc_floor.npz      the reference's TNC restarted 1-10 ulps away: how far its
                     own end point moves (legacy fit and the TNC fit cases)
  narrowband.*       GetTOAs.get_narrowband_TOAs with an archive template:
                     per-channel phases, errors, scales and .tim lines
  zap.npz            GetTOAs.get_channels_to_zap (after get_TOAs) and
                     ppzap.get_zap_channels on an archive with bad channels

Usage:  python tests/golden/make_golden_r2.py [fit|configs|align|headline|timing ...]
"""
import contextlib
import io
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import make_golden as MG  # noqa: E402
from tests.golden_consts import zap_perturb  # noqa: E402

MG.REF_FILES = MG.REF_FILES + ["ppzap.py"]  # get_zap_channels (ppzap.py:18-48)
from pulseportraiture_amd import synth  # noqa: E402

P0 = MG.P0
DM0 = MG.DM0
HEAD_SEED = 20240917


def quiet_call(fn, *a, **k):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **k)


# --------------------------------------------------------------------------
# fit_portrait_full: remaining get_nu_zeros branches, TNC, Newton-CG
# --------------------------------------------------------------------------
FIT_CASES = [
    # (nchan, nbin, tau_inj, flags, log10_tau, option, method, init tau, init alpha)
    (32, 512, 0.0, [1, 0, 1, 0, 0], False, 0, "trust-ncg", 0.0, 0.0),
    (16, 256, 4e-3, [0, 0, 0, 1, 1], True, 0, "trust-ncg", 3e-3, -4.0),
    (16, 256, 4e-3, [1, 1, 1, 1, 0], True, 0, "trust-ncg", 3e-3, -4.0),
    (16, 256, 4e-3, [1, 1, 1, 1, 0], True, 1, "trust-ncg", 3e-3, -4.0),
    (16, 256, 4e-3, [1, 1, 1, 1, 1], True, 0, "trust-ncg", 3e-3, -4.0),
    (32, 512, 0.0, [1, 1, 1, 0, 0], False, 1, "trust-ncg", 0.0, 0.0),
    (32, 512, 0.0, [1, 1, 0, 0, 0], False, 0, "TNC", 0.0, 0.0),
    (16, 256, 4e-3, [1, 1, 0, 1, 1], True, 0, "TNC", 3e-3, -4.0),
    (16, 256, 4e-3, [1, 1, 0, 1, 0], False, 0, "TNC", 3e-3, -4.0),
    (64, 512, 0.0, [1, 1, 0, 0, 0], False, 0, "TNC", 0.0, 0.0),
    (32, 512, 0.0, [1, 1, 0, 0, 0], False, 0, "Newton-CG", 0.0, 0.0),
]


def pptoas_tnc_bounds(nbin, log10_tau):
    """get_TOAs' default bounds for method='TNC' (pptoas.py:458-467)."""
    tau_b = (np.log10((10 * nbin) ** -1), None) if log10_tau else (0.0, None)
    return [(None, None), (None, None), (None, None), tau_b, (-10.0, 10.0)]


def gen_fit_r2(pplib, pptoaslib):
    rng = np.random.default_rng(8642)
    out = {}
    for ic, (nchan, nbin, tau, flags, log10_tau, option, method, t0, a0) in enumerate(FIT_CASES):
        phi = rng.uniform(-0.1, 0.1)
        dDM = rng.normal(3e-4, 2e-4)
        freqs, model, data = MG.make_portrait((pplib, pptoaslib), rng, nchan, nbin, phi, dDM,
                                              1.5 if nbin > 256 else 0.4, tau=tau)
        errs = pplib.get_noise(data, chans=True)
        nu_fit = pplib.guess_fit_freq(freqs)
        if flags[0]:
            phi0 = float(pplib.phase_transform(phi + 0.003, DM0 + dDM, 1500.0, nu_fit, P0,
                                               mod=True))
            DMi = DM0
        else:  # phase and DM not fitted: start at the injected values
            phi0 = float(pplib.phase_transform(phi, DM0 + dDM, 1500.0, nu_fit, P0, mod=True))
            DMi = DM0 + dDM
        tau_i = np.log10(t0) if (log10_tau and t0) else t0
        init = [phi0, DMi, 0.0, tau_i, a0]
        bounds = pptoas_tnc_bounds(nbin, log10_tau) if method == "TNC" else [(None, None)] * 5
        res = quiet_call(pptoaslib.fit_portrait_full, data, model, init, P0, freqs,
                         [nu_fit, nu_fit, nu_fit], [None, None, None], errs, flags,
                         bounds, log10_tau, option=option, method=method)
        key = "f%d_" % ic
        out[key + "data"] = data
        out[key + "model"] = model
        out[key + "freqs"] = freqs
        out[key + "errs"] = errs
        out[key + "init"] = np.array(init, dtype=float)
        out[key + "nu_fit"] = np.array(nu_fit)
        out[key + "flags"] = np.array(flags)
        out[key + "log10"] = np.array(log10_tau)
        out[key + "option"] = np.array(option)
        out[key + "method"] = np.array(method)
        out[key + "bounds"] = np.array([[np.nan if v is None else v for v in b] for b in bounds])
        for k in ["params", "param_errs", "scales", "scale_errs", "covariance_matrix",
                  "channel_snrs"]:
            out[key + k] = np.asarray(res[k], dtype=float)
        for k in ["phi", "phi_err", "DM", "DM_err", "GM", "GM_err", "tau", "tau_err", "alpha",
                  "alpha_err", "nu_DM", "nu_GM", "nu_tau", "chi2", "red_chi2", "snr"]:
            out[key + k] = np.array(float(res[k]))
        out[key + "nfeval"] = np.array(int(res["nfeval"]))
        out[key + "return_code"] = np.array(int(res["return_code"]))
        print("fit case %d %s %s opt %d: rc %d nfev %d nu %s" % (
            ic, method, flags, option, res["return_code"], res["nfeval"],
            [res["nu_DM"], res["nu_GM"], res["nu_tau"]]))
    out["ncase"] = np.array(len(FIT_CASES))
    out["P"] = np.array(P0)
    MG.save("fit_full_r2.npz", **out)


# --------------------------------------------------------------------------
# GetTOAs at configs 3 and 4 (synthetic archives from Philox seeds)
# --------------------------------------------------------------------------
CONFIGS = {
    # name: (nsub, nchan, nbin, seed, tau, gm, get_TOAs kwargs)
    "cfg3": (3, 512, 1024, 3003, 2e-3, 0.0, dict(fit_scat=True, log10_tau=True)),
    "cfg4": (4, 128, 2048, 4004, 0.0, 0.0, dict(fit_GM=True)),
}


def synth_archive(pplib, name, nsub, nchan, nbin, seed, tau, gm):
    """An in-memory load_data() bunch (pplib.py:2809-2819) of Philox portraits;
    the GPU test rebuilds the same subints with synth.make_workload."""
    w = synth.make_workload(nsub, nchan, nbin, seed=seed, tau=tau, gm=gm)
    data = synth.workload_data_host(w)
    subints = data[:, None]
    weights = np.ones((nsub, nchan))
    noise_stds = np.array([pplib.get_noise(subints[i, 0], chans=True) for i in range(nsub)])
    epochs = [MG.MJD(57300.0 + 0.001 * i) + 10.0 for i in range(nsub)]
    db = pplib.DataBunch(
        arch=None, backend="syn_be", backend_delay=2.0e-6, bw=800.0,
        doppler_factors=np.full(nsub, 1.00002), DM=DM0, dmc=0, epochs=epochs,
        filename=name, flux_prof=np.array([]), freqs=np.tile(w.freqs, (nsub, 1)),
        frontend="syn_rx", integration_length=30.0 * nsub,
        masks=np.ones((nsub, 1, nchan, nbin)), nbin=nbin, nchan=nchan,
        noise_stds=noise_stds[:, None], npol=1, nsub=nsub, nu0=1500.0,
        ok_ichans=[np.arange(nchan) for _ in range(nsub)], ok_isubs=np.arange(nsub),
        parallactic_angles=np.zeros(nsub), phases=pplib.get_bin_centers(nbin),
        prof=subints.mean(axis=(0, 1, 2)), prof_noise=1.0, prof_SNR=100.0,
        Ps=np.full(nsub, w.P), SNRs=np.ones((nsub, 1, nchan)), source="J1234-5678",
        state="Intensity", subints=subints, subtimes=[30.0] * nsub, telescope="GBT",
        telescope_code="1", weights=weights)
    return db


def gen_configs(pplib, pptoaslib, pptoas):
    out = {}
    meta = {}
    archives = {}
    for name, (nsub, nchan, nbin, seed, tau, gm, kw) in CONFIGS.items():
        archives[name + ".fits"] = synth_archive(pplib, name + ".fits", nsub, nchan, nbin, seed,
                                                 tau, gm)
    pptoas.load_data = lambda filename, **kw: archives[filename]
    pptoas.file_is_type = lambda f, t: False
    import shutil
    import tempfile
    tmpd = tempfile.mkdtemp()
    shutil.copy(MG.GMODEL, os.path.join(tmpd, "example.gmodel"))
    cwd = os.getcwd()
    os.chdir(tmpd)
    try:
        for name, (nsub, nchan, nbin, seed, tau, gm, kw) in CONFIGS.items():
            t0 = time.time()
            gt = quiet_call(pptoas.GetTOAs, name + ".fits", "example.gmodel", quiet=True)
            gt.datafiles = [name + ".fits"]
            quiet_call(gt.get_TOAs, quiet=True, **kw)
            dt = time.time() - t0
            lines = []
            for toa in gt.TOA_list:
                buf = io.StringIO()
                with contextlib.redirect_stdout(buf):
                    pplib.write_TOAs(toa, outfile=None)
                lines.append(buf.getvalue().strip())
            meta[name] = dict(kwargs=kw, tim=lines, nsub=nsub, nchan=nchan, nbin=nbin,
                              seed=seed, tau=tau, gm=gm, seconds=dt)
            p = name + "_"
            for attr in ["phis", "phi_errs", "DMs", "DM_errs", "GMs", "GM_errs", "taus",
                         "tau_errs", "alphas", "alpha_errs", "snrs", "red_chi2s", "rcs",
                         "nfevals", "scales", "scale_errs", "channel_snrs", "covariances"]:
                out[p + attr] = np.asarray(getattr(gt, attr)[0], dtype=float)
            out[p + "nu_refs"] = np.array(gt.nu_refs[0], dtype=float)
            out[p + "nu_fits"] = np.array(gt.nu_fits[0], dtype=float)
            out[p + "DeltaDM"] = np.array([gt.DeltaDM_means[0], gt.DeltaDM_errs[0]])
            out[p + "TOAs"] = np.array([[t.days, t.secs, t.fracsec] for t in gt.TOAs[0]])
            out[p + "noise_stds"] = archives[name + ".fits"].noise_stds
            print("%s: %d subints in %.1f s, rcs %s nfev %s" % (name, nsub, dt, gt.rcs[0],
                                                                gt.nfevals[0]))
    finally:
        os.chdir(cwd)
    MG.save("configs_r2.npz", **out)
    with open(os.path.join(HERE, "configs_r2.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


# --------------------------------------------------------------------------
# ppalign at config 5's shape
# --------------------------------------------------------------------------
ALIGN5 = dict(narch=6, nchan=256, nbin=2048, seed=5005, guess_rot=0.01)


def gen_align5(pplib, pptoaslib, ppalign):
    import types
    n, nchan, nbin = ALIGN5["narch"], ALIGN5["nchan"], ALIGN5["nbin"]
    names = ["a5_%d.fits" % i for i in range(n)]
    archives = {}
    for i, nm in enumerate(names):
        archives[nm] = synth_archive(pplib, nm, 1, nchan, nbin, ALIGN5["seed"] + i, 0.0, 0.0)
    w = synth.make_workload(1, nchan, nbin, seed=ALIGN5["seed"])
    guess = pplib.rotate_data(w.model, ALIGN5["guess_rot"])
    arch = MG._Arch(1, nchan, nbin)
    model_db = pplib.DataBunch(**dict(archives[names[0]]))
    model_db["subints"] = guess[None, None]
    model_db["arch"] = arch
    model_db["freqs"] = w.freqs[None]
    model_db["ok_ichans"] = [np.arange(nchan)]
    model_db["masks"] = np.ones((1, 1, nchan, nbin))

    def fake_load_data(filename, **kw):
        return model_db if filename == "guess.fits" else archives[filename]

    class _Popen(object):
        def __init__(self, *a, **k):
            self.stdout = io.StringIO("filename nchan nbin\nguess.fits %d %d\n" % (nchan, nbin))

    ppalign.load_data = fake_load_data
    ppalign.sub = types.SimpleNamespace(Popen=_Popen, PIPE=None)
    out = {}
    for niter in [1, 2]:
        arch.store[:] = 0.0
        t0 = time.time()
        quiet_call(ppalign.align_archives, list(names), "guess.fits", fit_dm=True, niter=niter,
                   quiet=True, outfile="x.fits")
        a = arch.store[0]
        k = np.arange(nbin)
        out["niter%d_chan_sum" % niter] = a.sum(axis=1)
        out["niter%d_chan_sum2" % niter] = (a ** 2).sum(axis=1)
        out["niter%d_chan_moment" % niter] = (a * k).sum(axis=1)
        if niter == 2:
            out["aligned_niter2_f32"] = a.astype(np.float32)
        out["niter%d_weights" % niter] = arch.weights.copy()
        print("align niter %d: %.1f s" % (niter, time.time() - t0))
    for key, v in ALIGN5.items():
        out["cfg_" + key] = np.array(v)
    out["noise_stds"] = np.array([archives[nm].noise_stds[0, 0] for nm in names])
    MG.save("align5.npz", **out)


# --------------------------------------------------------------------------
# 2000 headline subints: get_TOAs per-subint flow (pptoas.py:383-488)
# --------------------------------------------------------------------------
def ref_subint(ref, i, model, model_prof, perturb=True):
    pplib, pptoaslib = ref
    w = synth.make_workload(1, 64, 2048, seed=HEAD_SEED, sub0=i)
    port = synth.workload_data_host(w)[0]
    freqs = w.freqs
    errs = pplib.get_noise(port, chans=True)           # load_data noise_stds
    nu_fit = pplib.guess_fit_freq(freqs, np.ones(64))  # SNRs = 1
    nu_mean = freqs.mean()
    rot = pplib.rotate_data(port, 0.0, DM0, w.P, freqs, nu_mean)
    prof = np.average(rot, axis=0, weights=np.ones(64))
    phi_g = pplib.fit_phase_shift(prof, model_prof, Ns=100).phase
    phi_g = pplib.phase_transform(phi_g, DM0, nu_mean, nu_fit, w.P, mod=True)
    init = [phi_g, DM0, 0.0, 0.0, 0.0]

    def fit(x0):
        return pptoaslib.fit_portrait_full(port, model, x0, w.P, freqs, [nu_fit] * 3,
                                           [None] * 3, errs, [1, 1, 0, 0, 0], None, False,
                                           option=0, sub_id=None, method="trust-ncg",
                                           is_toa=True, quiet=True)
    r = fit(init)
    row = [r.phi, r.phi_err, r.DM, r.DM_err, r.nu_DM, r.return_code, r.nfeval, phi_g, nu_fit,
           r.red_chi2, r.snr]
    if perturb:
        for d in [np.inf, -np.inf]:
            x0 = list(init)
            x0[0] = np.nextafter(x0[0], d)
            q = fit(x0)
            row += [q.phi, q.DM, q.return_code, q.nu_DM]
    return row


def _headline_worker(args):
    lo, hi = args
    import warnings
    warnings.simplefilter("ignore")
    import shutil
    tmp, pplib, pptoaslib, _, _ = MG.load_reference()
    try:
        w = synth.make_workload(1, 64, 2048, seed=HEAD_SEED)
        model = w.model
        return [ref_subint((pplib, pptoaslib), i, model, model.mean(axis=0))
                for i in range(lo, hi)]
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


HEAD_COLS = ["phi", "phi_err", "DM", "DM_err", "nu_DM", "status", "nfev", "phi_guess",
             "nu_fit", "red_chi2", "snr", "up_phi", "up_DM", "up_status", "up_nu_DM",
             "dn_phi", "dn_DM", "dn_status", "dn_nu_DM"]


def gen_headline_2k(nsub=2000, nproc=8):
    from multiprocessing import Pool
    os.environ["OMP_NUM_THREADS"] = "1"
    step = (nsub + 4 * nproc - 1) // (4 * nproc)
    chunks = [(lo, min(nsub, lo + step)) for lo in range(0, nsub, step)]
    t0 = time.time()
    with Pool(nproc) as p:
        parts = p.map(_headline_worker, chunks)
    rows = np.array([r for part in parts for r in part], dtype=float)
    print("headline 2k: %.1f s" % (time.time() - t0))
    out = {c: rows[:, j] for j, c in enumerate(HEAD_COLS)}
    out["seed"] = np.array(HEAD_SEED)
    out["nsub"] = np.array(nsub)
    for tag in ["up", "dn"]:
        d = np.abs(out[tag + "_phi"] - out["phi"]) / out["phi_err"]
        print("floor %s: max %.3g p99 %.3g  status diff %d" % (
            tag, d.max(), np.percentile(d, 99), np.sum(out[tag + "_status"] != out["status"])))
    MG.save("headline_2k.npz", **out)


# --------------------------------------------------------------------------
# Oracle vs reference wall time (BASELINE.md:47)
# --------------------------------------------------------------------------
def gen_timing(pplib, pptoaslib, n=24):
    import warnings
    warnings.simplefilter("ignore")
    from oracle import ppfit_oracle as O
    w = synth.make_workload(1, 64, 2048, seed=HEAD_SEED)
    model = w.model
    mprof = model.mean(axis=0)
    ports = [synth.workload_data_host(synth.make_workload(1, 64, 2048, seed=HEAD_SEED,
                                                          sub0=i))[0] for i in range(n)]
    from threadpoolctl import threadpool_limits
    res = {}
    with threadpool_limits(limits=1):
        for rep in range(2):
            t0 = time.perf_counter()
            for i in range(n):
                ref_subint((pplib, pptoaslib), i, model, mprof, perturb=False)
            t_ref = (time.perf_counter() - t0) / n
            t0 = time.perf_counter()
            for i in range(n):
                d = ports[i]
                errs = O.get_noise_PS(d, chans=True)
                O.fit_subint_pptoas(d, model, w.freqs, np.ones(64), errs, np.ones(64), w.P,
                                    DM0, (1, 1, 0, 0, 0))
            t_orc = (time.perf_counter() - t0) / n
            res = dict(reference_s_per_toa=t_ref, oracle_s_per_toa=t_orc,
                       ratio_oracle_over_reference=t_orc / t_ref, subints=n,
                       threads=1, shape="64x2048 phase+DM get_TOAs guess + trust-ncg fit",
                       note="reference timing includes regenerating each subint (~30 ms); "
                            "oracle timing uses pre-generated subints")
    # the reference leg regenerates its subint: time that and remove it
    t0 = time.perf_counter()
    for i in range(n):
        synth.workload_data_host(synth.make_workload(1, 64, 2048, seed=HEAD_SEED, sub0=i))
    gen = (time.perf_counter() - t0) / n
    res["reference_s_per_toa"] -= gen
    res["ratio_oracle_over_reference"] = res["oracle_s_per_toa"] / res["reference_s_per_toa"]
    res["note"] = "per-subint data generation (%.1f ms) subtracted from the reference leg" % (
        gen * 1e3)
    print(res)
    with open(os.path.join(HERE, "timing_r2.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)


# --------------------------------------------------------------------------
# TNC's own floor: the reference restarted a few ulps away (legacy fit and
# the fit_full_r2 TNC cases).  TNC stops on |f_n - f_(n-1)| <= sqrt(eps)
# (scaled), so its end point moves by up to ~1e-2 sigma with the last bits.
# --------------------------------------------------------------------------
def gen_tnc_floor(pplib, pptoaslib):
    import warnings
    warnings.simplefilter("ignore")
    out = {}
    g = np.load(os.path.join(HERE, "legacy_fit_portrait.npz"))
    for ic in range(int(g["ncase"])):
        k = "l%d_" % ic
        rows = []
        for j in range(1, 11):
            init = np.array(g[k + "init"], float)
            init[0] += j * np.spacing(init[0]) * (1 if j % 2 else -1)
            r = quiet_call(pplib.fit_portrait, g[k + "data"], g[k + "model"], init, P0,
                           g[k + "freqs"], float(g[k + "nu_fit"]), None, g[k + "errs"])
            rows.append([(r.phase - float(g[k + "phase"])) / float(g[k + "phase_err"]),
                         (r.DM - float(g[k + "DM"])) / float(g[k + "DM_err"]), r.return_code])
        rows = np.array(rows)
        out[k + "phase_floor"] = np.abs(rows[:, 0]).max()
        out[k + "DM_floor"] = np.abs(rows[:, 1]).max()
        out[k + "rcs"] = np.unique(rows[:, 2]).astype(int)
        print("legacy %d floor: phase %.3g sigma, DM %.3g sigma, rcs %s" % (
            ic, out[k + "phase_floor"], out[k + "DM_floor"], out[k + "rcs"]))
    f = np.load(os.path.join(HERE, "fit_full_r2.npz"))
    for ic in range(int(f["ncase"])):
        k = "f%d_" % ic
        if str(f[k + "method"]) != "TNC":
            continue
        nu = float(f[k + "nu_fit"])
        bounds = [tuple(None if np.isnan(v) else float(v) for v in row) for row in f[k + "bounds"]]
        flags = list(f[k + "flags"])
        rows = []
        for j in range(1, 11):
            init = np.array(f[k + "init"], float)
            init[0] += j * np.spacing(init[0]) * (1 if j % 2 else -1)
            r = quiet_call(pptoaslib.fit_portrait_full, f[k + "data"], f[k + "model"], list(init),
                           P0, f[k + "freqs"], [nu] * 3, [None] * 3, f[k + "errs"], flags, bounds,
                           bool(f[k + "log10"]), option=0, method="TNC")
            row = []
            for i, nm in enumerate(["phi", "DM", "GM", "tau", "alpha"]):
                e = float(f[k + nm + "_err"])
                row.append(abs(r[nm] - float(f[k + nm])) / e if (flags[i] and e > 0) else 0.0)
            rows.append(row + [r.return_code])
        rows = np.array(rows)
        out[k + "param_floor"] = rows[:, :5].max(axis=0)
        out[k + "rcs"] = np.unique(rows[:, 5]).astype(int)
        print("fit_full TNC %d floor: %s rcs %s" % (ic, out[k + "param_floor"], out[k + "rcs"]))
    MG.save("tnc_floor.npz", **out)


# --------------------------------------------------------------------------
# Narrowband TOAs (pptoas.py:740-1125): per-channel fit_phase_shift.  The
# reference reads model_data.weights inside the channel loop, which exists
# only for an archive (FITS) template, and indexes it with the data's isub
# on a tscrunched (one-subint) model: so it runs with an archive template
# and one-subint archives, which is what is generated here.
# --------------------------------------------------------------------------
NB_ARCH = {"nbA.fits": (16, 256, 6006, 4), "nbB.fits": (8, 512, 6007, None)}


def nb_archive(pplib, name, nchan, nbin, seed, zero_chan):
    db = synth_archive(pplib, name, 1, nchan, nbin, seed, 0.0, 0.0)
    if zero_chan is not None:
        db["weights"][0, zero_chan] = 0.0
        db["ok_ichans"] = [np.compress(db["weights"][0], range(nchan))]
    return db


def nb_model(pplib, nchan, nbin, zero_model_chan):
    w = synth.make_workload(1, nchan, nbin, seed=1)
    db = pplib.DataBunch(subints=w.model[None, None], masks=np.ones((1, 1, nchan, nbin)),
                         weights=np.ones((1, nchan)), nbin=nbin, nchan=nchan,
                         freqs=w.freqs[None], nsub=1)
    if zero_model_chan is not None:
        db["weights"][0, zero_model_chan] = 0.0
    return db


def gen_narrowband(pplib, pptoaslib, pptoas):
    out, meta = {}, {}
    archives = {n: nb_archive(pplib, n, *v) for n, v in NB_ARCH.items()}
    import shutil
    import tempfile
    for name, (nchan, nbin, seed, zc) in NB_ARCH.items():
        model_db = nb_model(pplib, nchan, nbin, 2)  # template channel 2 has weight 0

        def fake_load(filename, **kw):
            return model_db if filename == "nbmodel.fits" else archives[filename]
        pptoas.load_data = fake_load
        pptoas.file_is_type = lambda f, t: (t == "FITS" and f == "nbmodel.fits")
        gt = quiet_call(pptoas.GetTOAs, name, "nbmodel.fits", quiet=True)
        quiet_call(gt.get_narrowband_TOAs, quiet=True)
        lines = []
        for toa in gt.TOA_list:
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                pplib.write_TOAs(toa, outfile=None)
            lines.append(buf.getvalue().strip())
        meta[name] = dict(tim=lines, nchan=nchan, nbin=nbin, seed=seed, zero_chan=zc,
                          zero_model_chan=2)
        p = name.split(".")[0] + "_"
        for attr in ["phis", "phi_errs", "scales", "scale_errs", "channel_snrs",
                     "channel_red_chi2s"]:
            out[p + attr] = np.asarray(getattr(gt, attr)[0], dtype=float)
        out[p + "TOAs"] = np.array([[t.days, t.secs, t.fracsec] if t else [0, 0, 0.0]
                                    for t in gt.TOAs[0].ravel()])
        print("narrowband %s: %d TOAs" % (name, len(lines)))
    MG.save("narrowband.npz", **out)
    with open(os.path.join(HERE, "narrowband.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


# --------------------------------------------------------------------------
# Channel zapping (pptoas.py:1201-1278 get_channels_to_zap after get_TOAs;
# ppzap.py:18-48 get_zap_channels): an archive with a spiky channel, a noisy
# channel and a weak one.
# --------------------------------------------------------------------------
ZAP = dict(name="zapA.fits", nsub=3, nchan=32, nbin=512, seed=7007)


def zap_archive(pplib):
    z = ZAP
    db = synth_archive(pplib, z["name"], z["nsub"], z["nchan"], z["nbin"], z["seed"], 0.0, 0.0)
    return db


def gen_zap(pplib, pptoaslib, pptoas, ppzap):
    import shutil
    import tempfile
    db = zap_archive(pplib)
    db["subints"] = zap_perturb(db["subints"])
    db["noise_stds"] = np.array([pplib.get_noise(db["subints"][i, 0], chans=True)
                                 for i in range(db["nsub"])])[:, None]
    pptoas.load_data = lambda filename, **kw: db
    pptoas.file_is_type = lambda f, t: False
    tmpd = tempfile.mkdtemp()
    shutil.copy(MG.GMODEL, os.path.join(tmpd, "example.gmodel"))
    cwd = os.getcwd()
    os.chdir(tmpd)
    out = {}
    try:
        for tag, kw in [("default", {}), ("snr30", dict(SNR_threshold=30.0, rchi2_threshold=1.2)),
                        ("noiter", dict(SNR_threshold=30.0, iterate=False))]:
            gt = quiet_call(pptoas.GetTOAs, ZAP["name"], "example.gmodel", quiet=True)
            quiet_call(gt.get_TOAs, quiet=True)
            quiet_call(gt.get_channels_to_zap, **kw)
            for isub in range(ZAP["nsub"]):
                out["%s_rchi2_%d" % (tag, isub)] = np.array(gt.channel_red_chi2s[0][isub])
                out["%s_zap_%d" % (tag, isub)] = np.array(gt.zap_channels[0][isub], dtype=int)
            print("zap %s: %s" % (tag, gt.zap_channels[0]))
        for nstd in [3, 1]:
            zc = ppzap.get_zap_channels(db, nstd=nstd)
            for isub in range(ZAP["nsub"]):
                out["median_nstd%d_%d" % (nstd, isub)] = np.array(zc[isub], dtype=int)
            print("get_zap_channels nstd %d: %s" % (nstd, zc))
        out["noise_stds"] = db["noise_stds"]
    finally:
        os.chdir(cwd)
    MG.save("zap.npz", **out)


# --------------------------------------------------------------------------
# Template portraits (gen_gaussian_portrait / read_model, pplib.py:853-930,
# 2873-2959) for the device generator: the headline shape with Doppler-
# shifted channel frequencies, both evolution codes, and a scattered model.
# --------------------------------------------------------------------------
MODEL_CASES = [  # name, nchan, nbin, CODE, TAU [s], freq scale
    ("hl", 64, 2048, "000", 0.0, 1.0001),
    ("lin", 32, 512, "101", 0.0, 1.0),
    ("lin2", 16, 256, "011", 0.0, 0.9999),
    ("scat", 128, 1024, "000", 0.0003, 1.0),
]


def gen_models_r2(pplib):
    import tempfile
    out = {}
    src = open(MG.GMODEL).read()
    for name, nchan, nbin, code, tau, scale in MODEL_CASES:
        txt = src.replace("CODE    000", "CODE    " + code).replace(
            "TAU     0.00000000 1", "TAU     %.8f 1" % tau)
        path = os.path.join(tempfile.mkdtemp(), name + ".gmodel")
        open(path, "w").write(txt)
        freqs = MG.channel_freqs(nchan) * scale
        phases = pplib.get_bin_centers(nbin)
        _, _, model = pplib.read_model(path, phases, freqs, P0, quiet=True)
        out[name + "_freqs"] = freqs
        out[name + "_model"] = model
        out[name + "_gmodel"] = np.frombuffer(txt.encode(), dtype=np.uint8)
        print("model %s: %s, max %.6g" % (name, model.shape, np.max(np.abs(model))))
    MG.save("models_r2.npz", **out)


def main():
    what = sys.argv[1:] or ["fit", "configs", "align", "headline", "timing", "tncfloor",
                            "narrowband", "zap", "models"]
    np.seterr(all="ignore")
    if "headline" in what:
        gen_headline_2k()
    rest = [x for x in what if x != "headline"]
    if not rest:
        return
    tmp, pplib, pptoaslib, pptoas, ppalign = MG.load_reference()
    import shutil
    try:
        if "fit" in rest:
            gen_fit_r2(pplib, pptoaslib)
        if "configs" in rest:
            gen_configs(pplib, pptoaslib, pptoas)
        if "align" in rest:
            gen_align5(pplib, pptoaslib, ppalign)
        if "timing" in rest:
            gen_timing(pplib, pptoaslib)
        if "tncfloor" in rest:
            gen_tnc_floor(pplib, pptoaslib)
        if "narrowband" in rest:
            gen_narrowband(pplib, pptoaslib, pptoas)
        if "models" in rest:
            gen_models_r2(pplib)
        if "zap" in rest:
            import ppzap
            gen_zap(pplib, pptoaslib, pptoas, ppzap)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
