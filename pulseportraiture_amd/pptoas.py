"""pptoas drop-in: wideband TOAs/DMs with the fits batched on the GPU.

``GetTOAs(datafiles, modelfile).get_TOAs(...)`` reproduces pptoas.py:81-738:
per archive it builds the per-subint templates, then hands every ok subint
to one ``ppf_fit_portrait_batch`` call (guess, fit and post-fit on device),
and assembles TOA records, Doppler-corrected DMs, flags and the DeltaDM mean
on the host.  Archives come from ``archive.load_data`` (PSRCHIVE is out of
scope; see archive.py).
"""
import time

import numpy as np

from . import archive as _arch
from .mjd import MJD
from .pplib import (DataBunch, F0_fact, phase_transform, guess_fit_freq, read_model,
                    gen_gaussian_portrait, scattering_alpha, weighted_mean, write_TOAs)
from .pptoaslib import fit_portraits_batch, report_failure

max_nfile = 999
rm_baseline = bool(F0_fact)  # pptoas.py:25-29


def _dist_info():
    """(rank, world) of an initialised torch.distributed group, else (0, 1)."""
    try:
        import torch.distributed as dist
    except ImportError:
        return 0, 1
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _shard_range(n, rank, world):
    """Contiguous [lo, hi) of n units for rank; sizes differ by at most one."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class TOA:
    """TOA record, pptoas.py:31-73."""

    def __init__(self, archive, frequency, MJD, TOA_error, telescope, telescope_code,
                 DM=None, DM_error=None, flags={}):
        self.archive = archive
        self.frequency = frequency
        self.MJD = MJD
        self.TOA_error = TOA_error
        self.telescope = telescope
        self.telescope_code = telescope_code
        self.DM = DM
        self.DM_error = DM_error
        self.flags = flags
        for k, v in flags.items():
            setattr(self, k, v)

    def write_TOA(self, inf_is_zero=True, outfile=None):
        return write_TOAs(self, inf_is_zero=inf_is_zero, outfile=outfile, append=True)


_LIST_ATTRS = ["obs", "doppler_fs", "nu0s", "nu_fits", "nu_refs", "ok_idatafiles", "ok_isubs",
               "epochs", "MJDs", "Ps", "phis", "phi_errs", "TOAs", "TOA_errs", "DM0s", "DMs",
               "DM_errs", "DeltaDM_means", "DeltaDM_errs", "GMs", "GM_errs", "taus",
               "tau_errs", "alphas", "alpha_errs", "scales", "scale_errs", "snrs",
               "channel_snrs", "profile_fluxes", "profile_flux_errs", "fluxes", "flux_errs",
               "flux_freqs", "red_chi2s", "channel_red_chi2s", "covariances", "nfevals",
               "rcs", "fit_durations", "order", "TOA_list", "zap_channels"]


class GetTOAs:
    """Measure TOAs and DMs from wideband data (pptoas.py:75-738)."""

    def __init__(self, datafiles, modelfile, quiet=False):
        if isinstance(datafiles, (list, tuple)):
            self.datafiles = list(datafiles)
        elif _arch.file_is_type(datafiles, "ASCII"):
            self.datafiles = [ln.strip() for ln in open(datafiles).readlines() if ln.strip()]
        else:
            self.datafiles = [datafiles]
        if len(self.datafiles) > max_nfile:
            raise SystemExit("Too many archives.  See/change max_nfile(=%d)." % max_nfile)
        self.is_FITS_model = _arch.file_is_type(modelfile, "FITS")
        self.modelfile = modelfile
        for a in _LIST_ATTRS:
            setattr(self, a, [])
        self.instrumental_response_dict = self.ird = {"DM": 0.0, "wids": [], "irf_types": []}
        self.quiet = quiet

    # -- per-subint templates ------------------------------------------------
    def _models(self, data, fit_scat, quiet):
        """Template portrait per ok subint (pptoas.py:351-378), de-duplicated."""
        nsub = data.nsub
        if self.is_FITS_model:
            md = _arch.load_data(self.modelfile)
            model = (md.masks * md.subints)[0, 0]
            if md.nbin != data.nbin or md.nchan != data.nchan:
                return None
            return np.asarray(model)[None], np.zeros(nsub, dtype=np.int32), None
        info = read_model(self.modelfile, quiet=True)
        name, code, nu_ref, ngauss, gparams, mflags, alpha, fit_alpha = info
        self.model_name, self.ngauss = name, ngauss
        if fit_scat:
            self.model_code, self.model_nu_ref = code, nu_ref
            self.gparams, self.alpha = gparams, alpha
        cache, models, idx = {}, [], np.zeros(nsub, dtype=np.int32)
        for isub in data.ok_isubs:
            P = data.Ps[isub]
            f = data.freqs[isub]
            key = (f.tobytes(), P if (gparams[1] != 0 and not fit_scat) else None)
            if key not in cache:
                if not fit_scat:
                    m = read_model(self.modelfile, data.phases, f, P, quiet=True)[2]
                else:
                    up = np.copy(gparams)
                    up[1] = 0.0
                    m = gen_gaussian_portrait(code, up, 0.0, data.phases, f, nu_ref)
                cache[key] = len(models)
                models.append(m)
            idx[isub] = cache[key]
        return np.array(models), idx, None

    def get_TOAs(self, datafile=None, tscrunch=False, nu_refs=None, DM0=None, bary=True,
                 fit_DM=True, fit_GM=False, fit_scat=False, log10_tau=True, scat_guess=None,
                 fix_alpha=False, print_phase=False, print_flux=False, print_parangle=False,
                 add_instrumental_response=False, addtnl_toa_flags={}, method="trust-ncg",
                 bounds=None, nu_fits=None, show_plot=False, quiet=None):
        """pptoas.py:150-738 with the subint loop batched on the device."""
        if quiet is None:
            quiet = self.quiet
        if add_instrumental_response and (self.ird["DM"] or len(self.ird["wids"])):
            raise NotImplementedError("instrumental response convolution (pptoas.py:387-393)")
        if tscrunch:
            raise NotImplementedError("tscrunch needs PSRCHIVE (out of scope)")
        already_warned = False
        warning = "You are using an experimental functionality of pptoas!"
        self.nfit = 1 + int(fit_DM) + int(fit_GM) + 2 * int(fit_scat) - int(fix_alpha)
        self.fit_phi, self.fit_DM, self.fit_GM = True, fit_DM, fit_GM
        self.fit_tau = self.fit_alpha = fit_scat
        if fit_scat:
            self.fit_alpha = not fix_alpha
        self.fit_flags = [int(self.fit_phi), int(self.fit_DM), int(self.fit_GM),
                          int(self.fit_tau), int(self.fit_alpha)]
        self.log10_tau = log10_tau
        if not fit_scat:
            self.log10_tau = log10_tau = False
        if self.fit_GM or fit_scat:
            if not quiet:
                print(warning)
            already_warned = True
        self.scat_guess = scat_guess
        self.DM0, self.bary = DM0, bary
        self._fit_flags_prev = None  # the reference's loop-carried fit_flags
        start = time.time()
        datafiles = self.datafiles if datafile is None else [datafile]
        # 1. load and prepare every archive (all ranks: host bookkeeping only)
        jobs = []
        for iarch, datafile in enumerate(datafiles):
            try:
                data = _arch.load_data(datafile, dedisperse=False, dededisperse=False,
                                       tscrunch=tscrunch, pscrunch=True, rm_baseline=rm_baseline,
                                       quiet=quiet)
                if data.dmc:
                    raise RuntimeError("dedispersed archive: dededispersion needs PSRCHIVE")
                if not len(data.ok_isubs):
                    if not quiet:
                        print("No subints to fit for %s.  Skipping it." % datafile)
                    continue
                self.ok_idatafiles.append(iarch)
            except RuntimeError:
                if not quiet:
                    print("Cannot load_data(%s).  Skipping it." % datafile)
                continue
            name = datafile if isinstance(datafile, str) else data.filename
            job = self._prepare(name, data, nu_refs, nu_fits, fit_scat, method, bounds, quiet)
            if job is not None:
                jobs.append(job)
        # 2. fit: the (archive, subint) units in get_TOAs order are split into
        #    contiguous shards, one per rank (torch.distributed, one process per
        #    GPU); no collective on the fit path
        rank, world = _dist_info()
        units = [(ij, isub) for ij, job in enumerate(jobs) for isub in job.ok_isubs]
        lo, hi = _shard_range(len(units), rank, world)
        results, durations = self._fit_units(jobs, units[lo:hi], fit_scat, method)
        # 3. gather every rank's per-subint results (small host dicts), then
        #    every rank assembles the same TOAs in the reference's order
        if world > 1:
            import torch.distributed as dist
            parts = [None] * world
            dist.all_gather_object(parts, (results, durations))
            results, durations = {}, {}
            for res_r, dur_r in parts:
                results.update(res_r)
                for ij, t in dur_r.items():
                    durations[ij] = durations.get(ij, 0.0) + t
        for ij, job in enumerate(jobs):
            res_all = {isub: results[(ij, isub)] for isub in job.ok_isubs}
            self._assemble(job.name, job.data, job.obs, job.DM0, job.MJDs, job.ok_isubs,
                           job.fit_flags_sub, res_all, job.nu_fits_a, job.nu_refs_a,
                           job.models, job.midx, print_phase, print_flux, print_parangle,
                           addtnl_toa_flags, durations.get(ij, 0.0), quiet)
        tot = time.time() - start
        if not quiet and len(self.ok_isubs):
            n = np.array([len(x) for x in self.ok_isubs]).sum()
            print("--------------------------")
            print("Total time: %.2f sec, ~%.4f sec/TOA" % (tot, tot / n))

    def _prepare(self, datafile, data, nu_ref_tuple, nu_fit_tuple, fit_scat, method, bounds,
                 quiet):
        """Per-archive set-up of pptoas.py:246-484: templates, reference
        frequencies, initial parameters and the per-subint fit flags."""
        nsub, nchan, nbin = data.nsub, data.nchan, data.nbin
        obs = DataBunch(telescope=data.telescope, backend=data.backend, frontend=data.frontend)
        DM_stored = data.DM
        DM0 = DM_stored if self.DM0 is None else self.DM0
        MJDs = np.array([data.epochs[i].in_days() for i in range(nsub)], dtype=np.double)
        ok_isubs = np.asarray(data.ok_isubs)
        mm = self._models(data, fit_scat, quiet)
        if mm is None:
            if not quiet:
                print("Model nbin/nchan mismatch for %s; skipping it." % datafile)
            return None
        models, midx, _ = mm
        mask = np.zeros((nsub, nchan), dtype=np.uint8)
        for isub in ok_isubs:
            mask[isub, data.ok_ichans[isub]] = 1
        # per-subint reference frequencies, guesses and flag sets (pptoas.py:383-484)
        nu_fits_a = np.zeros((nsub, 3))
        nu_refs_a = np.full((nsub, 3), np.nan)
        init = np.zeros((nsub, 5))
        guess_tau = np.zeros(nsub)
        fit_flags_sub = {}
        for isub in ok_isubs:
            ok = data.ok_ichans[isub]
            freqsx = data.freqs[isub, ok]
            P = data.Ps[isub]
            if nu_fit_tuple is None:
                nu_fit = guess_fit_freq(freqsx, data.SNRs[isub, 0, ok])
                nu_fits_a[isub] = [nu_fit] * 3
            else:
                nu_fits_a[isub] = [nu_fit_tuple[0], nu_fit_tuple[0], nu_fit_tuple[-1]]
            if nu_ref_tuple is not None:
                nu_refs_a[isub] = [nu_ref_tuple[0], nu_ref_tuple[0], nu_ref_tuple[-1]]
                if self.bary and nu_ref_tuple[-1]:
                    nu_refs_a[isub, 2] /= data.doppler_factors[isub]
            tau_g = alpha_g = 0.0
            if fit_scat:
                nu_fit_tau = nu_fits_a[isub, 2]
                if self.scat_guess is not None:
                    ts, tref, alpha_g = self.scat_guess
                    tau_g = (ts / P) * (nu_fit_tau / tref) ** alpha_g
                else:
                    alpha_g = self.alpha if hasattr(self, "alpha") else scattering_alpha
                    tau_g = (self.gparams[1] / P) * (nu_fit_tau / self.model_nu_ref) ** alpha_g \
                        if hasattr(self, "gparams") else 0.0
                guess_tau[isub] = tau_g
                if self.log10_tau:
                    if tau_g == 0.0:
                        tau_g = nbin ** -1
                    tau_g = np.log10(tau_g)
            init[isub] = [0.0, DM_stored, 0.0, tau_g, alpha_g]
            # pptoas.py:474-484 verbatim in effect: get_TOAs keeps one
            # fit_flags list across subints and archives, and a 2-channel
            # subint (fit_DM and fit_GM) zeroes GM in the *previous* subint's
            # list -- phase-only after a 1-channel subint, and an
            # UnboundLocalError when no subint came before it.
            if len(freqsx) == 1:
                ff = [1, 0, 0, 0, 0]
            elif len(freqsx) == 2 and self.fit_DM and self.fit_GM:
                if self._fit_flags_prev is None:
                    raise UnboundLocalError(
                        "local variable 'fit_flags' referenced before assignment")
                ff = list(self._fit_flags_prev)
                ff[2] = 0
            else:
                ff = list(self.fit_flags)
            self._fit_flags_prev = ff
            fit_flags_sub[isub] = ff
        if bounds is None and method == "TNC":
            # get_TOAs' default TNC bounds (pptoas.py:458-467)
            bounds = [(None, None), (None, None), (None, None),
                      (np.log10((10 * nbin) ** -1), None) if self.log10_tau else (0.0, None),
                      (-10.0, 10.0)]
        return DataBunch(name=datafile, data=data, obs=obs, DM0=DM0, MJDs=MJDs,
                         ok_isubs=ok_isubs, models=models, midx=midx, mask=mask,
                         nu_fits_a=nu_fits_a, nu_refs_a=nu_refs_a, init=init,
                         guess_tau=guess_tau, fit_flags_sub=fit_flags_sub, bounds=bounds)

    def _fit_units(self, jobs, units, fit_scat, method):
        """Fit this rank's (archive, subint) units: one batched device call per
        archive and flag set.  Returns {(archive, subint): one-row result dict}
        and the fit wall time per archive."""
        results, durations = {}, {}
        by_arch = {}
        for ij, isub in units:
            by_arch.setdefault(ij, []).append(isub)
        for ij, subs_all in by_arch.items():
            job = jobs[ij]
            data = job.data
            subints = np.asarray(data.subints)[:, 0]
            errs = None if data.get("noise_stds") is None else data.noise_stds[:, 0]
            flag_sets = {}
            for isub in subs_all:
                flag_sets.setdefault(tuple(job.fit_flags_sub[isub]), []).append(isub)
            for ff, subs in flag_sets.items():
                subs = np.array(subs)
                t0 = time.time()
                # errs None: the device estimates get_noise_PS per channel,
                # as load_data's noise_stds (pplib.py:2744-2748)
                res = fit_portraits_batch(
                    subints[subs], job.models, job.init[subs], data.Ps[subs], data.freqs[subs],
                    nu_fits=job.nu_fits_a[subs], nu_outs=job.nu_refs_a[subs],
                    errs=None if errs is None else errs[subs], fit_flags=list(ff),
                    log10_tau=self.log10_tau, option=0, is_toa=True,
                    chan_mask=job.mask[subs], weights=data.weights[subs],
                    model_idx=job.midx[subs], guess=True, guess_Ns=100, guess_wrap=True,
                    guess_nu=None, guess_tau=job.guess_tau[subs] if fit_scat else None,
                    method=method, bounds=job.bounds)
                durations[ij] = durations.get(ij, 0.0) + time.time() - t0
                for j, isub in enumerate(subs):
                    results[(ij, int(isub))] = {k: np.asarray(v)[j:j + 1] for k, v in res.items()}
        return results, durations

    def _assemble(self, datafile, data, obs, DM0, MJDs, ok_isubs, fit_flags_sub, res_all,
                  nu_fits_a, nu_refs_a, models, midx, print_phase, print_flux,
                  print_parangle, addtnl_toa_flags, fit_duration, quiet):
        """Host bookkeeping of pptoas.py:522-720 from the device results."""
        nsub, nchan, nbin = data.nsub, data.nchan, data.nbin
        z = lambda *s: np.zeros(s, dtype=np.float64)
        phis, phi_errs, DMs, DM_errs = z(nsub), z(nsub), z(nsub), z(nsub)
        GMs, GM_errs, taus, tau_errs = z(nsub), z(nsub), z(nsub), z(nsub)
        alphas, alpha_errs, snrs, red_chi2s = z(nsub), z(nsub), z(nsub), z(nsub)
        fluxes, flux_errs, flux_freqs = z(nsub), z(nsub), z(nsub)
        scales, scale_errs, chsnrs = z(nsub, nchan), z(nsub, nchan), z(nsub, nchan)
        pfl, pfle = z(nsub, nchan), z(nsub, nchan)
        covs = z(nsub, self.nfit, self.nfit)
        nfevals = np.zeros(nsub, dtype="int")
        rcs = np.zeros(nsub, dtype="int")
        TOAs = np.zeros(nsub, dtype="object")
        TOA_errs = np.zeros(nsub, dtype="object")
        nu_fits = list(nu_fits_a)
        nu_refs = [list(r) for r in nu_refs_a]
        for isub in ok_isubs:
            res, j = res_all[int(isub)], 0
            ff = fit_flags_sub[isub]
            ok = data.ok_ichans[isub]
            freqsx = data.freqs[isub, ok]
            P = data.Ps[isub]
            p, e = res["params"][j], res["param_errs"][j]
            phi, phi_err = p[0], e[0]
            DM, DM_err, GM, GM_err = p[1], e[1], p[2], e[2]
            report_failure(int(res["status"][j]), "%s_%d" % (datafile, isub))
            toa_mjd = data.epochs[isub] + MJD(((phi * P) + data.backend_delay) / (3600 * 24.))
            TOA_err = phi_err * P * 1e6
            if self.bary:
                df = data.doppler_factors[isub]
                if ff[1]:
                    DM *= df
                if ff[2]:
                    GM *= df ** 3
            else:
                df = 1.0
            sc = res["scales"][j][ok]
            sce = res["scale_errs"][j][ok]
            if print_flux:
                # scattering keeps each row's mean, so the scattered model's
                # channel means are the template's (pptoas.py:553-575)
                means = models[midx[isub]][ok].mean(axis=1)
                pfl[isub, ok] = means * sc
                pfle[isub, ok] = abs(means) * sce
                fluxes[isub], flux_errs[isub] = weighted_mean(pfl[isub, ok], pfle[isub, ok])
                flux_freqs[isub] = weighted_mean(freqsx, pfle[isub, ok])[0]
            nuo = res["nu_out"][j]
            nu_refs[isub] = [nuo[0], nuo[1], nuo[2]]
            phis[isub], phi_errs[isub] = phi, phi_err
            TOAs[isub], TOA_errs[isub] = toa_mjd, TOA_err
            DMs[isub], DM_errs[isub], GMs[isub], GM_errs[isub] = DM, DM_err, GM, GM_err
            taus[isub], tau_errs[isub] = p[3], e[3]
            alphas[isub], alpha_errs[isub] = p[4], e[4]
            nfevals[isub], rcs[isub] = res["nfev"][j], res["status"][j]
            scales[isub, ok], scale_errs[isub, ok] = sc, sce
            snrs[isub] = res["snr"][j]
            chsnrs[isub, ok] = res["channel_snrs"][j][ok]
            nf = int(np.sum(ff))
            cm = res["cov"][j][:nf, :nf]
            try:
                covs[isub] = cm
            except ValueError:
                for ii, ifit in enumerate(np.where(ff)[0]):
                    for jj, jfit in enumerate(np.where(ff)[0]):
                        covs[isub][ifit, jfit] = cm[ii, jj]
            red_chi2s[isub] = res["red_chi2"][j]
            flags = {}
            DM_out, DM_err_out = DM, DM_err
            if not ff[1]:
                DM_out = DM_err_out = None
            if ff[2]:
                flags["gm"] = GM
                flags["gm_err"] = GM_err
            if ff[3]:
                if self.log10_tau:
                    flags["scat_time"] = 10 ** p[3] * P / df * 1e6
                    flags["log10_scat_time"] = p[3] + np.log10(P / df)
                    flags["log10_scat_time_err"] = e[3]
                else:
                    flags["scat_time"] = p[3] * P / df * 1e6
                    flags["scat_time_err"] = e[3] * P / df * 1e6
                flags["scat_ref_freq"] = nuo[2] * df
                flags["scat_ind"] = p[4]
            if ff[4]:
                flags["scat_ind_err"] = e[4]
            flags["be"] = data.backend
            flags["fe"] = data.frontend
            flags["f"] = data.frontend + "_" + data.backend
            flags["nbin"] = nbin
            flags["nch"] = nchan
            flags["nchx"] = len(freqsx)
            flags["bw"] = freqsx.max() - freqsx.min()
            flags["chbw"] = abs(data.bw) / nchan
            flags["subint"] = int(isub)
            flags["tobs"] = data.subtimes[isub]
            flags["fratio"] = freqsx.max() / freqsx.min()
            flags["tmplt"] = self.modelfile
            flags["snr"] = res["snr"][j]
            if not np.isnan(nu_refs_a[isub][0]) and np.all(ff[:2]):
                flags["phi_DM_cov"] = cm[0, 1]
            flags["gof"] = res["red_chi2"][j]
            if print_phase:
                flags["phs"] = phi
                flags["phs_err"] = phi_err
            if print_flux:
                flags["flux"] = fluxes[isub]
                flags["flux_err"] = flux_errs[isub]
                flags["flux_ref_freq"] = flux_freqs[isub]
            if print_parangle:
                flags["par_angle"] = data.parallactic_angles[isub]
            for k, v in addtnl_toa_flags.items():
                flags[k] = v
            self.TOA_list.append(TOA(datafile, nuo[0], toa_mjd, TOA_err, data.telescope,
                                     data.telescope_code, DM_out, DM_err_out, flags))
        # DeltaDM weighted mean per archive (pptoas.py:664-681)
        DeltaDMs = DMs - DM0
        ok = ok_isubs
        w = DM_errs[ok] ** -2 if np.all(DM_errs[ok]) else np.ones(len(ok))
        mean, wsum = np.average(DeltaDMs[ok], weights=w, returned=True)
        var = wsum ** -1
        if len(ok) > 1:
            var *= np.sum(((DeltaDMs[ok] - mean) ** 2) * w) / (len(DeltaDMs[ok]) - 1)
        for attr, val in [("order", datafile), ("obs", obs), ("doppler_fs", data.doppler_factors),
                          ("nu0s", data.nu0), ("nu_fits", nu_fits), ("nu_refs", nu_refs),
                          ("ok_isubs", ok_isubs), ("epochs", data.epochs), ("MJDs", MJDs),
                          ("Ps", data.Ps), ("phis", phis), ("phi_errs", phi_errs),
                          ("TOAs", TOAs), ("TOA_errs", TOA_errs), ("DM0s", DM0),
                          ("DMs", DMs), ("DM_errs", DM_errs), ("DeltaDM_means", mean),
                          ("DeltaDM_errs", var ** 0.5), ("GMs", GMs), ("GM_errs", GM_errs),
                          ("taus", taus), ("tau_errs", tau_errs), ("alphas", alphas),
                          ("alpha_errs", alpha_errs), ("scales", scales),
                          ("scale_errs", scale_errs), ("snrs", snrs),
                          ("channel_snrs", chsnrs), ("profile_fluxes", pfl),
                          ("profile_flux_errs", pfle), ("fluxes", fluxes),
                          ("flux_errs", flux_errs), ("flux_freqs", flux_freqs),
                          ("covariances", covs), ("red_chi2s", red_chi2s),
                          ("nfevals", nfevals), ("rcs", rcs),
                          ("fit_durations", fit_duration)]:
            getattr(self, attr).append(val)
        if not quiet:
            print("--------------------------")
            print(datafile)
            print("~%.4f sec/TOA" % (fit_duration / len(ok_isubs)))
            print("Med. TOA error is %.3f us" % (np.median(phi_errs[ok_isubs]) *
                                                 data.Ps.mean() * 1e6))
