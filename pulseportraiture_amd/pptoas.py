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
                    load_spline_model_file,
                    read_model_device, gen_gaussian_portraits_device, scattering_alpha,
                    weighted_mean, write_TOAs)
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
        try:
            info = read_model(self.modelfile, quiet=True)
        except UnboundLocalError:  # not a .gmodel: a ppspline model (pptoas.py:375-378)
            return self._spline_models(data)
        name, code, nu_ref, ngauss, gparams, mflags, alpha, fit_alpha = info
        self.model_name, self.ngauss = name, ngauss
        if fit_scat:
            self.model_code, self.model_nu_ref = code, nu_ref
            self.gparams, self.alpha = gparams, alpha
        # one template per distinct (freqs, P-if-scattered) key, all built on
        # the device (ppf_gaussian_portraits): read_model per subint in the
        # reference (pptoas.py:351-378); fit_scat builds the unscattered one
        cache, keyf, keyP, idx = {}, [], [], np.zeros(nsub, dtype=np.int32)
        tau_P = gparams[1] != 0 and not fit_scat
        for isub in data.ok_isubs:
            P = data.Ps[isub]
            f = data.freqs[isub]
            key = (f.tobytes(), P if tau_P else None)
            if key not in cache:
                cache[key] = len(keyf)
                keyf.append(f)
                keyP.append(P)
            idx[isub] = cache[key]
        nbin = len(data.phases)
        models = np.empty((len(keyf), data.nchan, nbin))
        params = np.array(gparams, dtype=float)
        if fit_scat:
            params[1] = 0.0
            models[:] = gen_gaussian_portraits_device(code, params, 0.0, nbin, np.array(keyf),
                                                      nu_ref)
        elif not tau_P:
            models[:] = gen_gaussian_portraits_device(code, params, alpha, nbin, np.array(keyf),
                                                      nu_ref)
        else:  # read_model's TAU * nbin / P differs per period
            for P in sorted(set(keyP)):
                sel = [i for i, q in enumerate(keyP) if q == P]
                pp = np.copy(params)
                pp[1] *= nbin / P
                models[sel] = gen_gaussian_portraits_device(code, pp, alpha, nbin,
                                                            np.array([keyf[i] for i in sel]),
                                                            nu_ref)
        return models, idx, None

    def _spline_models(self, data):
        """ppspline templates: read_spline_model(modelfile, freqs[isub], nbin)
        per subint (pptoas.py:375-378), one device build per distinct channel
        frequency row (ppf_spline_portraits)."""
        name, source, datafile, mean_prof, eigvec, tck = load_spline_model_file(self.modelfile)
        self.model_name = name
        cache, keyf, idx = {}, [], np.zeros(data.nsub, dtype=np.int32)
        for isub in data.ok_isubs:
            f = data.freqs[isub]
            idx[isub] = cache.setdefault(f.tobytes(), len(keyf))
            if idx[isub] == len(keyf):
                keyf.append(f)
        from .engine import get_engine
        models = get_engine().spline_portraits(mean_prof, eigvec, tck, np.array(keyf),
                                               len(data.phases)).cpu().numpy()
        return models, idx, None

    def _irf_active(self):
        return bool(getattr(self, "add_instrumental_response", False)) and \
            bool(self.ird["DM"] or len(self.ird["wids"]))

    def _irf_models(self, models, midx, data, isubs):
        """Templates convolved with the instrumental response of each subint
        (pptoas.py:387-393: instrumental_response_port_FT(nbin, freqsx, DM, P,
        wids, irf_types) times rfft(modelx)), on the device.  The response
        depends on the subint only through P (DM smearing) and chan_bw =
        |freqsx[1] - freqsx[0]| of its ok channels; rows are convolved at
        every channel (masked ones are not fitted).  A one-channel subint,
        where the reference's chan_bw raises IndexError, gets chan_bw 0."""
        from .engine import get_engine
        eng = get_engine()
        ird = self.ird
        out, keys, idx = [], {}, np.zeros(data.nsub, dtype=np.int32)
        for isub in isubs:
            fx = data.freqs[isub, data.ok_ichans[isub]]
            cbw = abs(fx[1] - fx[0]) if len(fx) > 1 else 0.0
            P = data.Ps[isub]
            key = (int(midx[isub]), data.freqs[isub].tobytes(), cbw, P if ird["DM"] else None)
            if key not in keys:
                keys[key] = len(out)
                out.append(eng.instrumental_response_rows(
                    models[midx[isub]], data.freqs[isub], ird["DM"], P, ird["wids"],
                    ird["irf_types"], chan_bw=cbw).cpu().numpy())
            idx[isub] = keys[key]
        return np.stack(out), idx

    def get_TOAs(self, datafile=None, tscrunch=False, nu_refs=None, DM0=None, bary=True,
                 fit_DM=True, fit_GM=False, fit_scat=False, log10_tau=True, scat_guess=None,
                 fix_alpha=False, print_phase=False, print_flux=False, print_parangle=False,
                 add_instrumental_response=False, addtnl_toa_flags={}, method="trust-ncg",
                 bounds=None, nu_fits=None, show_plot=False, quiet=None):
        """pptoas.py:150-738 with the subint loop batched on the device."""
        if quiet is None:
            quiet = self.quiet
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
        self.tscrunch = tscrunch
        self.add_instrumental_response = add_instrumental_response
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

    def get_narrowband_TOAs(self, datafile=None, tscrunch=False, fit_scat=False,
                            log10_tau=True, scat_guess=None, print_phase=False,
                            print_flux=False, print_parangle=False,
                            add_instrumental_response=False, addtnl_toa_flags={},
                            method="trust-ncg", bounds=None, show_plot=False, quiet=None):
        """Narrowband TOAs: one FFTFIT per channel (pptoas.py:740-1125).

        Every (subint, channel) profile of every archive goes to the device in
        one ppf_phase_shift_batch call (brute force on linspace(-0.5, 0.5,
        100) + Nelder-Mead, pplib.py:2054-2100, with the load_data noise as
        err); TOAs, flags and the per-archive arrays follow the reference.
        As there, fit_scat is accepted but not fitted (tau = 0).  Reference
        quirks kept: channel_red_chi2s[isub] is set to the last channel's
        reduced chi2 for the whole row (pptoas.py:1011); channels whose
        template-archive weight is 0 are skipped (pptoas.py:966).  Where the
        reference cannot run -- a .gmodel template (model_data undefined,
        pptoas.py:966), isub > 0 of a tscrunched template, print_phase
        (results.phi, :1048) and print_flux (fluxes undefined, :1052) -- this
        build uses the template's single weight row, prints the fitted phase
        and prints the per-channel flux estimate.
        """
        if quiet is None:
            quiet = self.quiet
        self.nfit = 1 + 2 * int(bool(fit_scat))
        self.fit_phi, self.fit_tau = True, fit_scat
        self.fit_flags = [int(self.fit_phi), int(self.fit_tau)]
        self.log10_tau = log10_tau if fit_scat else False
        if not quiet:
            print("You are using an experimental functionality of pptoas!")
        self.scat_guess = scat_guess
        self.tscrunch = tscrunch
        self.add_instrumental_response = add_instrumental_response
        start = time.time()
        datafiles = self.datafiles if datafile is None else [datafile]
        from .pplib import get_bin_centers
        from .engine import get_engine
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
            nsub, nchan, nbin = data.nsub, data.nchan, data.nbin
            obs = DataBunch(telescope=data.telescope, backend=data.backend,
                            frontend=data.frontend)
            MJDs = np.array([data.epochs[i].in_days() for i in range(nsub)], dtype=np.double)
            mweights = None
            if self.is_FITS_model:
                md = _arch.load_data(self.modelfile)
                model = np.asarray((md.masks * md.subints)[0, 0])
                if md.nbin != nbin:
                    if not quiet:
                        print("Model nbin %d != data nbin %d for %s; skipping it." % (
                            md.nbin, nbin, name))
                    continue
                if md.nchan == 1:
                    model = np.tile(model[0], nchan).reshape(nchan, nbin)
                elif md.nchan != nchan:
                    if not quiet:
                        print("Model nchan %d != data nchan %d for %s; skipping it." % (
                            md.nchan, nchan, name))
                    continue
                mweights = np.asarray(md.weights)[0]
            models, midx = [], {}
            rows, mrows, noise, where = [], [], [], []
            subints = np.asarray(data.subints)
            irf = self._irf_active()
            spline = None
            for isub in data.ok_isubs:
                f = data.freqs[isub]
                kk = ("fits",) if self.is_FITS_model else (f.tobytes(), data.Ps[isub])
                if irf:  # modelx convolved per subint (pptoas.py:920-926)
                    kk = kk + (int(isub),)
                key = midx.setdefault(kk, len(models))
                if key == len(models):
                    if self.is_FITS_model:
                        m = model
                    else:
                        try:
                            m = read_model_device(self.modelfile, nbin, f, data.Ps[isub],
                                                  quiet=True)[2]
                        except UnboundLocalError:  # ppspline model (pptoas.py:912-915)
                            if spline is None:
                                spline = load_spline_model_file(self.modelfile)
                            m = get_engine().spline_portraits(spline[3], spline[4], spline[5],
                                                              f, nbin).cpu().numpy()
                    if irf:
                        fx = f[data.ok_ichans[isub]]
                        cbw = abs(fx[1] - fx[0]) if len(fx) > 1 else 0.0
                        m = get_engine().instrumental_response_rows(
                            np.asarray(m, dtype=np.float64), f, self.ird["DM"], data.Ps[isub],
                            self.ird["wids"], self.ird["irf_types"], chan_bw=cbw).cpu().numpy()
                    models.append(m)
                for ichan in data.ok_ichans[isub]:
                    if mweights is not None and mweights[ichan] == 0:
                        continue
                    rows.append(subints[isub, 0, ichan])
                    mrows.append(key * nchan + ichan)
                    ns = data.get("noise_stds")
                    noise.append(np.nan if ns is None else ns[isub, 0, ichan])
                    where.append((int(isub), int(ichan)))
            t0 = time.time()
            out = np.zeros((0, 6))
            if rows:
                mstack = np.concatenate(models, axis=0)
                out = get_engine().phase_shift_batch(
                    np.array(rows), mstack, noise=np.array(noise), Ns=100,
                    bounds=(-0.5, 0.5), model_idx=np.array(mrows, dtype=np.int32)).cpu().numpy()
            fit_duration = time.time() - t0
            z = lambda *sh: np.zeros(sh, dtype=np.float64)
            phis, phi_errs = z(nsub, nchan), z(nsub, nchan)
            TOAs = np.zeros([nsub, nchan], dtype="object")
            TOA_errs = np.zeros([nsub, nchan], dtype="object")
            taus, tau_errs = z(nsub, nchan), z(nsub, nchan)
            scales, scale_errs, channel_snrs = z(nsub, nchan), z(nsub, nchan), z(nsub, nchan)
            pfl, pfle = z(nsub, nchan), z(nsub, nchan)
            channel_red_chi2s = z(nsub, nchan)
            covariances = z(nsub, nchan, self.nfit, self.nfit)
            nfevals = np.zeros([nsub, nchan], dtype="int")
            rcs = np.zeros([nsub, nchan], dtype="int")
            for j, ((isub, ichan), (phase, phase_err, scale, scale_err, snr, red_chi2)) in \
                    enumerate(zip(where, out)):
                P = data.Ps[isub]
                toa = data.epochs[isub] + MJD(((phase * P) + data.backend_delay) / (3600 * 24.))
                toa_err = phase_err * P * 1e6
                if print_flux:
                    m = models[mrows[j] // nchan][ichan]
                    pfl[isub, ichan] = m.mean() * scale
                    pfle[isub, ichan] = abs(m.mean()) * scale_err
                phis[isub, ichan], phi_errs[isub, ichan] = phase, phase_err
                TOAs[isub, ichan], TOA_errs[isub, ichan] = toa, toa_err
                scales[isub, ichan], scale_errs[isub, ichan] = scale, scale_err
                channel_snrs[isub, ichan] = snr
                channel_red_chi2s[isub] = red_chi2  # the whole row (pptoas.py:1011)
                flags = {"be": data.backend, "fe": data.frontend,
                         "f": data.frontend + "_" + data.backend, "nbin": nbin,
                         "bw": abs(data.bw) / nchan, "subint": isub, "chan": ichan,
                         "tobs": data.subtimes[isub], "tmplt": self.modelfile, "snr": snr,
                         "gof": red_chi2}
                if print_phase:
                    flags["phs"] = phase
                    flags["phs_err"] = phase_err
                if print_flux:
                    flags["flux"] = pfl[isub, ichan]
                    flags["flux_err"] = pfle[isub, ichan]
                if print_parangle:
                    flags["par_angle"] = data.parallactic_angles[isub]
                for k, v in addtnl_toa_flags.items():
                    flags[k] = v
                self.TOA_list.append(TOA(name, data.freqs[isub, ichan], toa, toa_err,
                                         data.telescope, data.telescope_code, None, None,
                                         flags))
            for attr, val in [("order", name), ("obs", obs), ("doppler_fs", data.doppler_factors),
                              ("ok_isubs", np.asarray(data.ok_isubs)), ("epochs", data.epochs),
                              ("MJDs", MJDs), ("Ps", data.Ps), ("phis", phis),
                              ("phi_errs", phi_errs), ("TOAs", TOAs), ("TOA_errs", TOA_errs),
                              ("taus", taus), ("tau_errs", tau_errs), ("scales", scales),
                              ("scale_errs", scale_errs), ("channel_snrs", channel_snrs),
                              ("profile_fluxes", pfl), ("profile_flux_errs", pfle),
                              ("covariances", covariances),
                              ("channel_red_chi2s", channel_red_chi2s), ("nfevals", nfevals),
                              ("rcs", rcs), ("fit_durations", fit_duration)]:
                getattr(self, attr).append(val)
            if not quiet:
                print("--------------------------")
                print(name)
                print("~%.4f sec/TOA" % (fit_duration / max(len(self.TOA_list), 1)))
        if not quiet and len(self.ok_isubs):
            tot = time.time() - start
            print("--------------------------")
            print("Total time: %.2f sec, ~%.4f sec/TOA" % (tot, tot / max(len(self.TOA_list), 1)))

    # -- fitted portraits, residuals and channel zapping --------------------
    def _fitted_rows(self, datafile, isubs, quiet):
        """Inputs of show_fit (pptoas.py:1324-1402) for the subints isubs of
        one fitted archive, as device rows: for every ok channel of every
        subint, the data row, its rotate_portrait_full phase, its template
        row (de-duplicated templates + row index), the fitted scale, the
        scattering time [rot] and the channel noise."""
        from .pptoaslib import phase_shifts
        from .pplib import scattering_times
        ok_files = list(np.array(self.datafiles)[self.ok_idatafiles])
        ifile = ok_files.index(datafile)
        # rm_baseline=True as in show_fit; archives reach this build already
        # loaded (PSRCHIVE's baseline removal is out of scope, archive.py)
        data = _arch.load_data(datafile, dedisperse=False, dededisperse=False,
                               tscrunch=getattr(self, "tscrunch", False), pscrunch=True,
                               rm_baseline=True, quiet=quiet)
        if data.dmc:
            raise RuntimeError("dedispersed archive: dededispersion needs PSRCHIVE")
        nbin = data.nbin
        irf = self._irf_active()
        spline = None
        subints = np.asarray(data.subints)
        models, mkeys = [], {}
        rows, ph, mrow, sc, taus, noise, where = [], [], [], [], [], [], []
        for isub in isubs:
            phi = self.phis[ifile][isub]
            DM = self.DMs[ifile][isub]
            GM = self.GMs[ifile][isub]
            if self.bary:  # pptoas.py:1348-1350, whatever was fitted
                DM /= self.doppler_fs[ifile][isub]
                GM /= self.doppler_fs[ifile][isub] ** 3
            freqs = data.freqs[isub]
            nu_ref_DM, nu_ref_GM, nu_ref_tau = self.nu_refs[ifile][isub]
            P = data.Ps[isub]
            tau = self.taus[ifile][isub]
            if self.is_FITS_model:
                key = ("fits",)
            elif tau != 0.0:
                key = ("unscattered", freqs.tobytes())
            else:
                key = ("model", freqs.tobytes())
            if irf:  # the response depends on the subint (pptoas.py:1382-1388)
                key = key + (int(isub),)
            if key not in mkeys:
                mkeys[key] = len(models)
                if self.is_FITS_model:
                    md = _arch.load_data(self.modelfile)
                    m = np.asarray((md.masks * md.subints)[0, 0])
                    if md.nchan == 1:
                        m = np.tile(m[0], len(freqs)).reshape(len(freqs), md.nbin)
                elif tau != 0.0:
                    info = read_model(self.modelfile, quiet=True)
                    gparams = np.copy(info[4])
                    gparams[1] = 0.0
                    m = gen_gaussian_portraits_device(info[1], gparams, 0.0, nbin, freqs, info[2])
                else:
                    try:
                        m = read_model_device(self.modelfile, nbin, freqs, data.Ps.mean(),
                                              quiet=True)[2]
                    except UnboundLocalError:  # ppspline model (pptoas.py:1380-1381)
                        if spline is None:
                            spline = load_spline_model_file(self.modelfile)
                        from .engine import get_engine
                        m = get_engine().spline_portraits(spline[3], spline[4], spline[5],
                                                          freqs, nbin).cpu().numpy()
                if irf:
                    fx = freqs[data.ok_ichans[isub]]
                    cbw = abs(fx[1] - fx[0]) if len(fx) > 1 else 0.0
                    from .engine import get_engine
                    m = get_engine().instrumental_response_rows(
                        np.asarray(m, dtype=np.float64), freqs, self.ird["DM"], P,
                        self.ird["wids"], self.ird["irf_types"], chan_bw=cbw).cpu().numpy()
                models.append(np.asarray(m, dtype=np.float64))
            k = mkeys[key]
            phs = phase_shifts(phi, DM, GM, freqs, nu_ref_DM, nu_ref_GM, P)
            if tau != 0.0:
                t = 10 ** tau if self.log10_tau else tau
                tch = scattering_times(t, self.alphas[ifile][isub], freqs, nu_ref_tau)
            else:
                tch = np.zeros(len(freqs))
            ns = data.get("noise_stds")
            for ichan in data.ok_ichans[isub]:
                rows.append(subints[isub, 0, ichan])
                ph.append(phs[ichan])
                mrow.append(k * data.nchan + ichan)
                sc.append(self.scales[ifile][isub][ichan])
                taus.append(tch[ichan])
                noise.append(np.nan if ns is None else ns[isub, 0, ichan])
                where.append((int(isub), int(ichan)))
        return DataBunch(data=data, ifile=ifile, rows=np.array(rows).reshape(-1, nbin),
                         phase=np.array(ph), models=np.concatenate(models, 0) if models else
                         np.zeros((0, nbin)), model_row=np.array(mrow, dtype=np.int32),
                         scale=np.array(sc), tau=np.array(taus), noise=np.array(noise),
                         where=where)

    def show_fit(self, datafile=None, isub=0, rotate=0.0, show=True, return_fit=False,
                 savefig=False, quiet=None):
        """Fitted portrait and scaled template of one subint (pptoas.py:1310-1412):
        the data rotated by the fitted phi/DM/GM (rotate_portrait_full) and
        the (scattered) template times the fitted channel scales, formed on
        the device.  Plotting (show_residual_plot) is out of scope: show only
        prints a note."""
        if quiet is None:
            quiet = self.quiet
        if datafile is None:
            datafile = self.datafiles[0]
        from .engine import get_engine
        eng = get_engine()
        fr = self._fitted_rows(datafile, [isub], quiet)
        data = fr.data
        nchan, nbin = data.nchan, data.nbin
        ok = np.asarray(data.ok_ichans[isub])
        port = np.zeros((nchan, nbin))
        model_scaled = np.zeros((nchan, nbin))
        if len(ok):
            port[ok] = eng.scatter_rotate_rows(fr.rows, fr.phase + rotate).cpu().numpy()
            ms = eng.scatter_rotate_rows(fr.models[fr.model_row], np.full(len(ok), rotate),
                                         fr.tau).cpu().numpy()
            model_scaled[ok] = fr.scale[:, None] * ms
        # channels outside ok_ichans stay 0: masked data (port *= masks) and
        # a zero fitted scale
        port *= np.asarray(data.masks[isub, 0])
        if show and not quiet:
            print("show_fit: plotting is not part of this build; use return_fit=True")
        if return_fit:
            ns = data.get("noise_stds")
            noise = ns[isub, 0] if ns is not None else \
                eng.noise_rows(np.asarray(data.subints)[isub, 0]).cpu().numpy()
            return port, model_scaled, data.ok_ichans[isub], data.freqs[isub], noise

    def get_channels_to_zap(self, SNR_threshold=8.0, rchi2_threshold=1.3, iterate=True,
                            show=False):
        """Flag channels by reduced chi2 and S/N (pptoas.py:1201-1278); needs
        get_TOAs first.  Every ok channel of every ok subint of an archive
        goes to the device in one ppf_resid_chi2_rows call (rotation,
        scattering, scaling and the chi2 sum fused per channel); the
        thresholds and the iterated S/N cut run on the host as there."""
        from .engine import get_engine
        eng = get_engine()
        for iarch, ok_idatafile in enumerate(self.ok_idatafiles):
            datafile = self.datafiles[ok_idatafile]
            ok_isubs = list(self.ok_isubs[iarch])
            fr = self._fitted_rows(datafile, ok_isubs, True)
            data = fr.data
            chi2 = np.zeros(0)
            if len(fr.where):
                noise = fr.noise
                if np.isnan(noise).any():  # load_data's get_noise on the device
                    est = eng.noise_rows(fr.rows).cpu().numpy()
                    noise = np.where(np.isnan(noise), est, noise)
                chi2 = eng.resid_chi2_rows(fr.rows, fr.phase, fr.models, fr.scale, noise,
                                           data.nbin - 2, tau=fr.tau,
                                           model_row=fr.model_row).cpu().numpy()
            per_sub = {}
            for (isub, ichan), c in zip(fr.where, chi2):
                per_sub.setdefault(isub, []).append(c)
            channel_red_chi2s, zap_channels = [], []
            for isub in ok_isubs:
                ok_ichans = list(data.ok_ichans[isub])
                red_chi2s = list(per_sub.get(int(isub), []))
                channel_snrs = self.channel_snrs[iarch][isub]
                thr = (SNR_threshold ** 2.0 / len(ok_ichans)) ** 0.5
                bad = []
                for ok_ichan, c in zip(ok_ichans, red_chi2s):
                    if c > rchi2_threshold or np.isnan(c):
                        bad.append(ok_ichan)
                    elif SNR_threshold and channel_snrs[ok_ichan] < thr:
                        bad.append(ok_ichan)
                channel_red_chi2s.append(red_chi2s)
                zap_channels.append(bad)
                if iterate and SNR_threshold and len(bad):
                    old_len = len(bad)
                    added_new = True
                    while added_new and (len(ok_ichans) - len(bad)):
                        thr = (SNR_threshold ** 2.0 / (len(ok_ichans) - len(bad))) ** 0.5
                        for ok_ichan in ok_ichans:
                            if ok_ichan in bad:
                                continue
                            if channel_snrs[ok_ichan] < thr:
                                bad.append(ok_ichan)
                        added_new = bool(len(bad) - old_len)
                        old_len = len(bad)
                if show and len(bad):
                    print("%s, subint: %d  bad chans: %s" % (datafile, isub, bad))
            self.channel_red_chi2s.append(channel_red_chi2s)
            self.zap_channels.append(zap_channels)

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
        if self._irf_active():
            models, midx = self._irf_models(models, midx, data, ok_isubs)
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
