"""pptoas drop-in: wideband TOAs/DMs with the fits batched on the GPU.

``GetTOAs(datafiles, modelfile).get_TOAs(...)`` reproduces pptoas.py:81-738:
per archive it builds the per-subint templates, then hands every ok subint
to one ``ppf_fit_portrait_batch`` call (guess, fit and post-fit on device),
and assembles TOA records, Doppler-corrected DMs, flags and the DeltaDM mean
on the host.  Archives come from ``archive.load_data`` (PSRCHIVE is out of
scope; see archive.py).
"""
import gc
import time

import numpy as np

from . import archive as _arch
from .mjd import MJD, add_days_parts, epoch_parts
from .pplib import (DataBunch, F0_fact, phase_transform, guess_fit_freq, read_model,
                    load_spline_model_file,
                    read_model_device, gen_gaussian_portraits_device, scattering_alpha,
                    weighted_mean, write_TOAs)
from .pptoaslib import report_failure
from .toas import TOA, TOABlock, TOAList, FlagColumn, MJDArray  # noqa: F401

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


def _gather_objects(obj, rank, world, to_all=False, dst=0):
    """Every rank's obj, in rank order, on dst (None elsewhere) or on every
    rank (to_all) -- dist.gather_object / all_gather_object without their
    per-object pickles of the payload: obj is pickled with protocol 5, so its
    numpy arrays (a shard's columns: ~3.7 KB per subint at 128 channels)
    leave the pickle stream as out-of-band buffers; each rank's message is
    one flat byte tensor [stream | buffer 0 | buffer 1 | ...] (64-byte
    aligned pieces) moved by tensor collectives -- CPU tensors under gloo,
    device tensors under nccl (RCCL over xGMI) -- and rebuilt on the
    receiving rank with the arrays as views of the received bytes."""
    import pickle
    import torch
    import torch.distributed as dist
    bufs = []
    head = pickle.dumps(obj, protocol=5, buffer_callback=bufs.append)
    views = [b.raw() for b in bufs]
    sizes = [len(head)] + [v.nbytes for v in views]
    offs = np.zeros(len(sizes) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([(n + 63) // 64 * 64 for n in sizes])
    flat = np.empty(int(offs[-1]), dtype=np.uint8)
    flat[:len(head)] = np.frombuffer(head, dtype=np.uint8)
    for v, o in zip(views, offs[1:-1]):
        flat[o:o + v.nbytes] = np.frombuffer(v, dtype=np.uint8)
    del head, bufs, views
    dev = torch.device("cuda", torch.cuda.current_device()) \
        if dist.get_backend() == "nccl" else torch.device("cpu")
    meta = torch.tensor([len(flat), len(sizes)], dtype=torch.int64, device=dev)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta)
    metas = torch.stack(metas).cpu().numpy()
    ltot, lcnt = int(metas[:, 0].max()), int(metas[:, 1].max())
    sz = torch.zeros(lcnt, dtype=torch.int64, device=dev)
    sz[:len(sizes)] = torch.as_tensor(sizes, dtype=torch.int64)
    szs = [torch.empty_like(sz) for _ in range(world)]
    dist.all_gather(szs, sz)
    msg = torch.zeros(ltot, dtype=torch.uint8, device=dev)
    msg[:len(flat)] = torch.from_numpy(flat).to(dev)
    del flat
    if to_all:
        got = [torch.empty_like(msg) for _ in range(world)]
        dist.all_gather(got, msg)
    else:
        got = [torch.empty_like(msg) for _ in range(world)] if rank == dst else None
        dist.gather(msg, got, dst=dst)
        if rank != dst:
            return None
    out = []
    for r in range(world):
        a = got[r].cpu().numpy()
        n = int(metas[r, 1])
        s = szs[r][:n].cpu().numpy()
        o = np.zeros(n + 1, dtype=np.int64)
        o[1:] = np.cumsum((s + 63) // 64 * 64)
        out.append(pickle.loads(a[:s[0]].tobytes(),
                                buffers=[a[o[i]:o[i] + s[i]] for i in range(1, n)]))
        got[r] = None
    return out


_POOL = None


def _pool():
    """The host-thread pool of _par_concat / _par_map (None: one thread)."""
    global _POOL
    from .toas import _host_threads
    nt = min(4, _host_threads())
    if nt < 2:
        return None
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _POOL = ThreadPoolExecutor(max_workers=nt, thread_name_prefix="pptoas")
    return _POOL


def _par_map(fn, items):
    """[fn(x) for x in items], the calls on host threads."""
    pool = _pool()
    if pool is None:
        return [fn(x) for x in items]
    return [f.result() for f in [pool.submit(fn, x) for x in items]]


def _par_concat(parts):
    """{key: np.concatenate(pieces)} with the pieces copied into place on a
    few host threads (np.copyto releases the GIL); the same arrays as
    np.concatenate's."""
    pool = _pool()
    if pool is None:
        return {k: np.concatenate(v) for k, v in parts.items()}
    out, jobs = {}, []
    for k, v in parts.items():
        a = np.empty((sum(len(x) for x in v),) + v[0].shape[1:],
                     dtype=np.result_type(*[x.dtype for x in v]))
        o = 0
        for x in v:
            jobs.append(pool.submit(np.copyto, a[o:o + len(x)], x))
            o += len(x)
        out[k] = a
    for j in jobs:
        j.result()
    return out


def _gc_paused(fn):
    """Run fn with Python's cyclic collector paused: get_TOAs makes few
    containers, but a full collection of the caller's heap (a torch process
    holds ~10^5 objects) landing inside the call costs more than the call.
    The young generations are still collected after every fitted piece
    (_collect), so garbage does not accumulate over a long call."""
    import functools

    @functools.wraps(fn)
    def run(*a, **k):
        on = gc.isenabled()
        gc.disable()
        try:
            return fn(*a, **k)
        finally:
            if on:
                gc.enable()
    return run


def fit_pipeline(keys):
    """The batched-fit pipeline get_TOAs submits its pieces to
    (engine.FitPipeline on this process's device).  The CPU tests replace it
    at this boundary with pptoaslib.SyncPipeline over a stand-in fit."""
    from .engine import FitPipeline, get_engine
    return FitPipeline(get_engine(), keys=keys)


def _shard_range(n, rank, world):
    """Contiguous [lo, hi) of n units for rank; sizes differ by at most one."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


_LIST_ATTRS = ["obs", "doppler_fs", "nu0s", "nu_fits", "nu_refs", "ok_idatafiles", "ok_isubs",
               "epochs", "MJDs", "Ps", "phis", "phi_errs", "TOAs", "TOA_errs", "DM0s", "DMs",
               "DM_errs", "DeltaDM_means", "DeltaDM_errs", "GMs", "GM_errs", "taus",
               "tau_errs", "alphas", "alpha_errs", "scales", "scale_errs", "snrs",
               "channel_snrs", "profile_fluxes", "profile_flux_errs", "fluxes", "flux_errs",
               "flux_freqs", "red_chi2s", "channel_red_chi2s", "covariances", "nfevals",
               "rcs", "fit_durations", "order", "TOA_list", "zap_channels"]


class GetTOAs:
    """Measure TOAs and DMs from wideband data (pptoas.py:75-738).

    Under an initialised torch.distributed group the fits are sharded over
    the ranks (get_TOAs); ``gather_to`` says which ranks then hold the
    results: "root" (default) -- rank 0 receives every rank's result arrays
    and assembles all TOAs, the other ranks keep none (write from rank 0);
    "all" -- every rank assembles the same TOAs.  ``read_bytes_max`` bounds
    the bytes of one subint-range read of an archive that materialises its
    data (PSRFITS, .npz): a rank's shard is read and fitted in pieces of at
    most that size (registered in-memory archives are views, read whole)."""
    gather_to = "root"
    read_bytes_max = 8 << 30
    # device-resident subints of one call are fitted in pieces of these
    # fractions (at least pipeline_min_subints in all), each piece's TOA
    # records built while the next runs; pipeline_depth fits in flight
    pipeline_fracs = (0.7, 0.3)
    pipeline_min_subints = 4096
    pipeline_depth = 1

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
        self.TOA_list = TOAList()
        self.instrumental_response_dict = self.ird = {"DM": 0.0, "wids": [], "irf_types": []}
        self.quiet = quiet

    def _fits_model(self, nchan_data=None):
        """The FITS-archive template of get_TOAs (pptoas.py:323-338): tscrunched,
        baseline removed, masked; [nchan, nbin] (a 1-channel template tiled)."""
        md = _arch.load_data(self.modelfile, dedisperse=False, dededisperse=False,
                             tscrunch=True, pscrunch=True, rm_baseline=True, quiet=True)
        model = np.asarray((md.masks * md.subints)[0, 0])
        if md.nchan == 1 and nchan_data is not None:
            model = np.tile(model[0], nchan_data).reshape(nchan_data, md.nbin)
        return md, model

    @staticmethod
    def _row_keys(rows):
        """First-appearance index of every distinct row, and each row's index
        into those (np.unique on the rows, renumbered in order of appearance)."""
        rows = np.ascontiguousarray(rows)
        if (rows == rows[0]).all():
            return np.zeros(1, dtype=np.int64), np.zeros(len(rows), dtype=np.int64)
        v = rows.view(np.dtype((np.void, rows.dtype.itemsize * rows.shape[1]))).ravel()
        _, first, inv = np.unique(v, return_index=True, return_inverse=True)
        order = np.argsort(first, kind="stable")
        rank = np.empty_like(order)
        rank[order] = np.arange(len(order))
        return first[order], rank[inv.ravel()]

    # -- per-subint templates ------------------------------------------------
    def _models(self, data, fit_scat, quiet, uniform_freqs=False):
        """Template portrait per ok subint (pptoas.py:351-378), de-duplicated:
        one device build per distinct (channel frequencies, P when TAU is in
        bins of P) key."""
        nsub = data.nsub
        if self.is_FITS_model:
            md, model = self._fits_model(data.nchan)
            if md.nbin != data.nbin or md.nchan != data.nchan:  # pptoas.py:329-338
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
        tau_P = gparams[1] != 0 and not fit_scat
        ok = np.asarray(data.ok_isubs)
        if uniform_freqs and not tau_P:
            first, inv = np.zeros(1, dtype=np.int64), np.zeros(len(ok), dtype=np.int64)
        else:
            keyrows = data.freqs[ok]
            if tau_P:
                keyrows = np.concatenate([keyrows, data.Ps[ok][:, None]], axis=1)
            first, inv = self._row_keys(keyrows)
        idx = np.zeros(nsub, dtype=np.int32)
        idx[ok] = inv
        keyf = data.freqs[ok[first]]
        keyP = data.Ps[ok[first]]
        nbin = len(data.phases)
        models = np.empty((len(first), data.nchan, nbin))
        params = np.array(gparams, dtype=float)
        if fit_scat:
            params[1] = 0.0
            models[:] = gen_gaussian_portraits_device(code, params, 0.0, nbin, keyf, nu_ref)
        elif not tau_P:
            models[:] = gen_gaussian_portraits_device(code, params, alpha, nbin, keyf, nu_ref)
        else:  # read_model's TAU * nbin / P differs per period
            for P in sorted(set(keyP.tolist())):
                sel = np.flatnonzero(keyP == P)
                pp = np.copy(params)
                pp[1] *= nbin / P
                models[sel] = gen_gaussian_portraits_device(code, pp, alpha, nbin, keyf[sel],
                                                            nu_ref)
        return models, idx, None

    def _spline_models(self, data):
        """ppspline templates: read_spline_model(modelfile, freqs[isub], nbin)
        per subint (pptoas.py:375-378), one device build per distinct channel
        frequency row (ppf_spline_portraits)."""
        name, source, datafile, mean_prof, eigvec, tck = load_spline_model_file(self.modelfile)
        self.model_name = name
        ok = np.asarray(data.ok_isubs)
        first, inv = self._row_keys(data.freqs[ok])
        idx = np.zeros(data.nsub, dtype=np.int32)
        idx[ok] = inv
        from .engine import get_engine
        models = get_engine().spline_portraits(mean_prof, eigvec, tck, data.freqs[ok[first]],
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

    def _open(self, datafile, tscrunch, quiet, rm_base=None):
        """open_archive as get_TOAs loads (pptoas.py:250-264): no
        dedispersion; a dedispersed archive (dmc = 1) is reopened with
        dededisperse=True."""
        rb = rm_baseline if rm_base is None else rm_base
        a = _arch.open_archive(datafile, dedisperse=False, dededisperse=False, tscrunch=tscrunch,
                               pscrunch=True, rm_baseline=rb, quiet=quiet)
        if a.meta.dmc:
            if not quiet:
                print("%s is dedispersed (dmc = 1).  Reloading it." % datafile)
            a = _arch.open_archive(datafile, dedisperse=False, dededisperse=True,
                                   tscrunch=tscrunch, pscrunch=True, rm_baseline=rb,
                                   quiet=quiet)
        return a

    def _load(self, datafile, tscrunch, quiet, rm_base):
        """load_data as the reference's drivers call it (pptoas.py:808-820,
        1329-1344): reloaded with dededisperse=True when dmc = 1."""
        a = self._open(datafile, tscrunch, quiet, rm_base)
        b = DataBunch(**dict(a.meta))
        sub = a.read()
        if b.get("snr_deferred"):  # load_data's SNRs (pplib.py:2762-2770)
            b.SNRs = a.snrs(sub)
            b.snr_deferred = False
        b.subints = _arch.host_array(sub)
        return b

    @_gc_paused
    def get_TOAs(self, datafile=None, tscrunch=False, nu_refs=None, DM0=None, bary=True,
                 fit_DM=True, fit_GM=False, fit_scat=False, log10_tau=True, scat_guess=None,
                 fix_alpha=False, print_phase=False, print_flux=False, print_parangle=False,
                 add_instrumental_response=False, addtnl_toa_flags={}, method="trust-ncg",
                 bounds=None, nu_fits=None, show_plot=False, quiet=None):
        """pptoas.py:150-738 with the subint loop batched on the device.

        Every archive is opened for its metadata first (no DATA read); the
        (archive, subint) units in get_TOAs order are split into contiguous
        shards, one per rank of an initialised torch.distributed group, and a
        rank reads only the subint range of its shard (pptoas.py:246,343 is the
        loop being sharded).  Fits are submitted per archive and flag set, a
        large one in pieces (``pipeline_fracs``), through ``fit_pipeline``
        (engine.FitPipeline): the device fits piece i + 1 while the host turns
        piece i's results into records and text.  Every rank turns its own
        shard's results into columns -- the per-subint arrays and a TOABlock
        of its TOA records, with the .tim text already formatted when there
        is more than one rank -- and only those finished columns travel: to
        rank 0 (``gather_to`` "root", default), which concatenates them in
        unit order into the per-archive lists and TOA_list, or to every rank
        ("all").  With "root" the other ranks add nothing to their lists
        (their shard's blocks stay in ``shard_blocks``)."""
        if quiet is None:
            quiet = self.quiet
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
        if (self.fit_GM or fit_scat) and not quiet:
            print(warning)
        self.scat_guess = scat_guess
        self.DM0, self.bary = DM0, bary
        self.tscrunch = tscrunch
        self.add_instrumental_response = add_instrumental_response
        self._fit_flags_prev = None  # the reference's loop-carried fit_flags
        start = time.time()
        self.phase_s = tm = {}  # wall time per phase of this call (diagnostic)
        clock = time.perf_counter

        def mark(k, t0):
            tm[k] = tm.get(k, 0.0) + clock() - t0
            return clock()
        t = clock()
        datafiles = self.datafiles if datafile is None else [datafile]
        # 1. metadata of every archive (all ranks; no DATA read)
        jobs = []
        n_ok0 = len(self.ok_idatafiles)
        for iarch, datafile in enumerate(datafiles):
            try:
                t = clock()
                arch = self._open(datafile, tscrunch, quiet)
                meta = arch.meta
                t = mark("open", t)
                if not len(meta.ok_isubs):
                    if not quiet:
                        print("No subints to fit for %s.  Skipping it." % datafile)
                    continue
                self.ok_idatafiles.append(iarch)
            except RuntimeError:
                if not quiet:
                    print("Cannot load_data(%s).  Skipping it." % datafile)
                continue
            name = datafile if isinstance(datafile, str) else meta.filename
            job = self._prepare(name, meta, nu_refs, nu_fits, fit_scat, method, bounds, quiet)
            t = mark("prepare", t)
            if job is not None:
                job.arch = arch
                jobs.append(job)
        # 2. shard the units, read and fit this rank's subints, and turn the
        # results into columns (arrays + TOA records) on this rank
        rank, world = _dist_info()
        counts = [len(j.ok_isubs) for j in jobs]
        lo, hi = _shard_range(int(sum(counts)), rank, world)
        shards, durations, off = {}, {}, 0
        pipe = None
        pend = {}  # piece id -> [ij, a0, nsubs, groups left, result arrays]
        for ij, job in enumerate(jobs):
            a0, a1 = max(lo, off) - off, min(hi, off + counts[ij]) - off
            off += counts[ij]
            if a1 <= a0:
                continue
            if pipe is None:
                pipe = fit_pipeline(_RESULT_KEYS)
            t = clock()
            pa0 = a0
            for rsubs in self._read_pieces(job, job.ok_isubs[a0:a1]):
                s_lo, sub, errs = self._read(job, rsubs, fit_scat)
                t = mark("read", t)
                for subs in self._pipe_split(rsubs, sub):
                    self._submit(pipe, pend, (ij, pa0), job, subs, s_lo, sub, errs, fit_scat,
                                 method)
                    pa0 += len(subs)
                    t = mark("submit", t)
                    while len(pipe) > self.pipeline_depth:
                        self._collect(pipe, pend, jobs, shards, durations,
                                      (print_phase, print_flux, print_parangle,
                                       addtnl_toa_flags), mark)
                        t = clock()
        while pipe is not None and len(pipe):
            self._collect(pipe, pend, jobs, shards, durations,
                          (print_phase, print_flux, print_parangle, addtnl_toa_flags), mark)
        self.shard_blocks = [sh.block for ij in sorted(shards) for sh in shards[ij]]
        # 3. gather the finished columns: to rank 0 (gather_to "root") or to
        # every rank ("all")
        t = clock()
        if world > 1:
            got = _gather_objects((shards, durations), rank, world,
                                  to_all=self.gather_to == "all")
            if got is None:  # gather_to "root": the results live on rank 0
                del self.ok_idatafiles[n_ok0:]
                return
            shards, spans = {}, {}
            for s_r, d_r in got:
                for ij, v in s_r.items():
                    shards.setdefault(ij, []).extend(v)
                for ij, sp in d_r.items():  # summed over the ranks fitting the archive
                    spans[ij] = spans.get(ij, 0.0) + sp[1] - sp[0]
        else:
            spans = {ij: sp[1] - sp[0] for ij, sp in durations.items()}
        t = mark("gather", t)
        for ij, job in enumerate(jobs):
            self._finish(job, sorted(shards[ij], key=lambda v: v.a0), spans.get(ij, 0.0), quiet)
        mark("finish", t)
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
                data = self._load(datafile, tscrunch, quiet, rm_baseline)
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
                md, model = self._fits_model()
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
        data = self._load(datafile, getattr(self, "tscrunch", False), quiet, True)
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
                    md, m = self._fits_model(len(freqs))
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
                    # show_fit passes the full freqs row (pptoas.py:1384-1386),
                    # so chan_bw is |freqs[1] - freqs[0]| over all channels
                    cbw = abs(freqs[1] - freqs[0]) if len(freqs) > 1 else 0.0
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
        """Per-archive set-up of pptoas.py:246-484 on the metadata, as arrays:
        templates, reference frequencies, initial parameters and the
        per-subint fit flags."""
        nsub, nchan, nbin = data.nsub, data.nchan, data.nbin
        obs = DataBunch(telescope=data.telescope, backend=data.backend, frontend=data.frontend)
        DM_stored = data.DM
        DM0 = DM_stored if self.DM0 is None else self.DM0
        ep = data.get("epoch_parts") or epoch_parts(data.epochs)
        MJDs = ep[0] + (ep[1] + ep[2]) / 86400.0  # MJD.in_days elementwise
        ok_isubs = np.asarray(data.ok_isubs)
        wn = np.asarray(data.weights) != 0.0
        mask = wn.astype(np.uint8)
        # per-channel rows every ok subint shares (one row to the device,
        # one template key, one guess_fit_freq)
        dense = len(ok_isubs) == nsub

        def okrows(a):
            return a if dense else a[ok_isubs]

        def rows_equal(a):
            a = okrows(a)
            return bool(len(ok_isubs)) and bool((a == a[0]).all())
        # freqs and weights compared on two host threads (numpy releases the
        # GIL); equal weight rows make the mask rows equal too
        ru = _par_map(rows_equal, [data.freqs, data.weights])
        uniform = {"freqs": ru[0], "weights": ru[1], "mask": ru[1] or rows_equal(mask)}
        mm = self._models(data, fit_scat, quiet, uniform["freqs"])
        if mm is None:
            if not quiet:
                print("Model nbin/nchan mismatch for %s; skipping it." % datafile)
            return None
        models, midx, _ = mm
        if self._irf_active():
            models, midx = self._irf_models(models, midx, data, ok_isubs)
        nchx = np.count_nonzero(wn, axis=1)
        allok = nchx == nchan
        # the tobs flag's values: typed when the durations are numbers
        tobs = np.asarray(data.subtimes)
        if tobs.dtype.kind not in "fiu":
            tobs = np.asarray(data.subtimes, dtype=object)
        # reference frequencies (pptoas.py:396-415)
        nu_fits_a = np.zeros((nsub, 3))
        nu_refs_a = np.full((nsub, 3), np.nan)
        if nu_ref_tuple is not None:
            nu_refs_a[ok_isubs] = [nu_ref_tuple[0], nu_ref_tuple[0], nu_ref_tuple[-1]]
            if self.bary and nu_ref_tuple[-1]:
                nu_refs_a[ok_isubs, 2] /= np.asarray(data.doppler_factors)[ok_isubs]
        # initial guesses (pptoas.py:420-456; phi from the device guess)
        init = np.zeros((nsub, 5))
        guess_tau = np.zeros(nsub)
        init[ok_isubs, 1] = DM_stored
        self._nu_fit_and_tau(data, ok_isubs, wn, allok, nu_fit_tuple, fit_scat, nu_fits_a, init,
                             guess_tau, uniform["freqs"])
        # per-subint fit flags (pptoas.py:474-484): get_TOAs keeps one
        # fit_flags list across subints and archives, and a 2-channel subint
        # (fit_DM and fit_GM) zeroes GM in the *previous* subint's list --
        # phase-only after a 1-channel subint, and an UnboundLocalError when no
        # subint came before it.
        ff_all = np.zeros((nsub, 5), dtype=np.int64)
        special = (nchx[ok_isubs] == 1) | ((nchx[ok_isubs] == 2) & bool(self.fit_DM and self.fit_GM))
        if not special.any():
            ff_all[ok_isubs] = self.fit_flags
            self._fit_flags_prev = list(self.fit_flags)
        else:
            for isub in ok_isubs:
                n = nchx[isub]
                if n == 1:
                    ff = [1, 0, 0, 0, 0]
                elif n == 2 and self.fit_DM and self.fit_GM:
                    if self._fit_flags_prev is None:
                        raise UnboundLocalError(
                            "local variable 'fit_flags' referenced before assignment")
                    ff = list(self._fit_flags_prev)
                    ff[2] = 0
                else:
                    ff = list(self.fit_flags)
                self._fit_flags_prev = ff
                ff_all[isub] = ff
        if bounds is None and method == "TNC":
            # get_TOAs' default TNC bounds (pptoas.py:458-467)
            bounds = [(None, None), (None, None), (None, None),
                      (np.log10((10 * nbin) ** -1), None) if self.log10_tau else (0.0, None),
                      (-10.0, 10.0)]
        return _Job(name=datafile, data=data, obs=obs, DM0=DM0, MJDs=MJDs, epoch_parts=ep,
                    ok_isubs=ok_isubs, models=models, midx=midx, mask=mask, wn=wn,
                    nchx=nchx, nu_fits_a=nu_fits_a, nu_refs_a=nu_refs_a, init=init,
                    guess_tau=guess_tau, ff=ff_all, bounds=bounds, allok=allok,
                    nu_fit_tuple=nu_fit_tuple, uniform=uniform, tobs=tobs)

    def _nu_fit_and_tau(self, data, isubs, wn, allok, nu_fit_tuple, fit_scat, nu_fits_a, init,
                        guess_tau, uniform_freqs=False):
        """nu_fit (guess_fit_freq with the channel S/Ns, pptoas.py:396-415)
        and the scattering guess at nu_fit_tau (pptoas.py:420-440) of subints
        isubs, into nu_fits_a / init / guess_tau."""
        if not len(isubs):
            return
        nbin = data.nbin
        if nu_fit_tuple is None:
            nu_fits_a[isubs] = self._guess_fit_freqs(data, isubs, wn, allok,
                                                     uniform_freqs)[:, None]
        else:
            nu_fits_a[isubs] = [nu_fit_tuple[0], nu_fit_tuple[0], nu_fit_tuple[-1]]
        if fit_scat:
            P = data.Ps[isubs]
            nu_fit_tau = nu_fits_a[isubs, 2]
            if self.scat_guess is not None:
                ts, tref, alpha_g = self.scat_guess
                tau_g = (ts / P) * (nu_fit_tau / tref) ** alpha_g
            else:
                alpha_g = self.alpha if hasattr(self, "alpha") else scattering_alpha
                tau_g = (self.gparams[1] / P) * (nu_fit_tau / self.model_nu_ref) ** alpha_g \
                    if hasattr(self, "gparams") else np.zeros(len(isubs))
            tau_g = np.asarray(tau_g, dtype=np.float64) * np.ones(len(isubs))
            guess_tau[isubs] = tau_g
            if self.log10_tau:
                tau_g = np.log10(np.where(tau_g == 0.0, nbin ** -1, tau_g))
            init[isubs, 3] = tau_g
            init[isubs, 4] = alpha_g

    @staticmethod
    def _guess_fit_freqs(data, ok_isubs, wn, allok, uniform_freqs=False):
        """guess_fit_freq(freqsx, SNRsx) of every ok subint (pptoas.py:401,
        pplib.py:2618-2632): once when every such subint has the same
        frequencies, all channels on and the same S/Ns; whole rows at once
        where every channel is on (numpy's row sums are its 1-D sums), the
        compressed rows otherwise."""
        dense = len(ok_isubs) == data.nsub
        f = data.freqs if dense else data.freqs[ok_isubs]
        snr = np.asarray(data.SNRs)[:, 0] if dense else np.asarray(data.SNRs)[ok_isubs, 0]
        alla = bool(allok.all()) if dense else bool(allok[ok_isubs].all())
        if alla and uniform_freqs and (snr == snr[0]).all():
            return np.full(len(ok_isubs), guess_fit_freq(f[0], snr[0]))  # one distinct row
        if uniform_freqs:
            # one frequency row: its terms once, broadcast over the S/N rows
            # (the same elementwise operations on the same values)
            f0 = np.asarray(f[0], dtype=np.float64)
            nu0 = (f0.min() + f0.max()) * 0.5
            f2 = f0 ** -2
            out = nu0 + np.sum((f0 - nu0) * snr * f2, axis=1) / np.sum(snr * f2, axis=1)
        else:
            nu0 = (f.min(axis=1) + f.max(axis=1)) * 0.5
            f2 = f ** -2
            out = nu0 + np.sum((f - nu0[:, None]) * snr * f2, axis=1) / np.sum(snr * f2, axis=1)
        for j in np.flatnonzero(~allok[ok_isubs]):
            isub = ok_isubs[j]
            ok = wn[isub]
            out[j] = guess_fit_freq(data.freqs[isub, ok], np.asarray(data.SNRs)[isub, 0, ok])
        return out

    def _read_pieces(self, job, subs):
        """Split subs (ascending subint indices) into runs whose subint range
        reads at most read_bytes_max bytes (one run for views of registered
        archives)."""
        data = job.data
        if not getattr(job.arch, "owns_reads", True):
            return [subs]
        per = 8 * int(data.npol) * int(data.nchan) * int(data.nbin)
        span = max(1, int(self.read_bytes_max) // per)
        out, i = [], 0
        while i < len(subs):
            j = int(np.searchsorted(subs, subs[i] + span, side="left"))
            out.append(subs[i:j])
            i = j
        return out

    def _read(self, job, subs, fit_scat):
        """Read the subint range of subs (one read piece): (first subint,
        [n, nchan, nbin] numpy or device view, noise rows or None).  A
        PSRFITS archive's deferred SNRs (Profile::snr(), pplib.py:2762-2770)
        come from the data just read, then those subints' nu_fit and
        scattering guess."""
        data = job.data
        s_lo, s_hi = int(subs[0]), int(subs[-1]) + 1
        full = job.arch.read(s_lo, s_hi)  # [s_hi - s_lo, npol, nchan, nbin], numpy or device
        if data.get("snr_deferred"):
            from .engine import get_engine
            data.SNRs[s_lo:s_hi] = get_engine().profile_snr(full).cpu().numpy()
            self._nu_fit_and_tau(data, subs, job.wn, job.allok, job.nu_fit_tuple, fit_scat,
                                 job.nu_fits_a, job.init, job.guess_tau, job.uniform["freqs"])
        ns = data.get("noise_stds")
        return s_lo, full[:, 0], None if ns is None else np.asarray(ns)[:, 0]

    def _pipe_split(self, subs, sub):
        """Pipeline pieces of one read piece: host-resident subints in pieces
        of at most STREAM_CHUNK_BYTES (their copies overlap the fits), device-
        resident ones in shrinking fractions (pipeline_fracs) so that the
        host work after the last piece is small."""
        n = len(subs)
        if _arch._is_tensor(sub) and sub.device.type != "cpu":
            if n < self.pipeline_min_subints:
                return [subs]
            cuts = np.cumsum([0.0] + list(self.pipeline_fracs))
            cuts = np.unique(np.round(cuts / cuts[-1] * n).astype(int))
        else:
            from .pptoaslib import STREAM_CHUNK_BYTES
            per = 8 * int(np.prod(sub.shape[1:]))
            step = max(1, STREAM_CHUNK_BYTES // per)
            cuts = np.unique(np.append(np.arange(0, n, step), n))
        return [subs[i:j] for i, j in zip(cuts[:-1], cuts[1:]) if j > i]

    def _submit(self, pipe, pend, key, job, subs, s_lo, sub, errs, fit_scat, method):
        """Launch the fits of subints subs (one device call per fit-flag
        group) into the pipeline; piece key = (archive index, a0)."""
        data = job.data
        ffs = job.ff[subs]
        groups = [np.arange(len(subs))] if (ffs == ffs[0]).all() else \
            [np.flatnonzero((ffs == r).all(axis=1)) for r in np.unique(ffs, axis=0)]
        pend[key] = [len(groups), len(subs), None, time.time()]
        for g in groups:
            s = subs[g]
            rel = s - s_lo
            if len(rel) == rel[-1] - rel[0] + 1:  # contiguous: a view
                d = sub[int(rel[0]):int(rel[-1]) + 1]
            else:
                d = sub[rel] if not _arch._is_tensor(sub) else sub[_arch_index(rel, sub)]
            # errs None: the device estimates get_noise_PS per channel, as
            # load_data's noise_stds (pplib.py:2744-2748); per-channel rows
            # shared by every subint go as one row
            pipe.submit((key, g, _take(job.nu_fits_a, s)),
                        d, job.models, job.row("freqs", s), _take(data.Ps, s),
                        _take(job.init, s), list(ffs[g[0]]),
                        nu_fit=_take(job.nu_fits_a, s), nu_out=_take(job.nu_refs_a, s),
                        errs=None if errs is None else _take(errs, s),
                        log10_tau=self.log10_tau, option=0, is_toa=True,
                        chan_mask=job.row("mask", s), weights=job.row("weights", s),
                        model_idx=_take(job.midx, s), guess=True, guess_Ns=100,
                        guess_wrap=True, guess_nu=None,
                        guess_tau=_take(job.guess_tau, s) if fit_scat else None,
                        method=method, bounds=job.bounds)

    def _collect(self, pipe, pend, jobs, shards, durations, toa_args, mark):
        """Collect the oldest fit in the pipeline; when its piece is complete,
        turn it into columns on this rank (_shard; its .tim text formatted
        now, while later pieces still run on the device)."""
        t = time.perf_counter()
        (key, g, nu_fit), res = pipe.collect()
        t = mark("wait", t)
        p = pend[key]
        keep = {k: res[k] for k in _RESULT_KEYS if k in res}
        keep["nu_fit"] = nu_fit  # the assembling rank's nu_fits
        if p[0] == 1 and p[2] is None:
            out = keep
        else:
            if p[2] is None:
                p[2] = {k: np.zeros((p[1],) + v.shape[1:], dtype=v.dtype) for k, v in keep.items()}
            for k, v in keep.items():
                p[2][k][g] = v
            out = p[2]
        p[0] -= 1
        if p[0]:
            return
        del pend[key]
        ij, a0 = key
        # the archive's fit wall time on this rank: first submit to last
        # collect (its pieces overlap on the device, so no per-piece sum)
        t0, t1 = durations.get(ij, (p[3], p[3]))
        durations[ij] = (min(t0, p[3]), max(t1, time.time()))
        sh = self._shard(jobs[ij], a0, out, *toa_args)
        t = mark("shard", t)
        sh.block.preformat()  # the .tim text of these records
        mark("preformat", t)
        shards.setdefault(ij, []).append(sh)
        # the collector is paused over get_TOAs (_gc_paused): free this
        # piece's cyclic garbage from the young generations, so a long call
        # (a 125k-subint shard in many pieces) does not pile it up, without
        # a full collection of the caller's heap inside the call
        if not gc.isenabled():
            gc.collect(1)

    def _shard(self, job, a0, res, print_phase, print_flux, print_parangle, addtnl_toa_flags):
        """Columns of ok subints job.ok_isubs[a0:a0 + n] from their device
        results (pptoas.py:522-661), on the rank that fitted them: the
        per-subint values in ok order and a TOABlock of their TOA records
        (flags in the reference's insertion order, pptoas.py:606-661, then
        addtnl_toa_flags)."""
        data, datafile = job.data, job.name
        nchan = data.nchan
        p, e = res["params"], res["param_errs"]
        n = len(p)
        ok = job.ok_isubs[a0:a0 + n]
        status, nfev = res["status"].astype(np.int64), res["nfev"].astype(np.int64)
        for j in np.flatnonzero(~np.isin(status, (0, 1, 2, 4))):
            report_failure(int(status[j]), "%s_%d" % (datafile, ok[j]))
        ff = job.ff[ok]
        P = data.Ps[ok]
        phi, phi_err = p[:, 0], e[:, 0]
        DM, DM_err, GM, GM_err = p[:, 1].copy(), e[:, 1], p[:, 2].copy(), e[:, 2]
        mjd = add_days_parts(tuple(x[ok] for x in job.epoch_parts),
                             ((phi * P) + data.backend_delay) / (3600 * 24.))
        TOA_err = phi_err * P * 1e6
        if self.bary:
            df = np.asarray(data.doppler_factors, dtype=np.float64)[ok]
            DM = np.where(ff[:, 1] != 0, DM * df, DM)
            GM = np.where(ff[:, 2] != 0, GM * df ** 3, GM)
        else:
            df = np.ones(n)
        wn = _take(job.wn, ok)
        wall = bool(wn.all())
        sc = res["scales"] if wall else np.where(wn, res["scales"], 0.0)
        sce = res["scale_errs"] if wall else np.where(wn, res["scale_errs"], 0.0)
        chs = res["channel_snrs"] if wall else np.where(wn, res["channel_snrs"], 0.0)
        nuo = res["nu_out"]
        nf = ff.sum(axis=1)
        cov = res["cov"]
        full = nf == self.nfit
        if full.all():
            covs = np.ascontiguousarray(cov[:, :self.nfit, :self.nfit])
        else:
            covs = np.zeros((n, self.nfit, self.nfit))
            covs[full] = cov[full][:, :self.nfit, :self.nfit]
            for j in np.flatnonzero(~full):
                cm = cov[j][:nf[j], :nf[j]]
                try:  # the reference's assignment, broadcasting a 1x1 block
                    covs[j] = cm
                except ValueError:
                    w = np.where(ff[j])[0]
                    for ii, ifit in enumerate(w):
                        for jj, jfit in enumerate(w):
                            covs[j][ifit, jfit] = cm[ii, jj]
        if wall and job.uniform["freqs"]:  # every row the same: its extremes
            f0 = data.freqs[ok[0]]
            fmax, fmin = np.full(n, f0.max()), np.full(n, f0.min())
        else:
            fo = _take(data.freqs, ok)
            fmax = (fo if wall else np.where(wn, fo, -np.inf)).max(axis=1)
            fmin = (fo if wall else np.where(wn, fo, np.inf)).min(axis=1)
        flux = None
        if print_flux:
            # scattering keeps each row's mean, so the scattered model's
            # channel means are the template's (pptoas.py:553-575)
            pfl, pfle = np.zeros((n, nchan)), np.zeros((n, nchan))
            fluxes, flux_errs, flux_freqs = np.zeros(n), np.zeros(n), np.zeros(n)
            for j, isub in enumerate(ok):
                okc = wn[j]
                means = job.models[job.midx[isub]][okc].mean(axis=1)
                pfl[j, okc] = means * sc[j][okc]
                pfle[j, okc] = abs(means) * sce[j][okc]
                fluxes[j], flux_errs[j] = weighted_mean(pfl[j, okc], pfle[j, okc])
                flux_freqs[j] = weighted_mean(data.freqs[isub, okc], pfle[j, okc])[0]
            flux = (pfl, pfle, fluxes, flux_errs, flux_freqs)
        # TOA records as columns; a flag some rows lack carries a presence mask
        cols = []

        def col(key, vals, present=None):
            if present is not None:
                if not present.any():
                    return
                if present.all():
                    present = None
            cols.append(FlagColumn.of(key, vals, n, present))

        gp = ff[:, 2] != 0
        if gp.any():
            col("gm", GM, gp)
            col("gm_err", GM_err, gp)
        tp = ff[:, 3] != 0
        if tp.any():
            if self.log10_tau:
                col("scat_time", 10 ** p[:, 3] * P / df * 1e6, tp)
                col("log10_scat_time", p[:, 3] + np.log10(P / df), tp)
                col("log10_scat_time_err", e[:, 3], tp)
            else:
                col("scat_time", p[:, 3] * P / df * 1e6, tp)
                col("scat_time_err", e[:, 3] * P / df * 1e6, tp)
            col("scat_ref_freq", nuo[:, 2] * df, tp)
            col("scat_ind", p[:, 4], tp)
        col("scat_ind_err", e[:, 4], ff[:, 4] != 0)
        const = FlagColumn
        cols += [const("be", "const", data.backend), const("fe", "const", data.frontend),
                 const("f", "const", data.frontend + "_" + data.backend),
                 const("nbin", "const", data.nbin), const("nch", "const", nchan)]
        col("nchx", job.nchx[ok])
        col("bw", fmax - fmin)
        cols.append(const("chbw", "const", abs(data.bw) / nchan))
        col("subint", ok)
        col("tobs", _take(job.tobs, ok))
        col("fratio", fmax / fmin)
        cols.append(const("tmplt", "const", self.modelfile))
        col("snr", res["snr"])
        col("phi_DM_cov", cov[:, 0, 1],
            ~np.isnan(job.nu_refs_a[ok, 0]) & (ff[:, 0] != 0) & (ff[:, 1] != 0))
        col("gof", res["red_chi2"])
        if print_phase:
            col("phs", phi)
            col("phs_err", phi_err)
        if print_flux:
            col("flux", flux[2])
            col("flux_err", flux[3])
            col("flux_ref_freq", flux[4])
        if print_parangle:
            col("par_angle", np.asarray(data.parallactic_angles)[ok])
        dp = ff[:, 1] != 0
        block = TOABlock(datafile, data.telescope, data.telescope_code, nuo[:, 0], mjd, TOA_err,
                         dm=DM if dp.any() else None, dme=DM_err if dp.any() else None,
                         dm_present=None if dp.all() else dp, cols=cols)
        block.add_flags(list(addtnl_toa_flags.items()))
        return DataBunch(a0=a0, n=n, phi=phi, phi_err=phi_err, DM=DM, DM_err=DM_err, GM=GM,
                         GM_err=GM_err, tau=p[:, 3], tau_err=e[:, 3], alpha=p[:, 4],
                         alpha_err=e[:, 4], nfev=nfev, status=status, scales=sc, scale_errs=sce,
                         chsnrs=chs, snr=res["snr"], red_chi2=res["red_chi2"], covs=covs,
                         nu_out=nuo, nu_fit=res["nu_fit"], mjd=mjd, TOA_err=TOA_err, flux=flux,
                         block=block)

    def _finish(self, job, shards, fit_duration, quiet):
        """The per-archive lists of pptoas.py:662-720 (and the DeltaDM mean,
        :664-681) from the shards' columns, concatenated in unit order; the
        shards' TOABlocks join TOA_list."""
        data, datafile = job.data, job.name
        nsub, nchan = data.nsub, data.nchan
        ok = job.ok_isubs
        nok = len(ok)
        if len(shards) == 1:
            def cat(k):
                return shards[0][k]
        else:
            # the per-channel columns (most of the bytes) joined on host
            # threads: a fresh [nsub, nchan] array's first-touch page faults
            # and copies are most of _finish's time
            big = _par_concat({k: [sh[k] for sh in shards]
                               for k in ("scales", "scale_errs", "chsnrs")})

            def cat(k):
                return big[k] if k in big else np.concatenate([sh[k] for sh in shards])
        dense = nok == nsub  # ok_isubs is then every subint, in order

        def spread(v, tail=(), dtype=np.float64):
            if dense:
                return np.ascontiguousarray(v, dtype=dtype)
            out = np.zeros((nsub,) + tail, dtype=dtype)
            out[ok] = v
            return out

        phis, phi_errs = spread(cat("phi")), spread(cat("phi_err"))
        DMs, DM_errs = spread(cat("DM")), spread(cat("DM_err"))
        GMs, GM_errs = spread(cat("GM")), spread(cat("GM_err"))
        taus, tau_errs = spread(cat("tau")), spread(cat("tau_err"))
        alphas, alpha_errs = spread(cat("alpha")), spread(cat("alpha_err"))
        nfevals, rcs = spread(cat("nfev"), dtype="int"), spread(cat("status"), dtype="int")
        scales = spread(cat("scales"), (nchan,))
        scale_errs = spread(cat("scale_errs"), (nchan,))
        chsnrs = spread(cat("chsnrs"), (nchan,))
        snrs, red_chi2s = spread(cat("snr")), spread(cat("red_chi2"))
        covs = spread(cat("covs"), (self.nfit, self.nfit))
        if shards[0].flux is not None:
            fl = [np.concatenate([sh.flux[i] for sh in shards]) for i in range(5)]
            pfl, pfle = spread(fl[0], (nchan,)), spread(fl[1], (nchan,))
            fluxes, flux_errs, flux_freqs = spread(fl[2]), spread(fl[3]), spread(fl[4])
        else:
            pfl, pfle = np.zeros((nsub, nchan)), np.zeros((nsub, nchan))
            fluxes, flux_errs, flux_freqs = np.zeros(nsub), np.zeros(nsub), np.zeros(nsub)
        mjd = [shards[0].mjd[i] if len(shards) == 1 else
               np.concatenate([sh.mjd[i] for sh in shards]) for i in range(3)]
        if dense:
            TOAs = MJDArray(*mjd)
        else:
            parts = []
            for i, dt in enumerate((np.int64, np.int64, np.float64)):
                a = np.zeros(nsub, dtype=dt)
                a[ok] = mjd[i]
                parts.append(a)
            valid = np.zeros(nsub, dtype=bool)
            valid[ok] = True
            TOAs = MJDArray(*parts, valid=valid)
        if dense:
            TOA_errs = cat("TOA_err").astype(object)
            job.nu_fits_a[:] = cat("nu_fit")
        else:
            TOA_errs = np.zeros(nsub, dtype="object")
            TOA_errs[ok] = cat("TOA_err")
            job.nu_fits_a[ok] = cat("nu_fit")  # (computed by whichever rank read the subint)
        # the reference's list(np.zeros([nsub, 3])) with ok rows filled
        # (pptoas.py:283-284, 406, 527-530) as one [nsub, 3] array: indexed
        # by subint it gives the same rows
        nu_fits = job.nu_fits_a
        nu_refs = np.zeros((nsub, 3))
        nu_refs[ok] = cat("nu_out")
        for sh in shards:
            self.TOA_list.add_block(sh.block)
        # DeltaDM weighted mean per archive (pptoas.py:664-681)
        DeltaDMs = DMs - job.DM0
        dd, de = (DeltaDMs, DM_errs) if dense else (DeltaDMs[ok], DM_errs[ok])
        w = de ** -2 if np.all(de) else np.ones(nok)
        mean, wsum = np.average(dd, weights=w, returned=True)
        var = wsum ** -1
        if nok > 1:
            var *= np.sum(((dd - mean) ** 2) * w) / (len(dd) - 1)
        for attr, val in [("order", datafile), ("obs", job.obs),
                          ("doppler_fs", data.doppler_factors), ("nu0s", data.nu0),
                          ("nu_fits", nu_fits), ("nu_refs", nu_refs), ("ok_isubs", ok),
                          ("epochs", data.epochs), ("MJDs", job.MJDs), ("Ps", data.Ps),
                          ("phis", phis), ("phi_errs", phi_errs), ("TOAs", TOAs),
                          ("TOA_errs", TOA_errs), ("DM0s", job.DM0), ("DMs", DMs),
                          ("DM_errs", DM_errs), ("DeltaDM_means", mean),
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
            print("~%.4f sec/TOA" % (fit_duration / nok))
            print("Med. TOA error is %.3f us" % (np.median(phi_errs[ok]) *
                                                 data.Ps.mean() * 1e6))


class _Job(DataBunch):
    """One archive's get_TOAs set-up (GetTOAs._prepare)."""

    def row(self, key, s):
        """Per-subint [nsub, nchan] input key ("freqs", "weights", "mask")
        for subints s: one shared [nchan] row when every subint's is the
        same.  The shared row is the first ok subint's: `uniform` compares
        the ok subints' rows only, and a zapped subint 0 is not one of them."""
        a = self.mask if key == "mask" else self.data[key]
        if self.uniform[key]:
            return a[int(self.ok_isubs[0])]
        return _take(a, s)


def _take(a, s):
    """a[s]: a view when s is an ascending run of consecutive indices."""
    s = np.asarray(s)
    if len(s) and s[-1] - s[0] + 1 == len(s) and (len(s) < 3 or s[1] == s[0] + 1):
        return a[int(s[0]):int(s[-1]) + 1]
    return a[s]


_RESULT_KEYS = ["params", "param_errs", "nu_out", "cov", "scales", "scale_errs",
                "channel_snrs", "chi2", "red_chi2", "snr", "nfev", "status"]


def _arch_index(rel, t):
    import torch
    return torch.as_tensor(rel, device=t.device, dtype=torch.long)
