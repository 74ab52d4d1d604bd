"""ppalign drop-in: iterative align-and-average (ppalign.py:54-243) on the GPU.

Per iteration every (archive, subint) unit is fitted in one batched device
call (phase guess with Ns = nbin at nu_fit, then phase[+DM] trust-ncg), then
rotated and accumulated with weights scales/errs^2 in the Fourier domain
(ppf_rotate_accumulate; linear, so equal to summing irfft'd rotations).  With
torch.distributed initialised, units are sharded contiguously over ranks and
the only collective is one all-reduce (sum, fp64) of the [nchan, nbin/2+1]
spectrum and the channel weights per iteration -- RCCL over xGMI with the
"nccl" backend.  Every rank then divides locally and holds the new template.
"""
import gc
import itertools
import operator

import numpy as np
import torch

from . import archive as _arch
from .pplib import (DataBunch, Dconst, guess_fit_freq, gaussian_profile, rotate_data,
                    fit_phase_shift)
from .pptoaslib import fit_portraits_batch

# Keep every unit's data spectrum on the device after the first iteration's
# data pass (Engine.spec_cache): later iterations refit from it without
# transforming the data again, and the rotate-and-sum reads it instead of
# the time-domain rows.  Needs about the data's size again in HBM; off, or
# without the room, every iteration transforms the data twice as before.
SPEC_CACHE = True

rm_baseline = False


def shard_range(n, rank, world):
    """Contiguous [lo, hi) slice of n units for rank (sizes differ by <= 1)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def dist_info():
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed.get_rank(), torch.distributed.get_world_size()
    return 0, 1


def allreduce_sum(*tensors):
    """Sum tensors over all ranks in place (one fused buffer, one collective)."""
    rank, world = dist_info()
    if world == 1:
        return tensors
    flat = torch.cat([t.reshape(-1) for t in tensors])
    torch.distributed.all_reduce(flat, op=torch.distributed.ReduceOp.SUM)
    off = 0
    for t in tensors:
        n = t.numel()
        t.copy_(flat[off:off + n].reshape(t.shape))
        off += n
    return tensors


class _StackOpened(list):
    """_open_all's result when it is one register_archives stack, whole and
    in order (``stk``): _Bulk reads the stack without visiting the archives."""
    stk = None


def _open_stack(datafiles, reg, nbin, SNR_cutoff):
    """_open_all for exactly the archives of one register_archives stack, in
    registration order, each still registered as it was and passing the nbin
    and S/N checks: the checks as C-level maps over the bunches (their
    current values) instead of a Python visit per archive.  None when that
    does not apply (the per-archive path then runs, with its messages)."""
    if not reg or not datafiles or not isinstance(datafiles[0], str):
        return None
    b0 = reg.get(datafiles[0])
    s = b0.get("_stack") if b0 is not None else None
    if s is None or s[1] != 0:
        return None
    stk = s[0]
    bs = stk.bunches
    n = len(bs)
    if len(datafiles) != n or tuple(datafiles) != stk.names or \
            not all(map(operator.is_, map(reg.get, stk.names), bs)):
        return None
    nb = np.fromiter(map(operator.itemgetter("nbin"), bs), dtype=np.int64, count=n)
    snr = np.fromiter(map(operator.itemgetter("prof_SNR"), bs), dtype=np.float64, count=n)
    if (nb != nbin).any() or (snr < SNR_cutoff).any():
        return None
    out = _StackOpened(zip(stk.names, stk.views()))
    out.stk = stk
    return out


def _open_all(datafiles, model_data, SNR_cutoff, quiet, skip_these, tscrunch, pscrunch):
    """Metadata of every archive (ppalign.py:121-159's checks, no DATA read):
    [(name, Archive)] of the archives to align."""
    out = []
    # registered archives with nothing to process are read in place; with no
    # tscrunch / baseline removal asked that is every registered one
    reg = _arch._registry if not tscrunch and not rm_baseline else {}
    RV = _arch._RegisteredView
    nbin = model_data.nbin
    fast = _open_stack(datafiles, reg, nbin, SNR_cutoff)
    if fast is not None:
        return fast
    for name in datafiles:
        b = reg.get(name) if isinstance(name, str) else None
        if b is not None:
            a = RV(b)
        else:
            try:  # ppalign.py:123-127 (rm_baseline False: F0_fact = 0, pptoas.py:26-29)
                a = _arch.registered_view(name, dedisperse=False, tscrunch=tscrunch,
                                          rm_baseline=rm_baseline) or \
                    _arch.open_archive(name, dedisperse=False, tscrunch=tscrunch,
                                       pscrunch=pscrunch, rm_baseline=rm_baseline, quiet=True)
            except RuntimeError:
                if not quiet:
                    print("%s: cannot load_data().  Skipping it." % name)
                skip_these.append(name)
                continue
        m = a.meta
        if m.nbin != nbin:
            if not quiet:
                print("%s: %d != %d phase bins.  Skipping it." % (name, m.nbin, model_data.nbin))
            skip_these.append(name)
            continue
        if m.prof_SNR < SNR_cutoff:
            if not quiet:
                print("%s: %d < %d S/N cutoff.  Skipping it." % (name, m.prof_SNR, SNR_cutoff))
            skip_these.append(name)
            continue
        out.append((name, a))
    return out


class _All(np.ndarray):
    """Marker type of the shared every-channel index array (_units)."""


_ALL_CACHE = {}


def _all_index(nchan):
    """The shared every-channel index array for nchan channels:
    np.arange(nchan) viewed as _All, one read-only array per nchan (no
    per-call module state: calls with different nchan do not interfere)."""
    a = _ALL_CACHE.get(nchan)
    if a is None:
        a = np.arange(nchan).view(_All)
        a.setflags(write=False)
        a = _ALL_CACHE.setdefault(nchan, a)
    return a


class _Bulk:
    """Metadata of every opened archive stacked row-wise (one row per subint,
    archives in order; archive i's rows are offs[i]:offs[i + 1]), so the unit
    set-up indexes arrays instead of visiting 4,096 bunches one by one.  Built
    only when every archive holds plain arrays of its own nsub rows and needs
    nothing read to complete them (no snr_deferred); else ``build`` returns
    None and the per-archive path runs.  Rows: F freqs, W weights, S SNRs of
    polarisation 0, E noise_stds of polarisation 0 (NaN rows where an archive
    has none; ``has_e`` says which rows have them), P periods, DM; ``same``
    [narch]: every row of the archive equals the template's frequencies
    (ppalign.py:156's freq_diffs all 0); ``regs`` [narch]: the registered
    subints tensor of each archive or None; ``index``: name -> archive.
    Archives registered together (archive.register_archives) are rows of one
    stack already: their arrays are slices of it (no per-archive visit), with
    ``allok`` (every channel of every subint on) and ``rows_view`` (every
    row's [nchan, nbin] data as one view, npol 1) from the stack."""
    allok = False
    rows_view = None
    unit_rows = None  # [nunits] bulk row of each unit (set by _units)

    @staticmethod
    def build(opened, model_data, nchan):
        mfq = np.asarray(model_data.freqs)
        if len(opened) == 0 or mfq.ndim != 2 or mfq.shape[0] != 1 or mfq.shape[1] != nchan:
            return None
        b = _Bulk._from_stack(opened, mfq, nchan)
        if b is not None:
            return b
        metas = [a.meta for _, a in opened]
        if any(m.get("snr_deferred") for m in metas):
            return None
        nsubs = [m.nsub for m in metas]
        if min(nsubs) < 1:
            return None
        try:
            F = np.concatenate([m.freqs for m in metas])
            W = np.concatenate([m.weights for m in metas])
            S = np.concatenate([np.asarray(m.SNRs)[:, 0] for m in metas])
            P = np.concatenate([m.Ps for m in metas])
        except (ValueError, IndexError, TypeError):
            return None
        offs = np.zeros(len(metas) + 1, dtype=np.int64)
        np.cumsum(nsubs, out=offs[1:])
        R = int(offs[-1])
        if F.shape != (R, nchan) or W.shape != (R, nchan) or S.shape != (R, nchan) or \
                P.shape != (R,) or F.dtype != np.float64:
            return None
        if [len(m.freqs) for m in metas] != nsubs:  # each archive's own rows
            return None
        b = _Bulk()
        b.F, b.W, b.S, b.P, b.offs = F, W.astype(np.float64, copy=False), S, P, offs
        b.DM = np.repeat(np.array([float(m.DM) for m in metas]), nsubs)
        nss = [m.get("noise_stds") for m in metas]
        b.has_e = np.repeat(np.array([ns is not None for ns in nss]), nsubs)
        if b.has_e.all():
            b.E = np.concatenate([np.asarray(ns)[:, 0] for ns in nss])
        else:
            b.E = np.full((R, nchan), np.nan)
            for i, ns in enumerate(nss):
                if ns is not None:
                    b.E[offs[i]:offs[i + 1]] = np.asarray(ns)[:, 0]
        # same frequencies as the template: freq_diffs all exactly 0 (NaN never)
        b.same = np.logical_and.reduceat(((F - mfq) == 0.0).all(axis=1), offs[:-1])
        b.regs = [a.registered_rows() for _, a in opened]
        b.index = {name: i for i, (name, _) in enumerate(opened)}
        return b

    @staticmethod
    def _from_stack(opened, mfq, nchan):
        """build() for archives of one archive.register_archives stack, opened
        as registered views: slices (or one fancy index) of the stack."""
        if isinstance(opened, _StackOpened):  # the whole stack, in order
            stk = opened.stk
            if stk.nchan != nchan:
                return None
            n = len(opened)
            sel = slice(0, n)
        else:
            RV = _arch._RegisteredView
            if not all(type(a) is RV for _, a in opened):
                return None
            st = [a.meta.get("_stack") for _, a in opened]
            s0 = st[0]
            if s0 is None:
                return None
            stk = s0[0]
            if not all(s is not None and s[0] is stk for s in st) or stk.nchan != nchan:
                return None
            idx = np.fromiter((s[1] for s in st), dtype=np.int64, count=len(st))
            n = len(idx)
            if n == 1 or (np.diff(idx) == 1).all():
                sel = slice(int(idx[0]), int(idx[0]) + n)
            else:
                sel = idx
        nsub = stk.nsub
        R = n * nsub
        b = _Bulk()
        b.F = stk.freqs[sel].reshape(R, nchan)
        b.W = stk.weights[sel].reshape(R, nchan)
        b.S = stk.snrs0[sel].reshape(R, nchan)
        b.P = stk.Ps[sel].reshape(R)
        b.DM = np.repeat(stk.DM[sel], nsub)
        b.offs = np.arange(n + 1, dtype=np.int64) * nsub
        if stk.noise0 is not None:
            b.E = stk.noise0[sel].reshape(R, nchan)
            b.has_e = np.repeat(stk.has_noise[sel], nsub)
        else:
            b.E = None  # every row NaN
            b.has_e = np.zeros(R, dtype=bool)
        if np.isfinite(mfq).all():  # F - mfq == 0 exactly when F == mfq
            eq = (b.F == mfq).all(axis=1)
        else:
            eq = ((b.F - mfq) == 0.0).all(axis=1)
        b.same = eq.reshape(n, nsub).all(axis=1)
        b.allok = stk.allok
        if stk.rows is not None and stk.npol == 1 and isinstance(sel, slice):
            # a view only: archives opened out of stack order would make this
            # a device gather of every selected archive's subints on every
            # rank; they take the per-archive rows instead
            b.rows_view = stk.rows[sel].reshape(R, nchan, stk.nbin)
        b.regs = list(map(operator.itemgetter("subints"), stk.bunches)) \
            if isinstance(opened, _StackOpened) else [a.meta.subints for _, a in opened]
        b.index = dict(zip(map(operator.itemgetter(0), opened), range(n)))
        b.nsub = nsub
        return b


def _units(opened, model_data, bulk=None):
    """(name, subint, ichans, model_ichans) per ok subint (ppalign.py:153-177).
    A unit whose channels are all the template's (every channel on in both)
    carries the one shared index array ALL (its intersect1d)."""
    units = []
    mf = model_data.freqs[0]
    nch = len(mf)
    ALL = _all_index(nch)
    mok = model_data.ok_ichans[0]
    model_full = len(mok) == nch
    mfq = np.asarray(model_data.freqs)
    if bulk is not None and model_full and bulk.allok and bulk.same.all():
        # one register_archives stack, every channel on everywhere: every
        # subint a unit with the shared ALL, in bulk row order
        ns = bulk.nsub
        if ns == 1:
            names = map(operator.itemgetter(0), opened)
            units = list(zip(names, itertools.repeat(0), itertools.repeat(ALL),
                             itertools.repeat(ALL)))
        else:
            units = [(name, isub, ALL, ALL) for name, _ in opened for isub in range(ns)]
        bulk.unit_rows = np.arange(len(units), dtype=np.int64)
        return units
    if bulk is not None:
        if model_full:  # the common case: rows of every channel, one shared ALL
            for (name, a), same in zip(opened, bulk.same.tolist()):
                m = a.meta
                if same:
                    oic = m.ok_ichans
                    for isub in m.ok_isubs:
                        isub = int(isub)
                        oi = oic[isub]
                        if len(oi) == nch:
                            units.append((name, isub, ALL, ALL))
                        else:
                            ichans = np.intersect1d(oi, mok)
                            units.append((name, isub, ichans, ichans))
                else:
                    _units_of(units, name, m, False, mf, mok, model_full)
        else:
            for (name, a), same in zip(opened, bulk.same.tolist()):
                _units_of(units, name, a.meta, same, mf, mok, model_full)
        return units
    mbytes = mfq.tobytes()
    for name, a in opened:
        m = a.meta
        f = m.freqs
        if isinstance(f, np.ndarray) and f.shape == mfq.shape and f.dtype == mfq.dtype and \
                f.tobytes() == mbytes and not np.isnan(f).any():
            same = True  # identical values: fd is 0 everywhere
        else:
            try:
                fd = f - model_data.freqs
                same = fd.min() == fd.max() == 0.0
            except ValueError:
                same = False
        _units_of(units, name, m, same, mf, mok, model_full)
    return units


def _units_of(units, name, m, same, mf, mok, model_full):
    """One archive's units (see _units); same: its frequencies are the template's."""
    nch = len(mf)
    ALL = _all_index(nch)
    for isub in m.ok_isubs:
        if same:
            oi = m.ok_ichans[isub]
            if model_full and len(oi) == nch:  # ok_ichans are sorted, unique
                ichans = mich = ALL
            else:
                ichans = np.intersect1d(oi, mok)
                mich = ichans
        else:
            ichans = np.asarray(m.ok_ichans[isub])
            mich = np.array([np.argmin(abs(mf - m.freqs[isub, c])) for c in ichans])
        units.append((name, int(isub), ichans, mich))
    return units


def _guess_fit_freq_rows(freqs, snrs):
    """guess_fit_freq per row (pplib.py:2618-2632) for rows of equal length:
    numpy's row sums of a C-order 2-D array are its 1-D sums, so each value
    is the one guess_fit_freq(freqs[i], snrs[i]) returns."""
    f = np.ascontiguousarray(freqs, dtype=np.float64)
    w = np.ascontiguousarray(snrs, dtype=np.float64)
    if len(f) > 1 and (f == f[0]).all():
        if (w == w[0]).all():  # one distinct row
            return np.full(len(f), guess_fit_freq(f[0], w[0]))
        # one frequency row: its terms once, broadcast (the same elementwise
        # operations on the same values, so the same sums)
        f0 = f[0]
        nu0 = (f0.min() + f0.max()) * 0.5
        f2 = f0 ** -2
        return nu0 + np.sum((f0 - nu0) * w * f2, axis=1) / np.sum(w * f2, axis=1)
    nu0 = (f.min(axis=1) + f.max(axis=1)) * 0.5
    f2 = f ** -2
    return nu0 + np.sum((f - nu0[:, None]) * w * f2, axis=1) / np.sum(w * f2, axis=1)


def _is_full(ichans, mich, full_rows):
    """A unit with every channel of the template, in template order."""
    if isinstance(ichans, _All):
        return True
    return len(ichans) == len(full_rows) and np.array_equal(mich, full_rows) and \
        np.array_equal(ichans, mich)


def _strided_rows(rows):
    """rows: (t, j) pairs naming t[j] of float64 tensors [k, npol=1, nchan,
    nbin].  When every t[j] is a contiguous [1, nchan, nbin] row and they are
    equally spaced in one storage, returns one [n, nchan, nbin] view of them
    all (no copy); else None."""
    t0, j0 = rows[0]
    if t0.dim() != 4 or t0.shape[1] != 1 or t0.dtype != torch.float64:
        return None
    shape = t0.shape
    nchan, nbin = shape[2], shape[3]
    st0 = t0.stride()
    if (nbin > 1 and st0[3] != 1) or (nchan > 1 and st0[2] != nbin):
        return None
    # one storage: every row a view of t0's base (a cheap identity test), or
    # failing that the storages' own addresses; the same [1, nchan, nbin] row
    # shape and channel / bin strides (tested per distinct tensor: archives
    # may share one)
    base0 = t0._base
    ts = {id(t): t for t, _ in rows}.values() if len(rows) > 1 else (t0,)
    if base0 is not None:
        if not all(t._base is base0 for t in ts):
            return None
    else:
        sbase = t0.untyped_storage().data_ptr()
        if not all(t.untyped_storage().data_ptr() == sbase for t in ts):
            return None
    if not all(t.shape[1:] == shape[1:] and t.stride()[2:] == st0[2:] for t in ts):
        return None
    # the rows' addresses, equally spaced by st bytes
    q = np.fromiter((t.data_ptr() + j * t.stride(0) * 8 for t, j in rows), dtype=np.int64,
                    count=len(rows))
    st = int(q[1] - q[0]) if len(rows) > 1 else nchan * nbin * 8
    if st < nchan * nbin * 8 or st % 8 or (len(rows) > 2 and (np.diff(q) != st).any()):
        return None
    off = t0.storage_offset() + j0 * st0[0]
    return t0.as_strided((len(rows), nchan, nbin), (st // 8, nbin, 1), off)


class _UnitStack:
    """Device-resident inputs of this rank's units, built once and reused by
    every iteration (the reference re-reads every archive per iteration,
    ppalign.py:121-127; the data do not change): unit channel c sits in
    template slot mich[c], other slots are masked.  Units whose channels are
    the template's own (every channel, same order) are gathered with one
    device copy for all of them -- none when they already are equally spaced
    rows of one tensor -- and their host arrays stacked row-wise; the others
    take the per-channel path."""

    def __init__(self, eng, units, opened, model_freqs, npol, nchan, nbin, bulk=None,
                 urows=None):
        dev = eng.device
        n = len(units)
        f64 = dict(dtype=torch.float64, device=dev)
        self.n = n
        self.pols = [None] * npol
        if bulk is not None and npol == 1 and self._from_bulk(dev, units, bulk, urows):
            return
        freqs = np.tile(np.asarray(model_freqs, dtype=np.float64), (n, 1))
        errs = np.ones((n, nchan))
        mask = np.zeros((n, nchan), dtype=np.uint8)
        wts = np.zeros((n, nchan))
        P, DMg, nu_fit = np.zeros(n), np.zeros(n), np.zeros(n)
        need_noise = np.zeros(n, dtype=bool)
        arch = dict(opened)
        by_arch = {}
        for i, u in enumerate(units):
            by_arch.setdefault(u[0], []).append(i)
        full_rows = np.arange(nchan)
        frow, fsrc = [], []  # full units: stack row i <- (tensor, subint row)
        # the stack is allocated unless every unit is a full row of one
        # strided tensor (decided once all units are seen)
        partial_units = [i for i, u in enumerate(units) if not _is_full(u[2], u[3], full_rows)]
        if partial_units or npol != 1:
            self.pols = [torch.empty((n, nchan, nbin), **f64) for _ in range(npol)]
        full_f, full_w, full_s, full_e = [], [], [], []
        for name, idx in by_arch.items():
            a = arch[name]
            m = a.meta
            if len(idx) == 1:
                lo = units[idx[0]][1]
                hi = lo + 1
            else:
                isubs = [units[i][1] for i in idx]
                lo, hi = min(isubs), max(isubs) + 1
            reg = a.registered_rows()
            if reg is not None:  # the caller's own registered tensor, no slicing
                sub, lo = reg, 0
            else:
                sub = a.read(lo, hi)  # this rank's subint range only
            if not isinstance(sub, torch.Tensor):
                sub = torch.as_tensor(np.ascontiguousarray(sub), device=dev)
            snrs = m.SNRs
            if m.get("snr_deferred"):  # load_data's SNRs of the subints read
                snrs = np.array(m.SNRs, dtype=np.float64)
                snrs[lo:hi] = a.snrs(sub)
            ns = m.get("noise_stds")
            ns = None if ns is None else np.asarray(ns)
            Ps, DM, mfreqs, mwts = m.Ps, m.DM, m.freqs, m.weights
            # device rows, and the host arrays of this archive's units (full
            # units as (tensor, row) pairs, stacked once for all archives below)
            for i in idx:
                _, isub, ichans, mich = units[i]
                P[i] = Ps[isub]
                DMg[i] = DM
                if _is_full(ichans, mich, full_rows):
                    frow.append(i)
                    fsrc.append((sub, isub - lo))
                    full_f.append(mfreqs[isub])
                    full_w.append(mwts[isub])
                    full_s.append(snrs[isub, 0])
                    full_e.append(None if ns is None else ns[isub, 0])
                    continue
                ic = torch.as_tensor(ichans, device=dev, dtype=torch.long)
                mc = torch.as_tensor(mich, device=dev, dtype=torch.long)
                for ipol in range(npol):
                    self.pols[ipol][i].zero_()
                    self.pols[ipol][i].index_copy_(0, mc, sub[isub - lo, ipol].index_select(0, ic))
                freqs[i, mich] = mfreqs[isub, ichans]
                if ns is not None:
                    errs[i, mich] = ns[isub, 0, ichans]
                else:
                    need_noise[i] = True
                mask[i, mich] = 1
                wts[i, mich] = mwts[isub, ichans]
                nu_fit[i] = guess_fit_freq(mfreqs[isub, ichans], snrs[isub, 0, ichans])
        full_i = frow
        if full_i:
            rows = np.array(full_i)
            fr = np.stack(full_f)
            freqs[rows] = fr
            wts[rows] = np.stack(full_w)
            mask[rows] = 1
            have = np.array([e is not None for e in full_e])
            if have.any():
                errs[rows[have]] = np.stack([e for e in full_e if e is not None])
            need_noise[rows[~have]] = True
            nu_fit[rows] = _guess_fit_freq_rows(fr, np.stack(full_s))
        view = _strided_rows(fsrc) if (frow and npol == 1 and frow == list(range(n))) else None
        if view is not None:
            # every unit a full row of one strided tensor (rows of the caller's
            # own stack), in unit order: use it in place, no copy
            self.pols = [view]
        elif frow:  # one gather per polarisation for every full unit
            if self.pols[0] is None:
                self.pols = [torch.empty((n, nchan, nbin), **f64) for _ in range(npol)]
            dst = torch.as_tensor(np.array(frow), device=dev, dtype=torch.long)
            src = torch.stack([t[j] for t, j in fsrc])  # [nfull, npol, nchan, nbin]
            for ipol in range(npol):
                self.pols[ipol].index_copy_(0, dst, src[:, ipol])
            del src
        # load_data's noise_stds (pplib.py:2744-2748) where the archive has
        # none: NaN here, so the fit's data pass estimates them from the same
        # rows it transforms (get_noise_PS) and returns them (fit "errs")
        errs = np.where(need_noise[:, None] & (mask > 0), np.nan, errs)
        self.freqs, self.errs, self.mask, self.wts = freqs, errs, mask, wts
        self.P, self.DMg, self.nu_fit = P, DMg, nu_fit

    def _from_bulk(self, dev, units, bulk, urows=None):
        """The same stack when every unit is full (ALL) and every archive is
        registered: its host arrays are rows of the stacked metadata (one
        fancy index each), its data one strided view of the registered rows
        (or one gather).  urows: the bulk rows of these units when the caller
        has them (_units' unit_rows).  False (nothing set) when that does not
        apply."""
        if urows is not None and bulk.rows_view is not None:
            rows = urows  # one register_archives stack: every unit full
            n = len(rows)
            if n and rows[-1] - rows[0] == n - 1 and (n < 3 or (np.diff(rows) == 1).all()):
                rows = slice(int(rows[0]), int(rows[0]) + n)  # views, no copies
                view = bulk.rows_view[rows]
            else:
                view = bulk.rows_view[torch.as_tensor(rows, device=bulk.rows_view.device)]
            if view.device != dev:
                view = view.to(dev)
        else:
            if not all(type(u[2]) is _All for u in units):
                return False
            ix, regs = bulk.index, bulk.regs
            ai = [ix[u[0]] for u in units]
            src = [(regs[i], u[1]) for i, u in zip(ai, units)]
            if any(not isinstance(t, torch.Tensor) for t, _ in src):
                return False
            rows = bulk.offs[np.array(ai, dtype=np.int64)] + \
                np.fromiter((u[1] for u in units), dtype=np.int64, count=len(units))
            view = _strided_rows(src)
            if view is None:
                view = torch.stack([t[j, 0] for t, j in src]).to(dev)
        freqs = bulk.F[rows]
        # NaN rows: the data pass estimates them (see __init__)
        errs = torch.full(freqs.shape, float("nan"), dtype=torch.float64, device=dev) \
            if bulk.E is None else bulk.E[rows]
        self.pols = [view]
        self.freqs, self.errs, self.wts = freqs, errs, bulk.W[rows]
        self.mask = np.ones(freqs.shape, dtype=np.uint8)
        self.P, self.DMg = bulk.P[rows], bulk.DM[rows]
        self.nu_fit = _guess_fit_freq_rows(freqs, bulk.S[rows])
        return True

    def _spec_cache(self, eng):
        """The units' data-spectrum cache (SPEC_CACHE), made on first use
        when it fits in free device memory with a quarter to spare; None
        otherwise."""
        sc = getattr(self, "_spec", False)
        if sc is not False:
            return sc
        sc = None
        d = self.pols[0]
        if SPEC_CACHE and isinstance(d, torch.Tensor) and d.device.type == "cuda":
            n, nchan, nbin = d.shape
            from .engine import SpecCache
            need = SpecCache.bytes_for(eng, n, nchan, nbin)
            free, _ = torch.cuda.mem_get_info(d.device)
            if need < 0.75 * free:
                sc = eng.spec_cache(n, nchan, nbin)
        self._spec = sc
        return sc

    def fit_and_accumulate(self, eng, model_port, fit_dm, accum, tw, mark=None):
        """One iteration's fits (ppalign.py:178-195) and weighted rotate-and-sum
        (ppalign.py:202-208) in the Fourier domain.  The fit results stay on
        the device: the rotation phases and weights are formed there and fed
        to the rotate-and-sum without a host round trip."""
        import time
        t0 = time.perf_counter()
        n = self.n
        dev = eng.device
        if getattr(self, "_dv", None) is None:  # per-unit inputs, on the device once
            f64 = dict(dtype=torch.float64, device=dev)
            init = np.stack([np.zeros(n), self.DMg, np.zeros(n), np.zeros(n), np.zeros(n)], 1)
            self._dv = dict(P=torch.as_tensor(self.P, **f64),
                            f2=torch.as_tensor(self.freqs ** -2.0, **f64),
                            on=torch.as_tensor(self.mask > 0, device=dev),
                            init=torch.as_tensor(init, **f64),
                            freqs=torch.as_tensor(self.freqs, **f64),
                            errs=torch.as_tensor(self.errs, **f64),
                            mask=torch.as_tensor(self.mask, device=dev),
                            wts=torch.as_tensor(self.wts, **f64),
                            nu3=torch.as_tensor(np.stack([self.nu_fit] * 3, 1), **f64),
                            nu=torch.as_tensor(self.nu_fit, **f64))
        dv = self._dv
        flags = [1, int(bool(fit_dm)), 0, 0, 0]
        spec = self._spec_cache(eng)
        out = fit_portraits_batch(self.pols[0], model_port, dv["init"], dv["P"], dv["freqs"],
                                  nu_fits=dv["nu3"], errs=dv["errs"], fit_flags=flags,
                                  log10_tau=False, chan_mask=dv["mask"], weights=dv["wts"],
                                  guess=True, guess_Ns=model_port.shape[1], guess_wrap=False,
                                  guess_nu=dv["nu"], to_host=False, spec_cache=spec)
        if mark is not None:
            t0 = mark("fit", t0)
        out = {k: torch.as_tensor(out[k], device=dev) for k in ("params", "nu_out", "scales",
                                                                "errs")}
        phase = out["params"][:, 0]
        DM = out["params"][:, 1]
        nu_ref = out["nu_out"][:, 0]
        # rotate_data(port, phase, DM, P, freqs, nu_ref) per channel (pplib.py:2406-2415)
        ph = phase[:, None] + (Dconst * DM / dv["P"])[:, None] * (dv["f2"] - nu_ref[:, None] ** -2.0)
        e2 = torch.as_tensor(out["errs"], device=dev) ** 2  # the sigma each channel was fitted with
        w = torch.where(dv["on"], out["scales"] / e2, torch.zeros((), dtype=torch.float64,
                                                                 device=dev))
        for ipol, pol in enumerate(self.pols):
            if ipol == 0 and spec is not None:  # the fitted polarisation's cached spectra
                eng.rotate_accumulate_spec(spec, ph, w, accum[0])
            else:
                eng.rotate_accumulate(pol, ph, w, accum[ipol])
        tw += w.sum(dim=0).to(tw.device)
        if mark is not None:
            mark("accumulate", t0)
        return out


def align_archives(metafile, initial_guess, fit_dm=True, tscrunch=False, pscrunch=True,
                   SNR_cutoff=0.0, outfile=None, norm=None, rot_phase=0.0, place=None,
                   niter=1, quiet=False, return_weights=False, timings=None):
    """Iteratively align and average archives; returns aligned_port[npol, nchan, nbin].

    The reference writes the result into a PSRCHIVE archive; here the portrait
    is returned (and written with archive.save_archive when ``outfile`` ends in
    .npz).  ``timings`` (diagnostic): a dict that receives the wall time of
    each phase (open, unit stack, per-iteration fit / accumulate / exchange),
    with a device synchronisation at every phase boundary.
    """
    import time
    from .engine import get_engine

    def mark(key, t0):
        if timings is None:
            return 0.0
        torch.cuda.synchronize()
        t = time.perf_counter()
        timings[key] = timings.get(key, 0.0) + (t - t0)
        return t
    t0 = mark("start", 0.0) if timings is not None else 0.0
    if isinstance(metafile, str) and _arch.file_is_type(metafile, "ASCII"):
        datafiles = [ln.strip() for ln in open(metafile).readlines() if ln.strip()]
        if outfile is None:
            outfile = metafile + ".algnd.fits"
    else:
        datafiles = list(metafile) if not isinstance(metafile, str) else [metafile]
    # the initial guess: dedispersed, tscrunched, baseline removed (ppalign.py:103-106)
    model_data = _arch.load_data(initial_guess, dedisperse=True, dededisperse=False,
                                 tscrunch=True, pscrunch=pscrunch, rm_baseline=True, quiet=quiet)
    npol = 1 if pscrunch else model_data.npol
    model_port = np.asarray((model_data.masks * model_data.subints)[0, 0], dtype=np.float64)
    nchan, nbin = model_port.shape
    nharm = nbin // 2 + 1
    eng = get_engine()
    dev = eng.device
    rank, world = dist_info()
    skip_these = []
    # a few objects per archive and unit, none cyclic: keep the cyclic
    # collector (a full pass over every live object, tens of ms with 4,096
    # registered archives) out of the set-up
    gc_on = gc.isenabled()
    gc.disable()
    try:
        opened = _open_all(datafiles, model_data, SNR_cutoff, quiet, skip_these, tscrunch,
                           pscrunch)
        bulk = _Bulk.build(opened, model_data, nchan)
        units = _units(opened, model_data, bulk)
        t0 = mark("open", t0)
        lo, hi = shard_range(len(units), rank, world)
        mine = units[lo:hi]
        multi = [u for u in mine if len(u[2]) > 1]
        single = [u for u in mine if len(u[2]) <= 1]
        # bulk rows of this rank's units when _units made them in bulk order
        urows = bulk.unit_rows[lo:hi] if bulk is not None and bulk.unit_rows is not None and \
            not single else None
        stack = _UnitStack(eng, multi, opened, model_data.freqs[0], npol, nchan, nbin, bulk,
                           urows) if multi else None
        del bulk
    finally:
        if gc_on:
            gc.enable()
    t0 = mark("unit_stack", t0)
    archives = {}
    for name, a in (opened if single else ()):  # 1-channel hack units (rare): on the host
        if any(u[0] == name for u in single):
            archives[name] = _arch.load_data(name, dedisperse=False, tscrunch=tscrunch,
                                             pscrunch=pscrunch, rm_baseline=rm_baseline,
                                             quiet=True)
    count = 1
    aligned = None
    tw = None
    while niter:
        if not quiet and rank == 0:
            print("Doing iteration %d..." % count)
        accum = torch.zeros(npol, nchan, nharm, 2, dtype=torch.float64, device=dev)
        tw = torch.zeros(nchan, dtype=torch.float64, device=dev)
        if stack is not None:
            stack.fit_and_accumulate(eng, model_port, fit_dm, accum, tw, mark)
        t1 = t0 if stack is None else time.perf_counter()  # the 1-channel hack's start
        for u in single:  # 1-channel hack, ppalign.py:196-201
            _single_channel(u, archives, model_port, npol, accum, tw, dev)
        t0 = mark("accumulate", t1)
        allreduce_sum(accum, tw)
        spec = torch.view_as_complex(accum).reshape(npol * nchan, nharm)
        port = eng.irfft_rows(spec, nbin).reshape(npol, nchan, nbin)
        good = (tw > 0)[None, :, None]
        port = torch.where(good, port / tw[None, :, None], port)
        # the next iteration's template stays on the device (the 1-channel
        # hack and the caller take it on the host)
        model_port = port[0].cpu().numpy() if single else port[0]
        t0 = mark("exchange", t0)
        niter -= 1
        count += 1
    aligned = port.cpu().numpy()
    if norm in ("mean", "max", "prof", "rms", "abs"):
        from .pplib import get_noise
        for ipol in range(npol):
            aligned[ipol] = _normalize(aligned[ipol], norm, get_noise)
    if rot_phase:
        aligned = rotate_data(aligned, rot_phase)
    if place is not None:
        prof = np.average(aligned[0], axis=0)
        delta = prof.max() * gaussian_profile(len(prof), place, 0.0001)
        aligned = rotate_data(aligned, fit_phase_shift(prof, delta, Ns=nbin).phase)
    if outfile is not None and str(outfile).endswith(".npz") and rank == 0:
        w = np.where(tw.cpu().numpy() > 0, 1.0, 0.0)
        _arch.save_archive(outfile, dict(subints=aligned[None], freqs=model_data.freqs[0],
                                         Ps=model_data.Ps[:1], epochs=model_data.epochs[:1],
                                         weights=w[None], DM=0.0))
    if return_weights:
        return aligned, tw.cpu().numpy()
    return aligned


def _single_channel(u, archives, model_port, npol, accum, tw, dev):
    name, isub, ichans, mich = u
    d = archives[name]
    nbin = model_port.shape[1]
    errs = d.noise_stds[isub, 0, ichans] if d.get("noise_stds") is not None else [None]
    r = fit_phase_shift(d.subints[isub, 0, ichans][0], model_port[mich][0], errs[0], Ns=nbin)
    from .engine import get_engine
    eng = get_engine()
    w = np.array([[r.scale / errs[0] ** 2]]) if errs[0] is not None else np.array([[r.scale]])
    for ipol in range(npol):
        acc = torch.zeros_like(accum[ipol])
        eng.rotate_accumulate(d.subints[isub, ipol, ichans][None], np.array([[r.phase]]), w, acc)
        accum[ipol][int(mich[0])] += acc[0]
    tw[int(mich[0])] += float(w[0, 0])


def _normalize(port, method, get_noise):
    """normalize_portrait for the final template (pplib.py:2462-2507)."""
    out = np.zeros(port.shape)
    for i in range(len(port)):
        if not port[i].any():
            continue
        if method == "mean":
            nrm = port[i].mean()
        elif method == "max":
            nrm = port[i].max()
        elif method == "rms":
            nrm = get_noise(port[i])
        elif method == "abs":
            nrm = (port[i] ** 2).sum() ** 0.5
        else:
            good = np.where(port.sum(axis=1) != 0.0)[0]
            nrm = fit_phase_shift(port[i], np.average(port[good], axis=0)).scale
        out[i] = port[i] / nrm
    return out
