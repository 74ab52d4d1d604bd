"""Device engine: owns a libppfit context and marshals arrays to the C ABI.

torch is used only as plumbing: device allocations, H2D/D2H copies and the
HIP stream handle.  All numerics run in the HIP kernels of libppfit.so.
"""
import collections
import ctypes
import functools

import numpy as np
import torch

from . import _lib

_NAN = float("nan")


class PPFitError(RuntimeError):
    pass


def _dev_f64(x, dev, shape=None):
    if x is None:
        return None
    if isinstance(x, torch.Tensor):
        t = x.to(device=dev, dtype=torch.float64)
    else:
        t = torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device=dev)
    t = t.contiguous()
    if shape is not None:
        t = t.reshape(shape)
    return t


def _dev_i32(x, dev):
    if x is None:
        return None
    if isinstance(x, torch.Tensor):
        return x.to(device=dev, dtype=torch.int32).contiguous()
    return torch.as_tensor(np.ascontiguousarray(x, dtype=np.int32), device=dev)


def _dev_u8(x, dev):
    if x is None:
        return None
    if isinstance(x, torch.Tensor):
        return x.to(device=dev, dtype=torch.uint8).contiguous()
    return torch.as_tensor(np.array(x, dtype=np.uint8), device=dev)  # copy: inputs may be read-only views


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _nan_none(x):
    """Array-like that may contain None (reference 'use the default') -> float64 with NaN."""
    a = np.asarray(x)
    if a.dtype != object:  # no None in it
        return a.astype(np.float64)
    return np.array([np.nan if v is None else float(v) for v in a.ravel()],
                    dtype=np.float64).reshape(a.shape)


def _bcast(x, n, width, dev, fill=_NAN):
    """Per-subint row parameter: scalar, [width] or [n, width] -> [n, width] on dev."""
    if x is None:
        return torch.full((n, width), fill, dtype=torch.float64, device=dev)
    if isinstance(x, torch.Tensor):
        t = x.to(device=dev, dtype=torch.float64)
    else:
        t = torch.as_tensor(_nan_none(x), device=dev)
    if t.numel() == n * width:
        return t.reshape(n, width).contiguous()
    if t.numel() in (1, width):
        return t.reshape(1, -1).expand(n, width).contiguous()
    raise PPFitError("cannot broadcast %s to (%d, %d)" % (tuple(t.shape), n, width))


def _bcast_dev(t, n, width, dev, fill=_NAN):
    """_bcast for an input already on the device (None: fill)."""
    if t is None:
        return torch.full((n, width), fill, dtype=torch.float64, device=dev)
    if t.numel() == n * width:
        return t.reshape(n, width).contiguous()
    if t.numel() in (1, width):
        return t.reshape(1, -1).expand(n, width).contiguous()
    raise PPFitError("cannot broadcast %s to (%d, %d)" % (tuple(t.shape), n, width))


class _Stager:
    """The host (numpy) inputs of one call packed into one pinned buffer and
    copied to the device with one asynchronous H2D on the context stream, so
    the launches that follow on that stream see them; device tensors pass
    through unchanged.  add -> a token, run(), then get(token) -> tensor."""
    _ALIGN = 256

    def __init__(self, dev, stream):
        self.dev, self.stream = dev, stream
        self.host, self.nbytes = [], 0
        self.views = None

    def _add(self, a):
        if a is None or isinstance(a, torch.Tensor):
            return ("t", a)
        a = np.ascontiguousarray(a)
        off = self.nbytes
        self.host.append((off, a))
        self.nbytes = off + (a.nbytes + self._ALIGN - 1) // self._ALIGN * self._ALIGN
        return ("h", len(self.host) - 1)

    def f64(self, x):
        if isinstance(x, torch.Tensor):
            return ("t", x.to(device=self.dev, dtype=torch.float64))
        return self._add(None if x is None else np.asarray(x, dtype=np.float64))

    def rows(self, x):  # per-subint rows that may hold None (reference defaults)
        if isinstance(x, torch.Tensor):
            return ("t", x.to(device=self.dev, dtype=torch.float64))
        return self._add(None if x is None else _nan_none(x))

    def u8(self, x):
        if isinstance(x, torch.Tensor):
            return ("t", x.to(device=self.dev, dtype=torch.uint8))
        return self._add(None if x is None else np.asarray(x, dtype=np.uint8))

    def i32(self, x):
        if isinstance(x, torch.Tensor):
            return ("t", x.to(device=self.dev, dtype=torch.int32).contiguous())
        return self._add(None if x is None else np.asarray(x, dtype=np.int32))

    def run(self):
        self.views = []
        if not self.host:
            return
        pin = torch.empty(self.nbytes, dtype=torch.uint8, pin_memory=True)
        pv = pin.numpy()
        for off, a in self.host:
            pv[off:off + a.nbytes] = a.reshape(-1).view(np.uint8)
        buf = torch.empty(self.nbytes, dtype=torch.uint8, device=self.dev)
        with torch.cuda.stream(self.stream):
            buf.copy_(pin, non_blocking=True)
        self.buf = buf
        for off, a in self.host:
            v = buf[off:off + a.nbytes].view(_TORCH_DT[a.dtype.str]).reshape(a.shape)
            self.views.append(v)

    def get(self, tok):
        kind, v = tok
        if kind == "t":
            return None if v is None else v.contiguous()
        return self.views[v]


_TORCH_DT = {"<f8": torch.float64, "|u1": torch.uint8, "<i4": torch.int32}

# fit results: float64 keys and their widths per subint ("c" = nchan), in
# the order of one packed device buffer -- the keys the drivers read first,
# so their host copy is one contiguous prefix: the per-TOA scalars (params
# .. snr) then get_TOAs' per-channel keys (through channel_snrs)
RESULT_F64 = [("params", (5,)), ("param_errs", (5,)), ("nu_out", (3,)), ("chi2", ()),
              ("red_chi2", ()), ("snr", ()), ("cov", (5, 5)), ("scales", "c"),
              ("scale_errs", "c"), ("channel_snrs", "c"), ("init_used", (5,)), ("fun", ()),
              ("cov_nosc", (5, 5)), ("grad", (5,)), ("hess", (5, 5)), ("errs", "c")]
_LAYOUTS = {}


def _layout(nsub, nchan):
    """(key, offset, shape, size) of every float64 result and the total, for
    one (nsub, nchan) (cached: a batch loop asks for the same one each call)."""
    lay = _LAYOUTS.get((nsub, nchan))
    if lay is None:
        rows, o = [], 0
        for k, w in RESULT_F64:
            sh = (nsub, nchan) if w == "c" else (nsub,) + w
            n = int(np.prod(sh))
            rows.append((k, o, sh, n))
            o += n
        if len(_LAYOUTS) > 64:
            _LAYOUTS.clear()
        lay = _LAYOUTS[(nsub, nchan)] = (rows, o)
    return lay


def _result_tensors(nsub, nchan, dev):
    """Result tensors of one fit call as views of one float64 buffer (and
    nfev / status of one int32 buffer); "_packed" holds (buffer, int32
    buffer, layout)."""
    rows, total = _layout(nsub, nchan)
    flat = torch.empty(total, dtype=torch.float64, device=dev)
    iflat = torch.empty(2 * nsub, dtype=torch.int32, device=dev)
    out = {k: flat[o:o + n].view(sh) for k, o, sh, n in rows}
    lay = [(k, o, sh) for k, o, sh, _ in rows]
    out["nfev"], out["status"] = iflat[:nsub], iflat[nsub:]
    out["_packed"] = (flat, iflat, lay)  # not a tensor: key loops over tensors skip it
    return out


def results_to_host(out, keys=None, stream=None):
    """Host numpy copies of a fit call's results (keys None: all): one D2H
    of the packed buffer's span holding them, on the context stream (a copy
    into pageable memory waits for it).  Results without the packed layout
    (the streamed path) are copied key by key."""
    if "_packed" not in out:
        return {k: v.cpu().numpy() for k, v in out.items()
                if not k.startswith("_") and (keys is None or k in keys)}
    flat, iflat, layout = out["_packed"]
    lay = [(k, o, sh) for k, o, sh in layout if keys is None or k in keys]
    lo = min((o for _, o, _ in lay), default=0)
    hi = max((o + int(np.prod(sh)) for _, o, sh in lay), default=0)
    h = np.empty(max(hi - lo, 0))
    hi32 = np.empty(iflat.numel(), dtype=np.int32)
    with torch.cuda.stream(stream if stream is not None else torch.cuda.current_stream()):
        if hi > lo:
            torch.from_numpy(h).copy_(flat[lo:hi])
        torch.from_numpy(hi32).copy_(iflat)
    res = {k: h[o - lo:o - lo + int(np.prod(sh))].reshape(sh) for k, o, sh in lay}
    n = len(hi32) // 2
    for k, a in (("nfev", hi32[:n]), ("status", hi32[n:])):
        if keys is None or k in keys:
            res[k] = a
    return res


def results_to_host_async(out, keys, stream, side):
    """results_to_host deferred: marks the end of the fit call on `stream`
    now and returns a handle whose wait() copies the results on the `side`
    stream (behind that mark only) and returns them -- so the next call can
    be queued before this one's results are read."""
    return _PendingHost(out, keys, stream, side)


class Engine:
    """One libppfit context on one HIP device (one per process/GPU)."""

    def __init__(self, device=None, workspace_bytes=None):
        if not torch.cuda.is_available():
            raise PPFitError("no HIP device visible: libppfit has no CPU path")
        self.lib = _lib.load_library()
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", int(device))
        ctx = ctypes.c_void_p()
        rc = self.lib.ppf_ctx_create(int(device), ctypes.byref(ctx))
        if rc != 0:
            raise PPFitError("ppf_ctx_create failed (%d)" % rc)
        self.ctx = ctx
        if workspace_bytes is not None:
            self._chk(self.lib.ppf_set_workspace_limit(self.ctx, int(workspace_bytes)))
        self.bind_stream()

    # -- plumbing ----------------------------------------------------------
    def _chk(self, rc):
        if rc != 0:
            msg = self.lib.ppf_last_error(self.ctx)
            raise PPFitError("libppfit error %d: %s" % (rc, msg.decode() if msg else ""))

    def bind_stream(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        self.stream = s
        self._chk(self.lib.ppf_set_stream(self.ctx, ctypes.c_void_p(s.cuda_stream)))

    def synchronize(self):
        self._chk(self.lib.ppf_synchronize(self.ctx))

    def set_workspace_limit(self, nbytes):
        """Device workspace cap per fit call (ppf_set_workspace_limit)."""
        self._chk(self.lib.ppf_set_workspace_limit(self.ctx, int(nbytes)))

    def set_pipeline(self, pieces):
        """Pieces per chunk of the two-queue phase-family pipeline
        (ppf_set_pipeline; 0 = library default)."""
        self._chk(self.lib.ppf_set_pipeline(self.ctx, int(pieces)))

    def set_option(self, name, value):
        """Launch-schedule option of this context (ppf_set_option; names in
        _lib.OPTIONS).  No setting changes a result."""
        self._chk(self.lib.ppf_set_option(self.ctx, _lib.OPTIONS[name], int(value)))

    def get_option(self, name):
        v = ctypes.c_int32()
        self._chk(self.lib.ppf_get_option(self.ctx, _lib.OPTIONS[name], ctypes.byref(v)))
        return v.value

    def set_timing(self, on=True):
        self._chk(self.lib.ppf_set_timing(self.ctx, int(bool(on))))

    def set_trace(self, buf, cap):
        """Solver trace of the TNC / Newton-CG kernels and of the split
        trust-ncg scattering solve (ppf_set_trace): buf a float64 device
        tensor [nsub, cap, 32] or None (off)."""
        if buf is None or cap <= 0:
            self._chk(self.lib.ppf_set_trace(self.ctx, None, 0))
            self._trace = None
            return
        self._trace = buf
        self._chk(self.lib.ppf_set_trace(self.ctx, _ptr(buf), int(cap)))

    def kernel_time(self, name):
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        self._chk(self.lib.ppf_get_kernel_time(self.ctx, _lib.KERNEL_IDS[name],
                                               ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def phase_profile(self, enable):
        """k_fit_taylor phase clocks accumulated since the last call (ticks of
        wall_clock64, 100 MHz) as a list of PPF_PHASE_N ints; sets enable."""
        out = (ctypes.c_uint64 * _lib.PPF_PHASE_N)()
        self._chk(self.lib.ppf_phase_profile(self.ctx, int(bool(enable)), out))
        return list(out)

    def selftest(self):
        """Device check of the cross-lane primitives (DPP, permlane swaps);
        returns the per-test failing-lane counts (all 0 = pass)."""
        fails = (ctypes.c_int32 * _lib.PPF_SELFTEST_N)()
        self._chk(self.lib.ppf_selftest(self.ctx, fails))
        return list(fails)

    def reset_kernel_times(self):
        self._chk(self.lib.ppf_reset_kernel_times(self.ctx))

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.ppf_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- batched fit -------------------------------------------------------
    def fit_batch(self, data, model, freqs, P, init, fit_flags, nu_fit=None,
                  nu_out=None, errs=None, chan_mask=None, weights=None,
                  model_idx=None, log10_tau=False, option=0, is_toa=True,
                  guess=False, guess_Ns=100, guess_wrap=True, guess_nu=None,
                  guess_tau=None, exact=False, method="trust-ncg", bounds=None,
                  eval_only=False, guess_direct=False, spec_cache=None):
        """fit_portrait_full over a batch (pptoaslib.py:928-1096).

        data [nsub, nchan, nbin]; model [nmodel, nchan, nbin] (or [nchan, nbin]);
        freqs [nsub, nchan] or [nchan]; P [nsub] or scalar; init [nsub, 5] or [5].
        errs: time-domain sigma per channel; None or NaN entries are estimated
        on the device as get_noise_PS (pplib.py:2227-2253).
        exact=True forces the exact cross-spectrum sweeps for phase-family
        fits (default: per-channel Taylor moments, ppfit_taylor.hip).
        method: 'trust-ncg' | 'TNC' | 'Newton-CG' (pptoaslib.py:995-1014);
        bounds: 5 (low, high) pairs, None = unbounded (TNC only).
        eval_only: f, g, H and the post-fit at init, no solver step.
        guess_direct: brute-force guess grid by direct sums (no folded DFT).
        spec_cache: a SpecCache (Engine.spec_cache) for refits of the same
        subints against new templates (ppalign's iterations): its first fit
        stores the data spectra, later ones skip the data pass (ppfit.h,
        PPF_SPEC_*).  Phase-family trust-ncg fits only, with every input but
        the model the same as the first call's.
        Returns a dict of device tensors ("errs": the per-channel noise sigma
        each channel was fitted with, 0 for masked channels).
        """
        if method not in _lib.METHODS:
            raise PPFitError("Method '%s' is not implemented." % method)
        dev = self.device
        d = _dev_f64(data, dev)
        if d.dim() == 2:
            d = d.unsqueeze(0)
        nsub, nchan, nbin = d.shape
        # every host-side (numpy) input goes to the device in one pinned H2D
        # copy on the context stream; device tensors are used as they are
        st = _Stager(dev, self.stream)
        m = st.f64(model)
        fr = st.f64(freqs)
        Pt = st.f64(P)
        it, nf, no = st.rows(init), st.rows(nu_fit), st.rows(nu_out)
        er = st.f64(errs)
        mk = st.u8(chan_mask)
        wt = st.f64(weights)
        mi = st.i32(model_idx)
        gn, gt = st.rows(guess_nu), st.rows(guess_tau)
        st.run()
        m, fr, Pt, it, nf, no, er, mk, wt, mi, gn, gt = [
            st.get(x) for x in (m, fr, Pt, it, nf, no, er, mk, wt, mi, gn, gt)]
        if m.dim() == 2:
            m = m.unsqueeze(0)
        if m.shape[1:] != (nchan, nbin):
            raise PPFitError("model shape %s != (nmodel, %d, %d)" % (tuple(m.shape), nchan, nbin))
        fr = fr.reshape(-1, nchan).expand(nsub, nchan).contiguous()
        Pt = Pt.reshape(-1).expand(nsub).contiguous()
        it = _bcast_dev(it, nsub, 5, dev)
        nf = _bcast_dev(nf, nsub, 3, dev)
        no = _bcast_dev(no, nsub, 3, dev)
        er = None if er is None else er.reshape(-1, nchan).expand(nsub, nchan).contiguous()
        mk = None if mk is None else mk.reshape(-1, nchan).expand(nsub, nchan).contiguous()
        wt = None if wt is None else wt.reshape(-1, nchan).expand(nsub, nchan).contiguous()
        gn = None if guess_nu is None else _bcast_dev(gn, nsub, 1, dev).reshape(nsub).contiguous()
        gt = None if guess_tau is None else \
            _bcast_dev(gt, nsub, 1, dev, 0.0).reshape(nsub).contiguous()
        desc = _lib.FitDesc()
        desc.nsub, desc.nchan, desc.nbin, desc.nmodel = nsub, nchan, nbin, m.shape[0]
        for i in range(5):
            desc.fit_flags[i] = int(bool(fit_flags[i]))
        desc.log10_tau = int(bool(log10_tau))
        desc.option = int(option)
        desc.method = _lib.METHODS[method]
        desc.is_toa = int(bool(is_toa))
        desc.guess = int(bool(guess))
        desc.guess_Ns = int(guess_Ns)
        desc.guess_wrap = int(bool(guess_wrap))
        desc.solver_flags = ((_lib.PPF_SOLVE_EXACT if exact else 0) |
                             (_lib.PPF_SOLVE_EVAL if eval_only else 0) |
                             (_lib.PPF_GUESS_DIRECT if guess_direct else 0))
        bnd = None
        if bounds is not None:
            bnd = (ctypes.c_double * 10)(*[
                np.nan if v is None else float(v) for b in bounds for v in (list(b) + [None, None])[:2]])
        desc.bounds = ctypes.cast(bnd, ctypes.c_void_p) if bnd is not None else None
        keep = dict(d=d, m=m, fr=fr, P=Pt, it=it, nf=nf, no=no, er=er, mk=mk, wt=wt,
                    mi=mi, gn=gn, gt=gt, staged=getattr(st, "buf", None))
        desc.data, desc.model, desc.model_idx = _ptr(d), _ptr(m), _ptr(mi)
        desc.freqs, desc.errs, desc.chan_mask = _ptr(fr), _ptr(er), _ptr(mk)
        desc.weights, desc.P, desc.init = _ptr(wt), _ptr(Pt), _ptr(it)
        desc.nu_fit, desc.nu_out = _ptr(nf), _ptr(no)
        desc.guess_nu, desc.guess_tau = _ptr(gn), _ptr(gt)
        if spec_cache is not None:
            sc = spec_cache
            if (sc.nsub, sc.nchan, sc.nbin) != (nsub, nchan, nbin):
                raise PPFitError("spec_cache is for %s, data %s" % (
                    (sc.nsub, sc.nchan, sc.nbin), (nsub, nchan, nbin)))
            desc.spec_mode = _lib.PPF_SPEC_USE if sc.stored else _lib.PPF_SPEC_STORE
            desc.spec, desc.spec_sig = _ptr(sc.spec), _ptr(sc.sig)
            desc.spec_dsum, desc.spec_R = _ptr(sc.dsum), _ptr(sc.R)
            keep["spec"] = sc
        out = _result_tensors(nsub, nchan, dev)
        res = _lib.FitResult()
        for k in ["params", "param_errs", "nu_out", "cov", "scales", "scale_errs",
                  "channel_snrs", "chi2", "red_chi2", "snr", "nfev", "status",
                  "init_used", "fun", "cov_nosc", "grad", "hess"]:
            setattr(res, k, _ptr(out[k]))
        res.errs_out = _ptr(out["errs"])
        self._chk(self.lib.ppf_fit_portrait_batch(self.ctx, ctypes.byref(desc),
                                                  ctypes.byref(res)))
        if spec_cache is not None:
            spec_cache.stored = True
        out["_keep"] = keep  # inputs must outlive the stream-ordered call
        return out

    # -- other hot-path entry points ---------------------------------------
    def fit_batch_streamed(self, host_data, model, freqs, P, init, fit_flags, chunk=2048, **kw):
        """fit_batch over host-resident subints [nsub, nchan, nbin] that need
        not fit in HBM: chunk i + 1 is copied host -> device on a second
        stream while chunk i is fitted on the context stream (two device
        buffers).  host_data should be a pinned torch CPU tensor for full
        PCIe rate (an unpinned one is copied synchronously).  Per-subint
        arguments (leading dimension nsub) are sliced per chunk; results are
        those of one fit_batch call over all subints, concatenated on the
        device."""
        dev = self.device
        hd = host_data if isinstance(host_data, torch.Tensor) else torch.from_numpy(
            np.ascontiguousarray(host_data, dtype=np.float64))
        nsub, nchan, nbin = hd.shape
        chunk = max(1, min(int(chunk), nsub))
        # pageable input: each chunk is staged into one of two pinned buffers
        # on the host (a CPU copy that overlaps the previous chunk's fit),
        # then copied to the device asynchronously
        staged = not hd.is_pinned()
        pin = [torch.empty((chunk, nchan, nbin), dtype=torch.float64, pin_memory=True)
               for _ in range(2)] if staged else None

        # per-subint arguments and the ndim at which they carry a subint axis
        # (a [nchan] freqs row or a [5] init row is shared, never sliced)
        per_sub = {"freqs": 2, "P": 1, "init": 2, "nu_fit": 2, "nu_out": 2, "errs": 2,
                   "chan_mask": 2, "weights": 2, "model_idx": 1, "guess_nu": 1, "guess_tau": 1}

        def part(name, v, s0, s1):
            if v is None or isinstance(v, (int, float)):
                return v
            a = v if isinstance(v, torch.Tensor) else np.asarray(v)
            if a.ndim == per_sub[name] and a.shape[0] == nsub:
                return a[s0:s1]
            return a

        comp = self.stream
        copy = torch.cuda.Stream(dev)
        bufs = [torch.empty((chunk, nchan, nbin), dtype=torch.float64, device=dev)
                for _ in range(2)]
        copied = [torch.cuda.Event() for _ in range(2)]
        free = [torch.cuda.Event() for _ in range(2)]
        h2d_done = [None, None]
        nchunks = (nsub + chunk - 1) // chunk

        def issue(i):
            s0 = i * chunk
            n = min(chunk, nsub - s0)
            src = hd[s0:s0 + n]
            if staged:
                if h2d_done[i % 2] is not None:
                    h2d_done[i % 2].synchronize()  # the pinned buffer's last H2D finished
                pin[i % 2][:n].copy_(src)
                src = pin[i % 2][:n]
            with torch.cuda.stream(copy):
                if i >= 2:
                    copy.wait_event(free[i % 2])  # chunk i - 2 is done with the buffer
                bufs[i % 2][:n].copy_(src, non_blocking=True)
                copied[i % 2].record(copy)
                if staged:
                    h2d_done[i % 2] = torch.cuda.Event()
                    h2d_done[i % 2].record(copy)

        outs = []
        issue(0)
        for i in range(nchunks):
            s0 = i * chunk
            s1 = min(nsub, s0 + chunk)
            if i + 1 < nchunks:
                issue(i + 1)
            comp.wait_event(copied[i % 2])
            kwi = dict(kw)
            for k in per_sub:
                if k in kwi:
                    kwi[k] = part(k, kwi[k], s0, s1)
            r = self.fit_batch(bufs[i % 2][:s1 - s0], model, part("freqs", freqs, s0, s1),
                               part("P", P, s0, s1), part("init", init, s0, s1), fit_flags,
                               **kwi)
            free[i % 2].record(comp)
            outs.append(r)
        return {k: torch.cat([o[k] for o in outs]) for k in outs[0]
                if isinstance(outs[0][k], torch.Tensor) and not k.startswith("_")}

    def phase_shift_batch(self, data, model, noise=None, Ns=100, bounds=(-0.5, 0.5),
                          model_idx=None):
        """fit_phase_shift over rows (pplib.py:2054-2100) -> [nprof, 6] device tensor."""
        dev = self.device
        d = _dev_f64(data, dev)
        if d.dim() == 1:
            d = d.unsqueeze(0)
        nprof, nbin = d.shape
        m = _dev_f64(model, dev)
        if m.dim() == 1:
            m = m.unsqueeze(0)
        nz = None if noise is None else _bcast(noise, nprof, 1, dev).reshape(nprof).contiguous()
        mi = None if model_idx is None else _dev_i32(model_idx, dev)
        out = torch.empty(nprof, 6, dtype=torch.float64, device=dev)
        self._chk(self.lib.ppf_phase_shift_batch(self.ctx, nprof, nbin, _ptr(d), _ptr(m),
                                                 _ptr(mi), _ptr(nz), int(Ns),
                                                 float(bounds[0]), float(bounds[1]),
                                                 _ptr(out)))
        out._keep = (d, m, nz, mi)
        return out

    def rotate_rows(self, rows, phase, inplace=False):
        """irfft(rfft(row) e^{2 pi i k phase}) per row; inplace=True writes
        back into a contiguous float64 device tensor (each row is read whole
        into LDS before it is written)."""
        dev = self.device
        r = _dev_f64(rows, dev)
        shape = r.shape
        r = r.reshape(-1, shape[-1])
        ph = _dev_f64(phase, dev).reshape(-1).expand(r.shape[0]).contiguous()
        if inplace and not (isinstance(rows, torch.Tensor) and rows.data_ptr() == r.data_ptr()):
            raise PPFitError("rotate_rows(inplace=True) needs a contiguous float64 device tensor")
        out = r if inplace else torch.empty_like(r)
        self._chk(self.lib.ppf_rotate_rows(self.ctx, r.shape[0], r.shape[1], _ptr(r),
                                           _ptr(ph), _ptr(out)))
        out._keep = (r, ph)
        return out.reshape(shape)

    def gaussian_portraits(self, model_code, params, scattering_index, nbin, freqs, nu_ref):
        """gen_gaussian_portrait (pplib.py:853-930) on the device for every row
        of freqs ([..., nchan]); params as gen_gaussian_portrait takes them
        (TAU already in bins).  Returns a device tensor [..., nchan, nbin]."""
        dev = self.device
        f = _dev_f64(freqs, dev)
        shape = tuple(f.shape)
        f = f.reshape(-1).contiguous()
        params = np.asarray(params, dtype=np.float64)
        ngauss = (len(params) - 2) // 6
        code = (ctypes.c_int32 * 3)(*[int(c) for c in str(model_code)[:3]])
        par = (ctypes.c_double * len(params))(*params.tolist())
        out = torch.empty((f.numel(), nbin), dtype=torch.float64, device=dev)
        self._chk(self.lib.ppf_gaussian_portraits(
            self.ctx, f.numel(), nbin, ngauss, ctypes.cast(code, ctypes.c_void_p),
            ctypes.cast(par, ctypes.c_void_p), float(nu_ref), float(scattering_index), _ptr(f),
            _ptr(out)))
        out._keep = (f,)
        return out.reshape(shape + (nbin,))

    def spline_portraits(self, mean_prof, eigvec, tck, freqs, nbin=None):
        """gen_spline_portrait (pplib.py:932-956) on the device for every row
        of freqs ([..., nchan]): FITPACK splev of the projections, the
        eigenvector sum plus mean_prof, and (nbin != len(mean_prof)) the
        resample + rotate.  Returns a device tensor [..., nchan, nbin]."""
        dev = self.device
        f = _dev_f64(freqs, dev)
        shape = tuple(f.shape)
        f = f.reshape(-1).contiguous()
        mean = _dev_f64(np.asarray(mean_prof, dtype=np.float64), dev)
        nin = int(mean.numel())
        ev = np.asarray(eigvec, dtype=np.float64).reshape(nin, -1)
        neig = ev.shape[1]
        nb = nin if nbin is None else int(nbin)
        t, c, k = tck[0], tck[1], tck[2]
        if neig:
            t = np.ascontiguousarray(t, dtype=np.float64)
            c = np.ascontiguousarray(np.asarray(c, dtype=np.float64).reshape(neig, -1))
            tp, cp, nknot, ncoef = t.ctypes.data, c.ctypes.data, len(t), c.shape[1]
        else:
            tp = cp = None
            nknot = ncoef = 0
        evd = _dev_f64(ev, dev) if neig else mean
        out = torch.empty((f.numel(), nb), dtype=torch.float64, device=dev)
        self._chk(self.lib.ppf_spline_portraits(
            self.ctx, f.numel(), nin, nb, neig, _ptr(mean), _ptr(evd), nknot, int(k), tp, cp,
            ncoef, _ptr(f), _ptr(out)))
        out._keep = (f, mean, evd)
        return out.reshape(shape + (nb,))

    def _irf_call(self, nrow, nbin, rows, f, fh, DM, P, wids, irf_types, chan_bw, out):
        code = {"rect": 0, "gauss": 1}
        types = []
        for t in irf_types:
            if t not in code:
                raise ValueError("Unrecognized instrumental response function type '%s'." % t)
            types.append(code[t])
        wids = [float(w) for w in wids]
        if len(wids) != len(types):
            raise ValueError("wids and irf_types differ in length")
        if chan_bw is None:  # pptoaslib.py:174
            chan_bw = abs(fh[1] - fh[0]) if len(fh) > 1 else 0.0
        nw = len(wids)
        wa = (ctypes.c_double * max(nw, 1))(*wids)
        ta = (ctypes.c_int32 * max(nw, 1))(*types)
        self._chk(self.lib.ppf_instrumental_response_rows(
            self.ctx, nrow, nbin, _ptr(rows), nw, ctypes.cast(wa, ctypes.c_void_p),
            ctypes.cast(ta, ctypes.c_void_p), float(DM), float(chan_bw), float(P), _ptr(f),
            _ptr(out)))

    def instrumental_response_rows(self, rows, freqs, DM=0.0, P=1.0, wids=(), irf_types=(),
                                   chan_bw=None):
        """irfft(instrumental_response_port_FT * rfft(rows)) (pptoas.py:387-393)
        for rows [nrow, nbin] at freqs [nrow]; chan_bw defaults to
        |freqs[1] - freqs[0]| as pptoaslib.py:174 takes it."""
        dev = self.device
        fh = np.asarray(freqs, dtype=np.float64).reshape(-1)
        f = _dev_f64(fh, dev)
        r = _dev_f64(rows, dev)
        r2 = r.reshape(-1, r.shape[-1]).contiguous()
        out = torch.empty_like(r2)
        self._irf_call(r2.shape[0], r2.shape[1], r2, f, fh, DM, P, wids, irf_types, chan_bw, out)
        out._keep = (r2, f)
        return out.reshape(r.shape)

    def response_table(self, nbin, freqs, DM=0.0, P=1.0, wids=(), irf_types=(), chan_bw=None):
        """instrumental_response_port_FT (pptoaslib.py:145-179) as a real
        device tensor [nchan, nbin/2+1]."""
        dev = self.device
        fh = np.asarray(freqs, dtype=np.float64).reshape(-1)
        f = _dev_f64(fh, dev)
        out = torch.empty((len(fh), nbin // 2 + 1), dtype=torch.float64, device=dev)
        self._irf_call(len(fh), nbin, None, f, fh, DM, P, wids, irf_types, chan_bw, out)
        out._keep = f
        return out

    def tscrunch(self, subints, weights):
        """Weight-averaged subint (ppf_tscrunch): subints [nsub, npol, nchan,
        nbin], weights [nsub, nchan] -> ([1, npol, nchan, nbin], [1, nchan])
        device tensors."""
        dev = self.device
        d = _dev_f64(subints, dev).contiguous()
        w = _dev_f64(weights, dev).contiguous()
        nsub, npol, nchan, nbin = d.shape
        out = torch.empty((1, npol, nchan, nbin), dtype=torch.float64, device=dev)
        ws = torch.empty((1, nchan), dtype=torch.float64, device=dev)
        self._chk(self.lib.ppf_tscrunch(self.ctx, nsub, npol, nchan, nbin, _ptr(d), _ptr(w),
                                        _ptr(out), _ptr(ws)))
        out._keep = (d, w)
        return out, ws

    def remove_baseline(self, subints, weights, ntot=1, duty=0.15):
        """arch.remove_baseline() in place (ppf_remove_baseline): subints is a
        float64 device tensor [nsub, npol, nchan, nbin], weights [nsub, nchan].
        Returns the per-subint baseline window starts (int32 device tensor)."""
        d = subints
        if not (isinstance(d, torch.Tensor) and d.device == self.device and
                d.dtype == torch.float64 and d.is_contiguous() and d.dim() == 4):
            raise PPFitError("remove_baseline: need a contiguous float64 [nsub, npol, nchan, "
                             "nbin] tensor on %s" % self.device)
        nsub, npol, nchan, nbin = d.shape
        w = _dev_f64(weights, self.device).reshape(nsub, nchan).contiguous()
        width = max(1, int(duty * nbin))
        win = torch.empty(nsub, dtype=torch.int32, device=self.device)
        self._chk(self.lib.ppf_remove_baseline(self.ctx, nsub, npol, nchan, nbin, int(ntot), width,
                                               _ptr(d), _ptr(w), _ptr(win)))
        win._keep = w
        return win

    def profile_snr(self, rows, duty=0.15, threshold=0.1):
        """Profile::snr() of every row (ppf_profile_snr, PSRCHIVE's default
        phase S/N restated; parity unpinned): rows [..., nbin] -> [...]
        float64 device tensor."""
        d = _dev_f64(rows, self.device)
        shape = tuple(d.shape[:-1])
        nbin = int(d.shape[-1])
        d = d.reshape(-1, nbin).contiguous()
        out = torch.empty(d.shape[0], dtype=torch.float64, device=self.device)
        self._chk(self.lib.ppf_profile_snr(self.ctx, d.shape[0], nbin, _ptr(d),
                                           max(1, int(duty * nbin)), float(threshold), _ptr(out)))
        out._keep = d
        return out.reshape(shape)

    def irfft_rows(self, spec, nbin):
        dev = self.device
        if isinstance(spec, torch.Tensor) and spec.is_complex():
            sp = torch.view_as_real(spec.to(dev, torch.complex128).contiguous())
        else:
            sp = _dev_f64(np.stack([np.real(spec), np.imag(spec)], -1), dev)
        rows = sp.reshape(-1, nbin // 2 + 1, 2)
        out = torch.empty(rows.shape[0], nbin, dtype=torch.float64, device=dev)
        self._chk(self.lib.ppf_irfft_rows(self.ctx, rows.shape[0], nbin, _ptr(rows), _ptr(out)))
        out._keep = rows
        return out

    def noise_rows(self, rows):
        dev = self.device
        r = _dev_f64(rows, dev)
        r2 = r.reshape(-1, r.shape[-1])
        out = torch.empty(r2.shape[0], dtype=torch.float64, device=dev)
        self._chk(self.lib.ppf_noise_rows(self.ctx, r2.shape[0], r2.shape[1], _ptr(r2), _ptr(out)))
        out._keep = r2
        return out.reshape(r.shape[:-1])

    def resid_chi2_rows(self, data, phase, model, scale, errs, dof, tau=None,
                        model_row=None):
        """Per-row reduced chi2 of rotate(data, phase) - scale * scatter(model, tau)
        (ppf_resid_chi2_rows)."""
        dev = self.device
        d = _dev_f64(data, dev)
        d = d.reshape(-1, d.shape[-1])
        m = _dev_f64(model, dev)
        m = m.reshape(-1, m.shape[-1])
        nrow, nbin = d.shape
        row = lambda v: None if v is None else \
            _dev_f64(v, dev).reshape(-1).expand(nrow).contiguous()
        ph, sc, er, ta = row(phase), row(scale), row(errs), row(tau)
        mr = None if model_row is None else _dev_i32(model_row, dev)
        out = torch.empty(nrow, dtype=torch.float64, device=dev)
        self._chk(self.lib.ppf_resid_chi2_rows(self.ctx, nrow, nbin, _ptr(d), _ptr(ph), _ptr(m),
                                               _ptr(mr), _ptr(sc), _ptr(ta), _ptr(er),
                                               float(dof), _ptr(out)))
        out._keep = (d, m, ph, sc, er, ta, mr)
        return out

    def scatter_rotate_rows(self, rows, phase, tau=None):
        """irfft(rfft(rows) e^{2 pi i k phase} / (1 + 2 pi i k tau)) per row."""
        dev = self.device
        r = _dev_f64(rows, dev)
        shape = r.shape
        r = r.reshape(-1, shape[-1])
        ph = _dev_f64(phase, dev).reshape(-1).expand(r.shape[0]).contiguous()
        ta = None if tau is None else _dev_f64(tau, dev).reshape(-1).expand(r.shape[0]).contiguous()
        out = torch.empty_like(r)
        self._chk(self.lib.ppf_scatter_rotate_rows(self.ctx, r.shape[0], r.shape[1], _ptr(r),
                                                   _ptr(ph), _ptr(ta), _ptr(out)))
        out._keep = (r, ph, ta)
        return out.reshape(shape)

    def rotate_accumulate(self, data, phase, weight, accum):
        """accum [nchan, nharm, 2] (float64, device) += weighted rotated spectra."""
        dev = self.device
        d = _dev_f64(data, dev)
        nsub, nchan, nbin = d.shape
        ph = _dev_f64(phase, dev).reshape(nsub, nchan).contiguous()
        w = _dev_f64(weight, dev).reshape(nsub, nchan).contiguous()
        self._chk(self.lib.ppf_rotate_accumulate(self.ctx, nsub, nchan, nbin, _ptr(d), _ptr(ph),
                                                 _ptr(w), _ptr(accum)))
        return (d, ph, w)

    def spec_cache(self, nsub, nchan, nbin):
        """An empty data-spectrum cache for fit_batch(spec_cache=...) and
        rotate_accumulate_spec: nsub * nchan * NHP complex spectra (NHP =
        ppf_spec_nhp(nbin)) plus per-row sigma / sum |D|^2 and per-subint
        guess averages, on this engine's device."""
        return SpecCache(self, nsub, nchan, nbin)

    def rotate_accumulate_spec(self, cache, phase, weight, accum):
        """rotate_accumulate over the cached data spectra of a stored
        SpecCache (no transform): accum [nchan, nharm, 2] += weighted rotated
        spectra."""
        if not cache.stored:
            raise PPFitError("rotate_accumulate_spec: the cache holds no spectra yet")
        dev = self.device
        n, nchan, nbin = cache.nsub, cache.nchan, cache.nbin
        ph = _dev_f64(phase, dev).reshape(n, nchan).contiguous()
        w = _dev_f64(weight, dev).reshape(n, nchan).contiguous()
        self._chk(self.lib.ppf_rotate_accumulate_spec(self.ctx, n, nchan, nbin, _ptr(cache.spec),
                                                      _ptr(ph), _ptr(w), _ptr(accum)))
        return (cache, ph, w)

    def unpack_subints(self, raw, scl, offs, pmode=0, out=None):
        """PSRFITS samples to values on the device (ppf_unpack_subints):
        raw [nsub, npol, nchan, nbin] uint8 / int16 / float32 device tensor,
        scl / offs [nsub, npol, nchan] (DAT_SCL, DAT_OFFS); out [nsub, npo,
        nchan, nbin] float64, npo = 1 when pmode pscrunches."""
        rt = {torch.uint8: 1, torch.int16: 2, torch.float32: 3}[raw.dtype]
        nsub, npol, nchan, nbin = raw.shape
        npo = 1 if pmode else npol
        if out is None:
            out = torch.empty((nsub, npo, nchan, nbin), dtype=torch.float64, device=self.device)
        for t in (raw, scl, offs, out):
            if t.device != self.device or not t.is_contiguous():
                raise PPFitError("unpack_subints: contiguous tensors on %s" % self.device)
        if tuple(scl.shape) != (nsub, npol, nchan) or tuple(offs.shape) != (nsub, npol, nchan) \
                or tuple(out.shape) != (nsub, npo, nchan, nbin) or out.dtype != torch.float64 \
                or scl.dtype != torch.float64 or offs.dtype != torch.float64:
            raise PPFitError("unpack_subints: shapes / dtypes do not match raw")
        self._chk(self.lib.ppf_unpack_subints(self.ctx, nsub, npol, nchan, nbin, rt, _ptr(raw),
                                              _ptr(scl), _ptr(offs), int(pmode), _ptr(out)))
        return out

    def synth(self, model, phase, sigma, seed, sub0=0, out=None):
        """Synthetic portraits [nsub, nchan, nbin] on device (pplib.py:3342-3377 math)."""
        dev = self.device
        m = _dev_f64(model, dev)
        nchan, nbin = m.shape
        ph = _dev_f64(phase, dev)
        nsub = ph.numel() // nchan
        ph = ph.reshape(nsub, nchan).contiguous()
        if out is None:
            out = torch.empty(nsub, nchan, nbin, dtype=torch.float64, device=dev)
        self._chk(self.lib.ppf_synth_portraits(self.ctx, nsub, nchan, nbin, _ptr(m), _ptr(ph),
                                               float(sigma), int(seed) & (2 ** 64 - 1),
                                               int(sub0), _ptr(out)))
        out._keep = (m, ph)
        return out


def _on_engine_stream(fn):
    """Run an Engine call with its stream current: the temporaries it makes
    (device copies of host arguments, outputs) are then allocated for the
    stream its kernels run on, so the caching allocator cannot hand their
    memory to other work while those kernels may still use it (an engine
    bound to a side stream, e.g. a second context generating data beside the
    fits).  A no-op when the engine's stream is already current."""
    @functools.wraps(fn)
    def run(self, *args, **kw):
        if torch.cuda.current_stream(self.device) == self.stream:
            return fn(self, *args, **kw)
        with torch.cuda.stream(self.stream):
            return fn(self, *args, **kw)
    return run


for _name in ("fit_batch", "phase_shift_batch", "rotate_rows", "gaussian_portraits",
              "spline_portraits", "instrumental_response_rows", "response_table", "tscrunch",
              "remove_baseline", "profile_snr", "irfft_rows", "noise_rows", "resid_chi2_rows",
              "scatter_rotate_rows", "rotate_accumulate", "spec_cache", "rotate_accumulate_spec",
              "synth"):
    setattr(Engine, _name, _on_engine_stream(getattr(Engine, _name)))
del _name

_engines = {}


class _PendingHost:
    """Results of one fit call on their way to the host.  An event marks
    the end of the call on the context stream; wait() copies the needed
    span of the packed result buffer into fresh host memory on a side
    stream that waits for that event only, so later calls queued behind it
    keep running while the caller reads these results."""

    def __init__(self, out, keys, stream, side):
        self.flat, self.iflat, layout = out["_packed"]
        self.lay = [(k, o, sh) for k, o, sh in layout if keys is None or k in keys]
        self.keys, self.side = keys, side
        self.event = torch.cuda.Event()
        self.event.record(stream)

    def wait(self):
        lo = min((o for _, o, _ in self.lay), default=0)
        hi = max((o + int(np.prod(sh)) for _, o, sh in self.lay), default=0)
        h = np.empty(max(hi - lo, 0))
        hi32 = np.empty(self.iflat.numel(), dtype=np.int32)
        with torch.cuda.stream(self.side):
            self.side.wait_event(self.event)
            if hi > lo:
                torch.from_numpy(h).copy_(self.flat[lo:hi])
            torch.from_numpy(hi32).copy_(self.iflat)
        self.side.synchronize()
        res = {k: h[o - lo:o - lo + int(np.prod(sh))].reshape(sh) for k, o, sh in self.lay}
        n = len(hi32) // 2
        for k, a in (("nfev", hi32[:n]), ("status", hi32[n:])):
            if self.keys is None or k in self.keys:
                res[k] = a
        return res


class FitPipeline:
    """Batched fits submitted one piece at a time, run in submission order on
    the context stream, with each piece's results collected while later
    pieces still run -- so the caller's host work on piece i (get_TOAs' TOA
    records and .tim text) overlaps the device work of pieces i+1, ...

    Host-resident pieces (numpy or CPU tensors) are staged through two
    pinned buffers and copied to two device buffers on a second stream, the
    copy of piece i+1 overlapping the fit of piece i (as fit_batch_streamed).
    submit(tag, data, model, ...) takes fit_batch's arguments; collect()
    returns (tag, results as host numpy) in submission order."""

    def __init__(self, eng, keys=None):
        self.eng, self.keys = eng, keys
        self.pending = collections.deque()
        self.copy = self.side = None
        self.slots = [None, None]  # (pinned, device buffer, h2d event, free event)
        self.models = {}
        self.k = 0

    def __len__(self):
        return len(self.pending)

    def _stage(self, host):
        """Host piece -> device tensor, through slot k % 2."""
        eng = self.eng
        hd = host if isinstance(host, torch.Tensor) else torch.from_numpy(
            np.ascontiguousarray(host, dtype=np.float64))
        hd = hd.to(torch.float64)
        n = hd.numel()
        i = self.k % 2
        self.k += 1
        if self.copy is None:
            self.copy = torch.cuda.Stream(eng.device)
        slot = self.slots[i]
        if slot is None or slot[1].numel() < n:
            if slot is not None:  # in-flight users of the old buffers first
                for ev in slot[2:]:
                    if ev is not None:
                        ev.synchronize()
            slot = [None, torch.empty(n, dtype=torch.float64, device=eng.device), None, None]
            self.slots[i] = slot
        if hd.is_pinned():
            src = hd.reshape(-1)
        else:
            if slot[2] is not None:
                slot[2].synchronize()  # the pinned buffer's previous H2D is done
            if slot[0] is None or slot[0].numel() < n:
                slot[0] = torch.empty(n, dtype=torch.float64, pin_memory=True)
            slot[0][:n].copy_(hd.reshape(-1))
            src = slot[0][:n]
        dbuf, free = slot[1], slot[3]
        with torch.cuda.stream(self.copy):
            if free is not None:
                self.copy.wait_event(free)  # the fit that read the device buffer is done
            dbuf[:n].copy_(src, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy)
        slot[2] = ev
        eng.stream.wait_event(ev)
        return dbuf[:n].view(hd.shape), i

    def submit(self, tag, data, model, freqs, P, init, fit_flags, **kw):
        if isinstance(model, np.ndarray):  # one device copy per template array
            hit = self.models.get(id(model))
            if hit is None or hit[0] is not model:
                hit = self.models[id(model)] = (model, _dev_f64(model, self.eng.device))
            model = hit[1]
        slot = None
        if not isinstance(data, torch.Tensor) or data.device.type == "cpu":
            data, slot = self._stage(data)
        out = self.eng.fit_batch(data, model, freqs, P, init, fit_flags, **kw)
        if slot is not None:
            ev = torch.cuda.Event()
            ev.record(self.eng.stream)
            self.slots[slot][3] = ev
        if self.side is None:
            self.side = torch.cuda.Stream(self.eng.device)
        self.pending.append((tag, out, _PendingHost(out, self.keys, self.eng.stream, self.side)))

    def collect(self):
        tag, out, ph = self.pending.popleft()
        return tag, ph.wait()


class SpecCache:
    """Device arrays of the data-spectrum cache (ppfit.h, PPF_SPEC_*):
    spec [nsub, nchan, NHP, 2], sig / dsum [nsub, nchan], R [nsub, NHP, 2].
    stored: a fit has filled it (later fits read it)."""

    def __init__(self, eng, nsub, nchan, nbin):
        nhp = int(eng.lib.ppf_spec_nhp(int(nbin)))
        if nhp <= 0:
            raise PPFitError("nbin=%d: outside [16, 8192]" % nbin)
        f64 = dict(dtype=torch.float64, device=eng.device)
        self.nsub, self.nchan, self.nbin, self.nhp = int(nsub), int(nchan), int(nbin), nhp
        self.spec = torch.empty((nsub, nchan, nhp, 2), **f64)
        self.sig = torch.empty((nsub, nchan), **f64)
        self.dsum = torch.empty((nsub, nchan), **f64)
        self.R = torch.empty((nsub, nhp, 2), **f64)
        self.stored = False

    @property
    def nbytes(self):
        return sum(t.numel() * 8 for t in (self.spec, self.sig, self.dsum, self.R))

    @staticmethod
    def bytes_for(eng, nsub, nchan, nbin):
        """What __init__ allocates for this shape (NHP from the library, so
        the estimate follows its row padding)."""
        nhp = int(eng.lib.ppf_spec_nhp(int(nbin)))
        return (nsub * nchan * nhp + nsub * nhp) * 16 + 2 * nsub * nchan * 8


def get_engine(device=None):
    """Process-wide engine per device."""
    if device is None:
        device = torch.cuda.current_device() if torch.cuda.is_available() else 0
    key = int(device)
    if key not in _engines:
        _engines[key] = Engine(key)
    return _engines[key]
