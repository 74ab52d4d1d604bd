"""The drop-in drivers at world size 2 on CPU (gloo): GetTOAs.get_TOAs shards
its (archive, subint) units over ranks and gathers the results; ppalign
shards its units and all-reduces the Fourier-domain portrait sum.

The device calls are replaced at their boundaries by deterministic CPU
stand-ins -- pptoas.fit_pipeline / ppalign.fit_portraits_batch (one result per subint that
depends only on that subint's inputs) and, for ppalign, an engine whose
rotate_accumulate / irfft_rows are numpy (rfft * phasor, irfft).  What is
checked is the N > 1 bookkeeping: every unit is fitted on exactly one rank,
and every rank ends with exactly the single-process TOAs / template.
"""
import os
import socket
import tempfile

import numpy as np
import torch
import torch.multiprocessing as mp
from pulseportraiture_amd.pptoaslib import SyncPipeline  # noqa: E402

DM0 = 34.56789
P0 = 1.0 / 345.67890123456789


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def fake_fit(data, model, init, P, freqs, nu_fits=None, nu_outs=None, errs=None,
             fit_flags=(1, 1, 0, 0, 0), chan_mask=None, **kw):
    """Per-subint deterministic stand-in for fit_portraits_batch's results."""
    data = np.asarray(data)
    nsub, nchan, nbin = data.shape
    s = data.reshape(nsub, -1)
    a = s.sum(1)
    b = (s ** 2).sum(1)
    params = np.stack([0.01 * np.tanh(a), DM0 + 1e-4 * np.tanh(b / s.shape[1] - 1.0),
                       np.zeros(nsub), np.zeros(nsub), np.zeros(nsub)], 1)
    params = params * np.asarray(fit_flags, float) + np.asarray(init) * (1 - np.asarray(fit_flags))
    errs5 = np.tile([1e-4, 2e-4, 0.0, 0.0, 0.0], (nsub, 1)) * np.asarray(fit_flags, float)
    nu = np.asarray(nu_fits, float).reshape(nsub, 3)
    sc = 1.0 + 0.01 * np.abs(data).mean(axis=2)
    if chan_mask is not None:
        sc = sc * np.asarray(chan_mask)
    if kw.get("log_calls") is not None:
        kw["log_calls"].append(nsub)
    cov = np.zeros((nsub, 5, 5))
    cov[:, 0, 0], cov[:, 1, 1], cov[:, 0, 1] = 1e-8, 4e-8, 1e-9
    # the sigma each channel is fitted with: errs, get_noise_PS where NaN, 0 masked
    e = np.full((nsub, nchan), np.nan) if errs is None else \
        np.array(np.broadcast_to(np.asarray(errs, float), (nsub, nchan)))
    if np.isnan(e).any():
        from oracle import ppfit_oracle as O
        ps = O.get_noise_PS(data.reshape(-1, nbin), chans=True).reshape(nsub, nchan)
        e = np.where(np.isnan(e), ps, e)
    if chan_mask is not None:
        e = np.where(np.asarray(chan_mask) > 0, e, 0.0)
    return dict(params=params, param_errs=errs5, nu_out=nu.copy(), cov=cov, scales=sc, errs=e,
                scale_errs=0.1 * sc, channel_snrs=10 * sc, chi2=b, red_chi2=b / (nchan * nbin),
                snr=np.sqrt(b), nfev=np.full(nsub, 5, np.int32), status=np.full(nsub, 2, np.int32),
                duration=np.zeros(nsub))


def make_archives():
    from pulseportraiture_amd import archive, synth
    from pulseportraiture_amd.mjd import MJD
    names = []
    for i, (nsub, nchan) in enumerate([(5, 8), (3, 8), (4, 8)]):
        w = synth.make_workload(nsub, nchan, 64, seed=50 + i)
        data = synth.workload_data_host(w)
        wts = np.ones((nsub, nchan))
        wts[1, 2] = 0.0
        name = "dist%d.npz" % i
        archive.register_archive(name, dict(
            subints=data[:, None], freqs=w.freqs, Ps=np.full(nsub, w.P), weights=wts,
            noise_stds=np.full((nsub, 1, nchan), 1.5),
            epochs=[MJD(57000.0 + 0.01 * k) for k in range(nsub)], DM=DM0, backend="be",
            frontend="fe", telescope="GBT", telescope_code="1"))
        names.append(name)
    return names


def run_get_toas(log, reads=None, gather_to="root"):
    from pulseportraiture_amd import archive, pplib, pptoas, synth
    names = make_archives()
    if reads is not None:  # every subint range a rank reads (pptoas.py:246,343 sharded)
        orig = archive._Registered.read

        def read(self, lo, hi):
            reads.append((self.base.filename, lo, hi))
            return orig(self, lo, hi)
        archive._Registered.read = read

    def fit(*a, **k):
        k["log_calls"] = log
        return fake_fit(*a, **k)
    pptoas.fit_pipeline = lambda keys: SyncPipeline(fit, keys)
    # templates: the host restatement in place of the device generator
    pptoas.gen_gaussian_portraits_device = lambda code, params, alpha, nbin, freqs, nu_ref: \
        np.array([pplib.gen_gaussian_portrait(code, params, alpha, pplib.get_bin_centers(nbin), f,
                                              nu_ref) for f in np.atleast_2d(freqs)])
    gt = pptoas.GetTOAs(names, synth.EXAMPLE_GMODEL, quiet=True)
    gt.gather_to = gather_to
    gt.get_TOAs(quiet=True)
    # write_TOAs' bulk text first (no TOA object built yet), then the objects
    with tempfile.NamedTemporaryFile("r", suffix=".tim") as f:
        pplib.write_TOAs(gt.TOA_list, outfile=f.name, append=False)
        gt.bulk_lines = f.read().splitlines()
    return [pplib.toa_line(t) for t in gt.TOA_list], gt


def _toas_worker(rank, world, port, out_dir, gather_to):
    from pulseportraiture_amd.toas import _as_bytes
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        log, reads = [], []
        lines, gt = run_get_toas(log, reads, gather_to)
        subs = sorted((n, k) for n, lo, hi in reads for k in range(lo, hi))
        own = gt.shard_blocks  # the TOA records this rank built for its own shard
        np.savez(os.path.join(out_dir, "toas%d.npz" % rank), lines=np.array(lines),
                 bulk=np.array(gt.bulk_lines), nfit=sum(log), DeltaDM=np.array(gt.DeltaDM_means),
                 read=np.array(["%s:%d" % x for x in subs]),
                 own_rows=sum(b.n for b in own),
                 own_subints=np.concatenate([[c.values for c in b.cols if c.key == "subint"][0]
                                             for b in own]),
                 own_text=np.array([_as_bytes(b.text[1]).decode() for b in own]))
    finally:
        torch.distributed.destroy_process_group()


import pytest  # noqa: E402


@pytest.mark.parametrize("gather_to", ["root", "all"])
def test_get_toas_sharded_ws2_equals_single_process(gather_to):
    log = []
    ref_lines, gt = run_get_toas(log)
    assert sum(log) == 12  # every ok subint once
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_toas_worker, args=(2, _free_port(), d, gather_to), nprocs=2, join=True)
        r = [np.load(os.path.join(d, "toas%d.npz" % k)) for k in range(2)]
    assert int(r[0]["nfit"]) + int(r[1]["nfit"]) == 12  # disjoint shards cover all units
    assert int(r[0]["nfit"]) == 6 and int(r[1]["nfit"]) == 6
    # each rank read only the subints of its own shard: disjoint, covering all
    # 12 ok subints (archive 0's masked subint 1 sits inside rank 0's range)
    r0, r1 = set(r[0]["read"]), set(r[1]["read"])
    assert not (r0 & r1) and len(r0) + len(r1) <= 13 and len(r0 | r1) >= 12
    # gather_to "root": rank 0 assembles every TOA in the reference's order and
    # the other ranks hold none; "all": every rank holds them
    holders = r if gather_to == "all" else r[:1]
    assert gt.bulk_lines == ref_lines  # native .tim writer == per-TOA text
    for rk in holders:
        assert list(rk["lines"]) == ref_lines
        assert list(rk["bulk"]) == ref_lines
        np.testing.assert_array_equal(rk["DeltaDM"], np.array(gt.DeltaDM_means))
    if gather_to == "root":
        assert len(r[1]["lines"]) == 0 and len(r[1]["DeltaDM"]) == 0
    # every rank built its own shard's TOA records and .tim text: rank 1 the
    # last 6 ok units (archive 1's subint 2, archive 2's 4 subints ... in
    # unit order), and that text is exactly rank 0's lines for those units
    assert int(r[0]["own_rows"]) == 6 and int(r[1]["own_rows"]) == 6
    own = "".join(r[0]["own_text"]) + "".join(r[1]["own_text"])
    assert own.splitlines() == ref_lines
    assert "".join(r[1]["own_text"]).splitlines() == ref_lines[6:]


# ---------------------------------------------------------------------------
# ppalign: sharded fit + rotate-accumulate + all-reduce + divide
# ---------------------------------------------------------------------------
class NumpyEngine:
    """CPU stand-in for the engine calls align_archives makes."""
    device = torch.device("cpu")

    def rotate_accumulate(self, data, phase, weight, accum):
        d = np.asarray(data)
        k = np.arange(d.shape[-1] // 2 + 1)
        spec = np.fft.rfft(d, axis=-1) * np.exp(2j * np.pi * np.asarray(phase)[..., None] * k)
        s = np.sum(np.asarray(weight)[..., None] * spec, axis=0)
        accum += torch.as_tensor(np.stack([s.real, s.imag], -1))

    def irfft_rows(self, spec, nbin):
        return torch.as_tensor(np.fft.irfft(spec.numpy(), nbin, axis=-1))

    def noise_rows(self, rows):
        from oracle import ppfit_oracle as O
        return torch.as_tensor(O.get_noise_PS(np.asarray(rows), chans=True))


def run_align():
    from pulseportraiture_amd import archive, engine, ppalign, synth
    names = make_archives()
    engine.get_engine = lambda device=None: NumpyEngine()
    ppalign.fit_portraits_batch = fake_fit
    w = synth.make_workload(1, 8, 64, seed=50)
    # dmc=1: the registered guess is what load_data(dedisperse=True) returns
    archive.register_archive("dist_guess.npz", dict(subints=w.model[None, None], freqs=w.freqs,
                                                    Ps=[w.P], epochs=[(57000, 0, 0.0)], DM=DM0,
                                                    dmc=1))
    return ppalign.align_archives(names, "dist_guess.npz", fit_dm=True, niter=2, quiet=True)


def _align_worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        np.save(os.path.join(out_dir, "align%d.npy" % rank), run_align())
    finally:
        torch.distributed.destroy_process_group()


def test_align_archives_sharded_ws2_equals_single_process():
    ref = run_align()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_align_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        got = [np.load(os.path.join(d, "align%d.npy" % k)) for k in range(2)]
    for g in got:
        np.testing.assert_allclose(g, ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())
    assert np.array_equal(got[0], got[1])
