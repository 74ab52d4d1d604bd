#!/usr/bin/env python3
"""Round-3 golden fixtures from the reference PulsePortraiture source.

TEST INFRASTRUCTURE ONLY -- run in the build container, never on the GPU box
and never by the product.  The reference is loaded through the SURVEY.md
§8(c) shim exactly as in make_golden.py; only numbers (and the bytes of the
model files handed to it) are written into tests/golden/.

Two further Python-2 semantics are supplied at run time for the template
readers: text reads of a model file are byte-transparent (latin-1, as a
Python-2 ``open(f, "r")`` on a pickled model), and ``pickle.load`` takes
Python-2 strings as latin-1.  With them the reference's own get_TOAs falls
back from read_model to read_spline_model on a ppspline model
(pptoas.py:375-378) exactly as under Python 2.

Fixtures (templates_r3.npz / templates_r3.json):
  spl_*        gen_spline_portrait (pplib.py:932-956) for ppspline-style
               models (PCA eigenvectors of the example.gmodel portrait, the
               projections fitted by si.splprep): same nbin, upsampled,
               downsampled, degree 1 and 5, no eigenvectors (tiled mean),
               frequencies outside the knot span (ext=0 extrapolation)
  irf_*        instrumental_response_port_FT (pptoaslib.py:145-179): rect
               and gauss widths, with and without the DM smearing term
  gt_*         GetTOAs.get_TOAs with a spline model (same nbin and
               resampled) and with add_instrumental_response (rect + gauss
               widths and DM smearing): per-subint arrays and .tim lines

Usage:  python tests/golden/make_golden_r3.py
"""
import builtins
import contextlib
import io
import json
import os
import pickle
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import make_golden as MG  # noqa: E402
import make_golden_r2 as MG2  # noqa: E402
from pulseportraiture_amd import synth  # noqa: E402

# ppspline-style models: (name, nchan of the PCA portrait, nbin, neig, k)
SPLINE_MODELS = [("m3", 48, 512, 3, 3), ("m5", 40, 256, 2, 5), ("m1", 32, 512, 2, 1),
                 ("m0", 32, 512, 0, 3)]


def make_spline_model(name, nchan, nbin, neig, k):
    """mean profile, eigenvectors and splprep tck of the example.gmodel
    portrait, as ppspline.make_spline_model forms them (ppspline.py:82-146)."""
    import scipy.interpolate as si
    w = synth.make_workload(1, nchan, nbin, seed=3)
    port = w.model
    mean_prof = port.mean(axis=0)
    delta = port - mean_prof
    if neig == 0:
        return mean_prof, np.zeros((nbin, 0)), [np.array([]), np.array([]), 0], w.freqs
    u, s, vt = np.linalg.svd(delta, full_matrices=False)
    eigvec = np.ascontiguousarray(vt[:neig].T)
    proj = delta @ eigvec
    smooth = 1e-6 * nchan * np.sum(proj ** 2) / nchan
    (tck, _), fp, ier, msg = si.splprep(proj.T, u=w.freqs, k=k, s=smooth, full_output=1,
                                        quiet=1)
    tck = [np.asarray(tck[0]), [np.asarray(c) for c in tck[1]], int(tck[2])]
    return mean_prof, eigvec, tck, w.freqs


def spline_file_bytes(name, mean_prof, eigvec, tck):
    # the list ppspline.write_model pickles (ppspline.py:221-226)
    return pickle.dumps([name + ".spl", "J1234-5678", "synthetic.fits", mean_prof, eigvec,
                         tck], protocol=2)


def py2_io(pplib):
    """Python-2 file semantics the template readers rely on."""
    def open2(f, mode="r", *a, **k):
        if "b" not in mode:
            k.setdefault("encoding", "latin-1")
        return builtins.open(f, mode, *a, **k)

    class pickle2:
        @staticmethod
        def load(f):
            return pickle.load(f, encoding="latin1")

        dump = staticmethod(pickle.dump)
    pplib.open = open2
    pplib.pickle = pickle2


def gen_spline(pplib, out, meta):
    for name, nchan, nbin, neig, k in SPLINE_MODELS:
        mean_prof, eigvec, tck, freqs = make_spline_model(name, nchan, nbin, neig, k)
        raw = spline_file_bytes(name, mean_prof, eigvec, tck)
        path = os.path.join(tempfile.mkdtemp(), name + ".spl")
        open(path, "wb").write(raw)
        out["spl_%s_file" % name] = np.frombuffer(raw, dtype=np.uint8)
        # frequencies: the PCA channels, a Doppler-shifted set, and points
        # beyond the knot span (ext=0 extrapolates)
        cases = [("same", freqs, nbin), ("dopp", freqs * 1.0003, nbin),
                 ("wide", np.linspace(freqs[0] - 60.0, freqs[-1] + 45.0, 24), nbin),
                 ("up", freqs, 2 * nbin), ("down", freqs, nbin // 2)]
        meta[name] = dict(nchan=nchan, nbin=nbin, neig=neig, k=k, cases=[c[0] for c in cases])
        for tag, f, nb in cases:
            mname, port = pplib.read_spline_model(path, f, nb, quiet=True)
            out["spl_%s_%s_freqs" % (name, tag)] = f
            out["spl_%s_%s_nbin" % (name, tag)] = np.array(nb)
            out["spl_%s_%s_port" % (name, tag)] = port
        print("spline %s: neig %d k %d, max %.4g" % (name, neig, k, np.abs(port).max()))


IRF_CASES = [  # tag, nbin, nchan, DM, P, wids, irf_types
    ("rect", 512, 16, 0.0, MG.P0, [0.004], ["rect"]),
    ("gauss", 1024, 8, 0.0, MG.P0, [0.01], ["gauss"]),
    ("both_dm", 2048, 32, 10.0, MG.P0, [0.003, 0.02], ["rect", "gauss"]),
    ("dm", 256, 64, 1.0, 0.0015, [], []),
]


def gen_irf(pptoaslib, out, meta):
    for tag, nbin, nchan, DM, P, wids, types in IRF_CASES:
        f = MG.channel_freqs(nchan)
        R = pptoaslib.instrumental_response_port_FT(nbin, f, DM, P, wids, types)
        out["irf_%s" % tag] = np.asarray(R)
        out["irf_%s_freqs" % tag] = f
        meta["irf_" + tag] = dict(nbin=nbin, DM=DM, P=P, wids=wids, irf_types=types)
        print("irf %s: %s, min %.3g, max |imag| %.3g" % (tag, R.shape, np.min(R.real),
                                                          np.max(np.abs(np.imag(R)))))


GT_ARCH = ("splA.fits", 4, 32, 512, 8101)  # name, nsub, nchan, nbin, seed
GT_CASES = [  # tag, model, get_TOAs kwargs, instrumental response dict
    ("spline", "m3.spl", {}, None),
    ("spline_up", "m5.spl", {}, None),
    ("irf", "example.gmodel", {}, {"DM": 5.0, "wids": [0.004, 0.01], "irf_types": ["rect",
                                                                               "gauss"]}),
    ("irf_dmonly", "example.gmodel", dict(fit_GM=True), {"DM": 1.0, "wids": [],
                                                         "irf_types": []}),
]


def gen_get_toas(pplib, pptoas, out, meta):
    name, nsub, nchan, nbin, seed = GT_ARCH
    db = MG2.synth_archive(pplib, name, nsub, nchan, nbin, seed, 0.0, 0.0)
    pptoas.load_data = lambda filename, **kw: db
    pptoas.file_is_type = lambda f, t: False
    tmpd = tempfile.mkdtemp()
    shutil.copy(MG.GMODEL, os.path.join(tmpd, "example.gmodel"))
    for mname, _, _, _, _ in SPLINE_MODELS:
        open(os.path.join(tmpd, mname + ".spl"), "wb").write(
            bytes(out["spl_%s_file" % mname]))
    cwd = os.getcwd()
    os.chdir(tmpd)
    meta["gt_archive"] = dict(name=name, nsub=nsub, nchan=nchan, nbin=nbin, seed=seed)
    try:
        for tag, model, kw, ird in GT_CASES:
            gt = MG2.quiet_call(pptoas.GetTOAs, name, model, quiet=True)
            if ird is not None:
                gt.ird = gt.instrumental_response_dict = dict(ird)
                kw = dict(kw, add_instrumental_response=True)
            MG2.quiet_call(gt.get_TOAs, quiet=True, **kw)
            lines = []
            for toa in gt.TOA_list:
                buf = io.StringIO()
                with contextlib.redirect_stdout(buf):
                    pplib.write_TOAs(toa, outfile=None)
                lines.append(buf.getvalue().strip())
            meta["gt_" + tag] = dict(model=model, kwargs=kw, ird=ird, tim=lines)
            p = "gt_%s_" % tag
            for attr in ["phis", "phi_errs", "DMs", "DM_errs", "GMs", "GM_errs", "snrs",
                         "red_chi2s", "rcs", "scales"]:
                out[p + attr] = np.asarray(getattr(gt, attr)[0], dtype=float)
            print("get_TOAs %s: %d TOAs, rcs %s" % (tag, len(lines), gt.rcs[0]))
    finally:
        os.chdir(cwd)


def main():
    np.seterr(all="ignore")
    tmp, pplib, pptoaslib, pptoas, ppalign = MG.load_reference()
    py2_io(pplib)
    out, meta = {}, {}
    try:
        gen_spline(pplib, out, meta)
        gen_irf(pptoaslib, out, meta)
        gen_get_toas(pplib, pptoas, out, meta)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    MG.save("templates_r3.npz", **out)
    with open(os.path.join(HERE, "templates_r3.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
