#!/usr/bin/env python3
"""Config-1-shaped golden fixture: the reference's own GetTOAs.get_TOAs over
5 archives x 10 subints x 64 chan x 512 bin, phase+DM (BASELINE.json
configs[0], the examples/example.py plumbing run: example.gmodel template,
pptoas phase+DM fit).

TEST INFRASTRUCTURE ONLY -- run in the build container, never on the GPU box.
The reference is loaded through the SURVEY.md §8(c) shim (make_golden.py);
the subints are regenerated from Philox seeds on both sides
(synth.make_workload, seed = CFG1_SEED + archive index), and only numbers go
into tests/golden/config1.npz / config1.json.  One archive has a zapped
channel in two subints and one fully zapped subint (weights 0).

Usage:  python tests/golden/make_golden_cfg1.py
"""
import contextlib
import io
import json
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import make_golden as MG  # noqa: E402
import make_golden_r2 as M2  # noqa: E402

CFG1 = dict(narch=5, nsub=10, nchan=64, nbin=512, seed=1001)


def zap_weights(ia, nsub, nchan):
    """Archive 2: channel 9 zapped in subints 3 and 4, subint 7 fully zapped."""
    w = np.ones((nsub, nchan))
    if ia == 2:
        w[3, 9] = w[4, 9] = 0.0
        w[7] = 0.0
    return w


def main():
    np.seterr(all="ignore")
    tmp, pplib, pptoaslib, pptoas, _ = MG.load_reference()
    narch, nsub, nchan, nbin, seed = (CFG1[k] for k in ["narch", "nsub", "nchan", "nbin",
                                                         "seed"])
    archives = {}
    for ia in range(narch):
        name = "cfg1_%d.fits" % ia
        db = M2.synth_archive(pplib, name, nsub, nchan, nbin, seed + ia, 0.0, 0.0)
        w = zap_weights(ia, nsub, nchan)
        wn = np.where(w == 0.0, 0.0, 1.0)
        db["weights"] = w
        db["ok_isubs"] = np.compress(wn.mean(axis=1), range(nsub))
        db["ok_ichans"] = [np.compress(wn[i], range(nchan)) for i in range(nsub)]
        db["masks"] = np.einsum("j,ikl", np.ones(1), np.einsum("ij,k", wn, np.ones(nbin)))
        archives[name] = db
    pptoas.load_data = lambda filename, **kw: archives[filename]
    pptoas.file_is_type = lambda f, t: False
    tmpd = tempfile.mkdtemp()
    shutil.copy(MG.GMODEL, os.path.join(tmpd, "example.gmodel"))
    cwd = os.getcwd()
    os.chdir(tmpd)
    out, meta = {}, {"cfg": CFG1, "archives": sorted(archives)}
    try:
        gt = M2.quiet_call(pptoas.GetTOAs, "cfg1_0.fits", "example.gmodel", quiet=True)
        gt.datafiles = sorted(archives)
        M2.quiet_call(gt.get_TOAs, quiet=True)
        lines = []
        for toa in gt.TOA_list:
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                pplib.write_TOAs(toa, outfile=None)
            lines.append(buf.getvalue().strip())
        meta["tim"] = lines
        for ia in range(len(gt.phis)):
            p = "a%d_" % ia
            for attr in ["phis", "phi_errs", "DMs", "DM_errs", "snrs", "red_chi2s", "rcs",
                         "nfevals", "scales"]:
                out[p + attr] = np.asarray(gt.__dict__[attr][ia], dtype=float)
            out[p + "ok_isubs"] = np.asarray(gt.ok_isubs[ia])
            out[p + "nu_fits"] = np.array(gt.nu_fits[ia], dtype=float)
            out[p + "DeltaDM"] = np.array([gt.DeltaDM_means[ia], gt.DeltaDM_errs[ia]])
            out[p + "noise_stds"] = archives["cfg1_%d.fits" % ia].noise_stds
        print("config 1: %d TOAs" % len(lines))
    finally:
        os.chdir(cwd)
        shutil.rmtree(tmp, ignore_errors=True)
    MG.save("config1.npz", **out)
    with open(os.path.join(HERE, "config1.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
