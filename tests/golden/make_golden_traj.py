#!/usr/bin/env python3
"""Solver trajectories of the reference's TNC and Newton-CG fits.

TEST INFRASTRUCTURE ONLY -- run in the build container, never on the GPU box
and never by the product.  The reference is loaded through the SURVEY.md
§8(c) shim exactly as in make_golden.py; only numbers are written.

For every TNC / Newton-CG case of fit_full_r2.npz (pptoaslib.py:995-1014)
and legacy_fit_portrait.npz (pplib.py:2140-2148) the reference fit is run
again with its objective wrapped: each call of fit_portrait_full_function
(or pplib.fit_portrait_function) appends the point and the value, in call
order.  The GPU tests hold the device solver's own evaluation sequence
(ppf_set_trace) to this one: the same points up to the evaluation at which
the reference's f changes by no more than its own rounding (where a one-ulp
difference in f decides the next step), and the same end state.

Fixture solver_traj_r3.npz: <case>_x [nfev, 5], <case>_f [nfev] for
cases f6..f10 (fit_full_r2.npz) and l0, l1 (legacy).

Usage:  python tests/golden/make_golden_traj.py
"""
import contextlib
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import make_golden as MG  # noqa: E402


def recorder(fn, rec, npar):
    def wrapped(params, *args):
        f = fn(params, *args)
        x = np.zeros(5)
        x[:npar] = np.asarray(params, dtype=float)[:npar]
        rec.append((x, float(f)))
        return f
    return wrapped


def main():
    import warnings
    warnings.simplefilter("ignore")
    _, pplib, pptoaslib, _, _ = MG.load_reference()
    out = {}
    f = np.load(os.path.join(HERE, "fit_full_r2.npz"))
    orig = pptoaslib.fit_portrait_full_function
    for ic in range(int(f["ncase"])):
        k = "f%d_" % ic
        meth = str(f[k + "method"])
        if meth not in ("TNC", "Newton-CG"):
            continue
        rec = []
        pptoaslib.fit_portrait_full_function = recorder(orig, rec, 5)
        nu = float(f[k + "nu_fit"])
        bounds = [tuple(None if np.isnan(v) else float(v) for v in row) for row in f[k + "bounds"]]
        with contextlib.redirect_stdout(io.StringIO()):
            r = pptoaslib.fit_portrait_full(
                f[k + "data"], f[k + "model"], list(f[k + "init"]), MG.P0, f[k + "freqs"],
                [nu] * 3, [None] * 3, f[k + "errs"], [int(v) for v in f[k + "flags"]], bounds,
                bool(f[k + "log10"]), option=int(f[k + "option"]), method=meth)
        pptoaslib.fit_portrait_full_function = orig
        # the same fit as the fixture's (bitwise: same inputs, same code)
        assert int(r.nfeval) == int(f[k + "nfeval"]) and np.array_equal(
            np.asarray(r.params, float), f[k + "params"]), ic
        out["f%d_x" % ic] = np.array([x for x, _ in rec])
        out["f%d_f" % ic] = np.array([v for _, v in rec])
        print("f%d %s: %d objective calls, nfev %d" % (ic, meth, len(rec), r.nfeval))
    g = np.load(os.path.join(HERE, "legacy_fit_portrait.npz"))
    orig = pplib.fit_portrait_function
    for ic in range(int(g["ncase"])):
        k = "l%d_" % ic
        rec = []
        pplib.fit_portrait_function = recorder(orig, rec, 2)
        with contextlib.redirect_stdout(io.StringIO()):
            r = pplib.fit_portrait(g[k + "data"], g[k + "model"], g[k + "init"], MG.P0,
                                   g[k + "freqs"], float(g[k + "nu_fit"]), None, g[k + "errs"])
        pplib.fit_portrait_function = orig
        assert int(r.nfeval) == int(g[k + "nfeval"]) and r.phase == float(g[k + "phase"]), ic
        out["l%d_x" % ic] = np.array([x for x, _ in rec])
        out["l%d_f" % ic] = np.array([v for _, v in rec])
        print("l%d legacy TNC: %d objective calls, nfev %d" % (ic, len(rec), r.nfeval))
    MG.save("solver_traj_r3.npz", **out)


if __name__ == "__main__":
    main()
