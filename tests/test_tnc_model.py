"""tools/tnc_model.py -- the specification of the device TNC (ppfit_tnc.hip) --
against scipy's compiled TNC (scipy.optimize._moduleTNC, tnc.c).

The model must visit exactly the same points as scipy (every objective
evaluation, bitwise) and return the same status and nfev on the objectives
PulsePortraiture minimizes with TNC: the legacy phase+DM fit (pplib.py:2102,
n = 2) and fit_portrait_full with get_TOAs' bounds and minfev
(pptoaslib.py:1005-1007, n = 5, including a fit that runs into maxfun), plus
generic quadratic / Rosenbrock problems with and without bounds.

It also records why device-vs-reference TNC statuses are compared as a set:
scipy's own status for a converged fit flips between FCONVERGED (1) and
LSFAIL (4) when the start moves by a few ulps.
"""
import os
import sys
import warnings

import numpy as np
import pytest
from scipy.optimize import minimize

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ppfit_oracle as O  # noqa: E402
from tests.golden_consts import P0  # noqa: E402
from tools import tnc_model as TM  # noqa: E402


def scipy_points(fg, x0, bounds=None, **opts):
    pts = []

    def fun(x):
        pts.append(np.array(x, copy=True))
        return fg(x)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        r = minimize(fun, x0, jac=True, method="TNC", bounds=bounds, options=opts)
    return r, pts


def rosen(x):
    x = np.asarray(x)
    f = np.sum(100 * (x[1:] - x[:-1] ** 2) ** 2 + (1 - x[:-1]) ** 2)
    g = np.zeros_like(x)
    g[:-1] += -400 * x[:-1] * (x[1:] - x[:-1] ** 2) - 2 * (1 - x[:-1])
    g[1:] += 200 * (x[1:] - x[:-1] ** 2)
    return f, g


def quad(x):
    x = np.asarray(x)
    A = np.diag(np.arange(1, len(x) + 1.0))
    A[0, 1] = A[1, 0] = 0.3
    return 0.5 * x @ A @ x - x.sum(), A @ x - 1


def legacy_problem(golden, ic):
    g = golden("legacy_fit_portrait.npz")
    k = "l%d_" % ic
    data, model = g[k + "data"], g[k + "model"]
    dFT = np.fft.rfft(data, axis=1)
    dFT[:, 0] = 0
    mFT = np.fft.rfft(model, axis=1)
    mFT[:, 0] = 0
    e = g[k + "errs"] * np.sqrt(data.shape[1] / 2.0)
    p_n = np.real(np.sum(mFT * np.conj(mFT), axis=1))
    args = (mFT, p_n, dFT, e, P0, g[k + "freqs"], float(g[k + "nu_fit"]))
    return (lambda x: (O.legacy_function(x, *args), O.legacy_deriv(x, *args)),
            list(g[k + "init"]), None, dict(xtol=1e-10))


def full_problem(golden, ic):
    f = golden("fit_full_r2.npz")
    k = "f%d_" % ic
    data, model = f[k + "data"], f[k + "model"]
    nbin = data.shape[1]
    nu = float(f[k + "nu_fit"])
    dFT = np.fft.rfft(data, axis=-1)
    dFT[:, 0] = 0
    mFT = np.fft.rfft(model, axis=-1)
    mFT[:, 0] = 0
    e = f[k + "errs"] * np.sqrt(nbin / 2.0)
    flags = [bool(v) for v in f[k + "flags"]]
    args = (dFT, mFT, e, P0, f[k + "freqs"], nu, nu, nu, flags, bool(f[k + "log10"]))
    bounds = [tuple(None if np.isnan(v) else float(v) for v in row) for row in f[k + "bounds"]]
    Sd = np.sum((np.abs(dFT) ** 2).T / e ** 2)
    dof = data.size - (sum(flags) + len(f[k + "freqs"]))
    return (lambda x: (O.fit_function(x, *args), O.fit_function_deriv(x, *args)),
            list(f[k + "init"]), bounds, dict(xtol=1e-10, minfev=dof - Sd))


def assert_same_trajectory(fg, x0, bounds, opts):
    r, pts = scipy_points(fg, x0, bounds, **opts)
    kw = dict(xtol=opts.get("xtol", -1.0), fmin=opts.get("minfev", 0.0))
    m = TM.minimize_tnc(fg, x0, bounds, **kw)
    assert m["status"] == r.status and m["nfev"] == r.nfev, (m["status"], r.status, m["nfev"],
                                                             r.nfev)
    assert len(m["points"]) == len(pts)
    for a, b in zip(m["points"], pts):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(m["x"], r.x)


@pytest.mark.parametrize("name", ["legacy0", "legacy1", "full6", "full7", "full8", "full9"])
def test_model_matches_scipy_on_pulseportraiture(golden, name):
    if name.startswith("legacy"):
        prob = legacy_problem(golden, int(name[-1]))
    else:
        prob = full_problem(golden, int(name[4:]))
    assert_same_trajectory(*prob)


@pytest.mark.parametrize("case", [
    ("quad", [3.0, -2.0], None), ("quad", [3.0, -2.0, 1, 4, 0.5], None),
    ("rosen", [-1.2, 1.0], None), ("rosen", [-1.2, 1.0], [(-2, 0.5), (None, 2)]),
    ("quad", [3.0, -2.0, 1, 4, 0.5],
     [(None, None), (0, None), (None, 0.1), (-1, 1), (None, None)])])
def test_model_matches_scipy_generic(case):
    name, x0, bounds = case
    assert_same_trajectory({"quad": quad, "rosen": rosen}[name], x0, bounds, {})


def test_scipy_tnc_status_is_rounding_sensitive(golden):
    """FCONVERGED vs LSFAIL at the end of a converged TNC fit is decided by the
    last bits: the same problem restarted a few ulps away ends both ways."""
    fg, x0, bounds, opts = full_problem(golden, 6)
    seen = set()
    for k in range(8):
        x = list(x0)
        x[0] += k * np.spacing(x[0]) * (1 if k % 2 else -1)
        r, _ = scipy_points(fg, x, bounds, **opts)
        seen.add(int(r.status))
    assert seen == {1, 4}, seen
