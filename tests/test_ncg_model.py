"""tools/ncg_model.py (the scalar restatement ppfit_ncg.hip follows) against
scipy's own Newton-CG on the oracle objective, as fit_portrait_full calls it
(pptoaslib.py:1003-1004).  The model's dot products are sequential where
numpy's go through BLAS, so trajectories agree to rounding: same status,
parameters within 1e-6 sigma (the fixture's errors), nfev within a few."""
import os
import sys
import warnings

import numpy as np
import pytest
import scipy.optimize as opt

from oracle import ppfit_oracle as O
from tests.conftest import GOLDEN

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools"))
import ncg_model as M  # noqa: E402


def _args(z, k, data=None):
    data = z[k + "data"] if data is None else data
    nbin = data.shape[-1]
    dFT = np.fft.rfft(data, axis=-1)
    dFT[:, 0] = 0.0
    mFT = np.fft.rfft(z[k + "model"], axis=-1)
    mFT[:, 0] = 0.0
    errs_FT = np.asarray(z[k + "errs"]) * np.sqrt(nbin / 2.0)
    nu = float(z[k + "nu_fit"])
    flags = [bool(f) for f in z[k + "flags"]]
    return (dFT, mFT, errs_FT, float(z["P"]), z[k + "freqs"], nu, nu, nu, flags,
            bool(z[k + "log10"]))


def _fgh(args):
    def fgh(x):
        x = np.asarray(x, dtype=float)
        return (float(O.fit_function(x, *args)), list(O.fit_function_deriv(x, *args)),
                [list(r) for r in O.fit_function_2deriv(x, *args)])
    return fgh


@pytest.mark.parametrize("shift", [0.0, 0.002, -0.004])
def test_model_matches_scipy_newton_cg(shift):
    z = np.load(os.path.join(GOLDEN, "fit_full_r2.npz"))
    k = "f10_"
    args = _args(z, k)
    x0 = np.array(z[k + "init"], dtype=float)
    x0[0] += shift
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        ref = opt.minimize(O.fit_function, x0, args=args, method="Newton-CG",
                           jac=O.fit_function_deriv, hess=O.fit_function_2deriv,
                           options={"maxiter": 2000, "disp": False, "xtol": -1})
    x, f, nfev, status = M.newton_cg(_fgh(args), list(x0))
    assert status == ref.status
    err = z[k + "param_errs"]
    assert abs(x[0] - ref.x[0]) <= 1e-6 * err[0]
    assert abs(x[1] - ref.x[1]) <= 1e-6 * err[1]
    assert abs(nfev - ref.nfev) <= 6, (nfev, ref.nfev)


def test_model_golden_newton_cg():
    """The reference's own Newton-CG result (fit_full_r2.npz case f10) from the
    fixture's init: status 2 and the fitted phase / DM at nu_fit."""
    z = np.load(os.path.join(GOLDEN, "fit_full_r2.npz"))
    k = "f10_"
    args = _args(z, k)
    x, f, nfev, status = M.newton_cg(_fgh(args), list(np.array(z[k + "init"], float)))
    assert status == int(z[k + "return_code"])
    ref = O.fit_portrait_full(z[k + "data"], z[k + "model"], list(z[k + "init"]), float(z["P"]),
                              z[k + "freqs"], [float(z[k + "nu_fit"])] * 3, [None] * 3,
                              z[k + "errs"], list(z[k + "flags"]), log10_tau=False,
                              method="Newton-CG")
    assert ref.return_code == status
    assert abs(ref.DM - x[1]) <= 1e-6 * ref.DM_err
