#!/usr/bin/env python3
"""Device TNC / Newton-CG evaluation sequences against the reference's
(tests/golden/solver_traj_r3.npz, make_golden_traj.py).

Per case and evaluation i: the largest |x_dev - x_ref| over the fitted
parameters in units of the reference's parameter errors, |f_dev - f_ref| /
|f_ref|, and the reference's own step |f_ref[i] - f_ref[i-1]| / |f_ref| (how
close the solver is to its rounding floor there).

usage: traj_compare.py [out.json]    (GPU)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    from pulseportraiture_amd.engine import get_engine
    import solver_replay as SR
    eng = get_engine(0)
    g = os.path.join(ROOT, "tests", "golden")
    tr = np.load(os.path.join(g, "solver_traj_r3.npz"))
    z = np.load(os.path.join(g, "fit_full_r2.npz"))
    zl = np.load(os.path.join(g, "legacy_fit_portrait.npz"))
    out = []
    for legacy, src in ((False, z), (True, zl)):
        for case in SR.tnc_cases(src, legacy):
            tag = case["name"].split()[1] if legacy else case["name"].split()[0]
            meth = "TNC-legacy" if legacy else case["method"]
            res, rec = SR.device_fit(eng, case, meth)
            recc = rec[rec[:, 26] == 1.0]
            xr, fr = tr[tag + "_x"], tr[tag + "_f"]
            if legacy:
                sig = np.array([float(src[tag + "_phase_err"]), float(src[tag + "_DM_err"]), 1, 1, 1])
                fl = np.array([1, 1, 0, 0, 0])
            else:
                sig = np.array([float(src[tag + "_" + k + "_err"]) for k in
                                ["phi", "DM", "GM", "tau", "alpha"]])
                fl = np.array(case["flags"])
            sig = np.where(sig > 0, sig, 1.0)
            n = min(len(recc), len(xr))
            rows = []
            for i in range(n):
                dx = np.abs(recc[i, :5] - xr[i]) / sig * fl
                step = abs(fr[i] - fr[i - 1]) / abs(fr[i]) if i else np.nan
                rows.append(dict(i=i, dx_sigma=float(dx.max()),
                                 df_rel=float(abs(recc[i, 5] - fr[i]) / abs(fr[i])),
                                 ref_step_rel=float(step)))
            first = next((r["i"] for r in rows if r["dx_sigma"] > 1e-9), None)
            d = dict(case=tag, method=meth, device_nfev=int(res["nfev"]), ref_nfev=len(xr),
                     device_status=int(res["status"]), counted=len(recc),
                     first_divergent=first, rows=rows)
            print(json.dumps({k: v for k, v in d.items() if k != "rows"}), flush=True)
            for r in rows:
                print("   %3d dx %.3e sigma  df %.3e  ref step %.3e" % (
                    r["i"], r["dx_sigma"], r["df_rel"], r["ref_step_rel"]))
            out.append(d)
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
