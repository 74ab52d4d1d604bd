#!/usr/bin/env python3
"""Replay the device TNC and Newton-CG trajectories through their scalar
models (tools/tnc_model.py, tools/ncg_model.py: scipy restated, held to scipy
point for point by tests/test_tnc_model.py / test_ncg_model.py).

For every TNC / Newton-CG fixture case the device solver runs with its
solver trace on (ppf_set_trace: every objective sweep's point, f, gradient
and Hessian); the model is then driven by those same f/g/H values for as
long as it asks for the points the device visited.  If the model asks for a
point the device did not visit, that evaluation is the first divergent
iterate (the model then continues on device evaluations, PPF_SOLVE_EVAL).
A faithful device solver gives no divergence: the same points, nfev and
status as its model fed the same numbers -- what remains against the
reference is the reference's own sensitivity to the last bits of f
(tests/golden/tnc_floor.npz).

usage: solver_replay.py [out.json]    (GPU; writes a JSON summary)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def device_fit(eng, case, method, cap=512):
    import torch
    buf = torch.full((1, cap, 32), float("nan"), dtype=torch.float64, device=eng.device)
    eng.set_trace(buf, cap)
    try:
        out = eng.fit_batch(case["data"], case["model"], case["freqs"], case["P"], case["init"],
                            case["flags"], nu_fit=[case["nu"]] * 3, errs=case["errs"],
                            log10_tau=case["log10"], option=case["option"], method=method,
                            bounds=case.get("bounds"))
        torch.cuda.synchronize()
    finally:
        eng.set_trace(None, 0)
    rec = buf[0].cpu().numpy()
    n = int(np.sum(~np.isnan(rec[:, 27])))
    res = {k: v.cpu().numpy()[0] for k, v in out.items() if not k.startswith("_")}
    return res, rec[:n]


def device_eval(eng, case, x):
    out = eng.fit_batch(case["data"], case["model"], case["freqs"], case["P"], list(x),
                        case["flags"], nu_fit=[case["nu"]] * 3, errs=case["errs"],
                        log10_tau=case["log10"], option=case["option"], exact=True,
                        eval_only=True)
    f = float(out["fun"][0])
    g = out["grad"][0].cpu().numpy()
    H = out["hess"][0].cpu().numpy()
    return f, g, H


class Replay:
    """f/g(/H) from the device trace while the model follows it."""

    def __init__(self, rec, n, fallback, counted_only=False):
        self.rec = rec[rec[:, 26] == 1.0] if counted_only else rec
        self.n = n
        self.i = 0
        self.div = None
        self.fallback = fallback
        self.asked = 0

    def __call__(self, x):
        x = np.asarray(x, dtype=float)
        self.asked += 1
        if self.div is None and self.i < len(self.rec) and \
                np.array_equal(x[:self.n], self.rec[self.i, :self.n]):
            r = self.rec[self.i]
            self.i += 1
            return r[5], r[6:11][:self.n].copy(), _hess(r)
        if self.div is None:
            want = self.rec[self.i, :5].tolist() if self.i < len(self.rec) else None
            self.div = dict(index=self.i, model_point=x.tolist(), device_point=want)
        f, g, H = self.fallback(x)
        return f, g[:self.n], H


def _hess(r):
    from_pairs = np.zeros((5, 5))
    k = 11
    for i in range(5):
        for j in range(i, 5):
            from_pairs[i, j] = from_pairs[j, i] = r[k]
            k += 1
    return from_pairs


def tnc_cases(z, legacy):
    from tests.golden_consts import P0
    cases = []
    if legacy:
        for ic in range(int(z["ncase"])):
            k = "l%d_" % ic
            cases.append(dict(name="legacy l%d" % ic, data=z[k + "data"], model=z[k + "model"],
                              freqs=z[k + "freqs"], P=P0, errs=z[k + "errs"],
                              init=list(z[k + "init"]) + [0.0, 0.0, 0.0],
                              nu=float(z[k + "nu_fit"]), flags=[1, 1, 0, 0, 0], log10=False,
                              option=0, bounds=[(None, None)] * 5, n=2,
                              ref_status=int(z[k + "return_code"]),
                              ref_nfev=int(z[k + "nfeval"])))
        return cases
    for ic in range(int(z["ncase"])):
        k = "f%d_" % ic
        meth = str(z[k + "method"])
        if meth not in ("TNC", "Newton-CG"):
            continue
        b = z[k + "bounds"]
        cases.append(dict(name="f%d %s" % (ic, meth), method=meth, data=z[k + "data"],
                          model=z[k + "model"], freqs=z[k + "freqs"], P=float(z["P"]),
                          errs=z[k + "errs"], init=list(z[k + "init"]),
                          nu=float(z[k + "nu_fit"]), flags=[int(v) for v in z[k + "flags"]],
                          log10=bool(z[k + "log10"]), option=int(z[k + "option"]),
                          bounds=[tuple(None if np.isnan(v) else float(v) for v in row)
                                  for row in b], n=5,
                          ref_status=int(z[k + "return_code"]), ref_nfev=int(z[k + "nfeval"])))
    return cases


def run_tnc(eng, case, legacy):
    from tools import tnc_model as TM
    n = case["n"]
    res, rec = device_fit(eng, case, "TNC-legacy" if legacy else "TNC")
    rp = Replay(rec, n, lambda x: device_eval(eng, case, list(x) + [0.0] * (5 - len(x))))
    # minfev (pptoaslib.py:1005-1007) exactly as the device formed it: trace
    # record 0, field 29 (0 for the legacy fit, which passes none)
    kw = dict(xtol=1e-10, fmin=float(rec[0, 29]) if len(rec) else 0.0)
    m = TM.minimize_tnc(lambda x: rp(x)[:2], case["init"][:n],
                        case["bounds"][:n] if not legacy else None, **kw)
    return dict(case=case["name"], device_status=int(res["status"]), device_nfev=int(res["nfev"]),
                model_status=int(m["status"]), model_nfev=int(m["nfev"]),
                reference_status=case["ref_status"], reference_nfev=case["ref_nfev"],
                device_sweeps=len(rec), replayed=rp.i, divergence=rp.div,
                same_end=bool(np.array_equal(np.asarray(m["x"])[:n], res["params"][:n])))


def run_ncg(eng, case):
    from tools import ncg_model as NM
    res, rec = device_fit(eng, case, "Newton-CG")
    rp = Replay(rec, 5, lambda x: device_eval(eng, case, x))
    x, f, nfev, status = NM.newton_cg(lambda x: rp(x), case["init"])
    return dict(case=case["name"], device_status=int(res["status"]), device_nfev=int(res["nfev"]),
                model_status=int(status), model_nfev=int(nfev),
                reference_status=case["ref_status"], reference_nfev=case["ref_nfev"],
                device_sweeps=len(rec), replayed=rp.i, divergence=rp.div,
                same_end=bool(np.array_equal(np.asarray(x), res["params"])))


def main():
    from pulseportraiture_amd.engine import get_engine
    eng = get_engine(0)
    g = os.path.join(ROOT, "tests", "golden")
    z = np.load(os.path.join(g, "fit_full_r2.npz"))
    zl = np.load(os.path.join(g, "legacy_fit_portrait.npz"))
    out = []
    for case in tnc_cases(z, False):
        r = run_tnc(eng, case, False) if case["method"] == "TNC" else run_ncg(eng, case)
        print(json.dumps(r), flush=True)
        out.append(r)
    for case in tnc_cases(zl, True):
        r = run_tnc(eng, case, True)
        print(json.dumps(r), flush=True)
        out.append(r)
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
