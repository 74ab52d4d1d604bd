"""Diagnostic: device fit vs golden fit_full cases (prints, no asserts)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from pulseportraiture_amd.engine import Engine

f = np.load("tests/golden/fit_full.npz")
eng = Engine(0)
for ic in range(int(f["ncase"])):
    k = "f%d_" % ic
    nu = float(f[k + "nu_fit"])
    out = eng.fit_batch(f[k + "data"], f[k + "model"], f[k + "freqs"], float(f["P"]),
                        f[k + "init"], list(f[k + "flags"]), nu_fit=[nu, nu, nu],
                        errs=f[k + "errs"], log10_tau=bool(f[k + "log10"]))
    r = {kk: v.cpu().numpy()[0] for kk, v in out.items() if not kk.startswith("_")}
    print("case", ic, "flags", f[k + "flags"], "log10", bool(f[k + "log10"]))
    print("  params ", r["params"])
    print("  golden ", [float(f[k + n]) for n in ["phi", "DM", "GM", "tau", "alpha"]])
    print("  nu_out ", r["nu_out"], " golden", [float(f[k + n]) for n in ["nu_DM", "nu_GM", "nu_tau"]])
    print("  status", r["status"], "nfev", r["nfev"], "golden", int(f[k + "return_code"]), int(f[k + "nfeval"]))
    print("  chi2", r["chi2"], "golden", float(f[k + "chi2"]), "fun", r["fun"], "init", r["init_used"])
    print("  errs", r["param_errs"], "golden", [float(f[k + n + "_err"]) for n in ["phi", "DM", "GM", "tau", "alpha"]])
