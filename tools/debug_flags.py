"""Debug: Taylor vs exact on test_taylor_matches_exact_flags' batch."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import ppfit_oracle as O
from pulseportraiture_amd import synth
from pulseportraiture_amd.engine import Engine

flags = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "10000")]
eng = Engine(0)
w = synth.make_workload(5, 32, 512, seed=7, gm=2e-6)
data = synth.workload_data_host(w)
nu = O.guess_fit_freq(w.freqs)
init = np.array([[0.0, w.DM0, 0, 0, 0]] * 5)
res = {}
for name, ex in [("taylor", False), ("exact", True)]:
    if not ex:
        eng.phase_profile(True)
    o = eng.fit_batch(data, w.model, w.freqs, w.P, init, flags, nu_fit=[nu] * 3, guess=True, exact=ex)
    res[name] = {k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")}
    if not ex:
        print("phase clocks", eng.phase_profile(False)[:10])
t, e = res["taylor"], res["exact"]
for i in range(5):
    print(i, "nfev", t["nfev"][i], e["nfev"][i], "st", t["status"][i], e["status"][i],
          "phi %.15g %.15g err %.3g" % (t["params"][i, 0], e["params"][i, 0], e["param_errs"][i, 0]),
          "fun %.17g %.17g" % (t["fun"][i], e["fun"][i]), "init", t["init_used"][i, 0], e["init_used"][i, 0])
