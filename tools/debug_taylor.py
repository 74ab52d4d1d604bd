"""Debug: Taylor vs exact device fits on one synthetic batch (prints per subint)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import ppfit_oracle as O
from pulseportraiture_amd import synth
from pulseportraiture_amd.engine import Engine

nsub, nchan, nbin = (int(a) for a in sys.argv[1:4])
seed = int(sys.argv[4]) if len(sys.argv) > 4 else 100 + nbin
eng = Engine(0)
w = synth.make_workload(nsub, nchan, nbin, seed=seed)
data = synth.workload_data_host(w)
nu = O.guess_fit_freq(w.freqs)
init = np.array([[0.0, w.DM0, 0, 0, 0]] * nsub)
res = {}
for name, ex in [("taylor", False), ("exact", True)]:
    o = eng.fit_batch(data, w.model, w.freqs, w.P, init, [1, 1, 0, 0, 0], nu_fit=[nu] * 3,
                      guess=True, exact=ex)
    res[name] = {k: v.cpu().numpy() for k, v in o.items() if not k.startswith("_")}
t, e = res["taylor"], res["exact"]
for i in range(nsub):
    print(i, "nfev", t["nfev"][i], e["nfev"][i], "st", t["status"][i], e["status"][i],
          "dphi/sig %.2e dDM/sig %.2e" % ((t["params"][i, 0] - e["params"][i, 0]) / e["param_errs"][i, 0],
                                          (t["params"][i, 1] - e["params"][i, 1]) / e["param_errs"][i, 1]),
          "fun %.17g %.17g" % (t["fun"][i], e["fun"][i]), "init", t["init_used"][i, 0], e["init_used"][i, 0])
