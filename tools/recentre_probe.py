"""Taylor recentres per subint (k_fit_taylor's phase-profile counter [8]: one
more moment pass over the subint's X each) at the headline (64 ch), config 4
(128 ch, phase+DM+GM) and config 5 (256 ch, ppalign's guess grid) shapes, and
the X bytes they add over the first moment pass.
  python tools/recentre_probe.py [nsub]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pulseportraiture_amd import synth, pplib  # noqa: E402
from pulseportraiture_amd.engine import get_engine  # noqa: E402

CASES = [("headline", 64, 2048, [1, 1, 0, 0, 0], 100), ("gm", 128, 2048, [1, 1, 1, 0, 0], 100),
         ("ppalign", 256, 2048, [1, 1, 0, 0, 0], 2048)]


def main():
    nsub = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    eng = get_engine(0)
    dev = eng.device
    for name, nchan, nbin, flags, ns in CASES:
        w = synth.make_workload(nsub, nchan, nbin, seed=20240917)
        data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
        nu = pplib.guess_fit_freq(w.freqs)
        init = np.tile([0.0, w.DM0, 0.0, 0.0, 0.0], (nsub, 1))
        kw = dict(nu_fit=[nu] * 3, guess=True, guess_Ns=ns)
        if name == "ppalign":
            kw.update(guess_wrap=False, guess_nu=nu)
        eng.fit_batch(data, w.model, w.freqs, w.P, init, flags, **kw)
        torch.cuda.synchronize()
        eng.phase_profile(True)
        out = eng.fit_batch(data, w.model, w.freqs, w.P, init, flags, **kw)
        torch.cuda.synchronize()
        c = eng.phase_profile(False)
        nfev = out["nfev"].cpu().numpy()
        print("%-9s %3d ch: recentres %d over %d subints = %.3f per subint (X read %.3fx the "
              "first pass); evaluations [9] %d; mean nfev %.3f" % (
                  name, nchan, c[8], nsub, c[8] / nsub, 1 + c[8] / nsub, c[9], nfev.mean()),
              flush=True)
        del data


if __name__ == "__main__":
    main()
