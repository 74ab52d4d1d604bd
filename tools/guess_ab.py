"""A/B of the single-wave guess (k_guess_w) against the block guess: run the
headline batch (and a masked / scattering-guess variant) and save init_used
and the fitted params; run once with PPF_GUESS_WAVE=0 and once without, then
compare the two files bitwise.  usage: guess_ab.py OUT.npz | guess_ab.py A.npz B.npz"""
import sys

import numpy as np

if len(sys.argv) == 3:
    a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
    bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
    print("bitwise equal" if not bad else "DIFFER: %s" % bad)
    sys.exit(1 if bad else 0)

import torch  # noqa: E402

sys.path.insert(0, ".")
from pulseportraiture_amd import pplib, synth  # noqa: E402
from pulseportraiture_amd.engine import Engine  # noqa: E402

eng = Engine(0)
dev = eng.device
out = {}
for tag, nsub, nchan, nbin, mask_some in [("hl", 4000, 64, 2048, False), ("mk", 500, 64, 2048, True),
                                          ("sm", 800, 32, 512, False)]:
    w = synth.make_workload(nsub, nchan, nbin, seed=4242)
    data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
    nu = np.full((nsub, 3), pplib.guess_fit_freq(w.freqs))
    mask = np.ones((nsub, nchan), np.uint8)
    if mask_some:
        mask[::3, 5] = 0  # a third of the subints take the block guess
    init = np.array([[0.0, w.DM0, 0.0, 0.0, 0.0]] * nsub)
    r = eng.fit_batch(data, w.model, w.freqs, w.P, init, [1, 1, 0, 0, 0], nu_fit=nu,
                      chan_mask=mask, guess=True, guess_Ns=100)
    torch.cuda.synchronize()
    for k in ["init_used", "params", "param_errs", "status", "nfev"]:
        out[tag + "_" + k] = r[k].cpu().numpy()
np.savez(sys.argv[1], **out)
print("wrote", sys.argv[1])
