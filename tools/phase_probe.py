"""Attribute k_fit_taylor time to its phases by re-running the headline batch
with parts of the work removed (guess off with the guess's own start point;
start at the converged point).  Prints per-kernel ms for each variant."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pulseportraiture_amd import synth, pplib  # noqa: E402
from pulseportraiture_amd.engine import Engine  # noqa: E402

nsub = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
nchan, nbin = 64, 2048
eng = Engine(0)
if "sep" in sys.argv[2:]:  # the first moment pass in its own launch (k_moments)
    eng.set_option("fuse_moments", 0)
dev = eng.device
w = synth.make_workload(nsub, nchan, nbin, seed=20240917)
data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
model = torch.as_tensor(w.model, device=dev)
freqs = torch.as_tensor(w.freqs, device=dev)
P = torch.full((nsub,), w.P, dtype=torch.float64, device=dev)
nu = torch.full((nsub, 3), pplib.guess_fit_freq(w.freqs), dtype=torch.float64, device=dev)
init0 = torch.tensor([[0.0, w.DM0, 0.0, 0.0, 0.0]] * nsub, dtype=torch.float64, device=dev)
flags = [1, 1, 0, 0, 0]
names = ["data_xspec", "guess", "moments", "fit_taylor", "solve", "post", "model_fft"]


def run(init, guess, reps=3):
    out = eng.fit_batch(data, model, freqs, P, init, flags, nu_fit=nu, guess=guess, guess_Ns=100)
    torch.cuda.synchronize()
    eng.set_timing(True)
    eng.reset_kernel_times()
    for _ in range(reps):
        out = eng.fit_batch(data, model, freqs, P, init, flags, nu_fit=nu, guess=guess,
                            guess_Ns=100)
    torch.cuda.synchronize()
    kt = {k: eng.kernel_time(k)[0] / reps for k in names}
    eng.set_timing(False)
    return out, kt


base, kt = run(init0, True)
print("guess+fit      ", {k: round(v, 3) for k, v in kt.items()},
      "mean nfev", float(base["nfev"].double().mean()))
init_g = base["init_used"].clone()
o2, kt = run(init_g, False)
print("fit from guess ", {k: round(v, 3) for k, v in kt.items()},
      "mean nfev", float(o2["nfev"].double().mean()))
# converged point at nu_fit: params are at nu_out = nu_fit here (nu_out NaN -> nu_zero);
# use the fit's final x via a second fit from the first one's output
fin = torch.zeros_like(init0)
fin[:, 0] = base["params"][:, 0]
fin[:, 1] = base["params"][:, 1]
o3, kt = run(fin, False)
print("fit from final ", {k: round(v, 3) for k, v in kt.items()},
      "mean nfev", float(o3["nfev"].double().mean()))

# in-kernel phase clocks of k_fit_taylor (ppf_phase_profile), headline run
eng.phase_profile(True)
o4 = eng.fit_batch(data, model, freqs, P, init0, flags, nu_fit=nu, guess=True, guess_Ns=100)
torch.cuda.synchronize()
pt = eng.phase_profile(False)
nwg = max(pt[9], 1)
print("phase clocks per workgroup (us):",
      {n: round(pt[i] / nwg / 100.0, 2) for i, n in
       enumerate(["moment pass (fused)", "meta+T0", "centre", "sweep", "trstep"])},
      "recentres/subint", pt[8] / nwg, "workgroups", pt[9],
      "guess set-up+brute / NM us", round(pt[10] / nwg / 100.0, 2), round(pt[11] / nwg / 100.0, 2),
      "(of which set-up + fold sums %.2f, set-up + rm %.2f)" % (pt[26] / nwg / 100.0, pt[27] / nwg / 100.0), "NM calls", pt[12] / nwg)

# the fused kernel with one objective sweep and no solver steps (eval_only):
# the moment pass + meta + one sweep, i.e. the streaming part alone
eng.set_timing(True)
eng.reset_kernel_times()
for _ in range(3):
    eng.fit_batch(data, model, freqs, P, init0, flags, nu_fit=nu, guess=True, guess_Ns=100,
                  eval_only=True)
torch.cuda.synchronize()
print("eval_only      ", {k: round(eng.kernel_time(k)[0] / 3, 3) for k in names})
eng.set_timing(False)
