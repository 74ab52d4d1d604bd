"""Kernel times on the headline batch for the library named by PPF_LIB
(timing experiments: PPF_XP builds; results downstream of a crippled variant
are meaningless, only the kernel clock is read)."""
import os
import sys

import torch

sys.path.insert(0, ".")
from pulseportraiture_amd import synth, pplib  # noqa: E402
from pulseportraiture_amd.engine import Engine  # noqa: E402

nsub = 10000
eng = Engine(0)
dev = eng.device
w = synth.make_workload(nsub, 64, 2048, seed=20240917)
data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
model = torch.as_tensor(w.model, device=dev)
freqs = torch.as_tensor(w.freqs, device=dev)
P = torch.full((nsub,), w.P, dtype=torch.float64, device=dev)
nu = torch.full((nsub, 3), pplib.guess_fit_freq(w.freqs), dtype=torch.float64, device=dev)
init0 = torch.tensor([[0.0, w.DM0, 0.0, 0.0, 0.0]] * nsub, dtype=torch.float64, device=dev)
args = (data, model, freqs, P, init0, [1, 1, 0, 0, 0])
eng.fit_batch(*args, nu_fit=nu, guess=True, guess_Ns=100)
torch.cuda.synchronize()
eng.set_timing(True)
eng.reset_kernel_times()
for _ in range(3):
    eng.fit_batch(*args, nu_fit=nu, guess=True, guess_Ns=100)
torch.cuda.synchronize()
print(os.environ.get("PPF_LIB", "default"),
      " ".join("%s %.3f" % (k, eng.kernel_time(k)[0] / 3)
               for k in ["data_xspec", "guess", "moments", "fit_taylor", "post"]))
