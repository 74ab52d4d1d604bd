"""In-kernel phase clocks of k_fit_taylor and k_post on the headline batch
(ppf_phase_profile, wall_clock64 ticks at 100 MHz), per workgroup in us."""
import sys

import torch

sys.path.insert(0, ".")
from pulseportraiture_amd import synth, pplib  # noqa: E402
from pulseportraiture_amd.engine import Engine  # noqa: E402

nsub = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
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
eng.phase_profile(True)
eng.fit_batch(*args, nu_fit=nu, guess=True, guess_Ns=100)
torch.cuda.synchronize()
pt = eng.phase_profile(False)
nwg = max(pt[9], 1)
us = lambda v, n: round(v / max(n, 1) / 100.0, 2)
print("k_fit_taylor per WG (us):", {k: us(pt[i], nwg) for i, k in
      enumerate(["guess", "meta+moments0", "centre", "sweep", "trstep"])})
npost = pt[22]
print("k_post per WG (us):", {k: us(pt[16 + i], npost) for i, k in
      enumerate(["meta+Sd", "nu_zero", "out+centre", "ws_sweep", "inverse", "chan+store"])},
      "workgroups", npost)
