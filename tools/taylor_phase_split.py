"""Where k_fit_taylor's time goes: its phase clocks (ppf_phase_profile:
slot 0 the fused first moment pass, 1 set-up and T staging, 2 recentres,
3 the Taylor sweeps, 4 the trust-ncg steps) over one batch at the headline
(10,000 x 64 x 2048) and config-4 (2,000 x 128 x 2048) shapes, beside the
batch's kernel times.  python tools/taylor_phase_split.py"""
import sys, numpy as np, torch
sys.path.insert(0, ".")
import bench
from pulseportraiture_amd.engine import get_engine
eng = get_engine(0)
for cfg, n in (("headline", 10000), ("gm", 2000)):
    w, data, kw, _ = bench.synth_inputs(eng, cfg, n, 20240917, 0)
    flags = bench.CONFIGS[cfg][3]
    def fit():
        return eng.fit_batch(data, kw["model"], kw["freqs"], kw["P"], kw["init"], flags, nu_fit=kw["nu"],
                             guess=True, guess_Ns=100)
    fit(); torch.cuda.synchronize()
    eng.phase_profile(True)
    fit(); torch.cuda.synchronize()
    c = eng.phase_profile(False)
    tot = sum(c[i] for i in range(8))
    print(cfg, "slots 0-7 (ticks, fraction):", [(i, c[i], round(c[i] / max(tot, 1), 3)) for i in range(8)],
          "recentres", c[8], "fits", c[9], flush=True)
    eng.set_timing(True); eng.reset_kernel_times(); fit(); torch.cuda.synchronize()
    print(cfg, {k: round(eng.kernel_time(k)[0], 3) for k in ("data_xspec", "guess", "fit_taylor", "post")}, flush=True)
    eng.set_timing(False)
    del data
