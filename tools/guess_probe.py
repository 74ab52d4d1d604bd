#!/usr/bin/env python3
"""Where k_guess's time goes at ppalign's grid (Ns = nbin = 2048): one fit
call over NSUB synthetic 256 x 2048 subints with the phase clocks on
(ppf_phase_profile: slots 10 brute-force grid, 11 Nelder-Mead, 12 NM calls,
wall_clock64 ticks at 100 MHz summed over workgroups), with the
prime-factor grid and with the direct grid (guess_direct), and the HIP-event
kernel times of both.

Usage (GPU box):  python tools/guess_probe.py [NSUB]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(nsub=4096):
    import torch
    from pulseportraiture_amd import pplib, synth
    from pulseportraiture_amd.engine import get_engine
    eng = get_engine(0)
    w = synth.make_workload(nsub, 256, 2048, seed=31)
    data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
    nu = pplib.guess_fit_freq(w.freqs)
    args = dict(nu_fit=[nu] * 3, guess=True, guess_Ns=2048, guess_wrap=False,
                guess_nu=np.full(nsub, nu))
    eng.fit_batch(data, w.model, w.freqs, w.P, [0.0, w.DM0, 0, 0, 0], [1, 1, 0, 0, 0], **args)
    torch.cuda.synchronize()
    res = {}
    for direct in (False, True):
        eng.set_timing(True)
        eng.reset_kernel_times()
        eng.phase_profile(True)
        r = eng.fit_batch(data, w.model, w.freqs, w.P, [0.0, w.DM0, 0, 0, 0], [1, 1, 0, 0, 0],
                          guess_direct=direct, **args)
        torch.cuda.synchronize()
        clk = eng.phase_profile(False)
        kt = {k: eng.kernel_time(k) for k in ("data_xspec", "guess", "fit_taylor", "post")}
        eng.set_timing(False)
        res[direct] = r["init_used"][:, 0].cpu().numpy()
        print("%s grid: guess kernel %.3f ms; workgroup-summed clocks: brute %.1f ms, "
              "Nelder-Mead %.1f ms, %.1f NM calls per subint, %d grids re-taken directly; "
              "PFA setup / stage 1 / stage 2 %.1f / %.1f / %.1f ms; data pass %.3f ms, fit %.3f ms"
              % ("direct" if direct else "prime-factor", kt["guess"][0],
                 clk[10] / 1e5, clk[11] / 1e5, clk[12] / nsub, clk[13], clk[23] / 1e5,
                 clk[24] / 1e5, clk[25] / 1e5, kt["data_xspec"][0],
                 kt["fit_taylor"][0]))
    print("guesses identical:", bool(np.array_equal(res[False], res[True])),
          "max |d| %.3g" % np.max(np.abs(res[False] - res[True])))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4096)
