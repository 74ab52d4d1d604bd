#!/usr/bin/env python3
"""Device trust-ncg trajectories of config 3's scattering subints.

Fits the subints of tests/golden/scattering_200.npz exactly as
tests/test_gpu_scattering_floor.py does, with the solver trace on
(ppf_set_trace: every evaluation's point, f, g, H, the trust radius after
it, the predicted reduction and rho of the step that led to it), and saves
the traces and results for comparison with the reference's own sequence
(recorded in the build container by wrapping pptoaslib's objective).

Usage (GPU box):  python tools/scat_trace.py OUT.npz [CAP]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out, cap=64):
    import torch
    from pulseportraiture_amd import synth
    from pulseportraiture_amd.engine import get_engine
    from tests.golden_consts import DM0
    z = np.load(os.path.join(ROOT, "tests", "golden", "scattering_200.npz"))
    nsub, seed = int(z["nsub"]), int(z["seed"])
    nchan, nbin, tau = 512, 1024, 2e-3
    eng = get_engine(0)
    data = synth.workload_data_host_parallel(nsub, nchan, nbin, seed=seed, procs=16, tau=tau)
    w = synth.make_workload(1, nchan, nbin, seed=seed, tau=tau)
    nu = z["nu_fit"]
    init = np.stack([np.zeros(nsub), np.full(nsub, DM0), np.zeros(nsub), z["init_tau"],
                     z["init_alpha"]], 1)
    buf = torch.full((nsub, cap, 32), float("nan"), dtype=torch.float64, device=eng.device)
    eng.set_trace(buf, cap)
    try:
        r = eng.fit_batch(data, w.model, w.freqs, w.P, init, [1, 1, 0, 1, 1],
                          nu_fit=np.stack([nu] * 3, 1), log10_tau=True, guess=True,
                          guess_Ns=100, guess_tau=10.0 ** z["init_tau"])
        torch.cuda.synchronize()
    finally:
        eng.set_trace(None, 0)
    res = {k: v.cpu().numpy() for k, v in r.items() if not k.startswith("_")}
    np.savez(out, trace=buf.cpu().numpy(), **res)
    print("saved", out, "nfev mean", res["nfev"].mean())


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 64)
