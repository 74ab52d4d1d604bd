#!/usr/bin/env python3
"""Device trust-ncg trajectories of the headline_2k subints (64 x 2048,
phase + DM, Taylor path): fits them as tests/test_gpu_configs.py does with
the solver trace on (ppf_set_trace; k_fit_taylor records every counted
evaluation: point, f, g, H) and saves traces and results.

Usage (GPU box):  python tools/hl_trace.py OUT.npz [CAP]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out, cap=48):
    import torch
    from pulseportraiture_amd import synth
    from pulseportraiture_amd.engine import get_engine
    from tests.golden_consts import DM0
    z = np.load(os.path.join(ROOT, "tests", "golden", "headline_2k.npz"))
    nsub, seed = int(z["nsub"]), int(z["seed"])
    eng = get_engine(0)
    data = synth.workload_data_host_parallel(nsub, 64, 2048, seed=seed, procs=16)
    w = synth.make_workload(1, 64, 2048, seed=seed)
    buf = torch.full((nsub, cap, 32), float("nan"), dtype=torch.float64, device=eng.device)
    eng.set_trace(buf, cap)
    try:
        r = eng.fit_batch(data, w.model, w.freqs, w.P, [0.0, DM0, 0, 0, 0], [1, 1, 0, 0, 0],
                          nu_fit=np.stack([z["nu_fit"]] * 3, 1), guess=True, guess_Ns=100)
        torch.cuda.synchronize()
    finally:
        eng.set_trace(None, 0)
    res = {k: v.cpu().numpy() for k, v in r.items() if not k.startswith("_")}
    np.savez(out, trace=buf.cpu().numpy(), **res)
    print("saved", out)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 48)
