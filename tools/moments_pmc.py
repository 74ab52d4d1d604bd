"""One phase-family batch with the first moment pass in its own launch
(fuse_moments 0), for rocprofv3 --pmc passes on k_moments (its L2-miss
traffic against the X bytes it must read):
  python tools/moments_pmc.py [nsub] [nchan] [flags: pd|pdg]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pulseportraiture_amd import synth, pplib  # noqa: E402
from pulseportraiture_amd.engine import get_engine  # noqa: E402


def main():
    nsub = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    nchan = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    flags = [1, 1, 1, 0, 0] if (len(sys.argv) > 3 and sys.argv[3] == "pdg") else [1, 1, 0, 0, 0]
    nbin = 2048
    eng = get_engine(0)
    eng.set_option("fuse_moments", 0)
    w = synth.make_workload(nsub, nchan, nbin, seed=20240917)
    data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
    nu = pplib.guess_fit_freq(w.freqs)
    init = np.tile([0.0, w.DM0, 0.0, 0.0, 0.0], (nsub, 1))
    out = eng.fit_batch(data, w.model, w.freqs, w.P, init, flags, nu_fit=[nu] * 3, guess=True,
                        guess_Ns=100)
    torch.cuda.synchronize()
    nh = nbin // 2 + 1
    print("nsub %d nchan %d: X bytes %.4g, mean nfev %.3f" % (
        nsub, nchan, nsub * nchan * nh * 16.0, out["nfev"].float().mean().item()))


if __name__ == "__main__":
    main()
