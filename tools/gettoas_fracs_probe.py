"""get_TOAs + write_TOAs per call on the bench's 10,000 x 64 x 2048
device-resident archive for several piece splits (GetTOAs.pipeline_fracs):
median wall ms of 8 calls each, interleaved over 3 rounds.  Diagnostic."""
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from pulseportraiture_amd import archive, pplib, pptoas, synth  # noqa: E402
from pulseportraiture_amd.engine import get_engine  # noqa: E402
from pulseportraiture_amd.mjd import MJD  # noqa: E402

nsub = 10000
eng = get_engine(0)
w = synth.make_workload(nsub, 64, 2048, seed=20240917)
data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
archive.register_archive("gt", dict(subints=data[:, None], freqs=w.freqs, Ps=np.full(nsub, w.P),
                                    DM=w.DM0, telescope="GBT", telescope_code="gb",
                                    backend="bench", frontend="synth",
                                    epochs=[MJD(57000, int(30 * k), 0.0) for k in range(nsub)]))
tim = os.path.join(tempfile.gettempdir(), "fracs_%d.tim" % os.getpid())
SPLITS = [(0.7, 0.3), (0.8, 0.2), (0.6, 0.3, 0.1), (0.65, 0.25, 0.1), (0.5, 0.3, 0.2), (1.0,)]
res = {s: [] for s in SPLITS}
phases = {s: [] for s in SPLITS}


def call(split):
    pptoas.GetTOAs.pipeline_fracs = split
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gt = pptoas.GetTOAs(["gt"], synth.EXAMPLE_GMODEL, quiet=True)
    gt.get_TOAs(quiet=True)
    pplib.write_TOAs(gt.TOA_list, SNR_cutoff=0.0, outfile=tim, append=False)
    return time.perf_counter() - t0, dict(gt.phase_s)


for s in SPLITS:
    call(s)
for rnd in range(3):
    for s in SPLITS:
        for _ in range(3):
            t, ph = call(s)
            res[s].append(t)
            phases[s].append(ph)
for s in SPLITS:
    med = np.median(res[s]) * 1e3
    ph = {k: round(float(np.median([p.get(k, 0.0) for p in phases[s]])) * 1e3, 3)
          for k in phases[s][0]}
    print("%-20s %7.2f ms  %7.0f TOAs/s  %s" % (str(s), med, nsub / med * 1e3, ph), flush=True)
os.unlink(tim)
