"""cProfile of GetTOAs.get_TOAs + .tim text on the bench's registered
10,000 x 64 x 2048 device-resident archive (the get_toas leg of bench.py):
where the host time goes beside the ~9 ms of fits.  Diagnostic."""
import cProfile
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from pulseportraiture_amd import archive, pplib, pptoas, synth  # noqa: E402
from pulseportraiture_amd.engine import get_engine  # noqa: E402
from pulseportraiture_amd.mjd import MJD  # noqa: E402

nsub = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
eng = get_engine(0)
w = synth.make_workload(nsub, 64, 2048, seed=20240917)
data = eng.synth(w.template, w.phase, w.sigma, w.seed, sub0=w.sub0)
archive.register_archive("gt", dict(subints=data[:, None], freqs=w.freqs, Ps=np.full(nsub, w.P),
                                    DM=w.DM0, telescope="GBT", telescope_code="gb",
                                    backend="bench", frontend="synth",
                                    epochs=[MJD(57000, int(30 * k), 0.0) for k in range(nsub)]))


def run():
    gt = pptoas.GetTOAs(["gt"], synth.EXAMPLE_GMODEL, quiet=True)
    gt.get_TOAs(quiet=True)
    return [pplib.toa_line(t) for t in gt.TOA_list]


run()
torch.cuda.synchronize()
for _ in range(2):
    t0 = time.perf_counter()
    run()
    torch.cuda.synchronize()
    print("call %.1f ms" % ((time.perf_counter() - t0) * 1e3))
cProfile.run("run(); torch.cuda.synchronize()", "/tmp/gt.prof")
pstats.Stats("/tmp/gt.prof").sort_stats("tottime").print_stats(25)
pstats.Stats("/tmp/gt.prof").sort_stats("cumtime").print_stats(25)
