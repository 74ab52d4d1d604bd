"""cProfile (tottime) of GetTOAs.get_TOAs + write_TOAs on the bench's
registered 10,000 x 64 x 2048 device-resident archive.  Diagnostic."""
import cProfile
import pstats
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pulseportraiture_amd import archive, pplib, pptoas, synth  # noqa: E402
from pulseportraiture_amd.engine import get_engine  # noqa: E402
from pulseportraiture_amd.mjd import MJD  # noqa: E402

nsub = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
if len(sys.argv) > 2:
    pptoas.GetTOAs.pipeline_fracs = tuple(float(x) for x in sys.argv[2].split(","))
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
    pplib.write_TOAs(gt.TOA_list, outfile="/tmp/gt.tim", append=False)


for _ in range(3):
    run()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    run()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(45)
