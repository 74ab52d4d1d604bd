"""get_TOAs + write_TOAs on the bench's registered 10,000 x 64 x 2048
device-resident archive: GetTOAs.phase_s per call (median of 8), then one
cProfile of the whole call (cumulative and own time).  Diagnostic."""
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
    t0 = time.perf_counter()
    gt.get_TOAs(quiet=True)
    t1 = time.perf_counter()
    pplib.write_TOAs(gt.TOA_list, outfile="/tmp/gt.tim", append=False)
    t2 = time.perf_counter()
    return gt, t1 - t0, t2 - t1


for _ in range(3):
    run()
torch.cuda.synchronize()
rows = []
for _ in range(8):
    gt, a, b = run()
    rows.append(dict(gt.phase_s, call=a, write=b))
keys = list(rows[0])
med = {k: round(float(np.median([r.get(k, 0.0) for r in rows])) * 1e3, 3) for k in keys}
print("median ms over 8 calls:", med)
pr = cProfile.Profile()
pr.enable()
for _ in range(4):
    run()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(40)
st.sort_stats("tottime").print_stats(30)
st.print_callers("as_tensor")
st.print_callers("copy_")
# the same calls with the device drained before each one
rows = []
for _ in range(8):
    torch.cuda.synchronize()
    gt, a, b = run()
    rows.append(dict(gt.phase_s, call=a, write=b))
print("drained first, median ms over 8 calls:",
      {k: round(float(np.median([r.get(k, 0.0) for r in rows])) * 1e3, 3) for k in keys})
