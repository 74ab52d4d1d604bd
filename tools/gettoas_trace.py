"""Five timed GetTOAs.get_TOAs + write_TOAs calls on the bench's registered
10,000 x 64 x 2048 archive, each bracketed by roctx-free host timestamps
(printed), for a rocprofv3 kernel / memory-copy trace of the same process:
where the device idles inside a call.  Diagnostic."""
import sys
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
for rep in range(6):
    torch.cuda.synchronize()
    t0 = time.perf_counter_ns()
    gt = pptoas.GetTOAs(["gt"], synth.EXAMPLE_GMODEL, quiet=True)
    gt.get_TOAs(quiet=True)
    pplib.write_TOAs(gt.TOA_list, outfile="/tmp/gt.tim", append=False)
    t1 = time.perf_counter_ns()
    torch.cuda.synchronize()
    t2 = time.perf_counter_ns()
    print("rep %d: call %.2f ms, then sync %.2f ms; phases %s" % (
        rep, (t1 - t0) / 1e6, (t2 - t1) / 1e6,
        ", ".join("%s %.2f" % (k, v * 1e3) for k, v in gt.phase_s.items())), flush=True)
    time.sleep(0.05)  # a visible gap between calls in the trace
