"""Wall-clock split of GetTOAs.get_TOAs + write_TOAs on the bench's
registered 10,000 x 64 x 2048 device-resident archive: the call itself, the
device work still queued when it returns, the .tim writing, and the bare
fit_batch of the same subints for comparison.  Diagnostic."""
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
sync = torch.cuda.synchronize
# wrap the fit boundary pieces to split "fit" further
from pulseportraiture_amd import engine as E  # noqa: E402
acc = {}


def timed(name, fn):
    def f(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
    return f


E.Engine.fit_batch = timed("engine.fit_batch (launch)", E.Engine.fit_batch)
E.FitPipeline.submit = timed("pipeline submit", E.FitPipeline.submit)
E.FitPipeline.collect = timed("pipeline collect (wait)", E.FitPipeline.collect)
for fr in [None, (1.0,), (0.8, 0.2), (0.75, 0.25), (0.65, 0.35), (0.6, 0.3, 0.1), (0.55, 0.3, 0.15), (0.7, 0.3)]:
  if fr is not None:
    pptoas.GetTOAs.pipeline_fracs = fr
  print("pipeline_fracs", pptoas.GetTOAs.pipeline_fracs)
  for rep in range(4):
      sync()
      t0 = time.perf_counter()
      gt = pptoas.GetTOAs(["gt"], synth.EXAMPLE_GMODEL, quiet=True)
      gt.get_TOAs(quiet=True)
      t1 = time.perf_counter()
      sync()
      t2 = time.perf_counter()
      pplib.write_TOAs(gt.TOA_list, outfile="/tmp/gt.tim", append=False)
      t3 = time.perf_counter()
      sync()
      t4 = time.perf_counter()
      print("get_TOAs %.2f ms, queued after it %.2f ms, write_TOAs %.2f ms, idle sync %.3f ms"
            % ((t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3), flush=True)
      print("   phases (ms): " + ", ".join("%s %.2f" % (k, v * 1e3) for k, v in gt.phase_s.items()))
      print("   fit boundary (ms): " + ", ".join("%s %.2f" % (k, v * 1e3) for k, v in acc.items()))
      acc.clear()
nu = np.full((nsub, 3), 1400.0)
for rep in range(3):
    sync()
    t0 = time.perf_counter()
    out = eng.fit_batch(data, w.model, w.freqs, w.P, [0.0, w.DM0, 0, 0, 0], [1, 1, 0, 0, 0],
                        nu_fit=nu, guess=True, guess_Ns=100)
    sync()
    t1 = time.perf_counter()
    res = {k: v.cpu().numpy() for k, v in out.items() if not k.startswith("_")}
    t2 = time.perf_counter()
    print("fit_batch %.2f ms, results to host %.2f ms" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3),
          flush=True)
