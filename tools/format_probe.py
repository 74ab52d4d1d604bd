"""The .tim writer (libpptim.so ppt_format_rows) on get_TOAs-like records:
ms per call at 3,000 / 7,000 / 10,000 rows by host-thread count.  Run on the
GPU box's host (no GPU use).  Diagnostic."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from pulseportraiture_amd import toas as T  # noqa: E402


def fields(n, rng):
    name = b"bench_archive.npz"
    return [(T.PPT_TEXT, 0, name + b" ", None, None),
            (T.PPT_F64_FIXED, 8, rng.uniform(1e3, 2e3, n), None, None),
            (T.PPT_TEXT, 0, b" ", None, None), (T.PPT_I64, 0, np.full(n, 57000), None, None),
            (T.PPT_F64_FRAC, 15, rng.random(n), None, None),
            (T.PPT_TEXT, 0, b"   ", None, None), (T.PPT_F64_FIXED, 3, rng.random(n), None, None),
            (T.PPT_TEXT, 0, b"  gb -pp_dm ", None, None),
            (T.PPT_F64_FIXED, 7, rng.uniform(30, 40, n), None, None),
            (T.PPT_TEXT, 0, b" -pp_dme ", None, None),
            (T.PPT_F64_FIXED, 7, rng.random(n) * 1e-3, None, None),
            (T.PPT_TEXT, 0, b" -be bench -fe synth -f synth_bench -nbin 2048 -nch 64 -nchx ",
             None, None), (T.PPT_I64, 0, np.full(n, 64), None, None),
            (T.PPT_TEXT, 0, b" -bw ", None, None), (T.PPT_F64_FIXED, 3, np.full(n, 700.0), None, None),
            (T.PPT_TEXT, 0, b" -subint ", None, None), (T.PPT_I64, 0, np.arange(n), None, None),
            (T.PPT_TEXT, 0, b" -snr ", None, None), (T.PPT_F64_FIXED, 3, rng.random(n) * 100, None, None),
            (T.PPT_TEXT, 0, b" -gof ", None, None), (T.PPT_F64_FIXED, 3, rng.random(n) + 1, None, None)]


rng = np.random.default_rng(1)
for n in (3000, 7000, 10000):
    f = fields(n, rng)
    for nt in (1, 2, 4, 8):
        T._host_threads = lambda nt=nt: nt
        ts = []
        for _ in range(20):
            t = time.perf_counter()
            x = T.format_rows(n, f)
            ts.append(time.perf_counter() - t)
            del x
        print("rows %5d threads %d: %.3f ms" % (n, nt, np.median(ts) * 1e3), flush=True)
