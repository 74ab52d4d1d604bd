"""Host-side cost of align_archives' set-up (open, units, unit stack) on the
CPU: config 5's 4,096 registered single-subint archives with CPU tensors as
subints and a stand-in engine holding only a device.  No fit runs.

  python tools/ppalign_host_profile.py [narch] [--cprofile] [--slow] [--each]
"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))))
from pulseportraiture_amd import archive, ppalign  # noqa: E402


class _Eng:
    device = torch.device("cpu")


def main():
    narch = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 4096
    nchan, nbin = 256, 64  # nbin does not enter the host path
    data = torch.zeros((narch, nchan, nbin), dtype=torch.float64)
    freqs = np.linspace(1100.0, 1900.0, nchan)
    names = ["hp_%d" % i for i in range(narch)]
    bunches = [dict(subints=data[i:i + 1, None], freqs=freqs, Ps=[0.005],
                    epochs=[(57000 + i, 0, 0.0)], DM=10.0) for i in range(narch)]
    if "--each" in sys.argv:  # one register_archive call per archive (no stack)
        for nm, b in zip(names, bunches):
            archive.register_archive(nm, b)
    else:
        archive.register_archives(names, bunches)
    archive.register_archive("hp_guess", dict(subints=np.zeros((1, 1, nchan, nbin)), freqs=freqs,
                                              Ps=[0.005], epochs=[(57000, 0, 0.0)], DM=10.0,
                                              dmc=1))
    model = archive.load_data("hp_guess", dedisperse=True, tscrunch=True, rm_baseline=True,
                              quiet=True)

    def run():
        t = [time.perf_counter()]
        opened = ppalign._open_all(names, model, 0.0, True, [], False, True)
        t.append(time.perf_counter())
        bulk = None if "--slow" in sys.argv else ppalign._Bulk.build(opened, model, nchan)
        units = ppalign._units(opened, model, bulk)
        t.append(time.perf_counter())
        ppalign._UnitStack(_Eng(), units, opened, model.freqs[0], 1, nchan, nbin, bulk,
                           None if bulk is None else bulk.unit_rows)
        t.append(time.perf_counter())
        return np.diff(t) * 1e3
    run()
    best = min((run() for _ in range(5)), key=lambda x: x.sum())
    print("open %.2f ms  units %.2f ms  unit stack %.2f ms  (%d archives: %.2f us each)"
          % (best[0], best[1], best[2], narch, best.sum() * 1e3 / narch))
    if "--cprofile" in sys.argv:
        import cProfile
        import pstats
        cProfile.runctx("run()", globals(), locals(), "/tmp/pphost.prof")
        pstats.Stats("/tmp/pphost.prof").sort_stats("tottime").print_stats(15)


if __name__ == "__main__":
    main()
