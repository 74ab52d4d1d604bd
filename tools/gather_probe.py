#!/usr/bin/env python3
"""Rank-0 gather of get_TOAs at config-4 scale, on CPU (gloo): WORLD
processes, each fitting a PER_RANK-subint shard of one registered archive
(128 channels; the device fit replaced by tests/test_dist_drivers_cpu.fake_fit
at the fit_pipeline boundary), then gathering its finished columns to rank 0 (pptoas._gather_objects).
Reports per rank: the gather seconds (GetTOAs.phase_s), the pickled bytes
each rank sends, and peak RSS before / after the call.

  gather_probe.py [PER_RANK=125000] [WORLD=2] [NBIN=16] [GATHER_TO=root]
"""
import json
import os
import pickle
import resource
import socket
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _rss_mb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0


def _worker(rank, world, port, per_rank, nbin, gather_to, out):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests.test_dist_drivers_cpu import DM0, fake_fit
    from pulseportraiture_amd import archive, pplib, pptoas, synth
    from pulseportraiture_amd.mjd import MJD
    from pulseportraiture_amd.pptoaslib import SyncPipeline
    nchan, N = 128, per_rank * world
    w = synth.make_workload(1, nchan, nbin, seed=7)
    one = synth.workload_data_host(w)[0]
    # every subint the same samples (a broadcast view: no memory per subint)
    subints = np.broadcast_to(one, (N, 1, nchan, nbin))
    archive.register_archive("gather_probe.npz", dict(
        subints=subints, freqs=w.freqs, Ps=np.full(N, w.P), weights=np.ones((N, nchan)),
        noise_stds=np.full((N, 1, nchan), 1.5),
        epochs=[MJD(57000, 60 * k, 0.0) for k in range(N)],
        DM=DM0, backend="be", frontend="fe", telescope="GBT", telescope_code="1"))
    pptoas.fit_pipeline = lambda keys: SyncPipeline(fake_fit, keys)
    pptoas.gen_gaussian_portraits_device = lambda code, params, alpha, nb, freqs, nu_ref: \
        np.array([pplib.gen_gaussian_portrait(code, params, alpha, pplib.get_bin_centers(nb), f,
                                              nu_ref) for f in np.atleast_2d(freqs)])
    sent = {}
    orig = pptoas._gather_objects

    def gather(obj, *a, **k):  # the size of this rank's columns, pickled in-band
        sent["bytes"] = len(pickle.dumps(obj, protocol=5))
        t = time.perf_counter()
        dist.barrier()  # the slowest rank's fits, apart from the gather itself
        t1 = time.perf_counter()
        r = orig(obj, *a, **k)
        sent["wait_s"], sent["gather_s"] = t1 - t, time.perf_counter() - t1
        return r
    pptoas._gather_objects = gather
    gt = pptoas.GetTOAs(["gather_probe.npz"], synth.EXAMPLE_GMODEL, quiet=True)
    gt.gather_to = gather_to
    rss0 = _rss_mb()
    t0 = time.perf_counter()
    gt.get_TOAs(quiet=True, fit_GM=True)
    t1 = time.perf_counter()
    res = dict(rank=rank, world=world, per_rank=per_rank, nchan=nchan, gather_to=gather_to,
               call_s=round(t1 - t0, 3),
               phase_s={k: round(v, 4) for k, v in gt.phase_s.items()},
               sent_mb=round(sent.get("bytes", 0) / 1e6, 1),
               wait_s=round(sent.get("wait_s", 0.0), 3), gather_s=round(sent.get("gather_s", 0.0), 3),
               rss_before_mb=round(rss0, 1), rss_peak_mb=round(_rss_mb(), 1),
               toas_held=len(gt.TOA_list))
    with open(os.path.join(out, "r%d.json" % rank), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    per_rank = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    nbin = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    gather_to = sys.argv[4] if len(sys.argv) > 4 else "root"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, port, per_rank, nbin, gather_to, d), nprocs=world,
                 join=True)
        for r in range(world):
            print(open(os.path.join(d, "r%d.json" % r)).read())


if __name__ == "__main__":
    main()
