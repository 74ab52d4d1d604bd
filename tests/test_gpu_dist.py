"""The sharded drivers with the real device path: two ranks on the one GPU of
the box (gloo process group -- RCCL refuses two ranks on one device), each
fitting its own shard through libppfit.  GetTOAs.get_TOAs must give rank 0
the single-process TOAs (pptoas.py:246,343 sharded, the result arrays
gathered to rank 0; the other rank holds none), and ppalign.align_archives the single-process template
(sharded fits and rotate-accumulate, one fused all_reduce of the Fourier-
domain sum, ppalign.py:113-213).  tests/test_dist_drivers_cpu.py covers the
same bookkeeping on CPU with the fit replaced; here nothing is replaced.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
from tests._compare import tim_lines

pytestmark = pytest.mark.gpu

DM0 = 34.56789


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _archives():
    from pulseportraiture_amd import archive, synth
    from pulseportraiture_amd.mjd import MJD
    names = []
    for i, nsub in enumerate([5, 3, 4]):
        w = synth.make_workload(nsub, 16, 256, seed=70 + i)
        wts = np.ones((nsub, 16))
        wts[1, 3] = 0.0
        name = "gdist%d.npz" % i
        archive.register_archive(name, dict(
            subints=synth.workload_data_host(w)[:, None], freqs=w.freqs, Ps=np.full(nsub, w.P),
            weights=wts, epochs=[MJD(57000.0 + 0.01 * k) for k in range(nsub)], DM=DM0,
            backend="be", frontend="fe", telescope="GBT", telescope_code="1"))
        names.append(name)
    w = synth.make_workload(1, 16, 256, seed=70)
    archive.register_archive("gdist_guess.npz", dict(
        subints=w.model[None, None], freqs=w.freqs, Ps=[w.P], epochs=[(57000, 0, 0.0)],
        DM=DM0, dmc=1))
    return names


def _run():
    from pulseportraiture_amd import pplib, pptoas, ppalign, synth
    names = _archives()
    gt = pptoas.GetTOAs(names, synth.EXAMPLE_GMODEL, quiet=True)
    gt.get_TOAs(quiet=True)
    lines = tim_lines(gt)
    port = ppalign.align_archives(names, "gdist_guess.npz", fit_dm=True, niter=2, quiet=True)
    return lines, np.array(gt.DeltaDM_means), port


def _worker(rank, world, port, out_dir):
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lines, ddm, tmpl = _run()
        np.savez(os.path.join(out_dir, "r%d.npz" % rank), lines=np.array(lines), ddm=ddm,
                 tmpl=tmpl)
    finally:
        torch.distributed.destroy_process_group()


def test_drivers_two_ranks_on_device_equal_single_process():
    import torch
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    ref_lines, ref_ddm, ref_tmpl = _run()
    assert len(ref_lines) == 12
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        got = [np.load(os.path.join(d, "r%d.npz" % k)) for k in range(2)]
    # the same batched device fits on a subset of subints: identical lines on
    # rank 0, which assembles every TOA (GetTOAs.gather_to = "root")
    assert list(got[0]["lines"]) == ref_lines
    np.testing.assert_array_equal(got[0]["ddm"], ref_ddm)
    assert len(got[1]["lines"]) == 0
    for g in got:
        # the template is a sum over ranks (different fp64 addition order)
        np.testing.assert_allclose(g["tmpl"], ref_tmpl, rtol=0,
                                   atol=1e-12 * np.abs(ref_tmpl).max())
    assert np.array_equal(got[0]["tmpl"], got[1]["tmpl"])
