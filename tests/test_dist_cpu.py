"""Multi-process paths on CPU (gloo, world size 2): ppalign's sharding and its
one all-reduce, and the bench's per-rank weak-scaling inputs.

The device fit itself needs a GPU; what is tested here is everything around
it that decides correctness at N > 1: every unit lands on exactly one rank,
the fused fp64 all-reduce returns the single-process sum on every rank
(ppalign.py:202-213 sums over all archives), and a rank's synthetic subints
are the same subints a single process would generate at those indices.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from pulseportraiture_amd import ppalign, synth


def test_shard_range_partition():
    for n in range(0, 40):
        for world in range(1, 9):
            got = [ppalign.shard_range(n, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            for (lo, hi), (lo2, _) in zip(got, got[1:]):
                assert hi == lo2
            sizes = [hi - lo for lo, hi in got]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _unit_spectrum(i, nchan, nharm):
    """Deterministic stand-in for one unit's rotated, weighted spectrum."""
    rng = np.random.default_rng(1000 + i)
    spec = rng.standard_normal((nchan, nharm, 2))
    w = rng.uniform(0.5, 2.0, nchan)
    return spec * w[:, None, None], w


def _worker(rank, world, port, nunits, nchan, nharm, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r, w = ppalign.dist_info()
        assert (r, w) == (rank, world)
        lo, hi = ppalign.shard_range(nunits, rank, world)
        accum = torch.zeros(1, nchan, nharm, 2, dtype=torch.float64)
        tw = torch.zeros(nchan, dtype=torch.float64)
        for i in range(lo, hi):
            s, wt = _unit_spectrum(i, nchan, nharm)
            accum[0] += torch.as_tensor(s)
            tw += torch.as_tensor(wt)
        ppalign.allreduce_sum(accum, tw)
        np.savez(os.path.join(out_dir, "rank%d.npz" % rank), accum=accum.numpy(),
                 tw=tw.numpy(), lo=lo, hi=hi)
    finally:
        torch.distributed.destroy_process_group()


def test_gloo_ws2_allreduce_matches_single_process():
    nunits, nchan, nharm = 7, 6, 9
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), nunits, nchan, nharm, d), nprocs=2, join=True)
        ref_a = np.zeros((1, nchan, nharm, 2))
        ref_w = np.zeros(nchan)
        for i in range(nunits):
            s, wt = _unit_spectrum(i, nchan, nharm)
            ref_a[0] += s
            ref_w += wt
        r0 = np.load(os.path.join(d, "rank0.npz"))
        r1 = np.load(os.path.join(d, "rank1.npz"))
        assert (int(r0["lo"]), int(r0["hi"]), int(r1["lo"]), int(r1["hi"])) == (0, 4, 4, 7)
        for r in (r0, r1):
            np.testing.assert_allclose(r["accum"], ref_a, rtol=1e-13, atol=1e-13)
            np.testing.assert_allclose(r["tw"], ref_w, rtol=1e-13)
        # every rank holds the identical template afterwards (no broadcast needed)
        assert np.array_equal(r0["accum"], r1["accum"])


def test_single_process_allreduce_is_identity():
    a = torch.arange(6, dtype=torch.float64)
    (b,) = ppalign.allreduce_sum(a.clone())
    assert torch.equal(a, b)


def test_rank_slices_equal_single_process_subints():
    """bench.py rank r generates subints [r*nsub, (r+1)*nsub): same as one process."""
    nsub, nchan, nbin = 3, 4, 64
    whole = synth.make_workload(2 * nsub, nchan, nbin, seed=7)
    r1 = synth.make_workload(nsub, nchan, nbin, seed=7, sub0=nsub)
    np.testing.assert_array_equal(r1.phase, whole.phase[nsub:])
    np.testing.assert_array_equal(synth.workload_data_host(r1),
                                  synth.workload_data_host(whole)[nsub:])


def _gather_payload(rank):
    """Arrays of every layout the protocol-5 gather must carry: C and F order,
    strided views (pickled in-band), empty, odd byte counts, object arrays."""
    rng = np.random.default_rng(50 + rank)
    base = rng.standard_normal((5 + rank, 7))
    return {
        "rank": rank,
        "c": base,
        "f": np.asfortranarray(rng.standard_normal((3, 4 + rank))),
        "strided": base[::2, 1::3],
        "empty": np.zeros((0, 3), dtype=np.float32),
        "odd": rng.integers(0, 255, 13 + 2 * rank, dtype=np.uint8),
        "i16": rng.integers(-9, 9, (2, 3), dtype=np.int16),
        "obj": np.array(["a" * (rank + 1), None, 3], dtype=object),
        "tail": [np.float64(rank), "x" * 100 * (rank + 1)],
    }


def _gather_equal(a, b):
    assert a.keys() == b.keys()
    for k in a:
        if isinstance(a[k], np.ndarray):
            assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape, k
            assert a[k].tolist() == b[k].tolist(), k
        else:
            assert a[k] == b[k], k


def _gather_worker(rank, world, port, out_dir):
    from pulseportraiture_amd import pptoas
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        obj = _gather_payload(rank)
        root = pptoas._gather_objects(obj, rank, world)
        every = pptoas._gather_objects(obj, rank, world, to_all=True)
        dst1 = pptoas._gather_objects(obj, rank, world, dst=1)
        assert (root is None) == (rank != 0)
        assert (dst1 is None) == (rank != 1)
        for got in [g for g in (root, dst1) if g is not None] + [every]:
            assert len(got) == world
            for r in range(world):
                _gather_equal(got[r], _gather_payload(r))
        open(os.path.join(out_dir, "ok%d" % rank), "w").close()
    finally:
        torch.distributed.destroy_process_group()


def test_gloo_ws2_gather_objects_roundtrip():
    """get_TOAs' shard gather (pptoas._gather_objects) returns every rank's
    object unchanged, in rank order, to the root, to another rank and to all."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_gather_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        assert sorted(os.listdir(d)) == ["ok0", "ok1"]
