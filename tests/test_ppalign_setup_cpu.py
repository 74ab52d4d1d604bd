"""align_archives' unit set-up (ppalign.py:121-177 restated in
pulseportraiture_amd/ppalign.py): the stacked-metadata paths (_Bulk, from
per-archive registrations and from one register_archives stack) give the same
units and the same unit stack -- host arrays and data rows -- as the
per-archive path, on CPU tensors (no fit runs)."""
import numpy as np
import pytest
import torch

from pulseportraiture_amd import archive, ppalign


class _Eng:
    device = torch.device("cpu")


NCHAN, NBIN = 8, 16
FREQS = np.linspace(1200.0, 1600.0, NCHAN)


def _bunches(n, kind, rng):
    data = torch.as_tensor(rng.standard_normal((n, 2, 1, NCHAN, NBIN)))
    out = []
    for i in range(n):
        b = dict(subints=data[i], freqs=FREQS, Ps=[0.004 + 1e-5 * i, 0.004 + 2e-5 * i],
                 epochs=[(57000 + i, 0, 0.0), (57000 + i, 60, 0.0)], DM=10.0 + i,
                 SNRs=rng.uniform(5.0, 50.0, (2, 1, NCHAN)))
        if kind in ("noise", "mixed") and i % 2 == 0:
            b["noise_stds"] = rng.uniform(0.5, 2.0, (2, 1, NCHAN))
        if kind == "mixed":
            if i == 1:
                w = np.ones((2, NCHAN))
                w[0, 3] = 0.0  # one zapped channel in subint 0
                w[1] = 0.0  # a subint with no channel on
                b["weights"] = w
            if i == 2:
                b["freqs"] = FREQS + 0.5  # not the template's frequencies
        out.append(b)
    return out


def _setup(names, model, bulk_on):
    opened = ppalign._open_all(names, model, 0.0, True, [], False, True)
    bulk = ppalign._Bulk.build(opened, model, NCHAN) if bulk_on else None
    units = ppalign._units(opened, model, bulk)
    multi = [u for u in units if len(u[2]) > 1]
    urows = bulk.unit_rows if bulk is not None and bulk.unit_rows is not None and \
        len(multi) == len(units) else None
    st = ppalign._UnitStack(_Eng(), multi, opened, model.freqs[0], 1, NCHAN, NBIN, bulk, urows)
    return units, st, bulk


def _same_units(a, b):
    assert len(a) == len(b)
    for u, v in zip(a, b):
        assert u[0] == v[0] and u[1] == v[1]
        assert np.array_equal(u[2], v[2]) and np.array_equal(u[3], v[3])


def _same_stack(s, t):
    assert s.n == t.n
    for k in ("freqs", "mask", "wts", "P", "DMg", "nu_fit"):
        assert np.array_equal(np.asarray(getattr(s, k)), np.asarray(getattr(t, k))), k
    e1, e2 = np.asarray(s.errs), np.asarray(t.errs)
    assert np.array_equal(np.isnan(e1), np.isnan(e2))
    assert np.array_equal(e1[~np.isnan(e1)], e2[~np.isnan(e2)])
    assert torch.equal(s.pols[0], t.pols[0])


@pytest.mark.parametrize("kind", ["plain", "noise", "mixed"])
@pytest.mark.parametrize("stacked", [False, True])
def test_bulk_setup_equals_per_archive(kind, stacked):
    rng = np.random.default_rng(7)
    n = 6
    names = ["su_%s_%d_%d" % (kind, stacked, i) for i in range(n)]
    bs = _bunches(n, kind, rng)
    if stacked:
        archive.register_archives(names, bs)
    else:
        for nm, b in zip(names, bs):
            archive.register_archive(nm, b)
    archive.register_archive("su_guess", dict(subints=np.zeros((1, 1, NCHAN, NBIN)), freqs=FREQS,
                                              Ps=[0.004], epochs=[(57000, 0, 0.0)], DM=10.0,
                                              dmc=1))
    model = archive.load_data("su_guess", dedisperse=True, tscrunch=True, rm_baseline=True,
                              quiet=True)
    try:
        u0, s0, _ = _setup(names, model, False)
        u1, s1, bulk = _setup(names, model, True)
        assert bulk is not None
        if stacked and kind != "mixed":
            assert bulk.allok and bulk.rows_view is not None and bulk.unit_rows is not None
        _same_units(u0, u1)
        _same_stack(s0, s1)
        # every archive still loads on its own as registered
        d = archive.load_data(names[1], quiet=True)
        assert "_stack" not in d
        np.testing.assert_array_equal(d.freqs, bs[1]["freqs"] * np.ones((2, 1)))
    finally:
        for nm in names + ["su_guess"]:
            archive.unregister_archive(nm)


def test_register_archives_stack_views():
    rng = np.random.default_rng(3)
    names = ["sv_%d" % i for i in range(4)]
    bs = _bunches(4, "plain", rng)
    archive.register_archives(names, bs)
    try:
        stk = archive._registry[names[0]]["_stack"][0]
        assert stk.rows is not None and stk.rows.shape == (4, 2, 1, NCHAN, NBIN)
        for i, nm in enumerate(names):
            assert torch.equal(stk.rows[i], bs[i]["subints"])
            assert np.shares_memory(archive._registry[nm].freqs, stk.freqs)
        # subints that are not equally spaced views of one tensor: no rows view
        archive.register_archives(names[:2], [dict(bs[0], subints=bs[0]["subints"].clone()),
                                              bs[1]])
        assert archive._registry[names[0]]["_stack"][0].rows is None
    finally:
        for nm in names:
            archive.unregister_archive(nm)


def test_register_archives_mixed_shapes_register_each():
    """Archives of different subint counts are still each registered (no
    stack); the set-up then takes the per-archive stacked path and agrees
    with the per-archive one."""
    rng = np.random.default_rng(11)
    names = ["mx_%d" % i for i in range(3)]
    bs = _bunches(3, "noise", rng)
    bs[1] = dict(bs[1], subints=bs[1]["subints"][:1], Ps=bs[1]["Ps"][:1],
                 epochs=bs[1]["epochs"][:1], SNRs=bs[1]["SNRs"][:1])  # one subint
    archive.register_archives(names, bs)
    archive.register_archive("mx_guess", dict(subints=np.zeros((1, 1, NCHAN, NBIN)), freqs=FREQS,
                                              Ps=[0.004], epochs=[(57000, 0, 0.0)], DM=10.0,
                                              dmc=1))
    model = archive.load_data("mx_guess", dedisperse=True, tscrunch=True, rm_baseline=True,
                              quiet=True)
    try:
        assert all("_stack" not in archive._registry[nm] for nm in names)
        assert archive._registry[names[1]].nsub == 1
        u0, s0, _ = _setup(names, model, False)
        u1, s1, bulk = _setup(names, model, True)
        assert bulk is not None and bulk.rows_view is None
        _same_units(u0, u1)
        _same_stack(s0, s1)
    finally:
        for nm in names + ["mx_guess"]:
            archive.unregister_archive(nm)


def test_open_stack_fast_path():
    """_open_all on exactly one register_archives stack, in order, takes the
    stack path (_StackOpened: no per-archive visit) and opens the same
    archives as the per-archive loop; any other request declines it."""
    rng = np.random.default_rng(11)
    n = 5
    names = ["os_%d" % i for i in range(n)]
    bs = _bunches(n, "plain", rng)
    archive.register_archives(names, bs)
    archive.register_archive("os_guess", dict(subints=np.zeros((1, 1, NCHAN, NBIN)), freqs=FREQS,
                                              Ps=[0.004], epochs=[(57000, 0, 0.0)], DM=10.0,
                                              dmc=1))
    model = archive.load_data("os_guess", dedisperse=True, tscrunch=True, rm_baseline=True,
                              quiet=True)

    def opened(nms, cutoff=0.0):
        skip = []
        o = ppalign._open_all(nms, model, cutoff, True, skip, False, True)
        return o, skip

    try:
        o, skip = opened(names)
        assert isinstance(o, ppalign._StackOpened) and not skip
        assert [nm for nm, _ in o] == names
        assert all(a.meta is archive._registry[nm] for nm, a in o)
        # declined: another order, a subset, an S/N cut that skips one
        for nms in (names[::-1], names[:3]):
            o2, _ = opened(nms)
            assert not isinstance(o2, ppalign._StackOpened)
            assert [nm for nm, _ in o2] == nms
        archive._registry[names[2]]["prof_SNR"] = 1.0
        o3, skip = opened(names, cutoff=5.0)
        assert not isinstance(o3, ppalign._StackOpened) and skip == [names[2]]
        assert [nm for nm, _ in o3] == names[:2] + names[3:]
        archive._registry[names[2]]["prof_SNR"] = np.inf
        # one archive registered again on its own: not the stack any more
        archive.register_archive(names[1], dict(bs[1]))
        o4, _ = opened(names)
        assert not isinstance(o4, ppalign._StackOpened)
        assert o4[1][1].meta is archive._registry[names[1]]
        archive.unregister_archive(names[3])
        o5, skip = opened(names)
        assert not isinstance(o5, ppalign._StackOpened) and names[3] not in [nm for nm, _ in o5]
    finally:
        for nm in names + ["os_guess"]:
            archive.unregister_archive(nm)
