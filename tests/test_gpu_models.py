"""Device template portraits (ppf_gaussian_portraits) against the reference's
read_model / gen_gaussian_portrait (pplib.py:853-930, 2873-2959) run on the
same frequencies (tests/golden/models.npz, models_r2.npz from make_golden*.py):
both evolution codes, Doppler-shifted channels, the scattering branch, and
the headline 64 x 2048 shape.  The device's exp / log may differ from glibc's
in the last bit, so the bar is 1e-12 of the portrait's peak."""
import os

import numpy as np
import pytest

from tests.conftest import GOLDEN
from tests.golden_consts import P0

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from pulseportraiture_amd.engine import get_engine
    return get_engine(0)


def _close(got, ref):
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())


@pytest.mark.parametrize("case", ["hl", "lin", "lin2", "scat"])
def test_read_model_device_vs_reference(gpu, case, tmp_path):
    from pulseportraiture_amd import pplib
    z = np.load(os.path.join(GOLDEN, "models_r2.npz"))
    path = tmp_path / (case + ".gmodel")
    path.write_bytes(z[case + "_gmodel"].tobytes())
    ref = z[case + "_model"]
    nbin = ref.shape[1]
    _, _, got = pplib.read_model_device(str(path), nbin, z[case + "_freqs"], P0)
    _close(got, ref)
    # the host restatement agrees too (it makes the synthetic inputs)
    _, _, host = pplib.read_model(str(path), pplib.get_bin_centers(nbin), z[case + "_freqs"], P0,
                                  quiet=True)
    _close(got, host)


def test_models_npz_shapes(gpu):
    from pulseportraiture_amd import pplib, synth
    g = np.load(os.path.join(GOLDEN, "models.npz"))
    for shape in ["8x64", "16x256", "64x512"]:
        nbin = len(g["phases_" + shape])
        _, _, got = pplib.read_model_device(synth.EXAMPLE_GMODEL, nbin, g["freqs_" + shape], P0)
        _close(got, g["model_" + shape])


def test_batched_rows_equal_single(gpu):
    """One call over many subints' (Doppler-shifted) frequencies == per-subint calls."""
    from pulseportraiture_amd import pplib, synth
    info = pplib.read_model(synth.EXAMPLE_GMODEL, quiet=True)
    code, nu_ref, params, alpha = info[1], info[2], info[4], info[6]
    base = np.linspace(1100.0, 1900.0, 48)
    freqs = np.array([base * (1 + 1e-5 * k) for k in range(7)])
    many = pplib.gen_gaussian_portraits_device(code, params, alpha, 1024, freqs, nu_ref)
    for k in range(7):
        one = pplib.gen_gaussian_portraits_device(code, params, alpha, 1024, freqs[k], nu_ref)
        assert np.array_equal(many[k], one)


def test_abi_rejects_bad_model(gpu):
    import ctypes
    eng = gpu
    f = np.full(4, 1400.0)
    code = (ctypes.c_int32 * 3)(0, 2, 0)
    par = (ctypes.c_double * 8)(*([0.0] * 8))
    import torch
    ft = torch.as_tensor(f, device=eng.device)
    out = torch.empty(4, 64, dtype=torch.float64, device=eng.device)
    r = eng.lib.ppf_gaussian_portraits(eng.ctx, 4, 64, 1, ctypes.cast(code, ctypes.c_void_p),
                                       ctypes.cast(par, ctypes.c_void_p), 1400.0, 0.0,
                                       ctypes.c_void_p(ft.data_ptr()),
                                       ctypes.c_void_p(out.data_ptr()))
    assert r == -1  # PPF_ERR_INVALID
    code = (ctypes.c_int32 * 3)(0, 0, 0)
    r = eng.lib.ppf_gaussian_portraits(eng.ctx, 4, 64, 40, ctypes.cast(code, ctypes.c_void_p),
                                       ctypes.cast(par, ctypes.c_void_p), 1400.0, 0.0,
                                       ctypes.c_void_p(ft.data_ptr()),
                                       ctypes.c_void_p(out.data_ptr()))
    assert r == -3  # PPF_ERR_UNSUPPORTED
