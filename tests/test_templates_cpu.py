"""Template producers on the CPU: the oracle's restatements of
gen_spline_portrait (pplib.py:932-956) and instrumental_response_port_FT
(pptoaslib.py:145-179) against the reference's own outputs
(tests/golden/make_golden_r3.py), and the host side of the spline-model
reader (restricted unpickler, read_model's "not a .gmodel" signal)."""
import io
import json
import os
import pickle

import numpy as np
import pytest

from oracle import ppfit_oracle as O
from tests.conftest import GOLDEN


@pytest.fixture(scope="module")
def fx():
    return (np.load(os.path.join(GOLDEN, "templates_r3.npz")),
            json.load(open(os.path.join(GOLDEN, "templates_r3.json"))))


def test_oracle_spline_portraits(fx):
    from pulseportraiture_amd.pplib import load_spline_model_file
    z, meta = fx
    for name in ["m3", "m5", "m1", "m0"]:
        raw = bytes(z["spl_%s_file" % name])
        mn, src, df, mean, eigvec, tck = pickle.loads(raw)
        for tag in meta[name]["cases"]:
            p = "spl_%s_%s_" % (name, tag)
            port = O.gen_spline_portrait(mean, z[p + "freqs"], eigvec, tck, int(z[p + "nbin"]))
            ref = z[p + "port"]
            assert port.shape == ref.shape
            assert np.max(np.abs(port - ref)) <= 1e-13 * np.max(np.abs(ref)), (name, tag)


def test_spline_file_reader(fx, tmp_path):
    from pulseportraiture_amd.pplib import load_spline_model_file, read_model
    z, _ = fx
    for name in ["m3", "m5", "m1", "m0"]:  # every model the fixtures hold loads
        path = tmp_path / (name + ".spl")
        path.write_bytes(bytes(z["spl_%s_file" % name]))
        mn, src, df, mean, eigvec, tck = load_spline_model_file(str(path))
        assert mn == name + ".spl"
    path = tmp_path / "m3.spl"
    path.write_bytes(bytes(z["spl_m3_file"]))
    mn, src, df, mean, eigvec, tck = load_spline_model_file(str(path))
    ref = pickle.loads(bytes(z["spl_m3_file"]))
    assert mn == ref[0] and np.array_equal(mean, ref[3]) and np.array_equal(eigvec, ref[4])
    assert np.array_equal(tck[0], ref[5][0]) and tck[2] == ref[5][2]
    # read_model on a pickled model raises what the reference's does, which
    # get_TOAs takes as "spline model" (pptoas.py:375-378)
    with pytest.raises(UnboundLocalError):
        read_model(str(path), quiet=True)


def test_spline_reader_refuses_other_globals(tmp_path):
    from pulseportraiture_amd.pplib import load_spline_model_file

    class Evil:
        def __reduce__(self):
            return (os.getcwd, ())
    path = tmp_path / "evil.spl"
    path.write_bytes(pickle.dumps(["x", "s", "d", np.zeros(4), np.zeros((4, 0)),
                                   [np.array([]), [], 0], Evil()], protocol=2))
    with pytest.raises(pickle.UnpicklingError):
        load_spline_model_file(str(path))


def test_spline_reader_python2_protocol0(tmp_path):
    """A Python-2 ppspline file is a protocol-0 pickle whose array data are
    Python-2 str objects; written here opcode by opcode (numpy's py2
    __reduce__ form) and read back."""
    from pulseportraiture_amd.pplib import load_spline_model_file
    arr = np.array([1.5, -2.25, 3.0])

    def s(b):  # Python-2 repr of a byte string
        return "S'" + "".join("\\x%02x" % c for c in b) + "'\n"

    def nd(a):
        return ("cnumpy.core.multiarray\n_reconstruct\n(cnumpy\nndarray\n(I0\ntS'b'\ntR"
                "(I1\n(I%d\ntcnumpy\ndtype\n(S'f8'\nI0\nI1\ntR(I3\nS'<'\nNNNI-1\nI-1\nI0\ntb"
                "I00\n" % len(a) + s(a.tobytes()) + "tb")
    txt = ("(lp0\nS'm.spl'\naS'J0000+0000'\naS'd.fits'\na" + nd(arr) + "a" +
           "cnumpy.core.multiarray\n_reconstruct\n(cnumpy\nndarray\n(I0\ntS'b'\ntR"
           "(I1\n(I3\nI0\ntcnumpy\ndtype\n(S'f8'\nI0\nI1\ntR(I3\nS'<'\nNNNI-1\nI-1\nI0\ntb"
           "I00\nS''\ntba" + "(lp1\n" + nd(arr) + "a(lp2\naI0\naa.")
    path = tmp_path / "py2.spl"
    path.write_bytes(txt.encode("ascii"))
    mn, src, df, mean, eigvec, tck = load_spline_model_file(str(path))
    assert mn == "m.spl" and np.array_equal(mean, arr) and eigvec.shape == (3, 0)
    assert np.array_equal(tck[0], arr) and tck[2] == 0


def test_oracle_instrumental_response(fx):
    z, meta = fx
    for tag in ["rect", "gauss", "both_dm", "dm"]:
        m = meta["irf_" + tag]
        R = O.instrumental_response_port_FT(m["nbin"], z["irf_%s_freqs" % tag], m["DM"],
                                            m["P"], m["wids"], m["irf_types"])
        np.testing.assert_allclose(np.real(R), np.real(z["irf_" + tag]), rtol=0, atol=1e-15)
