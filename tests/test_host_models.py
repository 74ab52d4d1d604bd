"""Host-side template producer (read_model / gen_gaussian_portrait) vs golden."""
import os

import numpy as np

from pulseportraiture_amd import pplib, synth
from tests.golden_consts import P0


def test_example_models(golden):
    g = golden("models.npz")
    for shape in ["8x64", "16x256", "64x512"]:
        _, _, m = pplib.read_model(synth.EXAMPLE_GMODEL, g["phases_" + shape],
                                   g["freqs_" + shape], P0, quiet=True)
        np.testing.assert_allclose(m, g["model_" + shape], rtol=1e-13, atol=1e-13)
        np.testing.assert_array_equal(pplib.get_bin_centers(len(g["phases_" + shape])),
                                      g["phases_" + shape])
        np.testing.assert_array_equal(synth.channel_freqs(len(g["freqs_" + shape])),
                                      g["freqs_" + shape])


def test_scattered_model(golden, tmp_path):
    g = golden("models.npz")
    txt = open(synth.EXAMPLE_GMODEL).read().replace("TAU     0.00000000 1",
                                                    "TAU     0.00020000 1")
    p = os.path.join(tmp_path, "scat.gmodel")
    open(p, "w").write(txt)
    _, _, m = pplib.read_model(p, g["phases_scat_16x256"], g["freqs_scat_16x256"], P0,
                               quiet=True)
    np.testing.assert_allclose(m, g["model_scat_16x256"], rtol=1e-12, atol=1e-12)


def test_host_scalars(golden):
    u = golden("utils.npz")
    P = float(u["P"])
    for phi, DM, n1, n2, wrapped, raw in u["phase_transform"]:
        assert abs(pplib.phase_transform(phi, DM, n1, n2, P, mod=True) - wrapped) < 1e-14
        assert abs(pplib.phase_transform(phi, DM, n1, n2, P) - raw) < 1e-14
    assert pplib.guess_fit_freq(u["rot_freqs"], u["gff_snrs"]) == float(u["gff_out"])


def test_philox_known_answer():
    # Philox4x32-10 known-answer vectors (Salmon et al., Random123 kat_vectors)
    c = synth.philox4x32_10(0, 0, 0, 0, 0)
    assert [int(x) for x in c] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    m = 0xFFFFFFFF
    c = synth.philox4x32_10(m, m, m, m, m | (m << 32))
    assert [int(x) for x in c] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    c = synth.philox4x32_10(0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344,
                            0xA4093822 | (0x299F31D0 << 32))
    assert [int(x) for x in c] == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_synth_host_statistics():
    w = synth.make_workload(64, 16, 256, seed=5)
    d = synth.workload_data_host(w)
    resid = d - synth.synth_portraits_host(w.template, w.phase, 0.0, 0)
    assert abs(resid.std() - 1.5) < 0.03
    assert abs(resid.mean()) < 0.02
    assert np.all(np.abs(w.phi) <= 0.1)
