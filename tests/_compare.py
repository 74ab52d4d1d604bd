"""Shared parity comparisons for the CPU (oracle) and GPU tests."""
import numpy as np

DCONST = 0.000241 ** -1  # pplib.py:51

# trust-ncg / TNC return codes the reference treats as converged: it reports
# a fit as 'failed' only outside this set (pptoaslib.py:1022-1033)
CONVERGED = {1, 2, 4}


def phi_at(phi, DM, GM, nu_DM, nu_GM, to_DM, to_GM, P):
    """phi reported at (nu_DM, nu_GM) moved to (to_DM, to_GM), wrapped to
    [-0.5, 0.5) (phase_shifts / phase_transform, pptoaslib.py:181-214)."""
    out = phi + DCONST * DM / P * (to_DM ** -2 - nu_DM ** -2) + \
        DCONST ** 2 * GM / P * (to_GM ** -4 - nu_GM ** -4)
    return (out + 0.5) % 1.0 - 0.5


def phase_gap(phi, DM, GM, nu_DM, nu_GM, ref, P):
    """|phi - phi_ref| / sigma_phi with both phases at the reference's output
    frequencies.  The zero-covariance frequency is a ratio of Hessian sums
    that cancel heavily for multi-parameter fits, so two fits that agree to
    1e-5 sigma can report their TOA at frequencies 1e-8 apart; comparing the
    phases at one frequency separates the fit from that reporting choice."""
    p = phi_at(phi, DM, GM, nu_DM, nu_GM, ref["nu_DM"], ref["nu_GM"], P)
    d = abs(p - ref["phi"])
    return min(d, 1.0 - d) / ref["phi_err"]


def tim_lines(gt):
    """The .tim lines of gt.TOA_list as write_TOAs writes them (the native
    writer over the column-built records, none built as objects yet), held
    equal to toa_line over the TOA objects (which builds them)."""
    import os
    import tempfile
    from pulseportraiture_amd import pplib
    fd, path = tempfile.mkstemp(suffix=".tim")
    os.close(fd)
    try:
        pplib.write_TOAs(gt.TOA_list, outfile=path, append=False)
        bulk = open(path).read().splitlines()
    finally:
        os.unlink(path)
    objs = [pplib.toa_line(t) for t in gt.TOA_list]
    assert bulk == objs, "bulk .tim text differs from the per-TOA text"
    return bulk
