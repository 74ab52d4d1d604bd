"""pulseportraiture_amd -- MI355X (gfx950) implementation of PulsePortraiture's
wideband FFTFIT path (phase / DM / GM / scattering TOAs).

The numerics live in libppfit.so (hand-written HIP kernels, C ABI in
include/ppfit.h); the Python modules mirror the reference's call surface:
``pptoaslib.fit_portrait_full``, ``pplib.fit_phase_shift`` / ``fit_portrait``
/ ``rotate_data`` / ``get_noise`` / ``write_TOAs``, ``pptoas.GetTOAs`` and
``ppalign.align_archives``.
"""
__version__ = "0.1.0"
