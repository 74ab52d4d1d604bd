"""ctypes binding of libppfit.so (include/ppfit.h).

The shared library is built in-tree by ``pulseportraiture_amd.build`` (hipcc,
gfx950).  There is deliberately no CPU fallback: if the library or a HIP
device is missing, every entry point raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libppfit.so")

PPF_OK = 0
PPF_METHOD_TRUST_NCG = 0
PPF_METHOD_TNC = 1
PPF_METHOD_NEWTON_CG = 2
PPF_METHOD_TNC_LEGACY = 3
METHODS = {"trust-ncg": PPF_METHOD_TRUST_NCG, "TNC": PPF_METHOD_TNC,
           "Newton-CG": PPF_METHOD_NEWTON_CG, "TNC-legacy": PPF_METHOD_TNC_LEGACY}
KERNEL_IDS = {"model_fft": 0, "data_xspec": 1, "solve": 2, "phase_shift": 3,
              "rotate": 4, "rot_accum": 5, "synth": 6, "irfft": 7, "noise": 8,
              "guess": 9, "post": 10, "fit_taylor": 11, "moments": 12, "resid": 13, "unpack": 14}
PPF_SOLVE_EXACT = 1
PPF_SOLVE_EVAL = 2
PPF_GUESS_DIRECT = 4
PPF_SPEC_NONE = 0
PPF_SPEC_STORE = 1
PPF_SPEC_USE = 2
PPF_SELFTEST_N = 10
# ppf_set_option ids (include/ppfit.h)
OPTIONS = {"scat_graph": 0, "scat_split": 1, "scat_tail": 2, "fuse_moments": 3, "guess_wave": 4,
           "hbm_tables": 5}
PPF_PHASE_N = 32

_dp = ctypes.c_void_p  # device pointers travel as plain addresses


class FitDesc(ctypes.Structure):
    """ppf_fit_desc."""
    _fields_ = [("nsub", ctypes.c_int32), ("nchan", ctypes.c_int32),
                ("nbin", ctypes.c_int32), ("nmodel", ctypes.c_int32),
                ("fit_flags", ctypes.c_int32 * 5),
                ("log10_tau", ctypes.c_int32), ("option", ctypes.c_int32),
                ("method", ctypes.c_int32), ("is_toa", ctypes.c_int32),
                ("guess", ctypes.c_int32), ("guess_Ns", ctypes.c_int32),
                ("guess_wrap", ctypes.c_int32), ("solver_flags", ctypes.c_int32),
                ("data", _dp), ("model", _dp), ("model_idx", _dp),
                ("freqs", _dp), ("errs", _dp), ("chan_mask", _dp),
                ("weights", _dp), ("P", _dp), ("init", _dp), ("nu_fit", _dp),
                ("nu_out", _dp), ("guess_nu", _dp), ("guess_tau", _dp),
                ("bounds", _dp), ("spec_mode", ctypes.c_int32), ("spec", _dp),
                ("spec_sig", _dp), ("spec_dsum", _dp), ("spec_R", _dp)]


class FitResult(ctypes.Structure):
    """ppf_fit_result."""
    _fields_ = [("params", _dp), ("param_errs", _dp), ("nu_out", _dp),
                ("cov", _dp), ("scales", _dp), ("scale_errs", _dp),
                ("channel_snrs", _dp), ("chi2", _dp), ("red_chi2", _dp),
                ("snr", _dp), ("nfev", _dp), ("status", _dp),
                ("init_used", _dp), ("fun", _dp), ("cov_nosc", _dp),
                ("grad", _dp), ("hess", _dp), ("errs_out", _dp)]


EXPORTS = {
    "ppf_version": ([], ctypes.c_int),
    "ppf_ctx_create": ([ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "ppf_ctx_destroy": ([ctypes.c_void_p], None),
    "ppf_last_error": ([ctypes.c_void_p], ctypes.c_char_p),
    "ppf_set_stream": ([ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "ppf_synchronize": ([ctypes.c_void_p], ctypes.c_int),
    "ppf_set_pipeline": ([ctypes.c_void_p, ctypes.c_int32], ctypes.c_int),
    "ppf_set_workspace_limit": ([ctypes.c_void_p, ctypes.c_int64], ctypes.c_int),
    "ppf_set_timing": ([ctypes.c_void_p, ctypes.c_int], ctypes.c_int),
    "ppf_set_trace": ([ctypes.c_void_p, _dp, ctypes.c_int32], ctypes.c_int),
    "ppf_set_option": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32], ctypes.c_int),
    "ppf_get_option": ([ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)],
                       ctypes.c_int),
    "ppf_get_kernel_time": ([ctypes.c_void_p, ctypes.c_int,
                             ctypes.POINTER(ctypes.c_double),
                             ctypes.POINTER(ctypes.c_int64)], ctypes.c_int),
    "ppf_reset_kernel_times": ([ctypes.c_void_p], ctypes.c_int),
    "ppf_selftest": ([ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
    "ppf_phase_profile": ([ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64)],
                          ctypes.c_int),
    "ppf_fit_portrait_batch": ([ctypes.c_void_p, ctypes.POINTER(FitDesc),
                                ctypes.POINTER(FitResult)], ctypes.c_int),
    "ppf_phase_shift_batch": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                               _dp, _dp, _dp, _dp, ctypes.c_int32,
                               ctypes.c_double, ctypes.c_double, _dp], ctypes.c_int),
    "ppf_rotate_rows": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, _dp, _dp,
                         _dp], ctypes.c_int),
    "ppf_rotate_accumulate": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                               ctypes.c_int32, _dp, _dp, _dp, _dp], ctypes.c_int),
    "ppf_rotate_accumulate_spec": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_int32, _dp, _dp, _dp, _dp], ctypes.c_int),
    "ppf_spec_nhp": ([ctypes.c_int32], ctypes.c_int32),
    "ppf_irfft_rows": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, _dp, _dp],
                       ctypes.c_int),
    "ppf_noise_rows": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, _dp, _dp],
                       ctypes.c_int),
    "ppf_resid_chi2_rows": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, _dp, _dp, _dp,
                             _dp, _dp, _dp, _dp, ctypes.c_double, _dp], ctypes.c_int),
    "ppf_unpack_subints": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                            ctypes.c_int32, ctypes.c_int32, _dp, _dp, _dp, ctypes.c_int32, _dp],
                           ctypes.c_int),
    "ppf_gaussian_portraits": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                _dp, _dp, ctypes.c_double, ctypes.c_double, _dp, _dp],
                               ctypes.c_int),
    "ppf_scatter_rotate_rows": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, _dp, _dp, _dp,
                                 _dp], ctypes.c_int),
    "ppf_spline_portraits": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                              ctypes.c_int32, _dp, _dp, ctypes.c_int32, ctypes.c_int32, _dp, _dp,
                              ctypes.c_int32, _dp, _dp], ctypes.c_int),
    "ppf_instrumental_response_rows": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, _dp,
                                        ctypes.c_int32, _dp, _dp, ctypes.c_double,
                                        ctypes.c_double, ctypes.c_double, _dp, _dp],
                                       ctypes.c_int),
    "ppf_tscrunch": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                      ctypes.c_int32, _dp, _dp, _dp, _dp], ctypes.c_int),
    "ppf_remove_baseline": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                             ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _dp, _dp, _dp],
                            ctypes.c_int),
    "ppf_profile_snr": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, _dp, ctypes.c_int32,
                         ctypes.c_double, _dp], ctypes.c_int),
    "ppf_synth_portraits": ([ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                             ctypes.c_int32, _dp, _dp, ctypes.c_double,
                             ctypes.c_uint64, ctypes.c_int64, _dp], ctypes.c_int),
}

_lib = None


def load_library(path=None):
    """Load libppfit.so and declare every exported signature."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("PPF_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(
            "libppfit.so not found at %s: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950). "
            "There is no CPU fallback." % p)
    lib = ctypes.CDLL(p)
    for name, (argtypes, restype) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    if path is None:
        _lib = lib
    return lib
