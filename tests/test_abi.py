"""The C-ABI library builds, loads and exports every symbol of include/ppfit.h."""
import os
import re

from tests.conftest import ROOT


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "ppfit.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|void|const char\*)\s+(ppf_\w+)\s*\(", txt,
                                 re.M)))


def test_header_declares_entry_points():
    syms = header_symbols()
    for s in ["ppf_ctx_create", "ppf_fit_portrait_batch", "ppf_phase_shift_batch",
              "ppf_rotate_rows", "ppf_rotate_accumulate", "ppf_irfft_rows",
              "ppf_noise_rows", "ppf_synth_portraits"]:
        assert s in syms


def test_library_exports_all_header_symbols():
    from pulseportraiture_amd import build, _lib
    build.build()
    lib = _lib.load_library()
    for s in header_symbols():
        assert hasattr(lib, s), s
    assert lib.ppf_version() == 1


def test_spec_nhp_any_nbin():
    """ppf_spec_nhp (no device needed): the padded harmonic count for every
    nbin the library takes, [16, 8192] -- powers of two or not -- and -1
    outside it (include/ppfit.h)."""
    from pulseportraiture_amd import build, _lib
    build.build()
    lib = _lib.load_library()
    for nbin in (16, 17, 32, 63, 64, 96, 999, 1000, 1536, 2048, 6001, 8191, 8192):
        assert lib.ppf_spec_nhp(nbin) == ((nbin // 2 + 1) + 15) // 16 * 16, nbin
    for nbin in (0, 8, 15, 8193, 16384, -4):
        assert lib.ppf_spec_nhp(nbin) == -1, nbin


def test_binding_options_match_header():
    """_lib.OPTIONS carries every PPF_OPT_* of include/ppfit.h with its id."""
    from pulseportraiture_amd import _lib
    txt = open(os.path.join(ROOT, "include", "ppfit.h")).read()
    opts = {m.group(1).lower(): int(m.group(2))
            for m in re.finditer(r"#define PPF_OPT_([A-Z_]+) (\d+)", txt)}
    assert opts == _lib.OPTIONS
    n = int(re.search(r"#define PPF_NUM_OPTS (\d+)", txt).group(1))
    assert sorted(opts.values()) == list(range(n))


def test_binding_covers_header():
    from pulseportraiture_amd import _lib
    assert set(header_symbols()) == set(_lib.EXPORTS)


def test_no_device_fails_loudly():
    import torch
    import pytest
    if torch.cuda.is_available():
        pytest.skip("device present")
    from pulseportraiture_amd.engine import Engine, PPFitError
    with pytest.raises(PPFitError):
        Engine(0)


def test_ppfits_library_exports_header():
    """libppfits.so (include/ppfits.h, host PSRFITS reader) exports every entry point."""
    from pulseportraiture_amd import build, psrfits
    build.build_fits()
    txt = open(os.path.join(ROOT, "include", "ppfits.h")).read()
    syms = sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(ppfits_\w+)\s*\(", txt, re.M)))
    assert len(syms) == 7
    lib = psrfits.load_library()
    for s in syms:
        assert hasattr(lib, s), s


def test_pptim_library_exports_header():
    """libpptim.so (include/pptim.h, host .tim writer) exports every entry point."""
    from pulseportraiture_amd import build, toas
    build.build_tim()
    txt = open(os.path.join(ROOT, "include", "pptim.h")).read()
    syms = sorted(set(re.findall(r"^\s*(?:int|void|int64_t|const char\*)\s+(ppt_\w+)\s*\(",
                                 txt, re.M)))
    assert syms == sorted(["ppt_format_rows", "ppt_text_nparts", "ppt_text_part",
                           "ppt_text_size", "ppt_text_rows", "ppt_text_free"])
    lib = toas.load_tim_library()
    for s in syms:
        assert hasattr(lib, s), s


def test_libraries_carry_source_hash():
    """build.py reuses a library only when it carries today's source hash."""
    from pulseportraiture_amd import build
    build.build()
    for path in (build.OUT, build.FITS_OUT, build.TIM_OUT):
        assert not build.needs_build(path), path
        cmd, deps = build._lib_specs()[path]
        assert build.built_hash(path) == build.source_hash(cmd, deps)
