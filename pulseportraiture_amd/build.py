"""Build the in-tree libraries (no CUDA, no JIT cache):

- libppfit.so  -- the HIP library (hipcc, gfx950), include/ppfit.h;
- libppfits.so -- the host PSRFITS reader (g++), include/ppfits.h;
- libpptim.so  -- the host .tim writer (g++), include/pptim.h.

Each library carries the sha256 of its sources, headers and compile command
as the string "PPF_SRC_HASH=<hex>" (a -D define the sources export); a
library is rebuilt unless its file holds the hash of today's sources, so a
library built from other sources -- an A/B variant, a stale tree -- is never
taken for the current one (mtimes are not consulted).
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INC = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")

SOURCES = ["ppfit_lib.hip"]
DEPS = ["ppfit_lib.hip", "ppfit_spectra.hip", "ppfit_fit.hip", "ppfit_taylor.hip", "ppfit_tnc.hip",
        "ppfit_ncg.hip", "ppfit_models.hip", "ppfit_generic.hip", "ppfit_capi.hip", "ppfit_kernels.hpp",
        "ppfit_device.hpp"]
OUT = os.path.join(HERE, "libppfit.so")
FITS_OUT = os.path.join(HERE, "libppfits.so")
TIM_OUT = os.path.join(HERE, "libpptim.so")

HASH_TAG = b"PPF_SRC_HASH="


def _lib_specs():
    """(output, compiler command without -D/-o, dependency files) per library."""
    hip = ([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-I" + INC,
            "-I" + CSRC, os.path.join(CSRC, SOURCES[0])],
           [os.path.join(CSRC, f) for f in DEPS] + [os.path.join(INC, "ppfit.h")])
    fits = ([CXX, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-I" + INC,
             os.path.join(CSRC, "psrfits.cpp")],
            [os.path.join(CSRC, "psrfits.cpp"), os.path.join(INC, "ppfits.h")])
    tim = ([CXX, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-pthread", "-I" + INC,
            os.path.join(CSRC, "pptim.cpp")],
           [os.path.join(CSRC, "pptim.cpp"), os.path.join(INC, "pptim.h")])
    return {OUT: hip, FITS_OUT: fits, TIM_OUT: tim}


def source_hash(cmd, deps):
    h = hashlib.sha256()
    h.update(" ".join(os.path.basename(c) if os.path.isabs(c) else c for c in cmd).encode())
    for p in deps:
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:32]


def built_hash(path):
    """The PPF_SRC_HASH a library file carries (None if absent)."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        blob = f.read()
    i = blob.find(HASH_TAG)
    if i < 0:
        return None
    j = i + len(HASH_TAG)
    return blob[j:j + 32].decode("ascii", "replace")


def needs_build(path=OUT):
    cmd, deps = _lib_specs()[path]
    return built_hash(path) != source_hash(cmd, deps)


def _build_one(path, force, verbose):
    cmd, deps = _lib_specs()[path]
    hsh = source_hash(cmd, deps)
    if not force and built_hash(path) == hsh:
        return path
    full = cmd + ['-DPPF_SRC_HASH="%s"' % hsh, "-o", path + ".tmp"]
    if verbose:
        print(" ".join(full), file=sys.stderr)
    subprocess.check_call(full)
    os.replace(path + ".tmp", path)
    return path


def build_fits(force=False, verbose=False):
    return _build_one(FITS_OUT, force, verbose)


def build_tim(force=False, verbose=False):
    return _build_one(TIM_OUT, force, verbose)


def build(force=False, verbose=False):
    build_fits(force, verbose)
    build_tim(force, verbose)
    return _build_one(OUT, force, verbose)


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
