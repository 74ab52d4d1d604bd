"""Build libppfit.so in-tree with hipcc for gfx950 (no CUDA, no JIT cache)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["ppfit_lib.hip"]
DEPS = ["ppfit_lib.hip", "ppfit_spectra.hip", "ppfit_fit.hip", "ppfit_taylor.hip", "ppfit_tnc.hip", "ppfit_ncg.hip", "ppfit_models.hip", "ppfit_capi.hip",
        "ppfit_kernels.hpp", "ppfit_device.hpp"]
OUT = os.path.join(HERE, "libppfit.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    srcs = [os.path.join(CSRC, f) for f in DEPS] + [os.path.join(ROOT, "include", "ppfit.h")]
    return any(os.path.getmtime(s) > t for s in srcs)


# host-only PSRFITS reader (include/ppfits.h): plain C++, loadable without a GPU
FITS_OUT = os.path.join(HERE, "libppfits.so")
FITS_SRC = [os.path.join(CSRC, "psrfits.cpp"), os.path.join(ROOT, "include", "ppfits.h")]
CXX = os.environ.get("CXX", "g++")


def build_fits(force=False, verbose=False):
    if not force and os.path.exists(FITS_OUT) and \
            all(os.path.getmtime(s) <= os.path.getmtime(FITS_OUT) for s in FITS_SRC):
        return FITS_OUT
    cmd = [CXX, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-I" + os.path.join(ROOT, "include"), FITS_SRC[0], "-o", FITS_OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(FITS_OUT + ".tmp", FITS_OUT)
    return FITS_OUT


def build(force=False, verbose=False):
    build_fits(force, verbose)
    if not force and not needs_build():
        return OUT
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
           os.path.join(CSRC, SOURCES[0]), "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
