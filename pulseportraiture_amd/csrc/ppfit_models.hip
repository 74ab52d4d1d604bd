// ppfit_models.hip -- Gaussian-component template portraits on the device
// (SURVEY.md §8(f) next #2).
//
// gen_gaussian_portrait (pplib.py:853-930) as read_model builds it
// (pplib.py:2873-2959): per channel, every component's loc / wid / amp is
// evolved to the channel frequency (evolve_parameter, pplib.py:1030-1046:
// '0' power law exp((ln f - ln nu_ref) idx + ln p), '1' linear
// (f - nu_ref) slope + p), and the profile is DC + sum amp * gaussian_profile
// (pplib.py:770-825: bin centres wrapped to within half a turn of the mean,
// exp(-z^2/2) / (sigma sqrt(2 pi)) where |z| < 20, rescaled by
// exp(-z_max^2/2) / max at its first argmax, z_max taken from the unwrapped
// loc).  A non-zero TAU scatters the rows afterwards (k_rotate_rows with
// tau_n = TAU/nbin (f_n/nu_ref)^alpha, scattering_portrait_FT).  One
// workgroup per (portrait, channel) row; the host supplies the constants the
// reference forms with numpy (2 sqrt(2 ln 2), sqrt(2 pi)) so that only exp /
// log are the device's.
#include "ppfit_kernels.hpp"

namespace ppf {

// numpy.remainder(x, 1.0): the result takes the divisor's sign
__device__ __forceinline__ double py_mod1(double x) {
  double m = fmod(x, 1.0);
  if (m != 0.0) {
    if (m < 0.0) m += 1.0;
  } else {
    m = 0.0;
  }
  return m;
}

// numpy rounds every product and sum: no contraction into fma here
__device__ __forceinline__ double evolve(int code, double lf, double f, const GaussArgs& g,
                                         double par, double evo) {
  // power law: exp(outer(ln f - ln nu_ref, idx) + outer(1, ln par))
  if (code == 0) return exp(__dadd_rn(__dmul_rn(lf - g.lnu, evo), log(par)));
  return __dadd_rn(__dmul_rn(f - g.nu_ref, evo), par);  // linear
}

// bin centre j of get_bin_centers (numpy.linspace: j * step + start, the last
// one = stop), wrapped to within half a turn of mean (pplib.py:801-805)
__device__ __forceinline__ double locval(int j, int nbin, double start, double stop, double step,
                                         double mean) {
  double x = (j == nbin - 1) ? stop : __dadd_rn(__dmul_rn((double)j, step), start);
  if (mean < 0.5) {
    if (x > mean + 0.5) x -= 1.0;
  } else if (x < mean - 0.5) {
    x += 1.0;
  }
  return x;
}

__global__ __launch_bounds__(256) void k_gauss_port(GaussArgs g, const double* __restrict__ freqs,
                                                    double* __restrict__ out) {
  constexpr int NT = 256;
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nbin = g.nbin;
  const double f = freqs[r];
  const double lf = log(f);
  __shared__ double s_max[NT / 64];
  __shared__ int s_arg[NT / 64];
  // numpy.linspace(0.5 / nbin, 1 - 0.5 / nbin, nbin): i * step + start, last = stop
  const double start = 0.5 / (double)nbin, stop = 1.0 - 0.5 / (double)nbin;
  const double step = (stop - start) / (double)(nbin - 1);
  constexpr int QMAX = 32;  // nbin <= 8192 = 32 x 256
  double model[QMAX];
  const int nq = (nbin + NT - 1) / NT;
#pragma unroll
  for (int q = 0; q < QMAX; ++q) model[q] = g.params[0];  // zeros + DC
  for (int c = 0; c < g.ngauss; ++c) {
    const double* p = g.params + 2 + 6 * c;
    const double loc = evolve(g.code[0], lf, f, g, p[0], p[1]);
    const double wid = evolve(g.code[1], lf, f, g, p[2], p[3]);
    const double amp = evolve(g.code[2], lf, f, g, p[4], p[5]);
    if (!(wid > 0.0)) continue;  // wid <= 0 (zeroout) or NaN: adds zeros
    const double sigma = wid / g.fwhm;
    const double mean = py_mod1(loc);
    const double norm = __dmul_rn(sigma, g.sqrt2pi);
    // values and first argmax over the bins
    double best = -1.0;
    int bi = nbin;
    double rv[QMAX];
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      rv[q] = 0.0;
      const int j = tid + NT * q;
      if (q < nq && j < nbin) {
        const double z = (locval(j, nbin, start, stop, step, mean) - mean) / sigma;
        const double v = (fabs(z) < 20.0) ? exp(__dmul_rn(-0.5, __dmul_rn(z, z))) / norm : 0.0;
        rv[q] = v;
        if (v > best) { best = v; bi = j; }
      }
    }
    // block argmax, first index on ties (numpy.argmax)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const double ob = __shfl_xor(best, o);
      const int oi = __shfl_xor(bi, o);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (lane == 0) { s_max[w] = best; s_arg[w] = bi; }
    __syncthreads();
    double gb = s_max[0];
    int gi = s_arg[0];
    for (int v = 1; v < NT / 64; ++v)
      if (s_max[v] > gb || (s_max[v] == gb && s_arg[v] < gi)) { gb = s_max[v]; gi = s_arg[v]; }
    __syncthreads();
    double fact = 1.0;
    bool scale = gb != 0.0;
    if (scale) {  // locval at the argmax (wrapped), z from the unwrapped loc
      const double z = (locval(gi, nbin, start, stop, step, mean) - loc) / sigma;
      fact = exp(__dmul_rn(-0.5, __dmul_rn(z, z))) / gb;
    }
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      if (q < nq) {
        const double prof = scale ? __dmul_rn(fact, rv[q]) : rv[q];
        model[q] = __dadd_rn(model[q], __dmul_rn(amp, prof));
      }
    }
  }
  double* o = out + (size_t)r * nbin;
#pragma unroll
  for (int q = 0; q < QMAX; ++q) {
    const int j = tid + NT * q;
    if (q < nq && j < nbin) o[j] = model[q];
  }
}

// scattering_times(TAU / nbin, alpha, freqs, nu_ref) = tau (f / nu_ref)^alpha
__global__ void k_scat_taus(const double* __restrict__ freqs, int n, double tau, double alpha,
                            double nu_ref, double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = tau * pow(freqs[i] / nu_ref, alpha);
}

// ---------------------------------------------------------------------------
// PSRFITS unpacking (load_data's Archive_load + pscrunch, pplib.py:2670-2732):
// out[s][q][n][j] = sum over the polarisations q takes of
//   raw[s][p][n][j] * scl[s][p][n] + offs[s][p][n]
// with pmode 0: every polarisation kept (q = p), 1: q = 0 takes p = 0 and 1
// (AA + BB, coherence or 2-pol data), 2: q = 0 takes p = 0 (Stokes I).
// One thread per output sample (raw read once, coalesced along the bins).
// ---------------------------------------------------------------------------
template <typename T>
__global__ void k_unpack(const T* __restrict__ raw, const double* __restrict__ scl,
                         const double* __restrict__ offs, int nsub, int npol, int nchan,
                         int nbin, int pmode, double* __restrict__ out) {
  const int npo = pmode ? 1 : npol;
  const size_t total = (size_t)nsub * npo * nchan * nbin;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int j = (int)(i % nbin);
  size_t r = i / nbin;
  const int n = (int)(r % nchan);
  r /= nchan;
  const int q = (int)(r % npo);
  const size_t s = r / npo;
  auto val = [&](int p) {
    const size_t m = (s * npol + p) * nchan + n;
    return fma((double)raw[m * nbin + j], scl[m], offs[m]);
  };
  double v;
  if (pmode == 1) v = val(0) + val(1);
  else v = val(pmode == 2 ? 0 : q);
  out[i] = v;
}

template __global__ void k_unpack<uint8_t>(const uint8_t*, const double*, const double*, int, int,
                                           int, int, int, double*);
template __global__ void k_unpack<int16_t>(const int16_t*, const double*, const double*, int, int,
                                           int, int, int, double*);
template __global__ void k_unpack<float>(const float*, const double*, const double*, int, int, int,
                                         int, int, double*);

}  // namespace ppf
