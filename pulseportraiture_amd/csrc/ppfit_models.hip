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
// B-spline (PCA) template portraits, gen_spline_portrait (pplib.py:932-956)
// as read_spline_model builds them (pplib.py:2961-2993): row r at
// freqs[r] is mean_prof + sum_e splev(freqs[r], (t, c[e], k)) eigvec[:, e].
// splev is FITPACK's (splev.f with ext = 0: the knot interval search, then
// fpbspl.f's de Boor recurrence, every product and sum rounded as gfortran
// does without FMA); the eigenvector contraction (np.dot, a BLAS dgemm
// whose summation order is the library's) is a fused sum over e.
// ---------------------------------------------------------------------------
__device__ double fp_splev(const double* __restrict__ t, int n, int k,
                           const double* __restrict__ c, double x) {
  const int k1 = k + 1, nk1 = n - k1;
  // splev.f labels 35/40: the largest 1-based l in [k1, nk1] with t(l) <= x
  int l = k1;
  while (l != nk1 && x >= t[l]) ++l;  // t(l + 1) is t[l]
  double h[kMaxSplineK + 1], hh[kMaxSplineK];
  h[0] = 1.0;
#pragma unroll
  for (int j = 1; j <= kMaxSplineK; ++j) {
    if (j > k) break;
#pragma unroll
    for (int i = 0; i < kMaxSplineK; ++i)
      if (i < j) hh[i] = h[i];
    h[0] = 0.0;
#pragma unroll
    for (int i = 1; i <= kMaxSplineK; ++i) {
      if (i > j) break;
      const double tli = t[l + i - 1], tlj = t[l + i - j - 1];
      if (tli == tlj) {
        h[i] = 0.0;
        continue;
      }
      const double f = hh[i - 1] / (tli - tlj);
      h[i - 1] = __dadd_rn(h[i - 1], __dmul_rn(f, tli - x));
      h[i] = __dmul_rn(f, x - tlj);
    }
  }
  double sp = 0.0;
  const int ll = l - k1;
#pragma unroll
  for (int j = 0; j <= kMaxSplineK; ++j)
    if (j < k1) sp = __dadd_rn(sp, __dmul_rn(c[ll + j], h[j]));
  return sp;
}

__global__ __launch_bounds__(256) void k_spline_rows(SplineArgs s, const double* __restrict__ freqs,
                                                     double* __restrict__ out) {
  __shared__ double proj[kMaxEig];
  const int r = blockIdx.x;
  if ((int)threadIdx.x < s.neig)
    proj[threadIdx.x] = fp_splev(s.t, s.n, s.k, s.c + (size_t)threadIdx.x * s.ncoef, freqs[r]);
  __syncthreads();
  double* o = out + (size_t)r * s.nbin;
  for (int j = threadIdx.x; j < s.nbin; j += blockDim.x) {
    const double* ev = s.eigvec + (size_t)j * s.neig;
    double d = 0.0;
    for (int e = 0; e < s.neig; ++e) d = fma(proj[e], ev[e], d);
    o[j] = s.neig ? d + s.mean[j] : s.mean[j];  // eigvec.shape[1] == 0: the tiled mean
  }
}

// scipy.signal.resample (rfft branch) of rows from nin to nout bins followed
// by rotate_portrait(port, shift) (pplib.py:951-955), formed on the
// spectrum: Y_k = X_k for k < min(nin, nout) / 2 + 1, the shared Nyquist
// term x2 (down) or x0.5 (up), times nout / nin and e^{2 pi i k shift}; the
// Nyquist imaginary part is dropped first, as resample's irfft drops it.
__global__ void k_resample_spec(const double2* __restrict__ X, int nin, int nout, double shift,
                                int nrow, double2* __restrict__ Y) {
  const int ho = nout / 2 + 1, hi = nin / 2 + 1;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)nrow * ho) return;
  const int k = (int)(i % ho);
  const size_t r = i / ho;
  const int N = min(nin, nout);
  double2 y = cmk(0.0, 0.0);
  if (k < N / 2 + 1) y = X[r * hi + k];
  if (!(N & 1) && k == N / 2) {  // scipy adjusts the shared Nyquist bin of an even N only
    if (nout < nin) y = cscale(y, 2.0);
    else if (nin < nout) y = cscale(y, 0.5);
  }
  if (!(nout & 1) && k == nout / 2) y.y = 0.0;
  y = cscale(y, (double)nout / (double)nin);
  if (shift != 0.0) y = cmul(y, turn_phasor((double)k, shift));
  Y[i] = y;
}

// ---------------------------------------------------------------------------
// Instrumental response (pptoas.py:387-393): spec[r][k] *= R_r(k) with
// R_r = prod_w instrumental_response_FT(nbin, wids[w], types[w]) times, for
// DM != 0, the rect response of width 8.3e-6 chan_bw / (freq_r / 1e3)^3 / P
// (instrumental_response_port_FT, pptoaslib.py:145-179).  rect: np.sinc(k wid)
// = sin(pi x) / (pi x) with x = 0 -> 1; gauss: gaussian_profile_FT(nbin, 0,
// wid, 1) / its k = 0 term (pptoaslib.py:14-50, 136-139) =
// exp(-b^2) Re erf(a + i b) / erf(a), taken as exp(-b^2) / erf(a) -- exact
// to exp(-a^2) <= 2.4e-16 absolute for the widths the host admits (a >= 6).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double np_sinc(double x) {
  const double y = __dmul_rn(M_PI, x == 0.0 ? 1.0e-20 : x);
  return sin(y) / y;
}

__device__ __forceinline__ double irf_value(int type, double k, double wid, double fwhm) {
  if (type == 0) return np_sinc(__dmul_rn(k, wid));
  // gaussian_profile_FT: sigma = wid / (2 sqrt(2 ln 2)); sigma *= 2 pi; sigma = 1 / sigma
  double sigma = wid / fwhm;
  sigma = __dmul_rn(sigma, 2.0 * M_PI);
  sigma = 1.0 / sigma;
  const double a = sigma / __dmul_rn(1.0 / M_PI, M_SQRT2);
  const double b = k / __dmul_rn(sigma, M_SQRT2);
  return exp(-__dmul_rn(b, b)) / erf(a);
}

__global__ void k_ir_spec(double2* __restrict__ spec, double* __restrict__ resp, int nrow,
                          int nharm, IrArgs g, const double* __restrict__ freqs) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)nrow * nharm) return;
  const int k = (int)(i % nharm);
  const int r = (int)(i / nharm);
  double R = 1.0;
  for (int w = 0; w < g.nw; ++w) R = __dmul_rn(R, irf_value(g.type[w], (double)k, g.wid[w], g.fwhm));
  if (g.dm_wid_num != 0.0) {
    const double fr = freqs[r] / 1e3;
    const double wid = g.dm_wid_num / pow(fr, 3.0) / g.P;
    R = __dmul_rn(R, np_sinc(__dmul_rn((double)k, wid)));
  }
  if (resp) resp[i] = R;  // the response table itself
  else spec[i] = cscale(spec[i], R);
}

// ---------------------------------------------------------------------------
// tscrunch of fold-mode subints (load_data's arch.tscrunch(), pplib.py:2700):
// per (pol, channel, bin) the weight-averaged profile over the subints,
// out = sum_s w[s][n] d[s][p][n][j] / sum_s w[s][n] (0 where the weights sum
// to 0), and wsum[n] = sum_s w[s][n].  One thread per output sample, the
// subint loop in order (coalesced along the bins).
// ---------------------------------------------------------------------------
__global__ void k_tscrunch(const double* __restrict__ d, const double* __restrict__ w, int nsub,
                           int npol, int nchan, int nbin, double* __restrict__ out,
                           double* __restrict__ wsum) {
  const size_t total = (size_t)npol * nchan * nbin;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int j = (int)(i % nbin);
  const int n = (int)((i / nbin) % nchan);
  const int p = (int)(i / ((size_t)nbin * nchan));
  double acc = 0.0, ws = 0.0;
  for (int s = 0; s < nsub; ++s) {
    const double ww = w[(size_t)s * nchan + n];
    if (ww != 0.0) acc = fma(ww, d[(((size_t)s * npol + p) * nchan + n) * nbin + j], acc);
    ws += ww;
  }
  out[i] = ws != 0.0 ? acc / ws : 0.0;
  if (p == 0 && j == 0 && wsum) wsum[n] = ws;
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
__global__ __launch_bounds__(256) void k_unpack(const T* __restrict__ raw,
                                                const double* __restrict__ scl,
                                                const double* __restrict__ offs, int nsub,
                                                int npol, int nchan, int nbin, int pmode,
                                                double* __restrict__ out) {
  // one block per output profile (subint s, polarisation q, channel n): its
  // scale / offset once, then the row's samples coalesced
  const int npo = pmode ? 1 : npol;
  const size_t row = blockIdx.x;
  const int n = (int)(row % nchan);
  const size_t r = row / nchan;
  const int q = (int)(r % npo);
  const size_t s = r / npo;
  const size_t m0 = (s * npol + (pmode ? 0 : q)) * nchan + n;
  const size_t m1 = (s * npol + 1) * nchan + n;  // pmode 1 only (npol >= 2)
  const double sc0 = scl[m0], of0 = offs[m0];
  const double sc1 = pmode == 1 ? scl[m1] : 0.0, of1 = pmode == 1 ? offs[m1] : 0.0;
  const T* __restrict__ r0 = raw + m0 * nbin;
  const T* __restrict__ r1 = raw + (pmode == 1 ? m1 : m0) * nbin;
  double* __restrict__ o = out + row * nbin;
  for (int j = threadIdx.x; j < nbin; j += blockDim.x) {
    double v = fma((double)r0[j], sc0, of0);
    if (pmode == 1) v = v + fma((double)r1[j], sc1, of1);
    o[j] = v;
  }
  (void)nsub;
}

// ---------------------------------------------------------------------------
// remove_baseline (load_data's arch.remove_baseline(), pplib.py:2691), as
// PSRCHIVE's Integration::remove_baseline does it with the default baseline
// estimator: the off-pulse window is found once per subint on the total
// intensity profile (weighted frequency sum of the first ntot polarisations)
// as the circular window of `width` bins with the smallest sum (the minimum of
// the boxcar-smoothed profile; first window on ties), and every profile of
// the subint has its own mean over that window subtracted.  One workgroup per
// subint: t[j] in LDS (coalesced channel rows), each thread sums the windows
// that start at its bins directly (no prefix-sum cancellation), a block argmin,
// then one wave per profile row: window mean (wave sum), row -= mean in place.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_remove_baseline(double* __restrict__ data,
                                                         const double* __restrict__ w, int npol,
                                                         int nchan, int nbin, int ntot, int width,
                                                         int* __restrict__ win_out) {
  extern __shared__ __align__(16) unsigned char dyn[];
  double* t = reinterpret_cast<double*>(dyn);  // [nbin]
  __shared__ double bv[4];
  __shared__ int bi[4];
  __shared__ int s_j0;
  const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  double* sub = data + (size_t)s * npol * nchan * nbin;
  const double* ws = w + (size_t)s * nchan;
  for (int j = tid; j < nbin; j += 256) {
    double acc = 0.0;
    for (int n = 0; n < nchan; ++n) {
      const double wn = ws[n];
      if (wn == 0.0) continue;  // uniform over the block
      double v = 0.0;
      for (int p = 0; p < ntot; ++p) v += sub[((size_t)p * nchan + n) * nbin + j];
      acc = fma(wn, v, acc);
    }
    t[j] = acc;
  }
  __syncthreads();
  double best = INFINITY;
  int bj = 0x7fffffff;
  for (int j = tid; j < nbin; j += 256) {
    double b = 0.0;
    for (int i = 0; i < width; ++i) {
      int k = j + i;
      if (k >= nbin) k -= nbin;
      b += t[k];
    }
    if (b < best || (b == best && j < bj)) { best = b; bj = j; }
  }
  // block argmin, first index on ties
  for (int o = 32; o >= 1; o >>= 1) {
    const double ob = __shfl_xor(best, o);
    const int oj = __shfl_xor(bj, o);
    if (ob < best || (ob == best && oj < bj)) { best = ob; bj = oj; }
  }
  if (lane == 0) { bv[wv] = best; bi[wv] = bj; }
  __syncthreads();
  if (tid == 0) {
    double b = bv[0];
    int j0 = bi[0];
    for (int q = 1; q < 4; ++q)
      if (bv[q] < b || (bv[q] == b && bi[q] < j0)) { b = bv[q]; j0 = bi[q]; }
    s_j0 = j0;
    if (win_out) win_out[s] = j0;
  }
  __syncthreads();
  const int j0 = s_j0;
  const double iw = 1.0 / (double)width;
  for (int r = wv; r < npol * nchan; r += 4) {
    double* row = sub + (size_t)r * nbin;
    double m = 0.0;
    for (int i = lane; i < width; i += 64) {
      int k = j0 + i;
      if (k >= nbin) k -= nbin;
      m += row[k];
    }
    m = wave_sum(m) * iw;
    for (int j = lane; j < nbin; j += 64) row[j] -= m;
  }
}

// ---------------------------------------------------------------------------
// Profile::snr() for load_data's SNRs (pplib.py:2762-2770), PSRCHIVE's default
// phase S/N restated (include/ppfit.h ppf_profile_snr).  One wave per
// profile row, the row in LDS.  The window sums, the window statistics and
// the running sum are each formed in one fixed order: lane-contiguous
// segments of the circular row summed in sequence, then the lanes' totals
// in lane order (a serial exclusive scan over 64 values), so the result
// does not depend on the launch.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_profile_snr(const double* __restrict__ rows, int nbin,
                                                    int width, double thr,
                                                    double* __restrict__ out) {
  extern __shared__ __align__(16) unsigned char dyn[];
  double* x = reinterpret_cast<double*>(dyn);  // [nbin]
  __shared__ double seg[64];
  const int r = blockIdx.x, lane = threadIdx.x;
  const double* row = rows + (size_t)r * nbin;
  for (int j = lane; j < nbin; j += 64) x[j] = row[j];
  __syncthreads();
  // window of smallest sum (first start on ties)
  double best = INFINITY;
  int bj = 0x7fffffff;
  for (int j = lane; j < nbin; j += 64) {
    double b = 0.0;
    int k = j;
    for (int i = 0; i < width; ++i) {
      b += x[k];
      if (++k == nbin) k = 0;
    }
    if (b < best || (b == best && j < bj)) { best = b; bj = j; }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    const double ob = __shfl_xor(best, o);
    const int oj = __shfl_xor(bj, o);
    if (ob < best || (ob == best && oj < bj)) { best = ob; bj = oj; }
  }
  const int j0 = bj;
  // window mean and sample variance (serial over the window, lane 0's order
  // is the window's own: one pass for the mean, one for the squares)
  double m = 0.0, v = 0.0;
  if (lane == 0) {
    int k = j0;
    for (int i = 0; i < width; ++i) {
      m += x[k];
      if (++k == nbin) k = 0;
    }
    m /= (double)width;
    k = j0;
    for (int i = 0; i < width; ++i) {
      const double d = x[k] - m;
      v += d * d;
      if (++k == nbin) k = 0;
    }
    v = width > 1 ? v / (double)(width - 1) : 0.0;
  }
  m = __shfl(m, 0);
  v = __shfl(v, 0);
  // running sum of y = x - m from the bin after the window, in lane segments
  const int start = (j0 + width) % nbin;
  const int per = (nbin + 63) / 64;
  const int i0 = min(nbin, lane * per), i1 = min(nbin, i0 + per);
  double s = 0.0;
  for (int i = i0; i < i1; ++i) {
    int k = start + i;
    if (k >= nbin) k -= nbin;
    s += x[k] - m;
  }
  seg[lane] = s;
  __syncthreads();
  if (lane == 0) {
    double c = 0.0;
    for (int q = 0; q < 64; ++q) {
      const double t = seg[q];
      seg[q] = c;  // exclusive prefix
      c += t;
    }
    best = c;  // total C on lane 0
  }
  __syncthreads();
  const double C = __shfl(best, 0);
  // first crossings of thr C and (1 - thr) C: each lane rescans its segment
  int rise = 0x7fffffff, fall = 0x7fffffff;
  double crise = 0.0, cfall = 0.0, yrise = 0.0;
  {
    double c = seg[lane];
    for (int i = i0; i < i1; ++i) {
      int k = start + i;
      if (k >= nbin) k -= nbin;
      const double y = x[k] - m;
      c += y;
      if (rise == 0x7fffffff && c >= thr * C) { rise = i; crise = c; yrise = y; }
      if (fall == 0x7fffffff && c >= (1.0 - thr) * C) { fall = i; cfall = c; }
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    const int orise = __shfl_xor(rise, o), ofall = __shfl_xor(fall, o);
    const double ocr = __shfl_xor(crise, o), oyr = __shfl_xor(yrise, o),
                 ocf = __shfl_xor(cfall, o);
    if (orise < rise) { rise = orise; crise = ocr; yrise = oyr; }
    if (ofall < fall) { fall = ofall; cfall = ocf; }
  }
  if (lane == 0) {
    double snr = 0.0;
    if (C > 0.0 && v > 0.0 && rise != 0x7fffffff && fall != 0x7fffffff && fall >= rise)
      snr = (cfall - crise + yrise) / sqrt((double)(fall - rise + 1)) / sqrt(v);
    out[r] = snr;
  }
}

template __global__ void k_unpack<uint8_t>(const uint8_t*, const double*, const double*, int, int,
                                           int, int, int, double*);
template __global__ void k_unpack<int16_t>(const int16_t*, const double*, const double*, int, int,
                                           int, int, int, double*);
template __global__ void k_unpack<float>(const float*, const double*, const double*, int, int, int,
                                         int, int, double*);

}  // namespace ppf
