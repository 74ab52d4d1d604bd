// ppfit_generic.hip -- rfft-based kernels of libppfit for any nbin (gfx950).
//
// The reference transforms profiles with numpy's rfft / irfft of whatever
// length the archive has (pptoaslib.py:976-978, pplib.py:2338-2426).  The
// register and LDS FFTs of ppfit_spectra.hip are built per power of two; for
// every other nbin in [64, 8192] these kernels take their place in the fit
// entry point, the template spectra, the row rotations, FFTFIT, the noise
// rows, irfft, the zapping residuals and ppalign's rotate-and-sum: the same
// outputs from direct sums, O(nbin^2) per row instead of O(nbin log nbin).
//
// Bin k of a real row: D_k = sum_m x_m e^{-2 pi i m k / nbin}.  The phasor
// advances by one complex product per term and is re-seeded from the twiddle
// table at the exact index (m k) mod nbin every kSeed terms, so its rounding
// never grows past kSeed products (relative error ~1e-15, against the
// north_star tolerance of 1e-3 sigma on the fitted parameters).
#include "ppfit_kernels.hpp"

namespace ppf {

constexpr int kSeed = 32;

// D_k of x[0 .. nbin) (LDS); tw[j] = e^{-2 pi i j / nbin}, k < nbin.  The
// real input's symmetry halves the work: terms m and nbin - m share the
// phasor, D_k = x_0 + sum_{1 <= m < nbin/2} [(x_m + x_{nbin-m}) cos -
// i (x_m - x_{nbin-m}) sin](2 pi m k / nbin) + [nbin even] (-1)^k x_{nbin/2}.
__device__ __forceinline__ double2 dft_bin(const double* x, int nbin, int k,
                                           const double2* __restrict__ tw) {
  const double2 w = tw[k];
  const int M = (nbin - 1) / 2;  // pairs m = 1 .. M
  const int step = (int)(((long long)kSeed * k) % nbin);
  double re = x[0], im = 0.0;
  int seed = k;  // (m0 k) mod nbin at m0 = 1
  for (int m0 = 1; m0 <= M; m0 += kSeed) {
    double2 e = tw[seed];
    const int me = min(m0 + kSeed - 1, M);
    for (int m = m0; m <= me; ++m) {
      const double a = x[m], b = x[nbin - m];
      re = fma(a + b, e.x, re);
      im = fma(a - b, e.y, im);
      e = cmul(e, w);
    }
    seed += step;
    if (seed >= nbin) seed -= nbin;
  }
  if (!(nbin & 1)) re += (k & 1) ? -x[nbin / 2] : x[nbin / 2];
  return cmk(re, im);
}

// Two bins at once (k1, k2 < nbin): the same sums as dft_bin for each, the
// loads and pair sums shared and the two phasor chains interleaved.
__device__ __forceinline__ void dft_bin2(const double* x, int nbin, int k1, int k2,
                                         const double2* __restrict__ tw, double2& d1,
                                         double2& d2) {
  const double2 w1 = tw[k1], w2 = tw[k2];
  const int M = (nbin - 1) / 2;
  const int step1 = (int)(((long long)kSeed * k1) % nbin);
  const int step2 = (int)(((long long)kSeed * k2) % nbin);
  double re1 = x[0], im1 = 0.0, re2 = x[0], im2 = 0.0;
  int seed1 = k1, seed2 = k2;
  for (int m0 = 1; m0 <= M; m0 += kSeed) {
    double2 e1 = tw[seed1], e2 = tw[seed2];
    const int me = min(m0 + kSeed - 1, M);
    for (int m = m0; m <= me; ++m) {
      const double a = x[m], b = x[nbin - m];
      const double sp = a + b, sm = a - b;
      re1 = fma(sp, e1.x, re1);
      im1 = fma(sm, e1.y, im1);
      re2 = fma(sp, e2.x, re2);
      im2 = fma(sm, e2.y, im2);
      e1 = cmul(e1, w1);
      e2 = cmul(e2, w2);
    }
    seed1 += step1;
    if (seed1 >= nbin) seed1 -= nbin;
    seed2 += step2;
    if (seed2 >= nbin) seed2 -= nbin;
  }
  if (!(nbin & 1)) {
    const double xn = x[nbin / 2];
    re1 += (k1 & 1) ? -xn : xn;
    re2 += (k2 & 1) ? -xn : xn;
  }
  d1 = cmk(re1, im1);
  d2 = cmk(re2, im2);
}

// f(k, D_k) for every bin k < kend of the row, each thread taking k = tid +
// blockDim q in increasing q (the order of the one-bin loop), two at a time
template <typename F>
__device__ __forceinline__ void dft_each_bin(const double* x, int nbin, int kend,
                                             const double2* __restrict__ tw, F&& f) {
  const int nt = blockDim.x;
  for (int k = threadIdx.x; k < kend; k += 2 * nt) {
    const int k2 = k + nt;
    double2 d1, d2;
    dft_bin2(x, nbin, k, k2 < kend ? k2 : k, tw, d1, d2);
    f(k, d1);
    if (k2 < kend) f(k2, d2);
  }
}

// numpy irfft(X, n = nbin) at samples m and nbin - m (1 <= m < nbin/2):
// with A = sum_{1 <= k <= K} Re X_k cos(2 pi m k / nbin) and B = sum Im X_k
// sin(..), K = (nbin - 1) / 2, the two samples are (Re X_0 + 2 (A -+ B) +
// [nbin even] (-1)^m Re X_{nbin/2}) / nbin; m = 0 (and m = nbin/2) alone,
// with B = 0.  X[0 .. nbin/2] in LDS.
__device__ __forceinline__ void idft_pair(const double2* X, int nbin, int m,
                                          const double2* __restrict__ tw, double& out_m,
                                          double& out_nm) {
  const double2 w = cconj(tw[m]);  // e^{+2 pi i m / nbin}
  const int K = (nbin - 1) / 2;
  const int step = (int)(((long long)kSeed * m) % nbin);
  double A = 0.0, B = 0.0;
  int seed = m;  // (k0 m) mod nbin at k0 = 1
  for (int k0 = 1; k0 <= K; k0 += kSeed) {
    double2 e = cconj(tw[seed]);
    const int ke = min(k0 + kSeed - 1, K);
    for (int k = k0; k <= ke; ++k) {
      const double2 x = X[k];
      A = fma(x.x, e.x, A);
      B = fma(x.y, e.y, B);
      e = cmul(e, w);
    }
    seed += step;
    if (seed >= nbin) seed -= nbin;
  }
  double ny = 0.0;
  if (!(nbin & 1)) ny = (m & 1) ? -X[nbin / 2].x : X[nbin / 2].x;
  const double inv = 1.0 / (double)nbin;
  out_m = (fma(2.0, A - B, X[0].x) + ny) * inv;
  out_nm = (fma(2.0, A + B, X[0].x) + ny) * inv;
}

// every sample of irfft(X, n = nbin) into out[0 .. nbin), the block's threads
// taking the pairs (m, nbin - m)
__device__ __forceinline__ void idft_row(const double2* X, int nbin, const double2* __restrict__ tw,
                                         double* __restrict__ out) {
  const int half = nbin / 2;
  for (int m = threadIdx.x; m <= half; m += blockDim.x) {
    double a, b;
    idft_pair(X, nbin, m, tw, a, b);
    out[m] = a;
    if (m > 0 && nbin - m != m) out[nbin - m] = b;
  }
}

__device__ __forceinline__ void load_real_row(double* x, const double* __restrict__ row, int nbin) {
  for (int m = threadIdx.x; m < nbin; m += blockDim.x) x[m] = row[m];
}

// k_model_spec for any nbin: M[row][k], k <= nbin/2 (DC zeroed when
// zero_dc), zero padding up to NHP, p_n = sum_{k>=1} |M_k|^2, |M_k|^2 rows.
// Dynamic LDS: nbin doubles.
__global__ __launch_bounds__(kBlock) void k_model_spec_gen(const double* __restrict__ model,
                                                           double2* __restrict__ M,
                                                           double* __restrict__ pn, int NHP,
                                                           int zero_dc,
                                                           const double2* __restrict__ tw,
                                                           double* __restrict__ M2, int nbin) {
  extern __shared__ __align__(16) unsigned char gsm[];
  double* x = reinterpret_cast<double*>(gsm);
  __shared__ double red[kWaves];
  const int row = blockIdx.x, NH = nbin / 2 + 1;
  load_real_row(x, model + (size_t)row * nbin, nbin);
  __syncthreads();
  double p = 0.0;
  double2* out = M + (size_t)row * NHP;
  for (int k = threadIdx.x; k < NHP; k += kBlock) {
    double2 v = cmk(0.0, 0.0);
    if (k < NH) v = dft_bin(x, nbin, k, tw);
    if (k == 0 && zero_dc) v = cmk(0.0, 0.0);
    if (k >= 1 && k < NH) p += cabs2(v);
    out[k] = v;
    if (M2) M2[(size_t)row * NHP + k] = cabs2(v);
  }
  p = block_sum(p, red);
  if (threadIdx.x == 0 && pn) pn[row] = p;
}

// k_data_xspec for any nbin: one workgroup per subint, its channel rows in
// order.  Per fitted channel: D = rfft(row); sig = errs or get_noise_PS
// (pplib.py:2227-2253); dsum = sum_{k>=1} |D_k|^2; X_k = D_k conj(M_k) (0 at
// k = 0); R_k += w_n D_k e^{2 pi i k phi_n} (the guess's dedispersed, weighted
// average, pptoas.py:421-423), each R_k summed by one thread in channel order.
// Masked channels: sig = dsum = 0 and a zero X row.  No data-spectrum cache
// (the entry point refuses PPF_SPEC_* for these lengths).  Dynamic LDS: nbin
// doubles.
__global__ __launch_bounds__(kBlock) void k_data_xspec_gen(SpecArgs a, int nbin) {
  extern __shared__ __align__(16) unsigned char gsm[];
  double* x = reinterpret_cast<double*>(gsm);
  __shared__ double s_meta[4];
  __shared__ double red[kWaves];
  const int c = blockIdx.x, s = a.sub0 + c, tid = threadIdx.x;
  const int nchan = a.nchan, NH = nbin / 2 + 1;
  const double* fr = a.freqs + (size_t)s * nchan;
  const uint8_t* mask = a.mask ? a.mask + (size_t)s * nchan : nullptr;
  // nu_g (guess dedispersion reference): mean over fitted channels unless given
  if (tid == 0) {
    double fs = 0.0, ws = 0.0;
    int nok = 0;
    for (int q = 0; q < nchan; ++q) {
      if (mask && !mask[q]) continue;
      fs += fr[q];
      ws += a.weights ? a.weights[(size_t)s * nchan + q] : 1.0;
      ++nok;
    }
    double nug = a.guess_nu ? a.guess_nu[s] : NAN;
    if (isnan(nug)) nug = fs / nok;
    s_meta[0] = nug;
    s_meta[1] = ws;
    s_meta[2] = (double)nok;
    s_meta[3] = a.init ? a.init[(size_t)s * 5 + 1] : 0.0;
  }
  __syncthreads();
  const double nug2 = 1.0 / (s_meta[0] * s_meta[0]);
  const double wsum = s_meta[1];
  const double Dfac = kDconst * s_meta[3] / a.P[s];
  const int midx = a.model_idx ? a.model_idx[s] : 0;
  double2* Rr = a.R + (size_t)c * a.NHP;
  if (a.guess)
    for (int k = tid; k < a.NHP; k += kBlock) Rr[k] = cmk(0.0, 0.0);
  for (int n = 0; n < nchan; ++n) {
    double2* Xr = a.X + ((size_t)c * nchan + n) * a.NHP;
    if (mask && !mask[n]) {
      if (tid == 0) { a.sig[(size_t)c * nchan + n] = 0.0; a.dsum[(size_t)c * nchan + n] = 0.0; }
      for (int k = tid; k < a.NHP; k += kBlock) Xr[k] = cmk(0.0, 0.0);
      continue;
    }
    __syncthreads();  // the previous row's readers are done with x
    load_real_row(x, a.data + ((size_t)s * nchan + n) * nbin, nbin);
    __syncthreads();
    const double2* Mr = a.M + ((size_t)midx * nchan + n) * a.NHP;
    const double phi = Dfac * (1.0 / (fr[n] * fr[n]) - nug2);
    const double wq = a.weights ? a.weights[(size_t)s * nchan + n] : 1.0;
    double pn = 0.0, pd = 0.0;
    dft_each_bin(x, nbin, NH, a.tw, [&](int k, double2 d) {
      const double p2 = cabs2(d);
      if (k >= a.kc) pn += p2;
      if (k >= 1) pd += p2;
      Xr[k] = k >= 1 ? cmulc(d, Mr[k]) : cmk(0.0, 0.0);
      if (a.guess) Rr[k] = cadd(Rr[k], cmul(d, cscale(turn_phasor((double)k, phi), wq)));
    });
    for (int k = NH + tid; k < a.NHP; k += kBlock) Xr[k] = cmk(0.0, 0.0);
    pn = block_sum(pn, red);
    pd = block_sum(pd, red);
    if (tid == 0) {
      double sig = a.errs ? a.errs[(size_t)s * nchan + n] : NAN;
      if (isnan(sig)) sig = sqrt(pn / (double)nbin / (double)(NH - a.kc));
      a.sig[(size_t)c * nchan + n] = sig;
      a.dsum[(size_t)c * nchan + n] = pd;
    }
  }
  if (a.guess) {
    const double iw = 1.0 / wsum;
    for (int k = tid; k < a.NHP; k += kBlock) {
      double2 r = cmk(0.0, 0.0);
      if (k < NH) {
        r = cscale(Rr[k], iw);  // summed by this same thread
        if (k == 0) r = cmk(0.0, 0.0);
        if (!(nbin & 1) && k == nbin / 2) r.y = 0.0;  // irfft drops Im(X_N)
      }
      Rr[k] = r;
    }
  }
}

// k_rotate_rows for any nbin: rfft, times e^{2 pi i k phase} (rotate_data,
// pplib.py:2406-2415), divided by 1 + 2 pi i k tau (scattering_portrait_FT,
// pplib.py:4081-4101) when tau is given, irfft.  in == out is supported: the
// whole row is read before the first barrier.  Dynamic LDS: nbin doubles +
// (nbin/2 + 1) double2.
__global__ __launch_bounds__(kBlock) void k_rotate_rows_gen(const double* in,
                                                            const double* __restrict__ phase,
                                                            const double* __restrict__ tau,
                                                            double* out,
                                                            const double2* __restrict__ tw,
                                                            int nbin) {
  extern __shared__ __align__(16) unsigned char gsm[];
  double* x = reinterpret_cast<double*>(gsm);
  double2* X = reinterpret_cast<double2*>(gsm + (((size_t)nbin * sizeof(double) + 15) & ~(size_t)15));
  const int r = blockIdx.x, NH = nbin / 2 + 1;
  load_real_row(x, in + (size_t)r * nbin, nbin);
  __syncthreads();
  const double ph = phase ? phase[r] : 0.0;
  const double t2 = tau ? 2.0 * M_PI * tau[r] : 0.0;
  for (int k = threadIdx.x; k < NH; k += kBlock) {
    double2 v = dft_bin(x, nbin, k, tw);
    if (phase) v = cmul(v, turn_phasor((double)k, ph));
    if (t2 != 0.0) {
      const double w = t2 * (double)k, d = 1.0 / fma(w, w, 1.0);
      v = cmk(fma(v.y, w, v.x) * d, fma(-v.x, w, v.y) * d);
    }
    X[k] = v;
  }
  __syncthreads();
  idft_row(X, nbin, tw, out + (size_t)r * nbin);
}

// LDS layout of the kernels below: a real row (nbin doubles, 16-B aligned
// end) followed by one spectrum (nbin/2 + 1 double2)
__device__ __forceinline__ double2* gen_spec_after_row(unsigned char* sm, int nbin) {
  return reinterpret_cast<double2*>(sm + (((size_t)nbin * sizeof(double) + 15) & ~(size_t)15));
}

// k_phase_shift for any nbin: fit_phase_shift (pplib.py:2054-2100) on each
// profile -- spectrum, noise, then the shared brute-force + Nelder-Mead
// search (guess_search) on rm_k = D_k conj(M_k).
__global__ __launch_bounds__(kBlock) void k_phase_shift_gen(PhaseShiftArgs a, int nbin) {
  extern __shared__ __align__(16) unsigned char gsm[];
  double* x = reinterpret_cast<double*>(gsm);
  double2* rm = gen_spec_after_row(gsm, nbin);
  __shared__ GuessShared gs;
  const int r = blockIdx.x, tid = threadIdx.x, NH = nbin / 2 + 1;
  load_real_row(x, a.data + (size_t)r * nbin, nbin);
  __syncthreads();
  const int midx = a.model_idx ? a.model_idx[r] : 0;
  const double2* Mr = a.M + (size_t)midx * a.NHP;
  double pnoise = 0.0, dd = 0.0, pp = 0.0;
  for (int k = tid; k < NH; k += kBlock) {
    double2 v = dft_bin(x, nbin, k, a.tw);
    if (k >= a.kc) pnoise += cabs2(v);
    if (k == 0) v = cmk(0.0, 0.0);
    dd += cabs2(v);
    pp += cabs2(Mr[k]);
    rm[k] = cmulc(v, Mr[k]);
  }
  pnoise = block_sum(pnoise, gs.red);
  dd = block_sum(dd, gs.red);
  pp = block_sum(pp, gs.red);
  double noise = a.noise ? a.noise[r] : NAN;
  if (isnan(noise)) noise = sqrt(pnoise / (double)nbin / (double)(NH - a.kc));
  const double err = noise * sqrt(0.5 * (double)nbin);
  const double ie2 = 1.0 / (err * err);
  guess_search(rm, NH, ie2, a.Ns, a.lo, a.hi, gs);
  if (tid == 0) {
    const double fmin = gs.fx;
    gs.out[0] = gs.x;
    gs.out[1] = -fmin / (pp * ie2);
    gs.out[2] = dd * ie2;
    gs.out[3] = pp * ie2;
    gs.out[4] = fmin;
  }
  __syncthreads();
  double c2 = 0.0;  // second derivative at the phase (pplib.py:1270-1280)
  for (int k = tid; k < NH; k += kBlock) {
    const double2 w = cmul(rm[k], turn_phasor((double)k, gs.out[0]));
    c2 += (double)k * (double)k * w.x;
  }
  c2 = block_sum(c2, gs.red);
  if (tid == 0) {
    const double d2 = 4.0 * kPi * kPi * c2 * ie2;
    const double scale = gs.out[1], d = gs.out[2], p = gs.out[3], fmin = gs.out[4];
    double* o = a.out + (size_t)r * 6;
    o[0] = gs.out[0];
    o[1] = pow(scale * d2, -0.5);
    o[2] = scale;
    o[3] = pow(p, -0.5);
    o[4] = pow(scale * scale * p, 0.5);
    o[5] = (d - fmin * fmin / p) / (double)(nbin - 2);
  }
}

// spec[r][k] = rfft(in[r])[k], k <= nbin/2 (numpy layout)
__global__ __launch_bounds__(kBlock) void k_rfft_rows_gen(const double* __restrict__ in,
                                                          double2* __restrict__ spec,
                                                          const double2* __restrict__ tw, int nbin) {
  extern __shared__ __align__(16) unsigned char gsm[];
  double* x = reinterpret_cast<double*>(gsm);
  const int r = blockIdx.x, NH = nbin / 2 + 1;
  load_real_row(x, in + (size_t)r * nbin, nbin);
  __syncthreads();
  for (int k = threadIdx.x; k < NH; k += kBlock) spec[(size_t)r * NH + k] = dft_bin(x, nbin, k, tw);
}

// out[r] = irfft(spec[r], n = nbin)
__global__ __launch_bounds__(kBlock) void k_irfft_rows_gen(const double2* __restrict__ spec,
                                                           double* __restrict__ out,
                                                           const double2* __restrict__ tw,
                                                           int nbin) {
  extern __shared__ __align__(16) unsigned char gsm[];
  double2* X = reinterpret_cast<double2*>(gsm);
  const int r = blockIdx.x, NH = nbin / 2 + 1;
  for (int k = threadIdx.x; k < NH; k += kBlock) X[k] = spec[(size_t)r * NH + k];
  __syncthreads();
  idft_row(X, nbin, tw, out + (size_t)r * nbin);
}

// get_noise_PS per row (pplib.py:2227-2253)
__global__ __launch_bounds__(kBlock) void k_noise_rows_gen(const double* __restrict__ in,
                                                           double* __restrict__ out, int kc,
                                                           const double2* __restrict__ tw,
                                                           int nbin) {
  extern __shared__ __align__(16) unsigned char gsm[];
  double* x = reinterpret_cast<double*>(gsm);
  __shared__ double red[kWaves];
  const int r = blockIdx.x, NH = nbin / 2 + 1;
  load_real_row(x, in + (size_t)r * nbin, nbin);
  __syncthreads();
  double p = 0.0;
  for (int k = kc + threadIdx.x; k < NH; k += kBlock) p += cabs2(dft_bin(x, nbin, k, tw));
  p = block_sum(p, red);
  if (threadIdx.x == 0) out[r] = sqrt(p / (double)nbin / (double)(NH - kc));
}

// ppalign's weighted rotate-and-sum (ppalign.py:202-208) for any nbin:
// partial[p][n][k] = sum_{s in slice p} w[s][n] rfft(data[s][n])_k e^{2 pi i k ph[s][n]},
// each k summed by one thread in subint order.
__global__ __launch_bounds__(kBlock) void k_rot_accum_gen(const double* __restrict__ data,
                                                          const double* __restrict__ phase,
                                                          const double* __restrict__ weight,
                                                          double2* __restrict__ partial, int nsub,
                                                          int nchan, int nsplit,
                                                          const double2* __restrict__ tw,
                                                          int nbin) {
  extern __shared__ __align__(16) unsigned char gsm[];
  double* x = reinterpret_cast<double*>(gsm);
  const int n = blockIdx.x % nchan, p = blockIdx.x / nchan, NH = nbin / 2 + 1;
  const int per = (nsub + nsplit - 1) / nsplit;
  const int s0 = p * per, s1 = min(nsub, s0 + per);
  double2* out = partial + ((size_t)p * nchan + n) * NH;
  for (int k = threadIdx.x; k < NH; k += kBlock) out[k] = cmk(0.0, 0.0);
  for (int s = s0; s < s1; ++s) {
    const size_t row = (size_t)s * nchan + n;
    const double w = weight[row];
    if (w == 0.0) continue;  // uniform per block
    __syncthreads();
    load_real_row(x, data + row * nbin, nbin);
    __syncthreads();
    const double ph = phase[row];
    for (int k = threadIdx.x; k < NH; k += kBlock)
      out[k] = cadd(out[k], cscale(cmul(dft_bin(x, nbin, k, tw), turn_phasor((double)k, ph)), w));
  }
}

// k_resid_chi2 for any nbin (pptoas.py:1389-1402, get_red_chi2 pplib.py:727-749):
// Parseval on R = D e^{2 pi i k phase} - scale M / (1 + 2 pi i k tau); irfft
// keeps only Re R_0 (and Re R_{nbin/2} for even nbin).
__global__ __launch_bounds__(kBlock) void k_resid_chi2_gen(ResidArgs a,
                                                           const double2* __restrict__ tw,
                                                           int nbin) {
  extern __shared__ __align__(16) unsigned char gsm[];
  double* x = reinterpret_cast<double*>(gsm);
  double2* D = gen_spec_after_row(gsm, nbin);
  __shared__ double red[kWaves];
  const int r = blockIdx.x, NH = nbin / 2 + 1;
  load_real_row(x, a.data + (size_t)r * nbin, nbin);
  __syncthreads();
  const double ph = a.phase ? a.phase[r] : 0.0;
  for (int k = threadIdx.x; k < NH; k += kBlock)
    D[k] = cmul(dft_bin(x, nbin, k, tw), turn_phasor((double)k, ph));
  __syncthreads();
  load_real_row(x, a.model + (size_t)(a.model_row ? a.model_row[r] : r) * nbin, nbin);
  __syncthreads();
  const double sc = a.scale[r];
  const double t2 = a.tau ? 2.0 * M_PI * a.tau[r] : 0.0;
  double acc = 0.0;
  for (int k = threadIdx.x; k < NH; k += kBlock) {
    double2 m = dft_bin(x, nbin, k, tw);
    if (t2 != 0.0) {
      const double w = t2 * (double)k, d = 1.0 / fma(w, w, 1.0);
      m = cmk(fma(m.y, w, m.x) * d, fma(-m.x, w, m.y) * d);
    }
    const double2 q = cmk(fma(-sc, m.x, D[k].x), fma(-sc, m.y, D[k].y));
    const bool real_only = k == 0 || (!(nbin & 1) && k == nbin / 2);
    acc += real_only ? q.x * q.x : 2.0 * cabs2(q);
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) {
    const double e = a.errs[r];
    a.out[r] = acc / (double)nbin / (e * e) / a.dof;
  }
}

}  // namespace ppf
