// ppfit_generic.hip -- rfft-based kernels of libppfit for any nbin (gfx950).
//
// The reference transforms profiles with numpy's rfft / irfft of whatever
// length the archive has (pptoaslib.py:976-978, pplib.py:2338-2426).  The
// register and LDS FFTs of ppfit_spectra.hip are built per power of two; for
// every other nbin in [16, 8192] these kernels take their place in the fit
// entry point, the template spectra, the row rotations, FFTFIT, the noise
// rows, irfft, the zapping residuals and ppalign's rotate-and-sum: the same
// outputs from direct sums, O(nbin^2) per row instead of O(nbin log nbin).
//
// Bin k of a real row: D_k = sum_m x_m e^{-2 pi i m k / nbin}.  The fit's
// data pass forms all of them as a GEMM on the fp64 matrix cores against
// the twiddle table (k_dft_rows_mfma); the other row kernels sum one bin per
// thread, the phasor advancing by one complex product per term and re-seeded
// from the table at the exact index (m k) mod nbin every kSeed terms, so its
// rounding never grows past kSeed products (relative error ~1e-15, against
// the north_star tolerance of 1e-3 sigma on the fitted parameters).
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

// ---------------------------------------------------------------------------
// The data pass's transforms on the fp64 matrix cores: D = rfft of every row
// of the chunk as two GEMMs over the pair index m' = 1 .. M = (nbin - 1) / 2,
//   Re D_k = x_0 + [even] (-1)^k x_{nbin/2} + sum_m' (x_m' + x_{nbin-m'}) cos(2 pi m' k / nbin)
//   Im D_k =                                sum_m' (x_m' - x_{nbin-m'}) (-sin)(2 pi m' k / nbin)
// (dft_bin's sums, with every cos / sin an exact table value tw[(m' k) mod
// nbin] instead of a phasor chain).  Workgroup: 16 kGenRT rows x 256 bins,
// wave w the bins k0 + 64 w .. + 63 as four 16 x 16 tiles per row tile; per step of 4 pair
// indices one v_mfma_f64_16x16x4 per tile and part, A = the 16 rows' pair
// sums (lane l: row l & 15, m' = m0 + (l >> 4)), B = the table values
// (lane l: m' = m0 + (l >> 4), bin l & 15 of the tile).  Output: D into the
// X rows (k < nbin/2 + 1); k_data_post_gen turns them into X in place.
// ---------------------------------------------------------------------------
typedef double gen_f64x4 __attribute__((ext_vector_type(4)));
constexpr int kGenLdsTw = 4096;  // 64 KB of LDS

// LTW: the twiddle table staged in LDS (nbin <= kGenLdsTw), else read from L2.
// Each workgroup takes kGenRT tiles of 16 rows, so every table value a lane
// gathers feeds kGenRT MFMAs per part; the rows' pair sums go through LDS in
// chunks of kGenChunk pair indices, loaded coalesced (16 threads per row
// segment) by the whole workgroup.
#ifndef PPF_DFT_RT
#define PPF_DFT_RT 2  // A/B knob: row tiles per workgroup
#endif
constexpr int kGenChunk = 64;
constexpr int kGenRT = PPF_DFT_RT;
constexpr int kGenRows = 16 * kGenRT;
inline size_t dft_mfma_lds(int nbin, bool ltw) {
  return (ltw ? (size_t)nbin * sizeof(double2) : 0) +
         2 * (size_t)kGenChunk * kGenRows * sizeof(double);
}
template <bool LTW>
__global__ __launch_bounds__(kBlock) void k_dft_rows_mfma(const double* __restrict__ rows,
                                                          double2* __restrict__ D, int nrows,
                                                          int nbin, int NHP,
                                                          const double2* __restrict__ twg) {
  extern __shared__ __align__(16) unsigned char gsm[];
  const double2* tw = twg;
  double* sp_l = reinterpret_cast<double*>(gsm + (LTW ? (size_t)nbin * sizeof(double2) : 0));
  double* sm_l = sp_l + kGenChunk * kGenRows;
  if constexpr (LTW) {
    double2* t = reinterpret_cast<double2*>(gsm);
    for (int i = threadIdx.x; i < nbin; i += kBlock) t[i] = twg[i];
    tw = t;  // published by the chunk loop's first barrier
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int row0 = blockIdx.x * kGenRows, k0 = blockIdx.y * 256 + w * 64;
  const int NH = nbin / 2 + 1, M = (nbin - 1) / 2;
  const bool active = k0 < NH;  // wave-uniform: the wave has bins to compute
  const int ri = lane & 15, kk = lane >> 4;
  // the chunk loader: thread t fills pair indices 4 (t & 15) .. + 3 of rows
  // (t >> 4) + 16 q, q < kGenRT
  const int lr = tid >> 4, lq = tid & 15;
  // per tile j: the lane's bin and the table index (m' k) mod nbin at m' = 1 + kk
  int kj[4], idx[4], stp[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = k0 + 16 * j + ri;
    kj[j] = k < NH ? k : 0;  // bins past the end compute bin 0, never stored
    idx[j] = (int)(((long long)(1 + kk) * kj[j]) % nbin);
    stp[j] = (int)((4LL * kj[j]) % nbin);
  }
  gen_f64x4 cre[kGenRT][4], cim[kGenRT][4];
#pragma unroll
  for (int q = 0; q < kGenRT; ++q)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cre[q][j] = (gen_f64x4){0.0, 0.0, 0.0, 0.0};
      cim[q][j] = cre[q][j];
    }
  for (int c0 = 1; c0 <= M; c0 += kGenChunk) {
    __syncthreads();  // the previous chunk has been consumed
#pragma unroll
    for (int q = 0; q < kGenRT; ++q) {
      const int lrow = lr + 16 * q;
      const bool ok = row0 + lrow < nrows;
      const double* xl = rows + (size_t)(ok ? row0 + lrow : 0) * nbin;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mm = 4 * lq + i, m = c0 + mm;
        double a = 0.0, b = 0.0;
        if (ok && m <= M) {
          a = xl[m];
          b = xl[nbin - m];
        }
        sp_l[mm * kGenRows + lrow] = a + b;
        sm_l[mm * kGenRows + lrow] = a - b;
      }
    }
    __syncthreads();
    if (active) {
      const int nst = min(kGenChunk / 4, (M - c0) / 4 + 1);  // steps with any m' <= M
      for (int st = 0; st < nst; ++st) {
        double sp[kGenRT], sm[kGenRT];
#pragma unroll
        for (int q = 0; q < kGenRT; ++q) {
          sp[q] = sp_l[(4 * st + kk) * kGenRows + 16 * q + ri];
          sm[q] = sm_l[(4 * st + kk) * kGenRows + 16 * q + ri];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const double2 t = tw[idx[j]];
#pragma unroll
          for (int q = 0; q < kGenRT; ++q) {
            cre[q][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(sp[q], t.x, cre[q][j], 0, 0, 0);
            cim[q][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(sm[q], t.y, cim[q][j], 0, 0, 0);
          }
          idx[j] += stp[j];
          if (idx[j] >= nbin) idx[j] -= nbin;
        }
      }
    }
  }
  if (!active) return;
  // lane l holds rows (l >> 4) + 4 r of each row tile, bin l & 15 of each bin tile
#pragma unroll
  for (int q = 0; q < kGenRT; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 16 * q + kk + 4 * r;
      if (row >= nrows) continue;
      const double* xo = rows + (size_t)row * nbin;
      const double x0 = xo[0], xn = (nbin & 1) ? 0.0 : xo[nbin / 2];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + 16 * j + ri;
        if (k < NH) {
          const double re = cre[q][j][r] + x0 + ((k & 1) ? -xn : xn);
          D[(size_t)row * NHP + k] = cmk(re, cim[q][j][r]);
        }
      }
    }
}

// The data pass's per-subint part (k_data_xspec's outputs for any nbin) from
// the spectra k_dft_rows_mfma left in the X rows -- or, with the data-spectrum
// cache (a.D), in the cache's rows: sig, dsum, the guess average R (each R_k
// summed by one thread in channel order) and X = D conj(M) (0 at k = 0 and
// past nbin/2), in place or into X.  As k_data_xspec: under PPF_SPEC_STORE /
// _USE the Taylor-path subints get no X (their moment passes form it from
// D), under _USE they are not visited at all, and STORE leaves masked rows
// and the padding of the cached D rows zero.
__global__ __launch_bounds__(kBlock) void k_data_post_gen(SpecArgs a, int nbin) {
  __shared__ double s_meta[4];
  __shared__ double red[kWaves];
  const int c = blockIdx.x, s = a.sub0 + c, tid = threadIdx.x;
  const bool tsub = a.D && spec_taylor_sub(a, s);
  if (a.spec_mode == PPF_SPEC_USE && tsub) return;  // all of it cached
  const bool wx = !tsub;                                      // X rows wanted
  const bool wd = a.D != nullptr && a.spec_mode == PPF_SPEC_STORE;  // cache rows to tidy
  const int nchan = a.nchan, NH = nbin / 2 + 1;
  const double* fr = a.freqs + (size_t)s * nchan;
  const uint8_t* mask = a.mask ? a.mask + (size_t)s * nchan : nullptr;
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
    double2* Dr = a.D ? a.D + ((size_t)c * nchan + n) * a.NHP : Xr;  // the spectra
    if (mask && !mask[n]) {
      if (tid == 0) { a.sig[(size_t)c * nchan + n] = 0.0; a.dsum[(size_t)c * nchan + n] = 0.0; }
      for (int k = tid; k < a.NHP; k += kBlock) {
        if (wx) Xr[k] = cmk(0.0, 0.0);
        if (wd) Dr[k] = cmk(0.0, 0.0);
      }
      continue;
    }
    const double2* Mr = a.M + ((size_t)midx * nchan + n) * a.NHP;
    const double phi = Dfac * (1.0 / (fr[n] * fr[n]) - nug2);
    const double wq = a.weights ? a.weights[(size_t)s * nchan + n] : 1.0;
    double pn = 0.0, pd = 0.0;
    for (int k = tid; k < a.NHP; k += kBlock) {
      double2 xk = cmk(0.0, 0.0);
      if (k < NH) {
        const double2 d = Dr[k];
        const double p2 = cabs2(d);
        if (k >= a.kc) pn += p2;
        if (k >= 1) pd += p2;
        if (k >= 1) xk = cmulc(d, Mr[k]);
        if (a.guess) Rr[k] = cadd(Rr[k], cmul(d, cscale(turn_phasor((double)k, phi), wq)));
      } else if (wd) {
        Dr[k] = cmk(0.0, 0.0);
      }
      if (wx) Xr[k] = xk;
    }
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
        r = cscale(Rr[k], iw);
        if (k == 0) r = cmk(0.0, 0.0);
        if (!(nbin & 1) && k == nbin / 2) r.y = 0.0;
      }
      Rr[k] = r;
    }
  }
}

// k_synth for any nbin: data[s][n] = irfft(Mfull_n e^{2 pi i k phase[s][n]},
// n = nbin) + sigma * the Philox normals of k_synth (pair j of samples 2j,
// 2j + 1 from counter (j, n, s); at odd nbin the last sample takes the first
// normal of its pair -- synth.noise_block's layout).  Dynamic LDS: nbin/2 + 1
// double2.
__global__ __launch_bounds__(kBlock) void k_synth_gen(const double2* __restrict__ Mfull,
                                                      const double* __restrict__ phase,
                                                      double* __restrict__ data, int nchan,
                                                      int NHP, double sigma, uint64_t seed,
                                                      int64_t sub0,
                                                      const double2* __restrict__ tw, int nbin) {
  extern __shared__ __align__(16) unsigned char gsm[];
  double2* X = reinterpret_cast<double2*>(gsm);
  const int row = blockIdx.x, n = row % nchan, NH = nbin / 2 + 1;
  const int64_t s = row / nchan;
  const double ph = phase[row];
  for (int k = threadIdx.x; k < NH; k += kBlock)
    X[k] = cmul(Mfull[(size_t)n * NHP + k], turn_phasor((double)k, ph));
  __syncthreads();
  double* out = data + (size_t)row * nbin;
  idft_row(X, nbin, tw, out);
  if (sigma == 0.0) return;
  __syncthreads();  // the block's samples are stored (each pair is then one thread's)
  const uint64_t gs = (uint64_t)(s + sub0);
  for (int j = threadIdx.x; 2 * j < nbin; j += kBlock) {
    u32x4 ctr;
    ctr.v[0] = (uint32_t)j;
    ctr.v[1] = (uint32_t)n;
    ctr.v[2] = (uint32_t)gs;
    ctr.v[3] = (uint32_t)(gs >> 32);
    const double2 z = philox_normal2(ctr, seed);
    out[2 * j] = fma(sigma, z.x, out[2 * j]);
    if (2 * j + 1 < nbin) out[2 * j + 1] = fma(sigma, z.y, out[2 * j + 1]);
  }
}

}  // namespace ppf
