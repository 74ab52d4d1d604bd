// ppfit_spectra.hip -- FFT-based kernels of libppfit (gfx950).
//
// Kernels (a) and (b) of the hot path: one workgroup per
// subint streams its channel rows from HBM, transforms each row in LDS and
// writes the DC-zeroed cross-spectrum X_nk = D_nk conj(M_nk) that the fit
// kernel re-reads (pptoaslib.py:976-979, 431).  The per-channel noise level
// (get_noise_PS, pplib.py:2227-2253), the data power sum Sd (pptoaslib.py:985)
// and the dedispersed, weight-averaged guess profile of get_TOAs
// (pptoas.py:421-423 / ppalign.py:181-184) are fused into the same pass, so
// the data portrait is read exactly once.
#include "ppfit_kernels.hpp"

namespace ppf {

__global__ void k_twiddles(double2* tw, int nbin) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m < nbin) {
    double s, c;
    sincospi(2.0 * (double)m / (double)nbin, &s, &c);
    tw[m] = cmk(c, -s);
  }
}

// Load a real row of 2N doubles as N packed complex values into LDS.
template <int LOGN>
__device__ __forceinline__ void load_row(double2* buf, const double* __restrict__ row) {
  constexpr int N = 1 << LOGN;
  const double2* r2 = reinterpret_cast<const double2*>(row);
#pragma unroll
  for (int c = 0; c < (N + kBlock - 1) / kBlock; ++c) {
    const int j = threadIdx.x + c * kBlock;
    if (j < N) buf[j] = r2[j];
  }
}

// ---------------------------------------------------------------------------
// Template spectra: M[row][k] for k <= N (DC zeroed when zero_dc, F0_fact=0,
// pplib.py:66), zero padding up to NHP, and p_n = sum_{k>=1} |M_k|^2.
// ---------------------------------------------------------------------------
template <int LOGN>
__global__ __launch_bounds__(kBlock) void k_model_spec(const double* __restrict__ model,
                                                       double2* __restrict__ M,
                                                       double* __restrict__ pn, int NHP,
                                                       int zero_dc,
                                                       const double2* __restrict__ tw) {
  constexpr int N = 1 << LOGN;
  __shared__ double2 buf[N];
  __shared__ double red[kWaves];
  const int row = blockIdx.x;
  load_row<LOGN>(buf, model + (size_t)row * 2 * N);
  __syncthreads();
  lds_fft<LOGN, false>(buf, tw);
  double p = 0.0;
  double2* out = M + (size_t)row * NHP;
  for (int k = threadIdx.x; k < NHP; k += kBlock) {
    double2 x = cmk(0.0, 0.0);
    if (k <= N) x = rfft_post<LOGN>(buf, k, tw);
    if (k == 0 && zero_dc) x = cmk(0.0, 0.0);
    if (k >= 1 && k <= N) p += cabs2(x);
    out[k] = x;
  }
  p = block_sum(p, red);
  if (threadIdx.x == 0 && pn) pn[row] = p;
}

// ---------------------------------------------------------------------------
// Per-subint data pass.  For each fitted channel: rfft in LDS, then
//   X[c][n][k]  = D_nk conj(M_nk)      (k >= 1; DC = 0; pad = 0)
//   sig[c][n]   = errs[s][n] or sqrt(mean_{k>=kc} |D_k|^2 / nbin)
//   dsum[c][n]  = sum_{k>=1} |D_k|^2
//   R[c][k]    += w_n D_nk e^{2 pi i k phi_n},  phi_n = Dconst DM (nu_n^-2 -
//                 nu_g^-2) / P  (rotate_data with DM, pplib.py:2406-2415)
// ---------------------------------------------------------------------------
// Row prefetch into registers, kept as plain doubles (a double2 array
// carried across the channel loop is copied with memcpy and lands in scratch).
template <int LOGN>
struct RowRegs {
  static constexpr int N = 1 << LOGN;
  static constexpr int LI = N >= kBlock ? N / kBlock : 1;
  double x[LI], y[LI];
  __device__ __forceinline__ void load(const double* __restrict__ src) {
    const double2* r2 = reinterpret_cast<const double2*>(src);
#pragma unroll
    for (int i = 0; i < LI; ++i) {
      const int j = threadIdx.x + i * kBlock;
      if (N >= kBlock || j < N) {
        const double2 v = r2[j];
        x[i] = v.x;
        y[i] = v.y;
      }
    }
  }
  __device__ __forceinline__ void store(double2* buf) const {
#pragma unroll
    for (int i = 0; i < LI; ++i) {
      const int j = threadIdx.x + i * kBlock;
      if (N >= kBlock || j < N) buf[j] = cmk(x[i], y[i]);
    }
  }
};

// Latency hiding: the next channel row is loaded into registers while the
// current one is transformed, the template row and the rfft twiddles are in
// registers before the FFT starts, the FFT twiddles and the per-channel
// metadata sit in LDS (no global load inside the channel loop waits on the
// prefetch), and the guess phasor e^{2 pi i k phi_n} advances by one
// multiplication per 256 harmonics.  The per-channel sums are finished by
// thread 0 after the row's last barrier.
template <int LOGN>
__global__ __launch_bounds__(kBlock) void k_data_xspec(SpecArgs a) {
  constexpr int N = 1 << LOGN;
  constexpr int NH = N + 1;
  constexpr int KI = (NH + kBlock - 1) / kBlock;
  constexpr int NTW = 3 * N / 4;
  __shared__ double2 buf[N];
  __shared__ double2 twl[NTW];
  __shared__ double red[2][2 * kWaves];
  __shared__ double s_meta[4];
  extern __shared__ __align__(16) unsigned char dyn[];
  double2* cmeta = reinterpret_cast<double2*>(dyn);  // (phi_g, weight or NaN if masked)
  const int c = blockIdx.x;
  const int s = a.sub0 + c;
  const int tid = threadIdx.x;
  const int nchan = a.nchan;
  const int midx = a.model_idx ? a.model_idx[s] : 0;
  const double* fr = a.freqs + (size_t)s * nchan;
  const uint8_t* mask = a.mask ? a.mask + (size_t)s * nchan : nullptr;
  const double* drow0 = a.data + (size_t)s * nchan * (2 * N);

  RowRegs<LOGN> row;
  row.load(drow0);  // row 0 in flight first
  for (int e = tid; e < NTW; e += kBlock) twl[e] = a.tw[2 * e];
  double2 twp[KI];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = tid + i * kBlock;
    twp[i] = a.tw[k <= N ? k : 0];
  }
  // nu_g (guess dedispersion reference) default: mean over fitted channels
  if (tid == 0) {
    double fs = 0.0, ws = 0.0;
    int nok = 0;
    for (int n = 0; n < nchan; ++n) {
      if (mask && !mask[n]) continue;
      fs += fr[n];
      ws += a.weights ? a.weights[(size_t)s * nchan + n] : 1.0;
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
  const double wsum = s_meta[1];
  {
    const double nug = s_meta[0];
    const double Dfac = kDconst * s_meta[3] / a.P[s];
    const double nug2 = 1.0 / (nug * nug);
    for (int n = tid; n < nchan; n += kBlock) {
      const bool ok = !mask || mask[n];
      const double w = a.weights ? a.weights[(size_t)s * nchan + n] : 1.0;
      cmeta[n] = cmk(Dfac * (1.0 / (fr[n] * fr[n]) - nug2), ok ? w : NAN);
    }
  }
  __syncthreads();

  double2 racc[KI];
#pragma unroll
  for (int i = 0; i < KI; ++i) racc[i] = cmk(0.0, 0.0);

  for (int n = 0; n < nchan; ++n) {
    double2* Xr = a.X + ((size_t)c * nchan + n) * a.NHP;
    const double2 cm = cmeta[n];
    const bool ok = !isnan(cm.y);
    if (ok) row.store(buf);
    if (n + 1 < nchan) row.load(drow0 + (size_t)(n + 1) * 2 * N);
    if (!ok) {
      for (int k = tid; k < a.NHP; k += kBlock) Xr[k] = cmk(0.0, 0.0);
      if (tid == 0) { a.sig[(size_t)c * nchan + n] = 0.0; a.dsum[(size_t)c * nchan + n] = 0.0; }
      continue;
    }
    const double2* Mr = a.M + ((size_t)midx * nchan + n) * a.NHP;
    double2 mreg[KI];
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const int k = tid + i * kBlock;
      mreg[i] = Mr[k <= N ? k : 0];
    }
    __syncthreads();
    lds_fft_twl<LOGN>(buf, twl);
    const double w = cm.y;
    double2 ph = cmk(1.0, 0.0), phst = cmk(1.0, 0.0);
    if (a.guess) {
      ph = turn_phasor((double)tid, cm.x);
      phst = turn_phasor((double)kBlock, cm.x);
    }
    double pn = 0.0, pd = 0.0;
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const int k = tid + i * kBlock;
      if (i > 0) ph = cmul(ph, phst);
      if (k <= N) {
        const double2 x = rfft_post_w<LOGN>(buf, k, twp[i]);
        const double p2 = cabs2(x);
        if (k >= a.kc) pn += p2;
        if (k >= 1) pd += p2;
        Xr[k] = (k == 0) ? cmk(0.0, 0.0) : cmulc(x, mreg[i]);
        if (a.guess) racc[i] = cadd(racc[i], cscale(cmul(x, ph), w));
      }
    }
    for (int k = NH + tid; k < a.NHP; k += kBlock) Xr[k] = cmk(0.0, 0.0);
    pn = wave_sum(pn);
    pd = wave_sum(pd);
    double* rd = red[n & 1];
    if ((tid & 63) == 0) { rd[tid >> 6] = pn; rd[kWaves + (tid >> 6)] = pd; }
    __syncthreads();  // buf and rd complete; the next row may overwrite buf
    if (tid == 0) {
      double sn = 0.0, sd = 0.0;
      for (int i = 0; i < kWaves; ++i) { sn += rd[i]; sd += rd[kWaves + i]; }
      const double sig = a.errs ? a.errs[(size_t)s * nchan + n]
                                : sqrt(sn / (double)(2 * N) / (double)(NH - a.kc));
      a.sig[(size_t)c * nchan + n] = sig;
      a.dsum[(size_t)c * nchan + n] = sd;
    }
  }
  if (a.guess) {
    double2* Rr = a.R + (size_t)c * a.NHP;
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const int k = tid + i * kBlock;
      if (k <= N) {
        double2 r = cscale(racc[i], 1.0 / wsum);
        if (k == 0) r = cmk(0.0, 0.0);
        if (k == N) r.y = 0.0;  // irfft drops Im(X_N)
        Rr[k] = r;
      }
    }
    for (int k = NH + tid; k < a.NHP; k += kBlock) Rr[k] = cmk(0.0, 0.0);
  }
}

// ---------------------------------------------------------------------------
// fit_phase_shift on profiles: spectrum + noise in-kernel, then the shared
// brute-force + Nelder-Mead search (ppfit_guess.hpp).
// ---------------------------------------------------------------------------
template <int LOGN>
__global__ __launch_bounds__(kBlock) void k_phase_shift(PhaseShiftArgs a) {
  constexpr int N = 1 << LOGN;
  constexpr int NH = N + 1;
  __shared__ double2 buf[N + 1];
  __shared__ double2 rm[N + 1];
  __shared__ GuessShared gs;
  const int r = blockIdx.x;
  const int tid = threadIdx.x;
  load_row<LOGN>(buf, a.data + (size_t)r * 2 * N);
  __syncthreads();
  lds_fft<LOGN, false>(buf, a.tw);
  const int midx = a.model_idx ? a.model_idx[r] : 0;
  const double2* Mr = a.M + (size_t)midx * a.NHP;
  double pnoise = 0.0, dd = 0.0, pp = 0.0;
  double2 xs[(NH + kBlock - 1) / kBlock];
#pragma unroll
  for (int i = 0; i < (NH + kBlock - 1) / kBlock; ++i) {
    const int k = tid + i * kBlock;
    if (k <= N) {
      double2 x = rfft_post<LOGN>(buf, k, a.tw);
      if (k >= a.kc) pnoise += cabs2(x);
      if (k == 0) x = cmk(0.0, 0.0);
      xs[i] = x;
      dd += cabs2(x);
      pp += cabs2(Mr[k]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < (NH + kBlock - 1) / kBlock; ++i) {
    const int k = tid + i * kBlock;
    if (k <= N) rm[k] = cmulc(xs[i], Mr[k]);
  }
  pnoise = block_sum(pnoise, gs.red);
  dd = block_sum(dd, gs.red);
  pp = block_sum(pp, gs.red);
  double noise = a.noise ? a.noise[r] : NAN;
  if (isnan(noise)) noise = sqrt(pnoise / (double)(2 * N) / (double)(NH - a.kc));
  const double err = noise * sqrt((double)N);  // sqrt(nbin / 2)
  const double ie2 = 1.0 / (err * err);
  guess_search(rm, NH, ie2, a.Ns, a.lo, a.hi, gs);
  if (tid == 0) {
    const double phase = gs.x;
    const double fmin = gs.fx;
    const double d = dd * ie2, p = pp * ie2;
    const double scale = -fmin / p;
    gs.out[0] = phase;
    gs.out[1] = scale;
    gs.out[2] = d;
    gs.out[3] = p;
    gs.out[4] = fmin;
  }
  __syncthreads();
  // second derivative at the phase (pplib.py:1270-1280)
  double c2 = 0.0;
  for (int k = tid; k < NH; k += kBlock) {
    const double2 e = turn_phasor((double)k, gs.out[0]);
    const double2 w = cmul(rm[k], e);
    c2 += (double)k * (double)k * w.x;
  }
  c2 = block_sum(c2, gs.red);
  if (tid == 0) {
    const double d2 = 4.0 * kPi * kPi * c2 * ie2;  // -Re sum (-4 pi^2 k^2) ...
    const double scale = gs.out[1], d = gs.out[2], p = gs.out[3], fmin = gs.out[4];
    double* o = a.out + (size_t)r * 6;
    o[0] = gs.out[0];
    o[1] = pow(scale * d2, -0.5);
    o[2] = scale;
    o[3] = pow(p, -0.5);
    o[4] = pow(scale * scale * p, 0.5);
    o[5] = (d - fmin * fmin / p) / (double)(2 * N - 2);
  }
}

// ---------------------------------------------------------------------------
// Row rotation: out = irfft(rfft(in) e^{2 pi i k phase}) (rotate_data).
// ---------------------------------------------------------------------------
template <int LOGN>
__device__ void c2r_from_spectrum(double2* buf, double2 (&xs)[((1 << LOGN) + kBlock) / kBlock + 1],
                                  const double2* __restrict__ tw, double* __restrict__ out) {
  constexpr int N = 1 << LOGN;
  constexpr int KI = (N + 1 + kBlock - 1) / kBlock;
  const int tid = threadIdx.x;
  // stage X_k (k in [0, N]) in LDS, then form Z_k for k in [0, N)
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = tid + i * kBlock;
    if (k <= N) {
      double2 x = xs[i];
      if (k == 0 || k == N) x.y = 0.0;
      buf[k] = x;
    }
  }
  __syncthreads();
  double2 z[KI];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = tid + i * kBlock;
    if (k < N) z[i] = irfft_pre<LOGN>(buf[k], buf[N - k], k, tw);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = tid + i * kBlock;
    if (k < N) buf[k] = z[i];
  }
  __syncthreads();
  lds_fft<LOGN, true>(buf, tw);
  const double inv = 1.0 / (double)N;
  double2* o2 = reinterpret_cast<double2*>(out);
  for (int j = tid; j < N; j += kBlock) o2[j] = cscale(buf[j], inv);
}

template <int LOGN>
__global__ __launch_bounds__(kBlock) void k_rotate_rows(const double* __restrict__ in,
                                                        const double* __restrict__ phase,
                                                        double* __restrict__ out,
                                                        const double2* __restrict__ tw) {
  constexpr int N = 1 << LOGN;
  constexpr int KI = (N + 1 + kBlock - 1) / kBlock;
  __shared__ double2 buf[N + 1];
  const int r = blockIdx.x;
  load_row<LOGN>(buf, in + (size_t)r * 2 * N);
  __syncthreads();
  lds_fft<LOGN, false>(buf, tw);
  const double ph = phase[r];
  double2 xs[(N + kBlock) / kBlock + 1];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = threadIdx.x + i * kBlock;
    if (k <= N) xs[i] = cmul(rfft_post<LOGN>(buf, k, tw), turn_phasor((double)k, ph));
  }
  __syncthreads();
  c2r_from_spectrum<LOGN>(buf, xs, tw, out + (size_t)r * 2 * N);
}

template <int LOGN>
__global__ __launch_bounds__(kBlock) void k_irfft_rows(const double2* __restrict__ spec,
                                                       double* __restrict__ out,
                                                       const double2* __restrict__ tw) {
  constexpr int N = 1 << LOGN;
  constexpr int KI = (N + 1 + kBlock - 1) / kBlock;
  __shared__ double2 buf[N + 1];
  const int r = blockIdx.x;
  double2 xs[(N + kBlock) / kBlock + 1];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = threadIdx.x + i * kBlock;
    if (k <= N) xs[i] = spec[(size_t)r * (N + 1) + k];
  }
  c2r_from_spectrum<LOGN>(buf, xs, tw, out + (size_t)r * 2 * N);
}

template <int LOGN>
__global__ __launch_bounds__(kBlock) void k_noise_rows(const double* __restrict__ in,
                                                       double* __restrict__ out, int kc,
                                                       const double2* __restrict__ tw) {
  constexpr int N = 1 << LOGN;
  __shared__ double2 buf[N];
  __shared__ double red[kWaves];
  const int r = blockIdx.x;
  load_row<LOGN>(buf, in + (size_t)r * 2 * N);
  __syncthreads();
  lds_fft<LOGN, false>(buf, tw);
  double p = 0.0;
  for (int k = kc + threadIdx.x; k <= N; k += kBlock) p += cabs2(rfft_post<LOGN>(buf, k, tw));
  p = block_sum(p, red);
  if (threadIdx.x == 0) out[r] = sqrt(p / (double)(2 * N) / (double)(N + 1 - kc));
}

// ---------------------------------------------------------------------------
// Synthetic portraits: data[s][n] = irfft(Mfull_n e^{2 pi i k phase[s][n]})
//                                   + sigma * Philox normals.
// ---------------------------------------------------------------------------
template <int LOGN>
__global__ __launch_bounds__(kBlock) void k_synth(const double2* __restrict__ Mfull,
                                                  const double* __restrict__ phase,
                                                  double* __restrict__ data, int nchan,
                                                  int NHP, double sigma, uint64_t seed,
                                                  int64_t sub0,
                                                  const double2* __restrict__ tw) {
  constexpr int N = 1 << LOGN;
  constexpr int KI = (N + 1 + kBlock - 1) / kBlock;
  __shared__ double2 buf[N + 1];
  const int row = blockIdx.x;  // s * nchan + n
  const int n = row % nchan;
  const int64_t s = row / nchan;
  const double ph = phase[row];
  double2 xs[(N + kBlock) / kBlock + 1];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = threadIdx.x + i * kBlock;
    if (k <= N) xs[i] = cmul(Mfull[(size_t)n * NHP + k], turn_phasor((double)k, ph));
  }
  double* out = data + (size_t)row * 2 * N;
  c2r_from_spectrum<LOGN>(buf, xs, tw, out);
  __syncthreads();
  if (sigma != 0.0) {
    double2* o2 = reinterpret_cast<double2*>(out);
    const uint64_t gs = (uint64_t)(s + sub0);
    for (int j = threadIdx.x; j < N; j += kBlock) {
      u32x4 ctr;
      ctr.v[0] = (uint32_t)j;
      ctr.v[1] = (uint32_t)n;
      ctr.v[2] = (uint32_t)gs;
      ctr.v[3] = (uint32_t)(gs >> 32);
      const double2 z = philox_normal2(ctr, seed);
      double2 v = o2[j];
      v.x = fma(sigma, z.x, v.x);
      v.y = fma(sigma, z.y, v.y);
      o2[j] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// ppalign weighted rotate-and-sum in the Fourier domain (ppalign.py:202-208):
// partial[p][n][k] = sum_{s in slice p} w[s][n] rfft(data[s][n])_k e^{2 pi i k ph[s][n]}
// ---------------------------------------------------------------------------
template <int LOGN>
__global__ __launch_bounds__(kBlock) void k_rot_accum(const double* __restrict__ data,
                                                      const double* __restrict__ phase,
                                                      const double* __restrict__ weight,
                                                      double2* __restrict__ partial, int nsub,
                                                      int nchan, int nsplit,
                                                      const double2* __restrict__ tw) {
  constexpr int N = 1 << LOGN;
  constexpr int KI = (N + 1 + kBlock - 1) / kBlock;
  __shared__ double2 buf[N];
  const int n = blockIdx.x % nchan;
  const int p = blockIdx.x / nchan;
  const int per = (nsub + nsplit - 1) / nsplit;
  const int s0 = p * per, s1 = min(nsub, s0 + per);
  double2 acc[KI];
#pragma unroll
  for (int i = 0; i < KI; ++i) acc[i] = cmk(0.0, 0.0);
  for (int s = s0; s < s1; ++s) {
    const size_t row = (size_t)s * nchan + n;
    const double w = weight[row];
    if (w == 0.0) continue;  // uniform per block
    load_row<LOGN>(buf, data + row * 2 * N);
    __syncthreads();
    lds_fft<LOGN, false>(buf, tw);
    const double ph = phase[row];
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const int k = threadIdx.x + i * kBlock;
      if (k <= N)
        acc[i] = cadd(acc[i], cscale(cmul(rfft_post<LOGN>(buf, k, tw), turn_phasor((double)k, ph)), w));
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = threadIdx.x + i * kBlock;
    if (k <= N) partial[((size_t)p * nchan + n) * (N + 1) + k] = acc[i];
  }
}

__global__ void k_accum_reduce(const double2* __restrict__ partial, double2* __restrict__ accum,
                               int nsplit, size_t count) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  double2 s = accum[i];
  for (int p = 0; p < nsplit; ++p) s = cadd(s, partial[(size_t)p * count + i]);
  accum[i] = s;
}

// ---------------------------------------------------------------------------
// explicit instantiations (nbin = 64 ... 8192  <=>  LOGN = 5 ... 12)
// ---------------------------------------------------------------------------
#define PPF_INST(L)                                                                          \
  template __global__ void k_model_spec<L>(const double*, double2*, double*, int, int,       \
                                           const double2*);                                  \
  template __global__ void k_data_xspec<L>(SpecArgs);                                        \
  template __global__ void k_phase_shift<L>(PhaseShiftArgs);                                 \
  template __global__ void k_rotate_rows<L>(const double*, const double*, double*,           \
                                            const double2*);                                 \
  template __global__ void k_irfft_rows<L>(const double2*, double*, const double2*);        \
  template __global__ void k_noise_rows<L>(const double*, double*, int, const double2*);    \
  template __global__ void k_synth<L>(const double2*, const double*, double*, int, int,      \
                                      double, uint64_t, int64_t, const double2*);            \
  template __global__ void k_rot_accum<L>(const double*, const double*, const double*,       \
                                          double2*, int, int, int, const double2*);
PPF_INST(5)
PPF_INST(6)
PPF_INST(7)
PPF_INST(8)
PPF_INST(9)
PPF_INST(10)
PPF_INST(11)
PPF_INST(12)

}  // namespace ppf
