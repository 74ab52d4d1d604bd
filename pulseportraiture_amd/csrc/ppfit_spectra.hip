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
                                                       const double2* __restrict__ tw,
                                                       double* __restrict__ M2) {
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
    if (M2) M2[(size_t)row * NHP + k] = cabs2(x);  // |M_k|^2 for the scattering sweeps
  }
  p = block_sum(p, red);
  if (threadIdx.x == 0 && pn) pn[row] = p;
}

// ---------------------------------------------------------------------------
// Per-subint data pass.  For each fitted channel: rfft, then
//   sig[c][n]   = errs[s][n] or sqrt(mean_{k>=kc} |D_k|^2 / nbin)
//   dsum[c][n]  = sum_{k>=1} |D_k|^2
//   R[c][k]    += w_n D_nk e^{2 pi i k phi_n},  phi_n = Dconst DM (nu_n^-2 -
//                 nu_g^-2) / P  (rotate_data with DM, pplib.py:2406-2415)
//   X[c][n][k]  = D_nk conj(M_nk)   only for subints fitted with the exact
//                 (scattering) sweeps; phase-family subints get Taylor
//                 moments from k_moments instead (ppfit_taylor.hip)
// With the data-spectrum cache (a.D, PPF_SPEC_STORE) every row's spectrum
// D_nk, k = 0 .. N, is stored as well, and Taylor-path subints write no X
// (their moment passes form it from D).  PPF_SPEC_USE: those subints are not
// visited at all (sig, dsum and R are the cached ones); the others are
// processed as under STORE (the same values again) for their X.
// Channels go in groups of WPB: wave w transforms channel g*WPB + w in its
// own LDS buffer (wave-synchronous Stockham, next row already in registers)
// and post-processes the spectrum in (k, N-k) pairs straight from the packed
// FFT, leaving its weighted, rotated spectrum in the buffer.  One barrier per
// group, then every thread adds the group's WPB rows, in channel order, into
// the R harmonics it owns (k = tid + nthr q, in registers).
// ---------------------------------------------------------------------------
template <int LOGN>
struct XspecCfg {
  static constexpr int N = 1 << LOGN;
  // rows above 1024 points: one wave per workgroup, R accumulated in place
  // in the subint's global R row (too large for registers)
  static constexpr bool RREG = LOGN <= 10;
  static constexpr int WPB = RREG ? 4 : 1;
  // LOGN 10: register FFT (fft1024_wave) in the padded slot order
  static constexpr bool REGFFT = LOGN == 10;
  static constexpr int NB = REGFFT ? kFft1024Slots : N + 8;  // row buffer slots
  static constexpr int NPI = (N / 2 + 1 + 63) / 64;      // pair iterations (k <= N/2)
  static constexpr int NRQ = RREG ? (N + 1 + WPB * 64 - 1) / (WPB * 64) : 1;  // R slots/thread
};

// dynamic LDS of k_data_xspec: per-channel (phi_g, weight) then one
// active flag per channel (the group loop reads LDS, not the mask in HBM)
inline size_t xspec_dyn_lds(int nchan) {
  return (size_t)nchan * sizeof(double2) + (((size_t)nchan + 15) & ~(size_t)15);
}

template <int LOGN, bool WIDE>
__global__ __launch_bounds__(kBlock, 2) void k_data_xspec(SpecArgs a) {
  using Cfg = XspecCfg<LOGN>;
  constexpr int N = Cfg::N;
  constexpr int NH = N + 1;
  constexpr int WPB = Cfg::WPB;
  constexpr int NPI = Cfg::NPI;
  constexpr int NTW = PassTw<LOGN>::SIZE;
  constexpr bool RREG = Cfg::RREG;
  constexpr bool REGFFT = Cfg::REGFFT;
  constexpr int nthr = WPB * 64;
  __shared__ double2 bufs[WPB][Cfg::NB];
  // per-pass Stockham twiddles, or the register FFT's stage tables
  __shared__ __align__(16) unsigned char twraw[REGFFT ? sizeof(Fft1024Tw) : NTW * sizeof(double2)];
  double2* twl = reinterpret_cast<double2*>(twraw);
  Fft1024Tw* ftw = reinterpret_cast<Fft1024Tw*>(twraw);
  auto bi = [](int k) { return REGFFT ? fft1024_slot(k) : k; };
  __shared__ double s_meta[4];
  __shared__ int s_act[WPB];
  extern __shared__ __align__(16) unsigned char dyn[];
  unsigned char* ctab = chan_tables<WIDE>(a, dyn);
  double2* cmeta = reinterpret_cast<double2*>(ctab);  // (phi_g, weight or NaN if masked)
  uint8_t* cact = ctab + (size_t)a.nchan * sizeof(double2);  // fitted channel flags
  const int c = blockIdx.x;
  const int s = a.sub0 + c;
  const bool tsub = a.D && spec_taylor_sub(a, s);
  if (a.spec_mode == PPF_SPEC_USE && tsub) return;  // all of it cached
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: row pointers in SGPRs
  const int nchan = a.nchan;
  const int midx = a.model_idx ? a.model_idx[s] : 0;
  const double* fr = a.freqs + (size_t)s * nchan;
  const uint8_t* mask = a.mask ? a.mask + (size_t)s * nchan : nullptr;
  const double* drow0 = a.data + (size_t)s * nchan * (2 * N);
  double2* buf = bufs[w];
  auto active_g = [&](int q) { return q < nchan && (!mask || mask[q]); };
  // after the cmeta barrier; wave-uniform (q is), read as a scalar so that
  // no branch on it is divergent in the compiler's view (a divergent join
  // makes the wait-count pass drain every outstanding load and X store)
  auto active = [&](int q) {
    return q < nchan && __builtin_amdgcn_readfirstlane((int)cact[q]) != 0;
  };

  WaveRow<LOGN> row;
  bool have = active_g(w);  // the registers hold (or are loading) this wave's next row
  if (have) row.load(drow0 + (size_t)w * 2 * N, lane);  // first row in flight
  if constexpr (REGFFT) ftw[0].fill(a.tw, tid, nthr);
  else fill_pass_tw<LOGN>(twl, a.tw, tid, nthr);
  // nu_g (guess dedispersion reference) default: mean over fitted channels
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
  const double wsum = s_meta[1];
  const bool wx = a.X != nullptr && !tsub;
  const bool wd = a.D != nullptr && a.spec_mode == PPF_SPEC_STORE;
  {
    const double nug = s_meta[0];
    const double Dfac = kDconst * s_meta[3] / a.P[s];
    const double nug2 = 1.0 / (nug * nug);
    for (int q = tid; q < nchan; q += nthr) {
      const bool ok = !mask || mask[q];
      const double wq = a.weights ? a.weights[(size_t)s * nchan + q] : 1.0;
      cmeta[q] = cmk(Dfac * (1.0 / (fr[q] * fr[q]) - nug2), ok ? wq : NAN);
      cact[q] = ok;
    }
  }
  double2 rq[Cfg::NRQ];  // R harmonics owned by this thread (RREG)
#pragma unroll
  for (int q = 0; q < Cfg::NRQ; ++q) rq[q] = cmk(0.0, 0.0);
  double2* Rr = a.R + (size_t)c * a.NHP;
  if (!RREG && a.guess)
    for (int k = tid; k < a.NHP; k += nthr) Rr[k] = cmk(0.0, 0.0);
  double sw, cw;
  sincospi(-(double)lane / (double)N, &sw, &cw);
  const double2 w0 = cmk(cw, sw);                    // e^{-i pi lane / N}
  double ss, cs;
  sincospi(-64.0 / (double)N, &ss, &cs);
  const double2 wstep = cmk(cs, ss);                 // e^{-i pi 64 / N}
  __syncthreads();  // twl, cmeta

  const int ngroups = (nchan + WPB - 1) / WPB;
  for (int g = 0; g < ngroups; ++g) {
    const int n = g * WPB + w;
    const bool act = active(n);
    if (lane == 0) s_act[w] = act;
    if (act && !have) row.load(drow0 + (size_t)n * 2 * N, lane);
    have = false;
    // template harmonics k and N - k of this row, in flight during the FFT
    // (M is shared by every subint: L2-resident)
    const double2* Mr = a.M + ((size_t)midx * nchan + (act ? n : 0)) * a.NHP;
    // prefetch two pair iterations deep: (m0k, m0n) serve the even iterations
    // and (m1k, m1n) the odd ones, each reloaded for iteration i + 2 once
    // iteration i has used it; the first two are issued before the FFT.
    // Unpredicated (k clamped to N/2 past the end): no merge with the old
    // value, so the registers are reloaded in place, no copies
    auto mload = [&](int i, double2& mk, double2& mn) {
      const int k = min(lane + 64 * i, N / 2);
      mk = Mr[k];
      mn = Mr[N - k];
    };
    double2 m0k = cmk(0.0, 0.0), m0n = m0k, m1k = m0k, m1n = m0k;
    // next row of this wave: with the register FFT its load starts as soon
    // as stage A has moved the current row to LDS (stages B, C and the
    // spectrum pass cover it), else after the FFT
    const bool nxt = active(n + WPB);
    auto load_next = [&] {
      if (nxt) row.load(drow0 + (size_t)(n + WPB) * 2 * N, lane);
    };
    constexpr bool EARLY = REGFFT && PPF_EARLY_ROW;
    if (act) {
      mload(0, m0k, m0n);
      mload(1, m1k, m1n);
      if constexpr (REGFFT) {
        if constexpr (EARLY) fft1024_wave(row.x, row.y, buf, ftw[0], lane, load_next);
        else fft1024_wave(row.x, row.y, buf, ftw[0], lane);
      } else {
        row.store(buf, drow0 + (size_t)n * 2 * N, lane);
        fft_sync<true>();
        wave_fft<LOGN>(buf, twl, lane);
      }
    }
    if (!EARLY || !act) load_next();
    have = nxt;
    if (act) {
      const double2 cm = cmeta[n];
      const double wgt = cm.y;
      double2 e = cmk(1.0, 0.0), estep = e, EN = e;
      if (a.guess) {
        // the channel weight rides on the phasor chain (exact for the usual
        // weight 1): w e_k = (w e_0) estep^k
        e = cscale(turn_phasor((double)lane, cm.x), wgt);
        estep = turn_phasor(64.0, cm.x);
        EN = turn_phasor((double)N, cm.x);
      }
      double2* Xr = wx ? a.X + ((size_t)c * nchan + n) * a.NHP : nullptr;
      double2* Dr = wd ? a.D + ((size_t)c * nchan + n) * a.NHP : nullptr;
      double pn = 0.0, pd = 0.0;
      double2 tw = w0;
      // pair iteration i: k = lane + 64 i.  Every iteration but the last has
      // k < N/2 on every lane (a pair of two distinct harmonics); the last
      // holds k = N/2 (its own partner) on lane 0 only.  The full iterations
      // are branch-free so the stores and template loads keep a fixed count.
      // mk / mn hold iteration i's template harmonics and take iteration
      // i + 2's once used: the two register pairs alternate (no copies)
      auto pair = [&](int i, auto fullc, double2& mk, double2& mn) {
        constexpr bool FULL = decltype(fullc)::value;
        const int k = lane + 64 * i;
        if (i > 0) { tw = cmul(tw, wstep); e = cmul(e, estep); }
        if (FULL || k <= N / 2) {
          double2 xk, xn;
          rfft_pair_v(buf[bi(k)], buf[bi((N - k) & (N - 1))], tw, xk, xn);
          const int kn = N - k;
          const double p2k = cabs2(xk), p2n = cabs2(xn);
          const bool two = FULL || k < N / 2;  // k = N/2 is its own partner
          if (k >= a.kc) pn += p2k;
          if (two && kn >= a.kc) pn += p2n;
          if (k >= 1) pd += p2k;
          if (two) pd += p2n;
          if (wx) {
            st_stream((k == 0) ? cmk(0.0, 0.0) : cmulc(xk, mk), Xr + k);
            if (two) st_stream(cmulc(xn, mn), Xr + kn);
          }
          if (wd) {
            st_stream(xk, Dr + k);
            if (two) st_stream(xn, Dr + kn);
          }
          if (a.guess) {
            // e^{2 pi i (N-k) phi} = e^{2 pi i N phi} conj(e^{2 pi i k phi});
            // the pair's two slots are read and written by this lane only
            const double2 tk = cmul(xk, e);
            const double2 tn = cmul(xn, cmul(EN, cconj(e)));
            if (two) buf[bi(kn)] = tn;  // k = 0: the N slot
            buf[bi(k)] = tk;
          }
        }
        // reload for iteration i + 2 only if there is one: a trailing load
        // left in flight past the loop would be drained (with every X store
        // issued before it) when the registers are reused for the next row
        if (FULL && i + 2 < NPI) mload(i + 2, mk, mn);
      };
      static_assert(64 * (NPI - 1) <= N / 2 && 64 * (NPI - 1) + 63 >= N / 2, "pair split");
      constexpr int NFULL2 = (NPI - 1) & ~1;
#pragma unroll 1
      for (int i = 0; i < NFULL2; i += 2) {
        pair(i, std::true_type{}, m0k, m0n);
        pair(i + 1, std::true_type{}, m1k, m1n);
      }
      if constexpr (NFULL2 < NPI - 1) {
        pair(NPI - 2, std::true_type{}, m0k, m0n);
        pair(NPI - 1, std::false_type{}, m1k, m1n);
      } else {
        pair(NPI - 1, std::false_type{}, m0k, m0n);
      }
      if (wx)
        for (int k = NH + lane; k < a.NHP; k += 64) Xr[k] = cmk(0.0, 0.0);
      if (wd)
        for (int k = NH + lane; k < a.NHP; k += 64) Dr[k] = cmk(0.0, 0.0);
      pn = wave_sum(pn);
      pd = wave_sum(pd);
      if (lane == 0) {
        // errs NULL or NaN entry: get_noise_PS of the row (pplib.py:2227-2253)
        double sig = a.errs ? a.errs[(size_t)s * nchan + n] : NAN;
        if (isnan(sig)) sig = sqrt(pn / (double)(2 * N) / (double)(NH - a.kc));
        a.sig[(size_t)c * nchan + n] = sig;
        a.dsum[(size_t)c * nchan + n] = pd;
      }
    } else if (n < nchan) {  // masked channel
      if (lane == 0) { a.sig[(size_t)c * nchan + n] = 0.0; a.dsum[(size_t)c * nchan + n] = 0.0; }
      if (wx) {
        double2* Xr = a.X + ((size_t)c * nchan + n) * a.NHP;
        for (int k = lane; k < a.NHP; k += 64) Xr[k] = cmk(0.0, 0.0);
      }
      if (wd) {
        double2* Dr = a.D + ((size_t)c * nchan + n) * a.NHP;
        for (int k = lane; k < a.NHP; k += 64) Dr[k] = cmk(0.0, 0.0);
      }
    }
    if (a.guess) {
      __syncthreads();  // the group's rotated rows are complete
      if constexpr (RREG) {
        // branch-free: each sum is selected, not skipped (the same additions
        // in the same order as the guarded form)
        int actv[WPB];
#pragma unroll
        for (int v = 0; v < WPB; ++v) actv[v] = __builtin_amdgcn_readfirstlane(s_act[v]);
#pragma unroll
        for (int q = 0; q < Cfg::NRQ; ++q) {
          const int k = tid + nthr * q;
          const bool kin = k <= N;
          const int kk = kin ? k : N;
#pragma unroll
          for (int v = 0; v < WPB; ++v) {
            const double2 sum = cadd(rq[q], bufs[v][bi(kk)]);
            const bool use = kin && actv[v];
            rq[q] = cmk(use ? sum.x : rq[q].x, use ? sum.y : rq[q].y);
          }
        }
      } else {
        if (s_act[0])
          for (int k = tid; k <= N; k += nthr) Rr[k] = cadd(Rr[k], bufs[0][k]);
      }
      __syncthreads();  // buffers free for the next group
    } else {
      fft_sync<true>();
    }
  }
  if (a.guess) {
    const double iw = 1.0 / wsum;
    for (int k = tid; k < a.NHP; k += nthr) {
      double2 r = cmk(0.0, 0.0);
      if (k <= N) {
        if constexpr (RREG) {
#pragma unroll
          for (int q = 0; q < Cfg::NRQ; ++q)
            if (k == tid + nthr * q) r = rq[q];
        } else {
          r = Rr[k];  // accumulated by this same thread
        }
        r = cscale(r, iw);
        if (k == 0) r = cmk(0.0, 0.0);
        if (k == N) r.y = 0.0;  // irfft drops Im(X_N)
      }
      Rr[k] = r;
    }
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
// Row rotation: out = irfft(rfft(in) e^{2 pi i k phase}) (rotate_data),
// optionally scattered: / (1 + 2 pi i k tau) (scattering_portrait_FT).
// ---------------------------------------------------------------------------
// epi(j, v): the value stored at complex sample j (bins 2j, 2j + 1), given
// the transform's v -- a fused epilogue (k_synth adds its noise there)
struct C2rPlain {
  __device__ double2 operator()(int, double2 v) const { return v; }
};
template <int LOGN, typename Epi = C2rPlain>
__device__ void c2r_from_spectrum(double2* buf, double2 (&xs)[((1 << LOGN) + kBlock) / kBlock + 1],
                                  const double2* __restrict__ tw, double* __restrict__ out,
                                  Epi epi = Epi()) {
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
  for (int j = tid; j < N; j += kBlock) o2[j] = epi(j, cscale(buf[j], inv));
}

template <int LOGN>
// in == out is supported (ppf_rotate_rows in place, engine.rotate_rows):
// each workgroup loads its whole row into LDS and synchronises before any
// store, so in and out are deliberately not __restrict__.
__global__ __launch_bounds__(kBlock) void k_rotate_rows(const double* in,
                                                        const double* __restrict__ phase,
                                                        const double* __restrict__ tau,
                                                        double* out,
                                                        const double2* __restrict__ tw) {
  constexpr int N = 1 << LOGN;
  constexpr int KI = (N + 1 + kBlock - 1) / kBlock;
  __shared__ double2 buf[N + 1];
  const int r = blockIdx.x;
  load_row<LOGN>(buf, in + (size_t)r * 2 * N);
  __syncthreads();
  lds_fft<LOGN, false>(buf, tw);
  const double ph = phase ? phase[r] : 0.0;
  double2 xs[(N + kBlock) / kBlock + 1];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = threadIdx.x + i * kBlock;
    if (k <= N) {
      xs[i] = rfft_post<LOGN>(buf, k, tw);
      if (phase) xs[i] = cmul(xs[i], turn_phasor((double)k, ph));
    }
  }
  const double t2 = tau ? 2.0 * M_PI * tau[r] : 0.0;
  if (t2 != 0.0) {  // scattering_portrait_FT: x / (1 + 2 pi i k tau)
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const int k = threadIdx.x + i * kBlock;
      const double w = t2 * (double)k, d = 1.0 / fma(w, w, 1.0);
      if (k <= N) xs[i] = cmk(fma(xs[i].y, w, xs[i].x) * d, fma(-xs[i].x, w, xs[i].y) * d);
    }
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

// spec[r][k] = rfft(in[r])[k], k in [0, N] (numpy rfft layout; nothing zeroed)
template <int LOGN>
__global__ __launch_bounds__(kBlock) void k_rfft_rows(const double* __restrict__ in,
                                                      double2* __restrict__ spec,
                                                      const double2* __restrict__ tw) {
  constexpr int N = 1 << LOGN;
  __shared__ double2 buf[N];
  const int r = blockIdx.x;
  load_row<LOGN>(buf, in + (size_t)r * 2 * N);
  __syncthreads();
  lds_fft<LOGN, false>(buf, tw);
  for (int k = threadIdx.x; k <= N; k += kBlock)
    spec[(size_t)r * (N + 1) + k] = rfft_post<LOGN>(buf, k, tw);
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
  // the noise joins each sample pair as it is stored (one pass over the row)
  const uint64_t gs = (uint64_t)(s + sub0);
  c2r_from_spectrum<LOGN>(buf, xs, tw, out, [&](int j, double2 v) {
    if (sigma != 0.0) {
      u32x4 ctr;
      ctr.v[0] = (uint32_t)j;
      ctr.v[1] = (uint32_t)n;
      ctr.v[2] = (uint32_t)gs;
      ctr.v[3] = (uint32_t)(gs >> 32);
      const double2 z = philox_normal2(ctr, seed);
      v.x = fma(sigma, z.x, v.x);
      v.y = fma(sigma, z.y, v.y);
    }
    return v;
  });
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

// The same sum for nbin = 2048 (ppalign at config 5).  Workgroup (n, p)
// takes channel n of subint slice p; its four waves stream subints s0 + w,
// s0 + w + 4, ... (one row per wave per group, fft1024_wave into the wave's
// own LDS buffer, the next row's load started after stage A).  After a
// barrier every wave adds all four rows of the group, in subint order, into
// the harmonic pairs it owns: k = lane + 64 j and N - k for j = w, w + 4,
// w + 8 (j <= 8).  Spreading the pairs over the workgroup keeps 6 complex
// sums per lane instead of a whole channel spectrum (18), which spilled.
// The rotation e^{2 pi i k ph} w: turn_phasor at k = lane + 64 w per row,
// stepped by e^{2 pi i 256 ph}; the row's own wave forms that step and
// e^{2 pi i N ph} once and passes them with the weight through LDS.
__global__ __launch_bounds__(256, 2) void k_rot_accum_w(const double* __restrict__ data,
                                                       const double* __restrict__ phase,
                                                       const double* __restrict__ weight,
                                                       double2* __restrict__ partial, int nsub,
                                                       int nchan, int nsplit,
                                                       const double2* __restrict__ tw) {
  constexpr int LOGN = 10, N = 1 << LOGN, NJ = 3;  // j = w + 4 i <= 8
  __shared__ double2 bufs[4][kFft1024Slots];
  __shared__ Fft1024Tw ftw;
  __shared__ double2 s_step[4], s_EN[4];
  __shared__ double s_w[4], s_ph[4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = blockIdx.x % nchan, p = blockIdx.x / nchan;
  const int per = (nsub + nsplit - 1) / nsplit;
  const int s0 = p * per, s1 = min(nsub, s0 + per);
  const int ngrp = s1 > s0 ? (s1 - s0 + 3) / 4 : 0;
  ftw.fill(tw, tid, 256);
  double2* buf = bufs[w];
  double2 ak[NJ], an[NJ], tk[NJ];
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    ak[i] = an[i] = cmk(0.0, 0.0);
    double sw, cw;  // rfft post-processing twiddle e^{-i pi k / N} of pair k
    sincospi(-(double)(lane + 64 * (w + 4 * i)) / (double)N, &sw, &cw);
    tk[i] = cmk(cw, sw);
  }
  auto rowp = [&](int s) { return data + ((size_t)s * nchan + n) * 2 * N; };
  // weights and phases of this wave's rows 64 groups at a time (lane l: group
  // t0 + l), one window ahead, as vector loads: a scalar load per row would
  // hold up the FFT's LDS waits (they share lgkmcnt)
  auto wload = [&](int t0, double& wo, double& po) {
    const int s = s0 + 4 * (t0 + lane) + w;
    const size_t i = (size_t)(s < s1 ? s : s0) * nchan + n;
    wo = weight[i];
    po = phase[i];
    if (s >= s1) wo = 0.0;
  };
  double wv = 0.0, pv = 0.0, wv2 = 0.0, pv2 = 0.0;
  if (ngrp > 0) wload(0, wv2, pv2);
  WaveRow<LOGN> row;
  if (s0 + w < s1) row.load(rowp(s0 + w), lane);
  __syncthreads();  // ftw
  for (int t = 0; t < ngrp; ++t) {
    const int sc = s0 + 4 * t + w, sn = sc + 4;  // this wave's row now and next
    if ((t & 63) == 0) {
      wv = wv2;
      pv = pv2;
      if (t + 64 < ngrp) wload(t + 64, wv2, pv2);
    }
    const double wc = lane_of(wv, t & 63), pc = lane_of(pv, t & 63);  // 0 past s1
    auto load_next = [&] {
      if (sn < s1) row.load(rowp(sn), lane);
    };
    if (wc != 0.0) {
      if constexpr (PPF_EARLY_ROW) {
        fft1024_wave(row.x, row.y, buf, ftw, lane, load_next);
      } else {
        fft1024_wave(row.x, row.y, buf, ftw, lane);
        load_next();
      }
      const double2 st = turn_phasor(256.0, pc), en = turn_phasor((double)N, pc);
      if (lane == 0) { s_step[w] = st; s_EN[w] = en; s_ph[w] = pc; }
    } else {
      load_next();
    }
    if (lane == 0) s_w[w] = wc;
    __syncthreads();  // the group's four spectra and their rotations
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double wr = s_w[r];
      if (wr != 0.0) {  // uniform per workgroup
        const double pr = s_ph[r];
        const double2 st = s_step[r], EN = s_EN[r];
        const double2* br = bufs[r];
        double2 e = cscale(turn_phasor((double)(lane + 64 * w), pr), wr);
#pragma unroll
        for (int i = 0; i < NJ; ++i) {
          const int k = lane + 64 * (w + 4 * i);
          if (i > 0) e = cmul(e, st);
          if (k <= N / 2) {
            double2 xk, xn;
            rfft_pair_v(br[fft1024_slot(k)], br[fft1024_slot((N - k) & (N - 1))], tk[i], xk, xn);
            ak[i] = cadd(ak[i], cmul(xk, e));
            if (k < N / 2) an[i] = cadd(an[i], cmul(xn, cmul(EN, cconj(e))));
          }
        }
      }
    }
    __syncthreads();  // buffers and the row table free for the next group
  }
  double2* out = partial + ((size_t)p * nchan + n) * (N + 1);
#pragma unroll
  for (int i = 0; i < NJ; ++i) {
    const int k = lane + 64 * (w + 4 * i);
    if (k <= N / 2) {
      out[k] = ak[i];
      if (k < N / 2) out[N - k] = an[i];  // k = 0: the Nyquist harmonic
    }
  }
}

// The same sum from cached data spectra (PPF_SPEC_STORE's spec, [nsub][nchan]
// [NHP]): no transform, one streaming pass.  Workgroup (n, p) sums channel n
// over subint slice p in subint order; thread t owns harmonics k = kb + t +
// 256 i (i < kRotSpecK), with the row's rotation w e^{2 pi i k ph} from
// turn_phasor at kb + t stepped by e^{2 pi i 256 ph}.  The next row's
// harmonics load while this row's are added.  Rows of weight 0 add nothing.
constexpr int kRotSpecK = 5;  // 1280 harmonics per pass: nbin <= 2048 in one
__global__ __launch_bounds__(256) void k_rot_accum_spec(const double2* __restrict__ spec,
                                                        const double* __restrict__ phase,
                                                        const double* __restrict__ weight,
                                                        double2* __restrict__ partial, int nsub,
                                                        int nchan, int nsplit, int N, int NHP) {
  const int tid = threadIdx.x;
  const int n = blockIdx.x % nchan, p = blockIdx.x / nchan;
  const int per = (nsub + nsplit - 1) / nsplit;
  const int s0 = p * per, s1 = min(nsub, s0 + per);
  double2* out = partial + ((size_t)p * nchan + n) * (N + 1);
  for (int kb = 0; kb <= N; kb += 256 * kRotSpecK) {
    double2 acc[kRotSpecK], cur[kRotSpecK], nxt[kRotSpecK] = {};
    auto load = [&](int s, double2* v) {
      const double2* r = spec + ((size_t)s * nchan + n) * NHP;
#pragma unroll
      for (int i = 0; i < kRotSpecK; ++i) {
        const int k = kb + tid + 256 * i;
        v[i] = r[k <= N ? k : N];  // clamped, unpredicated; k > N unused
      }
    };
#pragma unroll
    for (int i = 0; i < kRotSpecK; ++i) acc[i] = cmk(0.0, 0.0);
    if (s0 < s1) load(s0, cur);
    for (int s = s0; s < s1; ++s) {
      const size_t row = (size_t)s * nchan + n;
      const double w = weight[row], ph = phase[row];
      if (s + 1 < s1) load(s + 1, nxt);
      if (w != 0.0) {  // uniform per workgroup
        const double2 st = turn_phasor(256.0, ph);
        double2 e = cscale(turn_phasor((double)(kb + tid), ph), w);
#pragma unroll
        for (int i = 0; i < kRotSpecK; ++i) {
          if (i > 0) e = cmul(e, st);
          acc[i] = cadd(acc[i], cmul(cur[i], e));
        }
      }
#pragma unroll
      for (int i = 0; i < kRotSpecK; ++i) cur[i] = nxt[i];
    }
#pragma unroll
    for (int i = 0; i < kRotSpecK; ++i) {
      const int k = kb + tid + 256 * i;
      if (k <= N) out[k] = acc[i];
    }
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
// Per-channel reduced chi2 of a fitted portrait, as GetTOAs.show_fit /
// get_channels_to_zap form it (pptoas.py:1389-1402, 1236; get_red_chi2,
// pplib.py:727-749).  With D = rfft(data[r]) e^{2 pi i k phase[r]} (the
// rotate_portrait_full of the data) and M = rfft(model[mrow]) / (1 + 2 pi i
// k tau[r]) (the scattered template), the time-domain residual sum follows
// from Parseval on R = D - scale[r] M (irfft drops Im R_0 and Im R_N):
//   out[r] = (Re(R_0)^2 + Re(R_N)^2 + 2 sum_{0<k<N} |R_k|^2) / nbin / errs[r]^2 / dof
// One workgroup per row; both FFTs in LDS, nothing materialised in HBM.
// ---------------------------------------------------------------------------
template <int LOGN>
__global__ __launch_bounds__(kBlock) void k_resid_chi2(ResidArgs a, const double2* __restrict__ tw) {
  constexpr int N = 1 << LOGN;
  constexpr int KI = (N + 1 + kBlock - 1) / kBlock;
  __shared__ double2 buf[N + 1];
  __shared__ double red[kWaves];
  const int r = blockIdx.x;
  load_row<LOGN>(buf, a.data + (size_t)r * 2 * N);
  __syncthreads();
  lds_fft<LOGN, false>(buf, tw);
  const double ph = a.phase ? a.phase[r] : 0.0;
  double2 xs[(N + kBlock) / kBlock + 1];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = threadIdx.x + i * kBlock;
    if (k <= N) xs[i] = cmul(rfft_post<LOGN>(buf, k, tw), turn_phasor((double)k, ph));
  }
  __syncthreads();
  load_row<LOGN>(buf, a.model + (size_t)(a.model_row ? a.model_row[r] : r) * 2 * N);
  __syncthreads();
  lds_fft<LOGN, false>(buf, tw);
  const double sc = a.scale[r];
  const double t2 = a.tau ? 2.0 * M_PI * a.tau[r] : 0.0;
  double acc = 0.0;
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = threadIdx.x + i * kBlock;
    if (k <= N) {
      double2 m = rfft_post<LOGN>(buf, k, tw);
      if (t2 != 0.0) {  // m / (1 + i w),  w = 2 pi k tau
        const double w = t2 * (double)k, d = 1.0 / fma(w, w, 1.0);
        m = cmk(fma(m.y, w, m.x) * d, fma(-m.x, w, m.y) * d);
      }
      const double2 q = cmk(fma(-sc, m.x, xs[i].x), fma(-sc, m.y, xs[i].y));
      // irfft keeps only the real part of the DC and Nyquist terms
      acc += (k == 0 || k == N) ? q.x * q.x : 2.0 * cabs2(q);
    }
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) {
    const double e = a.errs[r];
    a.out[r] = acc / (double)(2 * N) / (e * e) / a.dof;
  }
}

// ---------------------------------------------------------------------------
// explicit instantiations (nbin = 64 ... 8192  <=>  LOGN = 5 ... 12)
// ---------------------------------------------------------------------------
#define PPF_INST(L)                                                                          \
  template __global__ void k_model_spec<L>(const double*, double2*, double*, int, int,       \
                                           const double2*, double*);                         \
  template __global__ void k_data_xspec<L, false>(SpecArgs);                                 \
  template __global__ void k_data_xspec<L, true>(SpecArgs);                                  \
  template __global__ void k_phase_shift<L>(PhaseShiftArgs);                                 \
  template __global__ void k_rotate_rows<L>(const double*, const double*, const double*,     \
                                            double*, const double2*);                        \
  template __global__ void k_resid_chi2<L>(ResidArgs, const double2*);                       \
  template __global__ void k_irfft_rows<L>(const double2*, double*, const double2*);        \
  template __global__ void k_rfft_rows<L>(const double*, double2*, const double2*);         \
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
