// ppfit_taylor.hip -- the cross-spectrum-free solver for phase-family fits.
//
// For fits whose channels differ only by a phase shift phi_n (fit flags over
// phi, DM, GM with tau = 0; the get_TOAs headline path and ppalign), every
// quantity the objective, gradient and Hessian need from a channel is
//   C_n(phi_n)   = Re  sum_k X_nk e^{2 pi i k phi_n}        (pptoaslib.py:431)
//   dC_n/dphi_n  ∝ Im  sum_k k X_nk e^{2 pi i k phi_n}      (pptoaslib.py:437-449)
//   d2C_n/dphi_n2 ∝ Re sum_k k^2 X_nk e^{2 pi i k phi_n}    (pptoaslib.py:451-461)
// with X_nk = D_nk conj(M_nk).  Instead of writing X (16 B per cell) and
// re-reading it on every trust-region evaluation, k_moments transforms the
// data rows once more and reduces each channel to kMT Taylor moments about a
// centre phi_c,n:
//   T_nm = sum_k v_k^m X_nk e^{2 pi i k phi_c,n},   v_k = k / N,
// so that any later evaluation within |2 pi N (phi_n - phi_c,n)| <= kTaylorY
// is a kMTerm-term series (taylor_cells in ppfit_fit.hip) accurate to the
// fp64 rounding of the exact sums.  k_solve_taylor runs scipy's trust-ncg
// on those series; a proposal outside the radius of both stored centres
// parks the subint with its state saved, the host recentres it with one
// more k_moments pass over its data, and the solve resumes.  Per subint the
// data portrait is read twice (k_data_xspec, k_moments) and nothing of size
// nchan x nharm is written.
#include "ppfit_kernels.hpp"

namespace ppf {

// Reduce 2*NH values per lane over a wave so that, afterwards, each lane
// holds NH of them summed over the lanes that differ from it in bit `o`
// (lanes with that bit set keep the upper half).
template <int NH>
__device__ __forceinline__ void rs_step(const double* v, double* out, int o, bool upper) {
#pragma unroll
  for (int i = 0; i < NH; ++i) {
    const double keep = upper ? v[NH + i] : v[i];
    const double send = upper ? v[i] : v[NH + i];
    out[i] = keep + __shfl_xor(send, o);
  }
}

// The same step for o = 32 / 16 with v_permlane32_swap / v_permlane16_swap:
// swapping the upper half-wave (odd 16-lane rows) of `lo` with the lower half
// (even rows) of `hi` leaves lo + hi = the pair sum of the half each lane
// keeps, with no lane select and no LDS-routed shuffle.
template <int O>
__device__ __forceinline__ double pair_swap_sum(double lo, double hi) {
  const unsigned long long a = __double_as_longlong(lo), b = __double_as_longlong(hi);
  unsigned a0 = (unsigned)a, a1 = (unsigned)(a >> 32), b0 = (unsigned)b, b1 = (unsigned)(b >> 32);
  if constexpr (O == 32) {
    const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
    const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
    a0 = r0[0]; b0 = r0[1]; a1 = r1[0]; b1 = r1[1];
  } else {
    static_assert(O == 16, "permlane swaps exist for 16 and 32");
    const auto r0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
    const auto r1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
    a0 = r0[0]; b0 = r0[1]; a1 = r1[0]; b1 = r1[1];
  }
  return __longlong_as_double((long long)(((unsigned long long)a1 << 32) | a0)) +
         __longlong_as_double((long long)(((unsigned long long)b1 << 32) | b0));
}
template <int NH, int O>
__device__ __forceinline__ void rs_swap(const double* v, double* out) {
#pragma unroll
  for (int i = 0; i < NH; ++i) out[i] = pair_swap_sum<O>(v[i], v[NH + i]);
}

// Moment chunks: moments are formed 8 at a time (m in [8c, 8c + 8)); after
// chunk c the row's own absolute moments bound the truncation of a series
// that stops at Mt = 8c + 6 terms (T up to index Mt + 1 is stored):
//   |sum_{m >= Mt} (iy)^m/m! T_{m+p}| <= A_Mt e^Y Y^Mt / Mt!,
//   A_m = sum_k v_k^m (|Re W_k| + |Im W_k|)  (non-increasing in m, v <= 1),
// and the row stops once that is <= 2^-57 A_2, i.e. below the rounding of the
// exact sums (which is ~eps sum_k k^p |W_k|, and A_2 <= A_1 <= A_0).  Pulse
// spectra sit at low harmonics, so most rows stop after 2 chunks instead of
// the worst case 4.  The count of stored moments goes to Tcnt.
__device__ __forceinline__ double taylor_tail_factor(int Mt) {
  // e^3 * 3^Mt / Mt! for Mt = 6, 14, 22, 30 (kTaylorY = 3)
  switch (Mt) {
    case 6: return 20.085536923187668 * 729.0 / 720.0;
    case 14: return 20.085536923187668 * 4782969.0 / 87178291200.0;
    case 22: return 20.085536923187668 * 31381059609.0 / 1.1240007277776077e21;
    default: return 20.085536923187668 * 205891132094649.0 / 2.652528598121911e32;
  }
}

template <int LOGN>
struct MomentsCfg {
  static constexpr int N = 1 << LOGN;
  static constexpr int WPB = LOGN <= 10 ? 4 : (LOGN == 11 ? 2 : 1);
  static constexpr int NB = N + 8;
  static constexpr int NPI = (N / 2 + 1 + 63) / 64;
};

// ---------------------------------------------------------------------------
// k_moments: one workgroup per subint (or per listed subint when recentring);
// wave w transforms channels n = w, w + WPB, ... and writes T[c][wslot][n].
// ---------------------------------------------------------------------------
template <int LOGN>
__global__ __launch_bounds__(kBlock, 2) void k_moments(FitArgs a) {
  using Cfg = MomentsCfg<LOGN>;
  constexpr int N = Cfg::N;
  constexpr int WPB = Cfg::WPB;
  constexpr int NPI = Cfg::NPI;
  constexpr int NTW = PassTw<LOGN>::SIZE;
  constexpr int KW = (N + 1 + 63) / 64;   // harmonics per lane (k = lane + 64 i <= N)
  static_assert(kMT == 32, "moment chunks below assume 4 x 8 moments");
  __shared__ double2 bufs[WPB][Cfg::NB];
  __shared__ double2 twl[NTW];
  const int c = a.rq_list ? a.rq_list[blockIdx.x] : (int)blockIdx.x;
  const int s = a.sub0 + c;
  SolveState& st = a.st[c];
  if (!st.taylor) return;
  const int slot = st.wslot;
  const int nchan = a.nchan;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint8_t* mask = a.mask ? a.mask + (size_t)s * nchan : nullptr;
  const double* drow0 = a.data + (size_t)s * nchan * (2 * N);
  double2* buf = bufs[w];
  WaveRow<LOGN> row;
  int n = next_chan(w, WPB, nchan, mask);
  if (n < nchan) row.load(drow0 + (size_t)n * 2 * N, lane);
  fill_pass_tw<LOGN>(twl, a.tw, tid, WPB * 64);
  double xc[5], refs[3];
#pragma unroll
  for (int i = 0; i < 5; ++i) xc[i] = st.xc[slot][i];
#pragma unroll
  for (int i = 0; i < 3; ++i) refs[i] = st.refs[i];
  const double P = a.P[s];
  const int midx = a.model_idx ? a.model_idx[s] : 0;
  const double* fr = a.freqs + (size_t)s * nchan;
  const double iKs = 1.0 / (double)N;
  double sw, cw;
  sincospi(-(double)lane / (double)N, &sw, &cw);
  const double2 w0 = cmk(cw, sw);
  double ss, cs;
  sincospi(-64.0 / (double)N, &ss, &cs);
  const double2 wstep = cmk(cs, ss);
  __syncthreads();  // twl
  while (n < nchan) {
    row.store(buf, drow0 + (size_t)n * 2 * N, lane);
    const int nn = next_chan(n + WPB, WPB, nchan, mask);
    if (nn < nchan) row.load(drow0 + (size_t)nn * 2 * N, lane);
    fft_sync<true>();
    wave_fft<LOGN>(buf, twl, lane);
    // W_k = D_k conj(M_k) e^{2 pi i k phi_c}, written over the packed FFT in
    // (k, N-k) pairs (each pair's two slots are read and written by one lane)
    const double phic = phase_frac(xc, fr[n], refs, P);
    double2 e = turn_phasor((double)lane, phic);
    const double2 estep = turn_phasor(64.0, phic);
    const double2 EN = turn_phasor((double)N, phic);
    const double2* Mr = a.M + ((size_t)midx * nchan + n) * a.NHP;
    double2 tw = w0;
#pragma unroll 2
    for (int i = 0; i < NPI; ++i) {
      const int k = lane + 64 * i;
      if (i > 0) { tw = cmul(tw, wstep); e = cmul(e, estep); }
      if (k <= N / 2) {
        const double2 mk = Mr[k], mn = Mr[N - k];
        double2 xk, xn;
        rfft_pair<LOGN>(buf, k, tw, xk, xn);
        const double2 wk = cmul(cmulc(xk, mk), e);
        const double2 wn = cmul(cmulc(xn, mn), cmul(EN, cconj(e)));
        if (k < N / 2) buf[N - k] = wn;  // k = 0: W_N goes to the spare slot N
        buf[k] = wk;
      }
    }
    fft_sync<true>();
    double* Tn = reinterpret_cast<double*>(a.T + (((size_t)c * 2 + slot) * nchan + n) * kMT);
    int cnt = kMT;
    // sweep 0: moments 0..15 (the usual need) with A_2 and A_14
    double A2, At;
    {
      double acc[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) acc[j] = 0.0;
      double a2 = 0.0, at = 0.0;
#pragma unroll 1
      for (int i = 0; i < KW; ++i) {
        const int k = lane + 64 * i;
        if (k <= N) {
          const double2 W = buf[k];
          const double v = (double)k * iKs;
          const double aw = fabs(W.x) + fabs(W.y);
          double pw = 1.0;
#pragma unroll
          for (int m = 0; m < 16; ++m) {
            acc[2 * m] = fma(pw, W.x, acc[2 * m]);
            acc[2 * m + 1] = fma(pw, W.y, acc[2 * m + 1]);
            if (m == 2) a2 = fma(pw, aw, a2);
            if (m == 14) at = fma(pw, aw, at);
            if (m < 15) pw *= v;
          }
        }
      }
      // 32 -> 16 -> ... -> 1 value per lane pair: lane L holds value L >> 1
      double r16[16], r8[8], r4[4], r2[2], r1[1];
      rs_swap<16, 32>(acc, r16);
      rs_swap<8, 16>(r16, r8);
      rs_step<4>(r8, r4, 8, (lane & 8) != 0);
      rs_step<2>(r4, r2, 4, (lane & 4) != 0);
      rs_step<1>(r2, r1, 2, (lane & 2) != 0);
      r1[0] += __shfl_xor(r1[0], 1);
      if ((lane & 1) == 0) Tn[lane >> 1] = r1[0];
      A2 = wave_sum(a2);
      At = wave_sum(at);
    }
    if (!(At * taylor_tail_factor(14) <= 0x1p-57 * A2)) {
      // sweeps 1, 2: moments 16..23, 24..31 while the bound is not met
#pragma unroll 1
      for (int ch = 2; ch < 4; ++ch) {
        double acc[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = 0.0;
        double at = 0.0;
#pragma unroll 1
        for (int i = 0; i < KW; ++i) {
          const int k = lane + 64 * i;
          if (k <= N) {
            const double2 W = buf[k];
            const double v = (double)k * iKs;
            const double v2 = v * v, v4 = v2 * v2, v8 = v4 * v4, v16 = v8 * v8;
            double pw = ch == 2 ? v16 : v16 * v8;
            const double aw = fabs(W.x) + fabs(W.y);
#pragma unroll
            for (int m = 0; m < 8; ++m) {
              acc[2 * m] = fma(pw, W.x, acc[2 * m]);
              acc[2 * m + 1] = fma(pw, W.y, acc[2 * m + 1]);
              if (m == 6) at = fma(pw, aw, at);
              if (m < 7) pw *= v;
            }
          }
        }
        // 16 -> 8 -> 4 -> 2 -> 1 values per lane, then lane bits 1, 0
        double r8[8], r4[4], r2[2], r1[1];
        rs_swap<8, 32>(acc, r8);
        rs_swap<4, 16>(r8, r4);
        rs_step<2>(r4, r2, 8, (lane & 8) != 0);
        rs_step<1>(r2, r1, 4, (lane & 4) != 0);
        r1[0] += __shfl_xor(r1[0], 2);
        r1[0] += __shfl_xor(r1[0], 1);
        if ((lane & 3) == 0) Tn[16 * ch + (lane >> 2)] = r1[0];
        At = wave_sum(at);
        if (At * taylor_tail_factor(8 * ch + 6) <= 0x1p-57 * A2 || ch == 3) {
          cnt = 8 * ch + 8;
          break;
        }
      }
    } else {
      cnt = 16;
    }
    if (lane == 0) a.Tcnt[((size_t)c * 2 + slot) * nchan + n] = cnt;
    fft_sync<true>();  // every lane is done with buf before the next row lands
    n = nn;
  }
  if (tid == 0) st.mvalid |= 1 << slot;
}

// ---------------------------------------------------------------------------
// k_solve_taylor: k_solve<false> (ppfit_fit.hip) with every evaluation a
// Taylor series about one of the subint's two stored centres.  Same scipy
// trust-ncg control flow, same nfev / status semantics.
// ---------------------------------------------------------------------------
struct TaylorShared {
  double x[5], xp[5];
  double out[48];
  double red[kWaves][48];
  int done, nok, slot, park, tslot;
};

__device__ __forceinline__ int pick_centre(const FitArgs& a, const Meta& m, const SolveState& st,
                                           int c, const double* prm, const double* refs, double P,
                                           double* red, TaylorSrc& ts) {
  const double Ks = 0.5 * (double)a.nbin;
  int best = -1;
  double by = INFINITY;
  for (int q = 0; q < 2; ++q) {
    if (!(st.mvalid & (1 << q))) continue;
    const TaylorSrc tq{a.T + ((size_t)c * 2 + q) * a.nchan * kMT,
                       a.Tcnt + ((size_t)c * 2 + q) * a.nchan, st.xc[q], st.refs, true};
    const double y = taylor_reach(m, prm, refs, tq, P, Ks, red);
    if (y <= kTaylorY && y < by) { by = y; best = q; ts = tq; }
  }
  return best;
}

__global__ __launch_bounds__(kBlock) void k_solve_taylor(FitArgs a) {
  extern __shared__ __align__(16) unsigned char dyn[];
  __shared__ TaylorShared sh;
  __shared__ double refs[3];
  const int c = blockIdx.x, s = a.sub0 + c, tid = threadIdx.x;
  const int lane = tid & 63;
  SolveState& st = a.st[c];
  if (!st.taylor || st.fin) return;
  const Meta m = load_meta(a, c, s, dyn, &sh.nok);
  const double P = a.P[s];
  if (tid < 5) sh.x[tid] = st.x[tid];
  if (tid < 3) refs[tid] = st.refs[tid];
  if (tid == 0) { sh.done = (m.nok == 0); sh.slot = st.slot; sh.park = 0; sh.tslot = st.xslot; }
  __syncthreads();
  double* acc0 = a.acc + (size_t)c * 2 * a.nchan * NACC;
  // wave-0 solver state (lane i < 5 owns component i; scalars are uniform)
  double f = 0.0, g = 0.0, xl = 0.0, Hrow[5] = {0, 0, 0, 0, 0};
  double tr = 1.0, predv = 0.0, pl = 0.0;
  int hits = 0, k = 0, status = (m.nok == 0) ? -1 : 0, nfev = 0;
  int phase = st.phase;
  if (tid < 64 && phase == 1) {
    f = st.fun;
    g = lane < 5 ? st.g[lane] : 0.0;
    xl = lane < 5 ? sh.x[lane] : 0.0;
    if (lane < 5)
      for (int j = 0; j < 5; ++j) Hrow[j] = st.H[lane * 5 + j];
    tr = st.tr;
    k = st.kit;
    nfev = st.nfev;
  }
  auto load_fgh = [&](double& ff, double& gg, double (&HH)[5]) {
    ff = sh.out[0];
    gg = lane < 5 ? sh.out[1 + lane] : 0.0;
#pragma unroll
    for (int p = 0; p < 15; ++p) {
      const double v = sh.out[6 + p];
      if (lane == pair_i(p)) HH[pair_j(p)] = v;
      if (lane == pair_j(p)) HH[pair_i(p)] = v;
    }
  };
  // Park: save the wave-0 state, queue a recentre at p, leave.
  auto park = [&](const double* p) {
    if (tid < 64) {
      if (lane < 5) {
        st.g[lane] = g;
        for (int j = 0; j < 5; ++j) st.H[lane * 5 + j] = Hrow[j];
      }
      if (lane == 0) {
        st.fun = f;
        st.tr = tr;
        st.kit = k;
        st.nfev = nfev;
        st.phase = phase;
        st.slot = sh.slot;
        st.xslot = sh.tslot;
        const int wsl = sh.tslot ^ 1;
        st.wslot = wsl;
        st.mvalid &= ~(1 << wsl);
        for (int i = 0; i < 5; ++i) { st.xc[wsl][i] = p[i]; st.x[i] = sh.x[i]; }
        const int q = atomicAdd(a.rq_count, 1);
        a.rq_list[q] = c;
      }
    }
  };
  if (!sh.done && phase == 0) {
    TaylorSrc ts{};
    const int q = pick_centre(a, m, st, c, sh.x, refs, P, sh.red[0], ts);
    if (q < 0) { park(sh.x); return; }
    sweep<0, false>(a, m, c, s, sh.x, refs, P, acc0 + (size_t)sh.slot * a.nchan * NACC, sh.out,
                    sh.red, ts);
    if (tid < 64) {
      load_fgh(f, g, Hrow);
      xl = lane < 5 ? sh.x[lane] : 0.0;
      nfev = 1;
    }
    if (tid == 0) sh.tslot = q;
    phase = 1;
  }
  while (!sh.done) {
    if (tid < 64) {
      const double jm = sqrt(dot8(g, g));
      if (!(jm >= -1.0)) {  // NaN gradient: scipy's loop condition fails
        status = 0;
        if (lane == 0) sh.done = 1;
      } else {
        pl = steihaug(f, g, Hrow, tr, hits);
        predv = model_val(f, g, Hrow, pl);
        if (lane < 5) sh.xp[lane] = xl + pl;
      }
    }
    __syncthreads();
    if (sh.done) break;
    TaylorSrc ts{};
    const int q = pick_centre(a, m, st, c, sh.xp, refs, P, sh.red[0], ts);
    if (q < 0) {
      // the proposal is recomputed bit-identically from the saved state on resume
      park(sh.xp);
      return;
    }
    double* sl = acc0 + (size_t)(sh.slot ^ 1) * a.nchan * NACC;
    sweep<0, false>(a, m, c, s, sh.xp, refs, P, sl, sh.out, sh.red, ts);
    if (tid < 64) {
      double fp, gp, Hp[5] = {0, 0, 0, 0, 0};
      load_fgh(fp, gp, Hp);
      nfev += 1;
      const double actual = f - fp;
      const double pred = f - predv;
      if (pred <= 0.0) {
        status = 2;
        if (lane == 0) sh.done = 1;
      } else {
        const double rho = actual / pred;
        if (rho < 0.25) tr *= 0.25;
        else if (rho > 0.75 && hits) tr = fmin(2.0 * tr, 1000.0);
        if (rho > 0.15) {
          xl = xl + pl;
          f = fp;
          g = gp;
#pragma unroll
          for (int j = 0; j < 5; ++j) Hrow[j] = Hp[j];
          if (lane == 0) { sh.slot ^= 1; sh.tslot = q; }
          if (lane < 5) sh.x[lane] = xl;
        }
        k += 1;
        if (k >= 1000) {
          status = 1;
          if (lane == 0) sh.done = 1;
        }
      }
    }
    __syncthreads();
  }
  if (tid < 5) st.x[tid] = sh.x[tid];
  if (tid == 0) {
    st.fun = m.nok ? f : NAN;
    st.nfev = m.nok ? nfev : 0;
    st.status = status;
    st.slot = sh.slot;
    st.xslot = sh.tslot;
    st.fin = 1;
    st.scat_post = false;
  }
}

// ---------------------------------------------------------------------------
// Device self-test of the cross-lane primitives (DPP, permlane swaps,
// readlane) whose lane semantics the reductions above rely on.
// fails[t] counts the lanes where test t disagrees with its definition.
// ---------------------------------------------------------------------------
__global__ void k_selftest(int* fails) {
  const int l = threadIdx.x & 63;
  const double x = (double)l;
  auto chk = [&](int t, bool ok) { if (!ok) atomicAdd(&fails[t], 1); };
  chk(0, wave_sum(x) == 2016.0);
  chk(1, group8_sum(x) == (double)(8 * (l & ~7) + 28));
  chk(2, swap_rows<16>(x) == (double)(l ^ 16));
  chk(3, swap_rows<32>(x) == (double)(l ^ 32));
  chk(4, pair_swap_sum<32>(x, 100.0 + x) ==
             (l < 32 ? (double)(2 * l + 32) : 200.0 + (double)(2 * l - 32)));
  chk(5, pair_swap_sum<16>(x, 100.0 + x) ==
             ((l & 16) == 0 ? (double)(2 * l + 16) : 200.0 + (double)(2 * l - 16)));
  chk(6, wave_max(x * (l == 37 ? 2.0 : 1.0)) == 74.0);
  chk(7, lane0(x + 3.0) == 3.0 && lane_at<4>(x) == 4.0);
  chk(8, dpp_mov<0xB1>(x) == (double)(l ^ 1) && dpp_mov<0x4E>(x) == (double)(l ^ 2));
}

#define PPF_INST_TAYLOR(L) template __global__ void k_moments<L>(FitArgs);
PPF_INST_TAYLOR(5)
PPF_INST_TAYLOR(6)
PPF_INST_TAYLOR(7)
PPF_INST_TAYLOR(8)
PPF_INST_TAYLOR(9)
PPF_INST_TAYLOR(10)
PPF_INST_TAYLOR(11)
PPF_INST_TAYLOR(12)
#undef PPF_INST_TAYLOR

}  // namespace ppf
