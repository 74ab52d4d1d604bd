// ppfit_fit.hip -- the batched wideband fit (kernels (c), (d), (e) of SURVEY.md §8).
//
// One workgroup owns one subint for the whole fit and re-reads that subint's
// cross-spectrum X (written once by k_data_xspec) on every objective pass.
//   k_guess : initial phase of get_TOAs / ppalign (pptoas.py:420-456,
//             ppalign.py:180-185) -- FFTFIT brute force + Nelder-Mead.
//   k_solve : scipy trust-ncg (gtol=-1, pptoaslib.py:1001-1014) with Steihaug
//             CG, every pass one fused sweep giving f, g and H
//             (pptoaslib.py:525-643).
//   k_post  : zero-covariance frequencies (pptoaslib.py:733-906), phi/tau at
//             nu_out (1040-1065), the with-scales Hessian and its Woodbury
//             inverse (645-731, 1069-1077), snr and chi2 (1079-1085).
//
// Cell-pass lane layout: a wave holds 8 channels x 8 harmonic phases; lane
// (g, h) walks k = h, h+8, ... of channel g with the phasor advanced by the
// angle-addition recurrence and re-seeded exactly every 32 steps, so one
// wave load instruction covers 8 full 128-byte segments of X.
#include "ppfit_kernels.hpp"

namespace ppf {

constexpr int NACC = 10;
static_assert(NACC == kScatAcc, "k_scat_sweep's LDS rows (scat_sweep_lds)");
constexpr double kTwoPi = 2.0 * kPi;
constexpr double kFourPi2 = 4.0 * kPi * kPi;
constexpr double kDconst2 = kDconst * kDconst;  // Dconst**2

// upper-triangle pair p -> (i, j); compile-time so unrolled loops index
// ChanDeriv members statically (a runtime index would push it to scratch)
__host__ __device__ constexpr int pair_i(int p) {
  return p < 5 ? 0 : (p < 9 ? 1 : (p < 12 ? 2 : (p < 14 ? 3 : 4)));
}
__host__ __device__ constexpr int pair_j(int p) {
  return p < 5 ? p : (p < 9 ? p - 4 : (p < 12 ? p - 7 : (p < 14 ? p - 9 : 4)));
}

// ---------------------------------------------------------------------------
// per-subint channel metadata in LDS
// ---------------------------------------------------------------------------
struct Meta {
  int* chan;    // ok-channel ordinal -> channel index
  double* fr;   // frequency
  double* iw2;  // 1 / errs_FT^2, errs_FT = sigma sqrt(nbin/2) (pptoaslib.py:980-984)
  double* pn;   // sum_{k>=1} |M_nk|^2 (Sbp with tau = 0)
  double* d1;   // d phi_n / d DM at the subint's nu_fit  (pptoaslib.py:216-225)
  double* d2;   // d phi_n / d GM at the subint's nu_fit
  int nok;
};

__device__ __forceinline__ size_t meta_bytes(int nchan) {
  return (size_t)nchan * (5 * sizeof(double) + sizeof(int));
}

// refs = the subint's nu_fit (SolveState.refs, set by k_guess)
__device__ Meta load_meta(const FitArgs& a, int c, int s, unsigned char* dyn, int* s_nok) {
  Meta m;
  const int nchan = a.nchan;
  m.fr = reinterpret_cast<double*>(dyn);
  m.iw2 = m.fr + nchan;
  m.pn = m.iw2 + nchan;
  m.d1 = m.pn + nchan;
  m.d2 = m.d1 + nchan;
  m.chan = reinterpret_cast<int*>(m.d2 + nchan);
  const int tid = threadIdx.x, lane = tid & 63;
  const uint8_t* mask = a.mask ? a.mask + (size_t)s * nchan : nullptr;
  if (tid < 64) {
    int base = 0;
    for (int n0 = 0; n0 < nchan; n0 += 64) {
      const int n = n0 + lane;
      const bool ok = n < nchan && (!mask || mask[n]);
      const unsigned long long b = __ballot(ok);
      const int rank = __popcll(b & ((1ull << lane) - 1ull));
      if (ok) m.chan[base + rank] = n;
      base += __popcll(b);
    }
    if (lane == 0) *s_nok = base;
  }
  __syncthreads();
  m.nok = *s_nok;
  const int midx = a.model_idx ? a.model_idx[s] : 0;
  const double half = 0.5 * (double)a.nbin;
  const double P = a.P[s];
  const double* refs = a.st[c].refs;
  const double r0 = 1.0 / (refs[0] * refs[0]);
  const double r1 = 1.0 / (refs[1] * refs[1]);
  for (int j = tid; j < m.nok; j += kBlock) {
    const int n = m.chan[j];
    const double fr = a.freqs[(size_t)s * nchan + n];
    m.fr[j] = fr;
    const double sg = a.sig[(size_t)c * nchan + n];
    m.iw2[j] = 1.0 / (sg * sg * half);
    m.pn[j] = a.pn[(size_t)midx * nchan + n];
    const double f2 = 1.0 / (fr * fr);
    m.d1[j] = kDconst * (f2 - r0) / P;
    m.d2[j] = kDconst2 * (f2 * f2 - r1 * r1) / P;
  }
  __syncthreads();
  return m;
}

// Python's float % 1.0 (CPython float_rem): result in [0, 1).
__device__ __forceinline__ double pymod1(double x) {
  double r = fmod(x, 1.0);
  if (r != 0.0) {
    if (r < 0.0) r += 1.0;
  } else {
    r = 0.0;
  }
  return r;
}

// phase_transform(..., mod=True) wrap, pplib.py:2610-2613
__device__ __forceinline__ double wrap_half(double p) {
  if (fabs(p) >= 0.5) p = pymod1(p);
  if (p >= 0.5) p -= 1.0;
  return p;
}

// Sum N values over the block; result valid in all threads.
template <int N>
__device__ __forceinline__ void block_sum_vec(double (&v)[N], double (*red)[48]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const double t = wave_sum(v[i]);
    if (lane == 0) red[w][i] = t;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double t = 0.0;
    for (int q = 0; q < kWaves; ++q) t += red[q][i];
    v[i] = t;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Cell sweeps over one channel row of X (lane's harmonics k = h + 8 j)
// ---------------------------------------------------------------------------
// The row is streamed with the next U harmonics' loads in flight while the
// current U are accumulated (software pipelining: one HBM latency per row,
// not one per step); the accumulation order is unchanged.
constexpr int kPipe = 4;

// cells in flight per lane in the scattering sweep and k_scat_sweep's
// workgroups per CU (launch bound); A/B knobs for diagnostic builds.
// r05: k_scat_sweep's two-phase evaluation (sweep_scat_split) needs 167
// VGPRs at three workgroups per CU with no spills (the one-phase sweep: 223,
// two): config 3 solve 13.26-13.28 -> 12.68-12.74 ms, fits bitwise the same
// (U = 2 at three: 13.05-13.07; two-phase at two workgroups: 13.28)
#ifndef PPF_SCAT_U
#define PPF_SCAT_U 4
#endif
#ifndef PPF_SCAT_TWO_PHASE
#define PPF_SCAT_TWO_PHASE 1
#endif
#ifndef PPF_SCAT_WG_PER_CU
#define PPF_SCAT_WG_PER_CU (PPF_SCAT_TWO_PHASE ? 3 : 1)
#endif  // divides the 32-step re-seed period

__device__ __forceinline__ void cells_phase(const double2* __restrict__ Xr, int J, int h,
                                            double phif, double* acc) {
  const double2 step = turn_phasor(8.0, phif);
  const double2 zero = cmk(0.0, 0.0);
  double2 e = cmk(1.0, 0.0);
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  // the register-set alternation of cells_scat (no copies of in-flight loads)
  constexpr int U = kPipe;
  const int Jpad = (J + U - 1) / U * U;
  double2 xa[U], xb[U];
  auto load = [&](int jb, double2 (&x)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = Xr[h + 8 * min(jb + u, J - 1)];
  };
  auto consume = [&](int jb, const double2 (&xs)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int jj = jb + u;
      if (jj >= Jpad) break;
      const int k = h + 8 * jj;
      if ((jj & 31) == 0) e = turn_phasor((double)k, phif);
      else e = cmul(e, step);
      const double2 x = jj < J ? xs[u] : zero;
      const double wr = fma(x.x, e.x, -x.y * e.y);
      const double wi = fma(x.x, e.y, x.y * e.x);
      const double kd = (double)k;
      a0 += wr;
      a1 = fma(kd, wi, a1);
      a2 = fma(kd * kd, wr, a2);
    }
  };
  load(0, xa);
  load(U, xb);
  for (int jb = 0; jb < Jpad; jb += 2 * U) {
    consume(jb, xa);
    load(jb + 2 * U, xa);
    consume(jb + U, xb);
    load(jb + 3 * U, xb);
  }
  acc[0] = a0; acc[1] = a1; acc[2] = a2;
  for (int i = 3; i < NACC; ++i) acc[i] = 0.0;
}

// With scattering: B = 1/(1 + 2 pi i k tau_n), f = B(B-1)/tau_n and
// g1 = 2 B (B-1)^2 / tau_n^2 give every tau/alpha derivative of B through a
// per-channel real factor (pptoaslib.py:318-356).
// 1 / d for d >= 1 (the scattering denominators 1 + (2 pi k tau)^2): the
// hardware reciprocal refined by two Newton steps -- within an ulp of the
// correctly rounded quotient, at a third of the IEEE division sequence.
__device__ __forceinline__ double rcp_nr(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  return fma(r, fma(-d, r, 1.0), r);
}

// U cells in flight per lane: 4 (measured on config 3: solve 20.8 ms with 2,
// 19.9 with 4, 20.3 with 8, all at two waves per SIMD).
//
// The sweep is vector-issue bound (r04 SQ counters: the SIMDs' VALU issue
// ~0.9 busy), so the loop carries no work that is not arithmetic on a cell:
// the unrolled body covers whole blocks of 2U cells with unclamped,
// unselected loads (constant offsets from one pointer per row), and the
// J mod 2U cells past the last block (J = NHP / 8 is 2^m + 1 for a power-of-
// two nbin: one cell) run one at a time after it.  Each cell's operations and
// the order of the sums are those of the padded loop this replaced, minus
// its zero cells, which only ever added +0.0.
template <int U>
__device__ __forceinline__ void cells_scat(const double2* __restrict__ Xr,
                                           const double* __restrict__ M2r, int J, int h,
                                           double phif, double taun, double* acc) {
  const double2 step = turn_phasor(8.0, phif);
  const double itau = 1.0 / taun;
  const double w0 = kTwoPi * taun;
  double2 e = cmk(1.0, 0.0);
  double a[NACC];
  for (int i = 0; i < NACC; ++i) a[i] = 0.0;
  const double2* __restrict__ xp = Xr + h;
  const double* __restrict__ mp = M2r + h;
  auto cell = [&](int jj, double2 x, double m2) {
    const int k = h + 8 * jj;
    if ((jj & 31) == 0) e = turn_phasor((double)k, phif);
    else e = cmul(e, step);
    const double2 W = cmul(x, e);
    const double kd = (double)k;
    const double aa = w0 * kd;
    const double id = rcp_nr(fma(aa, aa, 1.0));
    const double2 B = cmk(id, -aa * id);
    const double2 Bm1 = cmk(B.x - 1.0, B.y);
    const double2 f = cscale(cmul(B, Bm1), itau);
    const double2 g1 = cscale(cmul(f, Bm1), 2.0 * itau);
    const double2 WB = cmulc(W, B);
    const double2 Wf = cmulc(W, f);
    const double2 Wg = cmulc(W, g1);
    a[0] += WB.x;
    a[1] = fma(kd, WB.y, a[1]);
    a[2] = fma(kd * kd, WB.x, a[2]);
    a[3] += Wf.x;
    a[4] = fma(kd, Wf.y, a[4]);
    a[5] += Wg.x;
    a[6] = fma(cabs2(B), m2, a[6]);
    a[7] = fma(fma(B.x, f.x, B.y * f.y), m2, a[7]);
    a[8] = fma(cabs2(f), m2, a[8]);
    a[9] = fma(fma(B.x, g1.x, B.y * g1.y), m2, a[9]);
  };
  static_assert(32 % U == 0, "phasor re-seed every 32 cells");
  const int Jmain = J / (2 * U) * (2 * U);  // cells of the unrolled blocks
  int jb = 0;
  if (Jmain >= 2 * U) {
    // two register sets of U cells alternate, each reloaded right after it
    // is consumed, so the loop carries no copies of in-flight loads
    double2 xa[U], xb[U];
    double ma[U], mb[U];
    auto load = [&](int j0, double2 (&x)[U], double (&m)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        x[u] = xp[8 * (j0 + u)];
        m[u] = mp[8 * (j0 + u)];
      }
    };
    auto consume = [&](int j0, const double2 (&xs)[U], const double (&ms)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u) cell(j0 + u, xs[u], ms[u]);
    };
    load(0, xa, ma);
    load(U, xb, mb);
    for (; jb + 4 * U <= Jmain; jb += 2 * U) {
      consume(jb, xa, ma);
      load(jb + 2 * U, xa, ma);
      consume(jb + U, xb, mb);
      load(jb + 3 * U, xb, mb);
    }
    consume(jb, xa, ma);
    consume(jb + U, xb, mb);
    jb += 2 * U;
  }
  for (; jb < J; ++jb) cell(jb, xp[8 * jb], mp[8 * jb]);
  for (int i = 0; i < NACC; ++i) acc[i] = a[i];
}

// ---------------------------------------------------------------------------
// Per-channel derived terms: C_n, its phase/scattering derivatives, S_n and
// its derivatives, all divided by errs_FT^2 (pptoaslib.py:390-523).
// ---------------------------------------------------------------------------
struct ChanDeriv {
  double C, C1, C2, F1, F1p, G1, S, SF, SFF, SG;
  double dph[3];   // d phi_n / d(phi, DM, GM)          pptoaslib.py:216-225
  double dts[2];   // d tau_n / d(tau, alpha)            pptoaslib.py:246-257
  double d2ts[3];  // tau-tau, tau-alpha, alpha-alpha    pptoaslib.py:259-274
};

template <bool SCAT>
__device__ __forceinline__ ChanDeriv derive(const double* acc, bool scat, double pn, double iw2,
                                            double fr, const double* prm, double tau_lin,
                                            const double* refs, double P, bool log10_tau,
                                            const double* dpre = nullptr) {
  ChanDeriv d;
  d.C = acc[0] * iw2;
  d.C1 = -kTwoPi * acc[1] * iw2;
  d.C2 = -kFourPi2 * acc[2] * iw2;
  if (SCAT && scat) {
    d.F1 = acc[3] * iw2;
    d.F1p = -kTwoPi * acc[4] * iw2;
    d.G1 = acc[5] * iw2;
    d.S = acc[6] * iw2;
    d.SF = acc[7] * iw2;
    d.SFF = acc[8] * iw2;
    d.SG = acc[9] * iw2;
  } else {
    d.F1 = d.F1p = d.G1 = d.SF = d.SFF = d.SG = 0.0;
    d.S = pn * iw2;
  }
  d.dph[0] = 1.0;
  if (dpre) {  // refs = nu_fit: precomputed in Meta
    d.dph[1] = dpre[0];
    d.dph[2] = dpre[1];
  } else {
    const double f2 = 1.0 / (fr * fr), f4 = f2 * f2;
    const double r0 = 1.0 / (refs[0] * refs[0]);
    const double r1 = 1.0 / (refs[1] * refs[1]);
    d.dph[1] = kDconst * (f2 - r0) / P;
    d.dph[2] = kDconst2 * (f4 - r1 * r1) / P;
  }
  if (!SCAT) {
    d.dts[0] = d.dts[1] = 0.0;
    d.d2ts[0] = d.d2ts[1] = d.d2ts[2] = 0.0;
    return d;
  }
  const double ratio = fr / refs[2];
  const double taus = tau_lin * pow(ratio, prm[4]);
  const double lnr = log(ratio);
  const bool has = tau_lin != 0.0;
  if (!log10_tau) {
    d.dts[0] = has ? taus / tau_lin : 0.0;
    d.dts[1] = lnr * taus;
    d.d2ts[0] = 0.0;
    d.d2ts[1] = has ? d.dts[1] / tau_lin : 0.0;
  } else {
    d.dts[0] = kLn10 * taus;
    d.dts[1] = lnr * taus;
    d.d2ts[0] = kLn10 * d.dts[0];
    d.d2ts[1] = kLn10 * d.dts[1];
  }
  d.d2ts[2] = lnr * d.dts[1];
  return d;
}

__device__ __forceinline__ double dC_(const ChanDeriv& d, int i) {
  return i < 3 ? d.C1 * d.dph[i] : d.dts[i - 3] * d.F1;
}
__device__ __forceinline__ double dS_(const ChanDeriv& d, int i) {
  return i < 3 ? 0.0 : 2.0 * d.dts[i - 3] * d.SF;
}
__device__ __forceinline__ double d2ts_(const ChanDeriv& d, int i, int j) {
  return (i == 0 && j == 0) ? d.d2ts[0] : ((i == 1 && j == 1) ? d.d2ts[2] : d.d2ts[1]);
}
__device__ __forceinline__ double d2C_(const ChanDeriv& d, int i, int j) {
  if (i < 3 && j < 3) return d.C2 * d.dph[i] * d.dph[j];
  if (i < 3) return d.dph[i] * d.dts[j - 3] * d.F1p;
  if (j < 3) return d.dph[j] * d.dts[i - 3] * d.F1p;
  return d.dts[i - 3] * d.dts[j - 3] * d.G1 + d2ts_(d, i - 3, j - 3) * d.F1;
}
__device__ __forceinline__ double d2S_(const ChanDeriv& d, int i, int j) {
  if (i < 3 || j < 3) return 0.0;
  return 2.0 * (d.dts[i - 3] * d.dts[j - 3] * (d.SFF + d.SG) + d2ts_(d, i - 3, j - 3) * d.SF);
}
// Hij_n of pptoaslib.py:624-628 (unmasked)
__device__ __forceinline__ double Hn_(const ChanDeriv& d, int i, int j) {
  const double C = d.C, S = d.S;
  const double dCi = dC_(d, i), dCj = dC_(d, j), dSi = dS_(d, i), dSj = dS_(d, j);
  return -2.0 * (C * C / S) *
         ((d2C_(d, i, j) / C) - (0.5 * d2S_(d, i, j) / S) + (dCi * dCj / (C * C)) +
          (dSi * dSj / (S * S)) - ((dCi * dSj) + (dSi * dCj)) / (C * S));
}

// The same terms with a lane-varying parameter index (i <= j): each operand
// chosen by selects, every case formed with the expression of the constant-
// index version, each operation rounded on its own as numpy rounds the
// reference's (pptoaslib.py:588-628; no contraction into fma).  Each pick selects
// between opaque copies: a select between fields of one aggregate would fold
// into a run-time-indexed load and keep the aggregate in scratch.
__device__ __forceinline__ double opq(double x) {
  asm("" : "+v"(x));
  return x;
}
struct LanePick {
  double ph0, ph1, ph2, ts0, ts1, t2a, t2b, t2c;
  __device__ __forceinline__ double dph(int i) const {
    const double a = opq(ph0), b = opq(ph1), c = opq(ph2);
    return i == 0 ? a : (i == 1 ? b : c);
  }
  __device__ __forceinline__ double dts(int i) const {  // i = 3, 4
    const double a = opq(ts0), b = opq(ts1);
    return i == 4 ? b : a;
  }
  __device__ __forceinline__ double d2ts(int i, int j) const {
    const double a = opq(t2a), b = opq(t2b), c = opq(t2c);
    return (i == 3 && j == 3) ? a : ((i == 4 && j == 4) ? c : b);
  }
};
__device__ __forceinline__ double dCr(const ChanDeriv& d, const LanePick& L, int i) {
#pragma clang fp contract(off)
  const double ph = d.C1 * L.dph(i);
  const double sc = L.dts(i) * d.F1;
  return i < 3 ? ph : sc;
}
__device__ __forceinline__ double dSr(const ChanDeriv& d, const LanePick& L, int i) {
#pragma clang fp contract(off)
  const double sc = 2.0 * L.dts(i) * d.SF;
  return i < 3 ? 0.0 : sc;
}
__device__ __forceinline__ double d2Cr(const ChanDeriv& d, const LanePick& L, int i, int j) {
#pragma clang fp contract(off)
  const double pp = d.C2 * L.dph(i) * L.dph(j);
  const double ps = L.dph(i) * L.dts(j) * d.F1p;
  const double ss = L.dts(i) * L.dts(j) * d.G1 + L.d2ts(i, j) * d.F1;
  return j < 3 ? pp : (i < 3 ? ps : ss);
}
__device__ __forceinline__ double d2Sr(const ChanDeriv& d, const LanePick& L, int i, int j) {
#pragma clang fp contract(off)
  const double ss = 2.0 * (L.dts(i) * L.dts(j) * (d.SFF + d.SG) + L.d2ts(i, j) * d.SF);
  return i < 3 ? 0.0 : ss;
}
__device__ __forceinline__ double Hnr(const ChanDeriv& d, const LanePick& L, int i, int j) {
#pragma clang fp contract(off)
  const double C = d.C, S = d.S;
  const double dCi = dCr(d, L, i), dCj = dCr(d, L, j), dSi = dSr(d, L, i), dSj = dSr(d, L, j);
  return -2.0 * (C * C / S) *
         ((d2Cr(d, L, i, j) / C) - (0.5 * d2Sr(d, L, i, j) / S) + (dCi * dCj / (C * C)) +
          (dSi * dSj / (S * S)) - ((dCi * dSj) + (dSi * dCj)) / (C * S));
}
// out-slot t of a MODE-0 sweep for one channel (q = C^2 / S): 0 f, 1 + i
// g_i, 6 + p H pair p; 0 for unfitted parameters and t >= 21
__device__ __forceinline__ double mode0_term(const ChanDeriv& d, const LanePick& L, double q,
                                             int t, int fm) {
#pragma clang fp contract(off)
  const int gi = min(max(t - 1, 0), 4);
  const int p = min(max(t - 6, 0), 14);
  const int pi = p < 5 ? 0 : (p < 9 ? 1 : (p < 12 ? 2 : (p < 14 ? 3 : 4)));
  const int pj = p < 5 ? p : (p < 9 ? p - 4 : (p < 12 ? p - 7 : (p < 14 ? p - 9 : 4)));
  const double gv = -q * (2.0 * dCr(d, L, gi) / d.C - dSr(d, L, gi) / d.S);
  const double hv = Hnr(d, L, pi, pj);
  const bool on = t == 0 || (t < 6 ? ((fm >> gi) & 1) : ((fm >> pi) & (fm >> pj) & 1));
  const double v = t == 0 ? -q : (t < 6 ? gv : hv);
  return (on && t < 21) ? v : 0.0;
}

#ifndef PPF_POST_WG_PER_CU
#define PPF_POST_WG_PER_CU 2  // k_post<false>'s launch bound (A/B knob)
#endif

// phi_n (pptoaslib.py:206-208), reduced to [0, 1)
__device__ __forceinline__ double phase_frac(const double* prm, double fr, const double* refs,
                                             double P) {
  const double f2 = 1.0 / (fr * fr);
  const double r0 = 1.0 / (refs[0] * refs[0]);
  const double r1 = 1.0 / (refs[1] * refs[1]);
  const double ph = prm[0] + kDconst * prm[1] * (f2 - r0) / P +
                    kDconst2 * prm[2] * (f2 * f2 - r1 * r1) / P;
  return ph - floor(ph);
}

// phi_n before reduction (pptoaslib.py:206-208)
__device__ __forceinline__ double phase_full(const double* prm, double fr, const double* refs,
                                             double P) {
  const double f2 = 1.0 / (fr * fr);
  const double r0 = 1.0 / (refs[0] * refs[0]);
  const double r1 = 1.0 / (refs[1] * refs[1]);
  return prm[0] + kDconst * prm[1] * (f2 - r0) / P + kDconst2 * prm[2] * (f2 * f2 - r1 * r1) / P;
}

// ---------------------------------------------------------------------------
// Taylor-moment evaluation of one channel (ppfit_taylor.hip builds T).
// With W_k = X_k e^{2 pi i k phi_c} and v_k = k / Ks, the sums the exact
// sweep forms at phi_c + delta are, for y = 2 pi Ks delta,
//   G_p = sum_k k^p W_k e^{2 pi i k delta} = Ks^p sum_m (i y)^m / m! T_{m+p}.
// (Moments about v = 0, not the band centre: pulse spectra sit at low k, and
// a centred expansion would cancel catastrophically in G_1, G_2.)
// Lane h of the channel's 8 lanes takes m = h, h+8, ... (< kMTerm); the
// result is linear in the partial series, so each lane returns its partial
// acc and the caller's group8_sum completes it exactly as for cells_phase.
// ---------------------------------------------------------------------------
__constant__ double c_inv_fact[kMT] = {
    1.0, 1.0, 0.5, 0.16666666666666666,
    0.041666666666666664, 0.008333333333333333, 0.001388888888888889, 0.0001984126984126984,
    2.48015873015873e-05, 2.7557319223985893e-06, 2.755731922398589e-07, 2.505210838544172e-08,
    2.08767569878681e-09, 1.6059043836821613e-10, 1.1470745597729725e-11, 7.647163731819816e-13,
    4.779477332387385e-14, 2.8114572543455206e-15, 1.5619206968586225e-16, 8.22063524662433e-18,
    4.110317623312165e-19, 1.9572941063391263e-20, 8.896791392450574e-22, 3.8681701706306835e-23,
    1.6117375710961184e-24, 6.446950284384474e-26, 2.4795962632247972e-27, 9.183689863795546e-29,
    3.279889237069838e-30, 1.1309962886447718e-31, 3.7699876288159054e-33, 1.2161250415535181e-34};

struct TaylorSrc {
  const double* T;     // this subint's compact moment rows for one centre: [nchan][kMT],
                       // or null (exact sweeps)
  const double* xc;    // centre params
  const double* refc;  // centre reference frequencies
  bool same = false;   // evaluation refs == refc: offsets from Meta d1/d2
  const double* ifact = nullptr;  // LDS copy of c_inv_fact, or null (constant memory)
  const double* Tl = nullptr;     // LDS copy of moments [0, nl) of these rows: [nchan][nl]
  int nl = 0;
};

// offset from the centre for evaluation refs == centre refs:
// delta_n = dphi + dDM d1_n + dGM d2_n
__device__ __forceinline__ double taylor_delta_lin(const double* prm, const double* xc, double d1,
                                                   double d2) {
  const double d = fma(prm[2] - xc[2], d2, fma(prm[1] - xc[1], d1, prm[0] - xc[0]));
  return d - rint(d);
}

// offset of phi_n(prm, refs) from the centre's phi_n, reduced to [-1/2, 1/2]
__device__ __forceinline__ double taylor_delta(const double* prm, const double* refs,
                                               const TaylorSrc& ts, double fr, double P) {
  double d = phase_full(prm, fr, refs, P) - phase_full(ts.xc, fr, ts.refc, P);
  return d - rint(d);
}

// Channel n's series G_j = sum_m T_{m+j} (i y)^m / m! (j = 0, 1, 2), this
// lane's terms m = h + 8 q.  i^m = i^h for every m of the lane (m = h mod 4),
// so of G_0, G_1, G_2 only Re G_0, Im G_1, Re G_2 are formed, and each reads
// one real part per moment: Re(i^m T_{m+j}) or Im(...) is +-Re T_{m+j} when
// m + j is even and +-Im T_{m+j} when it is odd -- the compact moment
// (kMT doubles per channel).  The lane's sums are those of the complex
// series' selected parts, operation for operation.
__device__ __forceinline__ void taylor_cells(const TaylorSrc& ts, int n, int h, double d,
                                             double Ks, double* acc) {
  // 1/m! by lane-varying m: from LDS when the caller staged it (a constant-
  // memory gather costs a memory round trip per call)
  const double* fz = ts.ifact ? ts.ifact : c_inv_fact;
  const double* __restrict__ Tg = ts.T + (size_t)n * kMT;
  const double* __restrict__ Tl = ts.Tl + (size_t)n * ts.nl;
  const int nl = ts.nl;
  // moment i of the channel: the LDS copy below nl, the HBM rows above
  auto tm = [&](int i) { return i < nl ? Tl[i] : Tg[i]; };
  const double y = kTwoPi * Ks * d;
  double yh = 1.0;
  for (int i = 0; i < h; ++i) yh *= y;
  const double y2 = y * y, y4 = y2 * y2, y8 = y4 * y4;
  double S0 = 0.0, S1 = 0.0, S2 = 0.0;
  double ym = yh;
#pragma unroll
  for (int q = 0; q < (kMTerm + 7) / 8; ++q) {
    const int m = h + 8 * q;
    if (m < kMTerm) {  // T up to index kMTerm + 1 = kMT - 1
      const double cf = ym * fz[m];
      S0 = fma(cf, tm(m), S0);
      S1 = fma(cf, tm(m + 1), S1);
      S2 = fma(cf, tm(m + 2), S2);
    }
    ym *= y8;
  }
  // the signs of i^h: Re G_0 (part of T_m), Im G_1 (T_{m+1}), Re G_2 (T_{m+2})
  double r0, i1, r2;
  switch (h & 3) {
    case 1: r0 = -S0; i1 = S1; r2 = -S2; break;
    case 2: r0 = -S0; i1 = -S1; r2 = -S2; break;
    case 3: r0 = S0; i1 = -S1; r2 = S2; break;
    default: r0 = S0; i1 = S1; r2 = S2; break;
  }
  acc[0] = r0;
  acc[1] = Ks * i1;
  acc[2] = (Ks * Ks) * r2;
  for (int i = 3; i < NACC; ++i) acc[i] = 0.0;
}

// Largest |y_n| of the fitted channels for evaluating prm (at refs) from the
// centre ts; every thread gets it.  red: >= kWaves doubles of LDS.
__device__ double taylor_reach(const Meta& m, const double* prm, const double* refs,
                               const TaylorSrc& ts, double P, double Ks, double* red) {
  double mx = 0.0;
  for (int j = threadIdx.x; j < m.nok; j += kBlock)
    mx = fmax(mx, fabs(ts.same ? taylor_delta_lin(prm, ts.xc, m.d1[j], m.d2[j])
                               : taylor_delta(prm, refs, ts, m.fr[j], P)));
  mx = wave_max(mx);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = mx;
  __syncthreads();
  double r = red[0];
  for (int i = 1; i < kWaves; ++i) r = fmax(r, red[i]);
  __syncthreads();
  return kTwoPi * Ks * r;
}

__device__ __forceinline__ int flag_mask(const FitArgs& a) {
  int fm = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) fm |= a.flags[i] ? 1 << i : 0;
  return fm;
}

// Solver sweep of a phase-family fit from Taylor moments (refs = nu_fit, so
// d phi_n / d(DM, GM) are Meta's d1, d2).  With tau = 0, S_n = p_n / errs^2
// does not depend on the parameters and every term of pptoaslib.py:525-643
// factors into a per-channel scalar times products of dphi_n:
//   f  = sum -C^2/S,  g_i = sum gc dph_i,  H_ij = sum hc dph_i dph_j,
//   gc = -2 C C1 / S,  hc = -2 (C C2 + C1^2) / S,
// so each lane carries 10 running sums over its channel groups and the wave
// reduces them once, instead of 21 reductions per group.
__device__ __forceinline__ void sweep_taylor0(const FitArgs& a, const Meta& m, const double* prm,
                              double* acc_slot, double* out, double (*red)[48],
                              const TaylorSrc& ts) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g8 = lane >> 3, h = lane & 7;
  const double Ks = 0.5 * (double)a.nbin;
  double t[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) t[i] = 0.0;
  const int ngroups = (m.nok + 7) >> 3;
  // a wave's groups two at a time (both series in flight), accumulated in
  // group order
  for (int gi = w; gi < ngroups; gi += 2 * kWaves) {
    double sg[2][3];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = (gi + u * kWaves) * 8 + g8;
      const int jj = j < m.nok ? j : m.nok - 1;
      double acc[NACC];
      taylor_cells(ts, m.chan[jj], h, taylor_delta_lin(prm, ts.xc, m.d1[jj], m.d2[jj]), Ks,
                   acc);
#pragma unroll
      for (int i = 0; i < 3; ++i) sg[u][i] = group8_sum(acc[i]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = (gi + u * kWaves) * 8 + g8;
      const bool valid = j < m.nok;
      const double s0 = sg[u][0], s1 = sg[u][1], s2 = sg[u][2];
      if (h == 0 && valid) {
        const double d1 = m.d1[j], d2 = m.d2[j];
        double* dst = acc_slot + (size_t)j * NACC;
        dst[0] = s0;
        dst[1] = s1;
        dst[2] = s2;
        const double iw2 = m.iw2[j];
        const double C = s0 * iw2, C1 = -kTwoPi * s1 * iw2, C2 = -kFourPi2 * s2 * iw2;
        const double iS = 1.0 / (m.pn[j] * iw2);
        const double gc = -2.0 * C * C1 * iS;
        const double hc = -2.0 * (C * C2 + C1 * C1) * iS;
        t[0] -= C * C * iS;
        t[1] += gc;
        t[2] = fma(gc, d1, t[2]);
        t[3] = fma(gc, d2, t[3]);
        t[4] += hc;
        t[5] = fma(hc, d1, t[5]);
        t[6] = fma(hc, d2, t[6]);
        t[7] = fma(hc * d1, d1, t[7]);
        t[8] = fma(hc * d1, d2, t[8]);
        t[9] = fma(hc * d2, d2, t[9]);
      }
    }
  }
  // only the channel lanes (h == 0) hold terms
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const double v = chan8_sum(t[i]);
    if (lane == 8) red[w][i] = v;
  }
  __syncthreads();
  if (tid < 21) {
    // out[0] f, out[1..5] g, out[6 + p] H pair p: (0,0) 0, (0,1) 1, (0,2) 2,
    // (1,1) 5, (1,2) 6, (2,2) 9; tau/alpha entries are 0
    // fit flags as a bit mask read with constant indices (scalar loads): a
    // lane-indexed a.flags[] would be a vector load from kernarg memory
    const int fm = flag_mask(a);
    int src = -1;
    bool on = true;
    if (tid == 0) src = 0;
    else if (tid < 4) { src = tid; on = (fm >> (tid - 1)) & 1; }
    else if (tid >= 6) {
      const int p = tid - 6, pi = pair_i(p), pj = pair_j(p);
      if (pj < 3) { src = 4 + (pi == 0 ? pj : 1 + pi + pj); on = (fm >> pi) & (fm >> pj) & 1; }
    }
    double v = 0.0;
    if (src >= 0 && on)
      for (int q = 0; q < kWaves; ++q) v += red[q][src];
    out[tid] = v;
  }
  __syncthreads();
}

// One sweep over all fitted channels at (prm, refs).  MODE 0: f, g, H for
// the solver (out[0..20]) and raw accumulators into acc_slot; MODE 1: the
// with-scales Hessian pieces (out[0..29]) and per-channel wsc rows.  SCAT
// compiles the scattering cell loop in; without it tau must be 0 (host-side
// dispatch guarantees it), which keeps the phase-only kernels lean.
// Each 8-channel group's contributions are reduced across the wave at once
// and added into the wave's own LDS row, so nothing is carried through the
// cell loop in registers.
// lrow (optional, kWaves * 8 rows of LDS): each channel lane (h == 0) adds its
// terms into its own row across groups and the block sums the rows once at
// the end, instead of NP wave reductions per channel group.
// [j0, j1) (multiples of 8 but the end): the fitted channels this block sums.
template <int MODE, bool SCAT>
__device__ __forceinline__ void sweep(const FitArgs& a, const Meta& m, int c, int s, const double* prm,
                      const double* refs, double P, double* acc_slot, double* out,
                      double (*red)[48], const TaylorSrc& ts, double (*lrow)[48] = nullptr,
                      int j0 = 0, int j1 = 1 << 30, double* gpart = nullptr) {
  if constexpr (MODE == 0 && !SCAT) {
    if (ts.T && ts.same) {
      sweep_taylor0(a, m, prm, acc_slot, out, red, ts);
      return;
    }
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g8 = lane >> 3, h = lane & 7;
  const int J = a.NHP >> 3;
  const bool log10_tau = a.log10_tau != 0;
  const double tau_lin = SCAT ? (log10_tau ? pow(10.0, prm[3]) : prm[3]) : 0.0;
  const bool scat = SCAT && tau_lin != 0.0;
  const int midx = a.model_idx ? a.model_idx[s] : 0;
  const int fm = flag_mask(a);
  constexpr int NP = MODE == 0 ? 21 : 45;
  if (lane < NP) red[w][lane] = 0.0;
  double* myrow = lrow ? lrow[w * 8 + g8] : nullptr;
  if (lrow && h == 0)
    for (int i = 0; i < NP; ++i) myrow[i] = 0.0;
  __syncthreads();
  const int jend = min(m.nok, j1);
  const int ngroups = (jend + 7) >> 3;
  for (int gi = (j0 >> 3) + w; gi < ngroups; gi += kWaves) {
    const int j = gi * 8 + g8;
    const bool valid = j < jend;
    const int jj = valid ? j : jend - 1;
    const int n = m.chan[jj];
    const double fr = m.fr[jj];
    double acc[NACC];
    if (!SCAT && ts.T) {
      const double dl = ts.same ? taylor_delta_lin(prm, ts.xc, m.d1[jj], m.d2[jj])
                                : taylor_delta(prm, refs, ts, fr, P);
      taylor_cells(ts, n, h, dl, 0.5 * (double)a.nbin, acc);
    } else if (!scat) {
      const double phif = phase_frac(prm, fr, refs, P);
      const double2* Xr = a.X + ((size_t)c * a.nchan + n) * a.NHP;
      cells_phase(Xr, J, h, phif, acc);
    } else {
      const double phif = phase_frac(prm, fr, refs, P);
      const double2* Xr = a.X + ((size_t)c * a.nchan + n) * a.NHP;
      const double* M2r = a.M2 + ((size_t)midx * a.nchan + n) * a.NHP;
      const double taun = tau_lin * pow(fr / refs[2], prm[4]);
      cells_scat<PPF_SCAT_U>(Xr, M2r, J, h, phif, taun, acc);
    }
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = group8_sum(acc[i]);
    if constexpr (MODE == 0) {
      if (!lrow) {
        // f, g and H terms spread over each channel's 8 lanes: lane h forms
        // out-slots h, h + 8, h + 16 (the channel's sums are on all 8 after
        // group8_sum), then one chan8_sum per slot row sums the group's 8
        // channels -- the additions wave_sum made on one lane's 21 terms, on
        // the same operands, so every slot is bitwise as before
        const double dpre[2] = {m.d1[jj], m.d2[jj]};
        const ChanDeriv d = derive<SCAT>(acc, scat, m.pn[jj], m.iw2[jj], fr, prm, tau_lin, refs,
                                         P, log10_tau, dpre);
        const double q = d.C * d.C / d.S;
        const LanePick L{d.dph[0], d.dph[1], d.dph[2], d.dts[0],
                         d.dts[1], d.d2ts[0], d.d2ts[1], d.d2ts[2]};
        if (h == 0 && valid) {
          double* dst = acc_slot + (size_t)j * NACC;
          for (int i = 0; i < NACC; ++i) dst[i] = acc[i];
        }
        const bool on = valid;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const double v = chan8_sum(on ? mode0_term(d, L, q, h + 8 * r, fm) : 0.0);
          const int t = (lane & 7) + 8 * r;
          if (lane >= 8 && lane < 16 && t < NP) {
            if (gpart) gpart[(size_t)gi * kScatPart + t] = v;  // summed by the caller
            else red[w][t] += v;
          }
        }
        continue;
      }
    }
    double ct[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) ct[i] = 0.0;
    if (h == 0 && valid) {
      const double dpre[2] = {m.d1[j], m.d2[j]};
      const ChanDeriv d = derive<SCAT>(acc, scat, m.pn[j], m.iw2[j], fr, prm, tau_lin, refs, P,
                                       log10_tau, MODE == 0 ? dpre : nullptr);
      const double q = d.C * d.C / d.S;
      if (MODE == 0) {
        double* dst = acc_slot + (size_t)j * NACC;
        for (int i = 0; i < NACC; ++i) dst[i] = acc[i];
        ct[0] = -q;
#pragma unroll
        for (int i = 0; i < 5; ++i)
          if (a.flags[i]) ct[1 + i] = -q * (2.0 * dC_(d, i) / d.C - dS_(d, i) / d.S);
#pragma unroll
                for (int p = 0; p < 15; ++p) {
          const int pi = pair_i(p), pj = pair_j(p);
          if (a.flags[pi] && a.flags[pj]) ct[6 + p] = Hn_(d, pi, pj);
        }
      } else {
        const double sc = d.C / d.S;
        double cross[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) cross[i] = -2.0 * (dC_(d, i) - sc * dS_(d, i));
        double* dst = a.wsc + ((size_t)c * a.nchan + j) * 8;
        dst[0] = sc;
        dst[1] = d.S;
#pragma unroll
        for (int i = 0; i < 5; ++i) dst[2 + i] = cross[i];
        const double ic = 1.0 / (2.0 * d.S);
#pragma unroll
                for (int p = 0; p < 15; ++p) {
          const int pi = pair_i(p), pj = pair_j(p);
          if (a.flags[pi] && a.flags[pj]) {
            ct[p] = -2.0 * q * ((d2C_(d, pi, pj) / d.C) - (0.5 * d2S_(d, pi, pj) / d.S));
            ct[15 + p] = cross[pi] * cross[pj] * ic;
            ct[30 + p] = Hn_(d, pi, pj);  // curvature without amplitude terms
          }
        }
      }
    }
    if (lrow) {
      if (h == 0 && valid)
#pragma unroll
        for (int i = 0; i < NP; ++i) myrow[i] += ct[i];
    } else {
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const double v = wave_sum(ct[i]);  // only h == 0 lanes hold terms
        if (lane == 0) {
          if (gpart) gpart[(size_t)gi * kScatPart + i] = v;  // summed by the caller
          else red[w][i] += v;
        }
      }
    }
  }
  __syncthreads();
  if (tid < NP) {
    double t = 0.0;
    if (lrow)
      for (int r = 0; r < kWaves * 8; ++r) t += lrow[r][tid];
    else
      for (int q = 0; q < kWaves; ++q) t += red[q][tid];
    out[tid] = t;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// k_guess
// ---------------------------------------------------------------------------
// Subints whose fit runs in k_fit_taylor (ppfit_taylor.hip): phase family
// (tau = 0 at the start and not fitted) when the Taylor path is on.
__device__ __forceinline__ bool fused_taylor(const FitArgs& a, int s) {
  if (!a.T) return false;
  const double t3 = a.init[(size_t)s * 5 + 3];
  const double tl = a.log10_tau ? pow(10.0, t3) : t3;
  return !((tl != 0.0) || a.flags[3]);
}

// Solver-state set-up and the get_TOAs initial phase of one subint (all
// threads of the block).  dyn: >= NHP double2 of LDS for the guess spectrum.
__device__ void guess_subint(const FitArgs& a, int c, int s, unsigned char* dyn, GuessShared& gs) {
  const int tid = threadIdx.x;
  const int nchan = a.nchan;
  const uint8_t* mask = a.mask ? a.mask + (size_t)s * nchan : nullptr;
  double fsum = 0.0, cnt = 0.0;
  for (int n = tid; n < nchan; n += kBlock)
    if (!mask || mask[n]) { fsum += a.freqs[(size_t)s * nchan + n]; cnt += 1.0; }
  fsum = block_sum(fsum, gs.red);
  cnt = block_sum(cnt, gs.red);
  const double fmean = fsum / cnt;
  SolveState& st = a.st[c];
  if (tid == 0) {
    for (int i = 0; i < 5; ++i) st.x[i] = a.init[(size_t)s * 5 + i];
    for (int i = 0; i < 3; ++i) {
      const double v = a.nu_fit[(size_t)s * 3 + i];
      st.refs[i] = isnan(v) ? fmean : v;
    }
    st.nfev = 0;
    st.status = -1;
    st.slot = 0;
    st.fun = NAN;
    const double tl = a.log10_tau ? pow(10.0, st.x[3]) : st.x[3];
    st.scat = (tl != 0.0) || a.flags[3];
    st.scat_post = st.scat;
    st.taylor = !st.scat && a.T != nullptr;
    st.kit = 0;
    st.sdone = 0;
    st.phase = 0;
    st.fin = 0;
    st.mvalid = 0;
    st.xslot = 0;
    st.wslot = 0;
    st.tr = 1.0;
  }
  if (!a.guess) {
    __syncthreads();
    if (tid == 0)
      for (int i = 0; i < 5; ++i) { st.init[i] = st.x[i]; st.xc[0][i] = st.x[i]; }
    return;
  }
  // rm_k = R_k conj(Mm_k B_k(tau_g)): the guess template is irfft(B rfft(mean
  // model)) when a scattering guess is given (pptoas.py:441-446).
  double2* rm = reinterpret_cast<double2*>(dyn);
  const double2* Rr = a.R + (size_t)c * a.NHP;
  const double tg = a.guess_tau ? a.guess_tau[s] : 0.0;
  const int N = a.NH - 1;
  const int midx = a.model_idx ? a.model_idx[s] : 0;
  const double2* Mb = a.M + (size_t)midx * nchan * a.NHP;
  const double inv_cnt = 1.0 / cnt;
  double pno = 0.0;
  for (int k = tid; k < a.NH; k += kBlock) {
    const double2 r = Rr[k];
    // modelx.mean(axis=0) over the fitted channels (pptoas.py:454); its
    // spectrum is the mean of the DC-zeroed channel spectra.
    double2 mm = cmk(0.0, 0.0);
    // every channel fitted: the mean template spectrum of k_model_mean (the
    // same sum in the same order, scaled by 1 / nchan as 1 / cnt)
    if ((!mask || cnt == (double)nchan) && a.Mmean) {
      mm = a.Mmean[(size_t)midx * a.NHP + k];
    } else {
      for (int n = 0; n < nchan; ++n)
        if (!mask || mask[n]) mm = cadd(mm, Mb[(size_t)n * a.NHP + k]);
      mm = cscale(mm, inv_cnt);
    }
    if (k == N) mm.y = 0.0;
    if (tg != 0.0) {
      const double aa = kTwoPi * (double)k * tg;
      const double id = 1.0 / fma(aa, aa, 1.0);
      mm = cmul(mm, cmk(id, -aa * id));
      if (k == N) mm.y = 0.0;
    }
    rm[k] = cmulc(r, mm);
    if (k >= a.kc) pno += cabs2(r);
  }
  pno = block_sum(pno, gs.red);  // includes the barrier that publishes rm
  // err = get_noise(rot_prof) * sqrt(nbin/2), pplib.py:2076-2080
  const double noise = sqrt(pno / (double)a.nbin / (double)(a.NH - a.kc));
  const double err2 = noise * noise * (0.5 * (double)a.nbin);
  // the prime-factor grid's scratch follows rm in the dynamic LDS
  // (ppf_fit_portrait_batch sizes it with pfa_scratch_slots)
  guess_search(rm, a.NH, 1.0 / err2, a.Ns, -0.5, 0.5, gs, !(a.solver_flags & PPF_GUESS_DIRECT),
               a.ptime ? a.ptime + 10 : nullptr,
               pfa_scratch_slots(a.Ns, a.NH) ? rm + a.NHP : nullptr);
  if (tid == 0) {
    double nug = a.guess_nu ? a.guess_nu[s] : NAN;
    if (isnan(nug)) nug = fmean;
    const double P = a.P[s];
    const double DM = st.x[1];
    double phi = gs.x;
    // phase_transform(phi, DM_guess, nu_g, nu_fit_DM, P, mod), pplib.py:2609
    phi = phi + (kDconst * DM * (1.0 / P) *
                 (pow(st.refs[0], -2.0) - pow(nug, -2.0)));
    if (a.guess_wrap) phi = wrap_half(phi);
    st.x[0] = phi;
    for (int i = 0; i < 5; ++i) { st.init[i] = st.x[i]; st.xc[0][i] = st.x[i]; }
  }
}

__device__ bool guess_wave_ok(const FitArgs& a, int s);  // below, with k_guess_w

__global__ __launch_bounds__(kBlock) void k_guess(FitArgs a) {
  extern __shared__ __align__(16) unsigned char dyn[];
  __shared__ GuessShared gs;
  const int c = blockIdx.x, s = a.sub0 + c;
  if (guess_wave_ok(a, s)) return;  // k_guess_w's subint
  guess_subint(a, c, s, dyn, gs);
}

// ---------------------------------------------------------------------------
// k_guess_w: the get_TOAs guess of one subint per wave (64 threads) in the
// common case -- every channel fitted (the guess template is Mmean), the
// folded grid (lo, hi) = (-1/2, 1/2) with 2 <= Ns - 1 <= kBlock / 2 and
// NH > 2 (Ns - 1), NH <= 17 * 64.  Lane l plays k_guess's threads l + 64 q
// (q < 4): rm_k for k = l + 64 m (m < 17) lives in registers; every sum is
// formed with k_guess's operations in its order (per virtual thread, then
// the wave's DPP tree, then the four waves in order), and the grid argmin is
// a total order, so st.x / st.init come out bitwise k_guess's.  k_guess
// skips the subints taken here.  No block barrier, 17 complex registers
// instead of a 16.5 KB LDS spectrum: many more subints in flight per CU.
// ---------------------------------------------------------------------------
constexpr int kGwM = 17;  // rm registers per lane: k = lane + 64 m

__device__ bool guess_wave_ok(const FitArgs& a, int s) {
  if (!a.guess_wave || !a.guess || !a.Mmean || (a.solver_flags & PPF_GUESS_DIRECT)) return false;
  const int L = a.Ns - 1;
  if (!(L >= 2 && L <= kBlock / 2 && a.NH > 2 * L && a.NH <= kGwM * 64)) return false;
  if (a.mask)
    for (int n = 0; n < a.nchan; ++n)
      if (!a.mask[(size_t)s * a.nchan + n]) return false;
  return true;
}

// rm_k = R_k conj(Mm_k B_k(tg)) exactly as guess_subint forms it (unmasked)
__device__ __forceinline__ double2 guess_rm(const FitArgs& a, const double2* Rr,
                                            const double2* Mm, double tg, int k) {
  const int N = a.NH - 1;
  const double2 r = Rr[k];
  double2 mm = Mm[k];
  if (k == N) mm.y = 0.0;
  if (tg != 0.0) {
    const double aa = kTwoPi * (double)k * tg;
    const double id = 1.0 / fma(aa, aa, 1.0);
    mm = cmul(mm, cmk(id, -aa * id));
    if (k == N) mm.y = 0.0;
  }
  return cmulc(r, mm);
}

// The four virtual threads' wave sums of v_q, added in wave order: block_sum
__device__ __forceinline__ double vsum4(const double (&v)[4]) {
  double t = 0.0;
#pragma unroll
  for (int q = 0; q < 4; ++q) t += wave_sum(v[q]);
  return t;
}

// block_eval_phase at phi over the registers (see there for the order)
__device__ __forceinline__ double wave_eval_phase(const double2 (&rm)[kGwM], int NH, double phi,
                                                  int lane) {
  const double2 st = turn_phasor((double)kBlock, phi);
  double acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    double2 e = turn_phasor((double)(lane + 64 * q), phi);
    double v = 0.0;
#pragma unroll
    for (int i = 0; i * 4 + q < kGwM; ++i) {
      const int k = lane + 64 * (q + 4 * i);
      if (k < NH) {
        const double2 r = rm[q + 4 * i];
        v = fma(r.x, e.x, v);
        v = fma(-r.y, e.y, v);
        e = cmul(e, st);
      }
    }
    acc[q] = wave_sum(v);
  }
  return ((acc[0] + acc[1]) + acc[2]) + acc[3];
}

// row_eval_phase over rm recomputed from R and Mm (the direct-sum recheck)
__device__ double row_eval_phase_g(const FitArgs& a, const double2* Rr, const double2* Mm,
                                   double tg, int k0, int k1, double phi) {
  const double2 z = turn_phasor(1.0, phi);
  double acc = 0.0;
  for (int kb = k0; kb < k1; kb += 64) {
    double2 e = turn_phasor((double)kb, phi);
    const int ke = min(kb + 64, k1);
    for (int k = kb; k < ke; ++k) {
      const double2 r = guess_rm(a, Rr, Mm, tg, k);
      acc = fma(r.x, e.x, acc);
      acc = fma(-r.y, e.y, acc);
      e = cmul(e, z);
    }
  }
  return acc;
}

__global__ __launch_bounds__(64) void k_guess_w(FitArgs a) {
  __shared__ double2 fb[kBlock / 2], fw[kBlock / 2];
  const int c = blockIdx.x, s = a.sub0 + c, lane = threadIdx.x;
  if (!guess_wave_ok(a, s)) return;
  const int nchan = a.nchan;
  // fmean over the (all fitted) channels: block_sum of the threads' sums
  double fv[4], cv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    fv[q] = 0.0;
    cv[q] = 0.0;
    for (int n = lane + 64 * q; n < nchan; n += kBlock) {
      fv[q] += a.freqs[(size_t)s * nchan + n];
      cv[q] += 1.0;
    }
  }
  const double fsum = vsum4(fv), cnt = vsum4(cv);
  const double fmean = fsum / cnt;
  SolveState& st = a.st[c];
  if (lane == 0) {
    for (int i = 0; i < 5; ++i) st.x[i] = a.init[(size_t)s * 5 + i];
    for (int i = 0; i < 3; ++i) {
      const double v = a.nu_fit[(size_t)s * 3 + i];
      st.refs[i] = isnan(v) ? fmean : v;
    }
    st.nfev = 0;
    st.status = -1;
    st.slot = 0;
    st.fun = NAN;
    const double tl = a.log10_tau ? pow(10.0, st.x[3]) : st.x[3];
    st.scat = (tl != 0.0) || a.flags[3];
    st.scat_post = st.scat;
    st.taylor = !st.scat && a.T != nullptr;
    st.kit = 0;
    st.sdone = 0;
    st.phase = 0;
    st.fin = 0;
    st.mvalid = 0;
    st.xslot = 0;
    st.wslot = 0;
    st.tr = 1.0;
  }
  const double2* Rr = a.R + (size_t)c * a.NHP;
  const double tg = a.guess_tau ? a.guess_tau[s] : 0.0;
  const int NH = a.NH;
  const int midx = a.model_idx ? a.model_idx[s] : 0;
  const double2* Mm = a.Mmean + (size_t)midx * a.NHP;
  // diagnostic clocks (ppf_phase_profile, lane 0): [10] set-up + brute
  // force, [11] Nelder-Mead, [12] NM calls, [26] up to the fold sums, [27] up to rm
  unsigned long long* clk = a.ptime ? a.ptime + 10 : nullptr;
  const unsigned long long c0 = clk ? wall_clock64() : 0ull;
  double2 rm[kGwM];
  double pv[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int m = 0; m < kGwM; ++m) {
    const int k = lane + 64 * m;
    rm[m] = cmk(0.0, 0.0);
    if (k < NH) {
      rm[m] = guess_rm(a, Rr, Mm, tg, k);
      if (k >= a.kc) pv[m & 3] += cabs2(Rr[k]);
    }
  }
  const double pno = vsum4(pv);
  if (clk && lane == 0) atomicAdd(&clk[17], wall_clock64() - c0);  // [27] set-up + rm
  const double noise = sqrt(pno / (double)a.nbin / (double)(NH - a.kc));
  const double err2 = noise * noise * (0.5 * (double)a.nbin);
  const double ie2 = 1.0 / err2;
  // ---- folded brute force (guess_search, FOLD) ----
  const int Ns = a.Ns, L = Ns - 1;
  const double lo = -0.5, hi = 0.5;
  const double step = (hi - lo) / (double)(Ns - 1);
  for (int t = lane; t < L; t += 64) {
    double2 b = cmk(0.0, 0.0);
    for (int k = t; k < NH; k += L) {
      const double2 r = guess_rm(a, Rr, Mm, tg, k);
      b = (k & 1) ? csub(b, r) : cadd(b, r);
    }
    fb[t] = b;
    double sn, cs;
    sincospi(2.0 * (double)t / (double)L, &sn, &cs);
    fw[t] = cmk(cs, sn);
  }
  __syncthreads();  // one wave: orders the LDS writes before the reads
  if (clk && lane == 0) atomicAdd(&clk[16], wall_clock64() - c0);
  const int jm = (L + 1) / 2;
  double myf[2] = {NAN, NAN};
  double bv = NAN;
  int bi = 0x7fffffff;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int g = lane + 64 * u;
    if (g < Ns) {
      double part[2];
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int j0 = half ? jm : 0, j1 = half ? L : jm;
        double pt = 0.0;
        int mi = (j0 * g) % L;
        for (int j = j0; j < j1; ++j) {
          const double2 b = fb[j], wv = fw[mi];
          pt = fma(b.x, wv.x, pt);
          pt = fma(-b.y, wv.y, pt);
          mi += g;
          if (mi >= L) mi -= L;
        }
        part[half] = pt;
      }
      const double f = -(part[0] + part[1]) * ie2;
      myf[u] = f;
      if (argmin_better(f, g, bv, bi)) { bv = f; bi = g; }
    }
  }
  auto wave_argmin = [&](double& v, int& i) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double ov = __shfl_xor(v, o);
      const int oi = __shfl_xor(i, o);
      if (argmin_better(ov, oi, v, i)) { v = ov; i = oi; }
    }
  };
  wave_argmin(bv, bi);
  // near tie on the folded grid: retake the grid by direct sums
  bool near = false;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int g = lane + 64 * u;
    const bool endpair = (bi == 0 && g == Ns - 1) || (bi == Ns - 1 && g == 0);
    if (g < Ns && g != bi && !endpair && !(fabs(myf[u] - bv) > 1e-12 * fabs(bv))) near = true;
  }
  if (__any(near)) {
    const int kmid = (NH + 1) / 2;
    bv = NAN;
    bi = 0x7fffffff;
    for (int u = 0; u < 2; ++u) {
      const int g = lane + 64 * u;
      if (g < Ns) {
        const double ph = (g == Ns - 1) ? hi : __dadd_rn(__dmul_rn((double)g, step), lo);
        const double p0 = row_eval_phase_g(a, Rr, Mm, tg, 0, kmid, ph);
        const double p1 = row_eval_phase_g(a, Rr, Mm, tg, kmid, NH, ph);
        const double f = -(p0 + p1) * ie2;
        if (argmin_better(f, g, bv, bi)) { bv = f; bi = g; }
      }
    }
    wave_argmin(bv, bi);
  }
  const double x0 = (bi == Ns - 1) ? hi : __dadd_rn(__dmul_rn((double)bi, step), lo);
  const unsigned long long c1 = clk ? wall_clock64() : 0ull;
  // ---- Nelder-Mead polish (guess_search) ----
  const int maxfun = 200;
  int fcalls = 0;
  bool stop = false;
  auto F = [&](double xv) -> double {
    if (fcalls >= maxfun) { stop = true; return 0.0; }
    ++fcalls;
    return -wave_eval_phase(rm, NH, xv, lane) * ie2;
  };
  double s0, f0, s1, f1;
  nm_polish(F, stop, fcalls, maxfun, x0, s0, f0, s1, f1);
  if (clk && lane == 0) {
    atomicAdd(&clk[0], c1 - c0);
    atomicAdd(&clk[1], wall_clock64() - c1);
    atomicAdd(&clk[2], (unsigned long long)fcalls);
  }
  if (lane == 0) {
    double nug = a.guess_nu ? a.guess_nu[s] : NAN;
    if (isnan(nug)) nug = fmean;
    const double P = a.P[s];
    const double DM = st.x[1];
    double phi = s0;
    // phase_transform(phi, DM_guess, nu_g, nu_fit_DM, P, mod), pplib.py:2609
    phi = phi + (kDconst * DM * (1.0 / P) * (pow(st.refs[0], -2.0) - pow(nug, -2.0)));
    if (a.guess_wrap) phi = wrap_half(phi);
    st.x[0] = phi;
    for (int i = 0; i < 5; ++i) { st.init[i] = st.x[i]; st.xc[0][i] = st.x[i]; }
  }
}

// Mean of the DC-zeroed channel spectra of each template (unmasked guess
// template, pptoas.py:454): Mmean[t][k] = sum_n M[t][n][k] / nchan.
__global__ void k_model_mean(const double2* __restrict__ M, double2* __restrict__ Mmean, int nchan,
                             int NHP) {
  const int t = blockIdx.y;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= NHP) return;
  const double2* Mt = M + (size_t)t * nchan * NHP;
  double2 mm = cmk(0.0, 0.0);
  for (int n = 0; n < nchan; ++n) mm = cadd(mm, Mt[(size_t)n * NHP + k]);
  Mmean[(size_t)t * NHP + k] = cscale(mm, 1.0 / (double)nchan);
}

// ---------------------------------------------------------------------------
// k_solve: scipy.optimize._trustregion._minimize_trust_region with the
// CGSteihaugSubproblem (scipy 1.15, _trustregion.py / _trustregion_ncg.py):
// initial radius 1, max 1000, eta 0.15, gtol -1, maxiter 200 * 5.
// ---------------------------------------------------------------------------
// The 5-parameter trust-region step runs on wave 0 with lane i < 5 holding
// component i of every vector (lanes >= 5 hold zeros): dot products are an
// 8-lane shuffle sum broadcast from lane 0, H.v gathers v by lane shuffles.
// Every lane then runs the same scalar control flow, so the step needs a few
// registers per lane instead of dozens of 5-vectors on one thread.
__device__ __forceinline__ double dot8(double a, double b) {
  return lane0(group8_sum(a * b));
}
// scipy's ScalarFunction memoises the last point it evaluated
// (_differentiable_functions.py: fun(x) re-evaluates only when x differs,
// np.array_equal): a trust-ncg proposal bitwise equal to the last evaluated
// point -- after a rejection the interior Steihaug step is often the same
// step again -- reuses its f (and g, H) and does not count in nfev.  Lane
// i < 5 holds component i of both points; wave-uniform result.
__device__ __forceinline__ bool same_point8(int lane, double p, double e) {
  return lane0(group8_sum((lane < 5 && !(p == e)) ? 1.0 : 0.0)) == 0.0;
}
__device__ __forceinline__ double hvec(const double (&Hrow)[5], double v) {
  double s = 0.0;
  s += Hrow[0] * lane_at<0>(v);
  s += Hrow[1] * lane_at<1>(v);
  s += Hrow[2] * lane_at<2>(v);
  s += Hrow[3] * lane_at<3>(v);
  s += Hrow[4] * lane_at<4>(v);
  return s;
}
// m(p) = f + g.p + 0.5 p.(H p)   (BaseQuadraticSubproblem.__call__)
__device__ __forceinline__ double model_val(double f, double g, const double (&Hrow)[5], double p) {
  return f + dot8(g, p) + 0.5 * dot8(p, hvec(Hrow, p));
}
// get_boundaries_intersections: ||z + t d|| = tr, sorted roots
__device__ __forceinline__ void boundary_t(double z, double d, double tr, double& ta, double& tb) {
  const double a = dot8(d, d), b = 2.0 * dot8(z, d), c = dot8(z, z) - tr * tr;
  const double sq = sqrt(b * b - 4.0 * a * c);
  const double aux = b + copysign(sq, b);
  double t1 = -aux / (2.0 * a), t2 = -2.0 * c / aux;
  if (t1 > t2) { const double t = t1; t1 = t2; t2 = t; }
  ta = t1;
  tb = t2;
}

// CG-Steihaug, Nocedal & Wright alg. 7.2 as in scipy's CGSteihaugSubproblem.
// Returns this lane's component of the step p.
__device__ __forceinline__ double steihaug(double f, double g, const double (&Hrow)[5], double tr,
                                           int& hits) {
  const double jm = sqrt(dot8(g, g));
  const double tol = fmin(0.5, sqrt(jm)) * jm;
  if (jm < tol) { hits = 0; return 0.0; }
  double z = 0.0, r = g, d = -g;
  for (int it = 0; it < 64; ++it) {
    const double Bd = hvec(Hrow, d);
    const double dBd = dot8(d, Bd);
    if (dBd <= 0.0) {
      double ta, tb;
      boundary_t(z, d, tr, ta, tb);
      const double pa = z + ta * d, pb = z + tb * d;
      hits = 1;
      return model_val(f, g, Hrow, pa) < model_val(f, g, Hrow, pb) ? pa : pb;
    }
    const double r2 = dot8(r, r);
    const double alpha = r2 / dBd;
    const double zn = z + alpha * d;
    if (sqrt(dot8(zn, zn)) >= tr) {
      double ta, tb;
      boundary_t(z, d, tr, ta, tb);
      hits = 1;
      return z + tb * d;
    }
    const double rn = r + alpha * Bd;
    const double rn2 = dot8(rn, rn);
    if (sqrt(rn2) < tol) { hits = 0; return zn; }
    const double beta = rn2 / r2;
    d = -rn + beta * d;
    z = zn;
    r = rn;
  }
  hits = 0;  // a 5-D CG ends well before this
  return z;
}

// scipy's result jac (and the Hessian) at the final point: lane i < 5 of
// wave 0 holds g_i and row i of H
__device__ __forceinline__ void store_grad_hess(const FitArgs& a, int s, int lane, bool ok,
                                                double g, const double (&Hrow)[5]) {
  if (a.o_grad) a.o_grad[(size_t)s * 5 + lane] = ok ? g : NAN;
  if (a.o_hess)
    for (int j = 0; j < 5; ++j) a.o_hess[(size_t)s * 25 + lane * 5 + j] = ok ? Hrow[j] : NAN;
}

struct SolveShared {
  double x[5], xp[5];
  double out[48];
  double red[kWaves][48];
  int done, nok, slot;  // slot: accumulator half holding the accepted point
  int same;             // the proposal repeats the last evaluated point
};

template <bool SCAT, bool WIDE>
__global__ __launch_bounds__(kBlock) void k_solve(FitArgs a) {
  extern __shared__ __align__(16) unsigned char dyn[];
  __shared__ SolveShared sh;
  __shared__ double refs[3];
  const int c = blockIdx.x, s = a.sub0 + c, tid = threadIdx.x;
  const int lane = tid & 63;
  if (a.method != PPF_METHOD_TRUST_NCG) return;  // k_tnc owns TNC fits
  if ((a.st[c].scat != 0) != SCAT) return;  // the other variant owns this subint
  const Meta m = load_meta(a, c, s, chan_tables<WIDE>(a, dyn), &sh.nok);
  SolveState& st = a.st[c];
  const double P = a.P[s];
  if (tid < 5) sh.x[tid] = st.x[tid];
  if (tid < 3) refs[tid] = st.refs[tid];
  if (tid == 0) { sh.done = (m.nok == 0); sh.slot = 0; }
  __syncthreads();
  double* acc0 = a.acc + (size_t)c * 2 * a.nchan * NACC;
  // wave-0 solver state (lane i < 5 owns component i; scalars are uniform)
  double f = 0.0, g = 0.0, xl = 0.0, Hrow[5] = {0, 0, 0, 0, 0};
  double tr = 1.0, predv = 0.0, pl = 0.0;
  int hits = 0, k = 0, status = (m.nok == 0) ? -1 : 0, nfev = 0;
  double xe = 0.0;  // lane i < 5: the last evaluated point (same_point8)
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
  if (!sh.done) {
    sweep<0, SCAT>(a, m, c, s, sh.x, refs, P, acc0, sh.out, sh.red, TaylorSrc{});
    if (tid < 64) {
      load_fgh(f, g, Hrow);
      xl = lane < 5 ? sh.x[lane] : 0.0;
      xe = xl;
      nfev = 1;
      if (a.solver_flags & PPF_SOLVE_EVAL) {  // objective at init only
        status = 1;
        if (lane == 0) sh.done = 1;
      }
    }
  }
  __syncthreads();
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
        const bool same = same_point8(lane, xl + pl, xe);
        if (lane == 0) sh.same = same;
      }
    }
    __syncthreads();
    if (sh.done) break;
    // every wave writes the proposal into the half the accepted point is not in
    // (a repeat of the last evaluated point reuses its sweep: sh.out and the
    // accumulators in that half are still its own)
    const bool fresh = !sh.same;
    double* sl = acc0 + (size_t)(sh.slot ^ 1) * a.nchan * NACC;
    if (fresh) sweep<0, SCAT>(a, m, c, s, sh.xp, refs, P, sl, sh.out, sh.red, TaylorSrc{});
    if (tid < 64) {
      double fp, gp, Hp[5] = {0, 0, 0, 0, 0};
      load_fgh(fp, gp, Hp);
      if (fresh) {
        nfev += 1;
        xe = xl + pl;
      }
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
          if (lane == 0) sh.slot ^= 1;
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
  if (tid < 5) store_grad_hess(a, s, lane, m.nok > 0, g, Hrow);
  if (tid == 0) {
    st.fun = m.nok ? f : NAN;
    st.nfev = m.nok ? nfev : 0;
    st.status = status;
    st.slot = sh.slot;
    const double tl = a.log10_tau ? pow(10.0, sh.x[3]) : sh.x[3];
    st.scat_post = SCAT && tl != 0.0;
  }
}

// ---------------------------------------------------------------------------
// Split scattering solve: k_solve<true>'s trust-ncg with every evaluation
// spread over `split` workgroups per subint.  One exact scattering sweep of a
// 512-channel subint is ~4 MB of X; a single workgroup streaming it nfev
// times ran at 0.2 of HBM (r02 config 3).  Per iteration the host launches
//   k_scat_sweep (subint x split blocks): partial f, g, H over a channel
//     range at the subint's point (x at init, else the proposal xp), and the
//     per-channel accumulators into the proposal's slot;
//   k_scat_step (one wave per subint): the per-group terms summed in the
//     order one k_solve block sums them, then k_solve's accept / reject and
//     the next Steihaug proposal, with the solver state kept in SolveState
//     between launches;
// until no subint is left running.  Every sum is formed in k_solve<true>'s
// order, so the trajectory, nfev, status and result are bitwise k_solve's.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool scat_split_owner(const FitArgs& a, const SolveState& st) {
  return a.method == PPF_METHOD_TRUST_NCG && st.scat != 0 && !st.sdone;
}

// The solver step of one subint (one wave, 64 lanes; out: kScatPart doubles
// of LDS): the group partials summed in k_solve's order, then k_solve's
// accept / reject and the next Steihaug proposal, the state in SolveState.
__device__ __forceinline__ void scat_step_wave(const FitArgs& a, const double* part, int init,
                                               int* active, double* out, int c) {
  const int s = a.sub0 + c, lane = threadIdx.x & 63;
  SolveState& st = a.st[c];
  // fitted channels: the mask loads all in flight, then one count
  int cnt = 0;
#pragma unroll 8
  for (int n0 = 0; n0 < a.nchan; n0 += 64) {
    const int n = n0 + lane;
    const bool ok = n < a.nchan && (!a.mask || a.mask[(size_t)s * a.nchan + n]);
    cnt += __popcll(__ballot(ok));
  }
  const int nok = cnt;
  // group terms summed exactly as one k_solve block sums them: wave w's
  // running sum over groups w, w + kWaves, ..., then the waves in order.
  // The terms of kBatch groups are loaded before any is added, so the loads
  // overlap instead of each waiting for the previous add (the additions, and
  // so the sums, are unchanged)
  if (lane < 21) {
    const double* pc = part + (size_t)c * ((a.nchan + 7) >> 3) * kScatPart + lane;
    const int ng = (nok + 7) >> 3;
    constexpr int kBatch = 16;
    double t = 0.0;
    for (int w = 0; w < kWaves; ++w) {
      double r = 0.0;
      for (int g0 = w; g0 < ng; g0 += kWaves * kBatch) {
        double v[kBatch];
#pragma unroll
        for (int b = 0; b < kBatch; ++b) {
          const int gi = min(g0 + kWaves * b, ng - 1);
          v[b] = pc[(size_t)gi * kScatPart];
        }
#pragma unroll
        for (int b = 0; b < kBatch; ++b)
          if (g0 + kWaves * b < ng) r += v[b];
      }
      t += r;
    }
    out[lane] = t;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  auto load_fgh = [&](double& ff, double& gg, double (&HH)[5]) {
    ff = out[0];
    gg = lane < 5 ? out[1 + lane] : 0.0;
#pragma unroll
    for (int p = 0; p < 15; ++p) {
      const double v = out[6 + p];
      if (lane == pair_i(p)) HH[pair_j(p)] = v;
      if (lane == pair_j(p)) HH[pair_i(p)] = v;
    }
  };
  double f, g, xl, Hrow[5] = {0, 0, 0, 0, 0}, tr, predv, pl;
  int hits, k, status, nfev, slot;
  bool done = false;
  // solver trace (ppf_set_trace): the point this sweep evaluated, its f, g, H
  const double xev = lane < 5 ? (init ? st.x[lane] : st.xp[lane]) : 0.0;
  double rho_tr = NAN, pred_tr = NAN;
  // k_solve's post-sweep block for the point xev (whose f, g, H are in out);
  // counted: a fresh sweep (scipy's nfev), else a repeat of the same point
  auto advance = [&](bool counted) {
    double fp, gp, Hp[5] = {0, 0, 0, 0, 0};
    load_fgh(fp, gp, Hp);
    if (counted) nfev += 1;
    const double actual = f - fp;
    const double pred = f - predv;
    pred_tr = pred;
    if (pred <= 0.0) {
      status = 2;
      done = true;
    } else {
      const double rho = actual / pred;
      rho_tr = rho;
      if (rho < 0.25) tr *= 0.25;
      else if (rho > 0.75 && hits) tr = fmin(2.0 * tr, 1000.0);
      if (rho > 0.15) {
        xl = xl + pl;
        f = fp;
        g = gp;
#pragma unroll
        for (int j = 0; j < 5; ++j) Hrow[j] = Hp[j];
        slot ^= 1;
      }
      k += 1;
      if (k >= 1000) { status = 1; done = true; }
    }
  };
  if (init) {
    load_fgh(f, g, Hrow);
    xl = lane < 5 ? st.x[lane] : 0.0;
    tr = 1.0;
    predv = pl = 0.0;
    hits = k = status = 0;
    nfev = 1;
    slot = 0;
    if (nok == 0) { status = -1; nfev = 0; done = true; }
    if (a.solver_flags & PPF_SOLVE_EVAL) { status = 1; done = true; }
  } else {
    f = st.fun;
    g = lane < 5 ? st.g[lane] : 0.0;
    if (lane < 5)
      for (int j = 0; j < 5; ++j) Hrow[j] = st.H[lane * 5 + j];
    xl = lane < 5 ? st.x[lane] : 0.0;
    tr = st.tr;
    predv = st.predv;
    pl = lane < 5 ? st.pl[lane] : 0.0;
    hits = st.hits;
    k = st.kit;
    status = st.status;
    nfev = st.nfev;
    slot = st.slot;
    advance(true);
  }
  if (a.trace && nok) {
    double xv[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) xv[i] = __shfl(xev, i);
    const int isw = nfev - 1;
    if (lane == 0 && isw < a.trace_cap) {
      trace_sweep(a, s, isw, xv, out, 21, true);
      double* r = a.trace + ((size_t)s * a.trace_cap + isw) * kTraceRec;
      r[28] = tr;  // radius after this evaluation's update
      r[29] = pred_tr;
      r[30] = rho_tr;
      r[31] = (double)hits;  // the Steihaug boundary flag of the step that led here
    }
  }
  // k_solve's loop head: NaN gradient, else the next proposal; a proposal
  // that repeats xev (the point just evaluated) is decided on its memoised
  // f, g, H without a sweep and without counting, as scipy's ScalarFunction
  // does, until a new point (for the next sweep) or the end
  while (!done) {
    const double jm = sqrt(dot8(g, g));
    if (!(jm >= -1.0)) {
      status = 0;
      done = true;
      break;
    }
    pl = steihaug(f, g, Hrow, tr, hits);
    predv = model_val(f, g, Hrow, pl);
    if (!same_point8(lane, xl + pl, xev)) break;
    advance(false);
  }
  // state back (lanes < 5 own the vectors; lane 0 the scalars)
  if (lane < 5) {
    st.x[lane] = xl;
    st.g[lane] = g;
    for (int j = 0; j < 5; ++j) st.H[lane * 5 + j] = Hrow[j];
    st.pl[lane] = pl;
    st.xp[lane] = xl + pl;
  }
  if (done && lane < 5) store_grad_hess(a, s, lane, nok > 0, g, Hrow);
  if (lane == 0) {
    st.fun = nok ? f : NAN;
    st.tr = tr;
    st.predv = predv;
    st.hits = hits;
    st.kit = k;
    st.status = status;
    st.nfev = nok ? nfev : 0;
    st.slot = slot;
    if (done) st.sdone = 1;
    else atomicAdd(active, 1);
  }
  if (done) {
    const double x3 = __shfl(xl, 3);
    if (lane == 0) {
      const double tl = a.log10_tau ? pow(10.0, x3) : x3;
      st.scat_post = tl != 0.0;
    }
  }
}

// k_scat_sweep's evaluation: sweep<0, true>'s arithmetic over channels
// [j0, j1) in two phases.  Phase 1 runs every group's cell loop and parks the
// group-summed accumulators in LDS (chA, one row per channel of the block);
// phase 2, after a barrier, forms each channel's f / g / H terms from them.
// The same numbers in the same order as the one-phase loop (the accumulators
// pass through LDS unchanged), but nothing the terms need is live across the
// cell loop: the loop's registers alone set the kernel's, not the loop's
// plus everything derive() holds (223 VGPRs in one phase, two waves per SIMD).
__device__ __forceinline__ void sweep_scat_split(const FitArgs& a, const Meta& m, int c, int s,
                                                 const double* prm, const double* refs, double P,
                                                 double* acc_slot, int j0, int j1, double* gpart,
                                                 double* chA) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g8 = lane >> 3, h = lane & 7;
  const int J = a.NHP >> 3;
  const bool log10_tau = a.log10_tau != 0;
  const int jend = min(m.nok, j1);
  const int ngroups = (jend + 7) >> 3;
  const int gfirst = (j0 >> 3) + w;
  // phase 0: each channel's phase and tau_n (phase_frac, pow: the same calls
  // on the same operands as in the loop, by one thread each) into chP, so
  // the cell-loop phase carries neither
  double2* chP = reinterpret_cast<double2*>(chA + (size_t)(((j1 - j0) + 7) & ~7) * NACC);
  const bool scat = (log10_tau ? pow(10.0, prm[3]) : prm[3]) != 0.0;
  for (int jl = tid; jl < jend - j0; jl += kBlock) {
    const double fr = m.fr[j0 + jl];
    const double tau_lin = log10_tau ? pow(10.0, prm[3]) : prm[3];
    chP[jl] = cmk(phase_frac(prm, fr, refs, P), scat ? tau_lin * pow(fr / refs[2], prm[4]) : 0.0);
  }
  __syncthreads();
  {
    const int midx = a.model_idx ? a.model_idx[s] : 0;
    for (int gi = gfirst; gi < ngroups; gi += kWaves) {
      const int j = gi * 8 + g8;
      const bool valid = j < jend;
      const int jj = valid ? j : jend - 1;
      const int n = m.chan[jj];
      const double2 pt = chP[jj - j0];
      const double2* Xr = a.X + ((size_t)c * a.nchan + n) * a.NHP;
      double acc[NACC];
      if (!scat) {
        cells_phase(Xr, J, h, pt.x, acc);
      } else {
        const double* M2r = a.M2 + ((size_t)midx * a.nchan + n) * a.NHP;
        cells_scat<PPF_SCAT_U>(Xr, M2r, J, h, pt.x, pt.y, acc);
      }
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = group8_sum(acc[i]);
      if (h == 0 && valid) {
        double* row = chA + (size_t)(j - j0) * NACC;
        double* dst = acc_slot + (size_t)j * NACC;
#pragma unroll
        for (int i = 0; i < NACC; ++i) {
          row[i] = acc[i];
          dst[i] = acc[i];
        }
      }
    }
  }
  __syncthreads();  // chA complete (and nothing below is hoisted above the cell loops)
  const double tau_lin = log10_tau ? pow(10.0, prm[3]) : prm[3];
  const int fm = flag_mask(a);
  constexpr int NP = 21;
  for (int gi = gfirst; gi < ngroups; gi += kWaves) {
    const int j = gi * 8 + g8;
    const bool valid = j < jend;
    const int jj = valid ? j : jend - 1;
    const double fr = m.fr[jj];
    double acc[NACC];
    const double* row = chA + (size_t)(jj - j0) * NACC;
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = row[i];
    const double dpre[2] = {m.d1[jj], m.d2[jj]};
    const ChanDeriv d = derive<true>(acc, scat, m.pn[jj], m.iw2[jj], fr, prm, tau_lin, refs, P,
                                     log10_tau, dpre);
    const double q = d.C * d.C / d.S;
    const LanePick L{d.dph[0], d.dph[1], d.dph[2], d.dts[0],
                     d.dts[1], d.d2ts[0], d.d2ts[1], d.d2ts[2]};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const double v = chan8_sum(valid ? mode0_term(d, L, q, h + 8 * r, fm) : 0.0);
      const int t = (lane & 7) + 8 * r;
      if (lane >= 8 && lane < 16 && t < NP) gpart[(size_t)gi * kScatPart + t] = v;
    }
  }
}

__global__ __launch_bounds__(kBlock, PPF_SCAT_WG_PER_CU) void k_scat_sweep(FitArgs a, double* part,
                                                                          int split, int init) {
  extern __shared__ __align__(16) unsigned char dyn[];
  __shared__ SolveShared sh;
  const int c = blockIdx.x, q = blockIdx.y, s = a.sub0 + c, tid = threadIdx.x;
  const SolveState& st = a.st[c];
  if (!scat_split_owner(a, st)) return;
  const Meta m = load_meta(a, c, s, dyn, &sh.nok);
  if (m.nok == 0) return;
  // channel range of this block: whole groups of 8, blocks in order; each
  // group's wave-reduced terms go to part[c][group] (k_scat_step sums them
  // in k_solve's order)
  const int ng = (m.nok + 7) >> 3;
  const int per = (ng + split - 1) / split;
  const int j0 = q * per * 8, j1 = min(m.nok, (q + 1) * per * 8);
  const double* prm = init ? st.x : st.xp;
  const int slot = init ? 0 : (st.slot ^ 1);
  double* acc = a.acc + ((size_t)c * 2 + slot) * a.nchan * NACC;
#if PPF_SCAT_TWO_PHASE
  // the block's channel rows of group sums (dynamic LDS after the Meta arrays)
  double* chA = reinterpret_cast<double*>(dyn + scat_meta_lds(a.nchan));
  if (j0 < j1)
    sweep_scat_split(a, m, c, s, prm, st.refs, a.P[s], acc, j0, j1,
                     part + (size_t)c * ((a.nchan + 7) >> 3) * kScatPart, chA);
#else
  if (j0 < j1)
    sweep<0, true>(a, m, c, s, prm, st.refs, a.P[s], acc, sh.out, sh.red, TaylorSrc{}, nullptr,
                   j0, j1, part + (size_t)c * ((a.nchan + 7) >> 3) * kScatPart);
#endif
  (void)tid;
}

// The solver step of every running subint (one wave each).  ctrs: the
// running counts by iteration parity -- this launch adds to ctrs[par] and
// clears ctrs[par ^ 1] for the next one, so no memset runs between launches.
__global__ __launch_bounds__(64) void k_scat_step(FitArgs a, const double* part, int init,
                                                  int* ctrs, int par) {
  __shared__ double out[kScatPart];
  const int c = blockIdx.x;
  if (c == 0 && threadIdx.x == 0) ctrs[par ^ 1] = 0;
  if (!scat_split_owner(a, a.st[c])) return;
  scat_step_wave(a, part, init, ctrs + par, out, c);
}

// ---------------------------------------------------------------------------
// k_post
// ---------------------------------------------------------------------------
// The post-fit's serial sections (thread 0) index small arrays at run time;
// they live in the block's LDS workspace (PostWs), not in per-lane scratch.
struct PostWs {
  double c[7], pol[7][7], prev[7], pts[9], cur[7], brk[8];  // poly_real_roots
  double bound;
  int kind[8], d, np, npts, deg;
  double co[7], nz[3];                                      // nz_solve
  double M[5][10];                                 // invert_small
  double A[25], Ci[25];                            // with-scales / no-scales blocks
};

// Real roots of sum_i c[i] y^(deg-i) (deg <= 6) in ascending order: the roots
// of the derivative bracket them; each bracket is bisected to convergence.
// All threads of the block call it (uniform deg): thread 0 builds the
// derivative ladder and the brackets of each level, thread q bisects bracket
// q, and thread 0 gathers the level's roots in bracket order -- the same
// arithmetic, per bracket, as a serial sweep, so the roots are bitwise those
// of one.  Returns the root count (block-uniform); roots in w.prev.
__device__ int poly_real_roots(const double* cin, int deg, PostWs& w, int tid) {
  auto& pol = w.pol;
  if (tid == 0) {
    double* c = w.c;
    int off = 0;
    while (off <= deg && cin[off] == 0.0) ++off;  // np.roots strips leading zeros
    int d = deg - off;
    for (int i = 0; i <= d; ++i) c[i] = cin[off + i];
    while (d > 0 && c[d] == 0.0) --d;             // trailing zeros: roots at 0 (not > 0)
    w.d = d;
    if (d > 0) {
      for (int i = 0; i <= d; ++i) pol[d][i] = c[i] / c[0];
      for (int o = d - 1; o >= 1; --o)
        for (int i = 0; i <= o; ++i)
          pol[o][i] = pol[o + 1][i] * (double)(o + 1 - i) / (double)(o + 1);
      double bound = 0.0;
      for (int i = 1; i <= d; ++i) bound = fmax(bound, fabs(pol[d][i]));
      w.bound = 1.0 + bound;
      w.prev[0] = -pol[1][1];  // linear
      w.np = 1;
    } else {
      w.np = 0;
    }
  }
  __syncthreads();
  const int d = w.d;
  for (int o = 2; o <= d; ++o) {
    auto ev = [&](double x) {
      double v = pol[o][0];
      for (int i = 1; i <= o; ++i) v = v * x + pol[o][i];
      return v;
    };
    if (tid == 0) {
      const double bound = w.bound;
      double* pts = w.pts;
      int npts = 0;
      pts[npts++] = -bound;
      for (int i = 0; i < w.np; ++i) pts[npts++] = fmin(fmax(w.prev[i], -bound), bound);
      pts[npts++] = bound;
      w.npts = npts;
    }
    __syncthreads();
    if (tid + 1 < w.npts) {
      double lo = w.pts[tid], hi = w.pts[tid + 1];
      double flo = ev(lo);
      const double fhi = ev(hi);
      int kind = 0;  // 0: no root, 1: root at lo, 2: bisected root
      double r = lo;
      if (flo == 0.0) {
        kind = 1;
      } else if ((flo < 0.0) != (fhi < 0.0)) {
        for (int it = 0; it < 200; ++it) {
          const double mid = 0.5 * (lo + hi);
          if (mid == lo || mid == hi) break;
          const double fm = ev(mid);
          if ((fm < 0.0) == (flo < 0.0)) { lo = mid; flo = fm; } else { hi = mid; }
        }
        kind = 2;
        r = 0.5 * (lo + hi);
      }
      w.kind[tid] = kind;
      w.brk[tid] = r;
    }
    __syncthreads();
    if (tid == 0) {
      double* cur = w.cur;
      int nc = 0;
      for (int q = 0; q + 1 < w.npts; ++q) {
        const int kind = w.kind[q];
        if (kind == 1) {
          if (nc == 0 || cur[nc - 1] != w.brk[q]) cur[nc++] = w.brk[q];
        } else if (kind == 2) {
          cur[nc++] = w.brk[q];
        }
      }
      if (ev(w.bound) == 0.0) cur[nc++] = w.bound;
      w.np = nc;
      for (int i = 0; i < nc; ++i) w.prev[i] = cur[i];
    }
    __syncthreads();
  }
  return w.np;
}

// Gauss-Jordan inverse with partial pivoting (np.linalg.inv), n <= 5.
__device__ bool invert_small(const double* A, int n, double* Ai, PostWs& w) {
  auto& M = w.M;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 2 * n; ++j) M[i][j] = j < n ? A[i * n + j] : (j - n == i ? 1.0 : 0.0);
  for (int col = 0; col < n; ++col) {
    int piv = col;
    for (int r = col + 1; r < n; ++r)
      if (fabs(M[r][col]) > fabs(M[piv][col])) piv = r;
    if (M[piv][col] == 0.0) return false;
    if (piv != col)
      for (int j = 0; j < 2 * n; ++j) { const double t = M[col][j]; M[col][j] = M[piv][j]; M[piv][j] = t; }
    const double iv = 1.0 / M[col][col];
    for (int j = 0; j < 2 * n; ++j) M[col][j] *= iv;
    for (int r = 0; r < n; ++r) {
      if (r == col) continue;
      const double fct = M[r][col];
      if (fct == 0.0) continue;
      for (int j = 0; j < 2 * n; ++j) M[r][j] -= fct * M[col][j];
    }
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) Ai[i * n + j] = M[i][j + n];
  return true;
}

// The fitted block of a 5x5 symmetric matrix, inverted in registers: A is
// padded with the identity on unfitted rows/columns, which Gauss-Jordan with
// partial pivoting leaves untouched (their pivots are 1, their off-diagonal
// entries 0 and never chosen as pivots), so the fitted entries of the result
// are bitwise those of invert_small on the compacted nf x nf block.  Fully
// unrolled: the pivot row swap is a select over the candidate rows.  Returns
// false (singular) like invert_small; Ai gets 0 outside the fitted block.
__device__ __forceinline__ bool invert5_fitted(const double (&A)[5][5], const bool (&fit)[5],
                                               double (&Ai)[5][5]) {
  double M[5][10];
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 10; ++j)
      M[i][j] = j < 5 ? ((fit[i] && fit[j]) ? A[i][j] : (i == j ? 1.0 : 0.0))
                      : (j - 5 == i ? 1.0 : 0.0);
  bool ok = true;
#pragma unroll
  for (int col = 0; col < 5; ++col) {
    int piv = col;
    double best = fabs(M[col][col]);
#pragma unroll
    for (int r = col + 1; r < 5; ++r)
      if (fabs(M[r][col]) > best) { best = fabs(M[r][col]); piv = r; }
    if (best == 0.0) ok = false;
#pragma unroll
    for (int r = col + 1; r < 5; ++r) {
      if (piv == r) {
#pragma unroll
        for (int j = 0; j < 10; ++j) { const double t = M[col][j]; M[col][j] = M[r][j]; M[r][j] = t; }
      }
    }
    const double iv = 1.0 / M[col][col];
#pragma unroll
    for (int j = 0; j < 10; ++j) M[col][j] *= iv;
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      if (r == col) continue;
      const double fct = M[r][col];
      if (fct == 0.0) continue;
#pragma unroll
      for (int j = 0; j < 10; ++j) M[r][j] -= fct * M[col][j];
    }
  }
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) Ai[i][j] = (fit[i] && fit[j]) ? M[i][j + 5] : 0.0;
  return ok;
}

// Per-channel contributions to the zero-covariance sums (pptoaslib.py:746-901).
// Returns the number of sums; the branch id is chosen by the caller.
enum { NZ_NONE = 0, NZ_PD, NZ_PG, NZ_TA, NZ_PDT, NZ_PDG, NZ_PDTA, NZ_PDGT };

__device__ __forceinline__ int nz_branch(const int* ff) {
  const int code = ff[0] * 16 + ff[1] * 8 + ff[2] * 4 + ff[3] * 2 + ff[4];
  switch (code) {
    case 0b11000: return NZ_PD;
    case 0b10100: return NZ_PG;
    case 0b00011: return NZ_TA;
    case 0b11010: return NZ_PDT;
    case 0b11100: return NZ_PDG;
    case 0b11011: return NZ_PDTA;
    case 0b11111: return NZ_PDTA;  // approximated with [1,1,0,1,1] (pptoaslib.py:893-901)
    case 0b11110: return NZ_PDGT;
    default: return NZ_NONE;
  }
}

__device__ __forceinline__ void nz_terms(int br, int option, const ChanDeriv& d, double fr, const double* refs,
                         const int* fl, double* t) {
  const double f2 = 1.0 / (fr * fr), f4 = f2 * f2, lnf = log(fr);
  auto H = [&](int i, int j) { return (fl[i] && fl[j]) ? Hn_(d, i, j) : 0.0; };
  for (int i = 0; i < 22; ++i) t[i] = 0.0;
  switch (br) {
    case NZ_PD: {
      const double h = H(1, 0) / d.dph[1];
      t[0] = f2 * h; t[1] = h;
    } break;
    case NZ_PG: {
      const double h = H(0, 2) / d.dph[2];
      t[0] = f4 * h; t[1] = h;
    } break;
    case NZ_TA: {
      // taus_deriv[1] / taus = ln(fr / nu_tau)
      const double h = H(3, 4) / log(fr / refs[2]);
      t[0] = lnf * h; t[1] = h;
    } break;
    case NZ_PDT: {
      const double h21 = H(1, 0) / d.dph[1], h23 = H(1, 3) / d.dph[1];
      t[0] = f2 * h23; t[1] = f2 * h21; t[2] = h23; t[3] = h21; t[4] = H(3, 0); t[5] = H(3, 3);
    } break;
    case NZ_PDG: {
      if (option == 0) {
        const double h21 = H(1, 0) / d.dph[1], h23 = H(1, 2) / d.dph[1];
        const double h31 = H(2, 0) / d.dph[2], h33 = H(2, 2) / d.dph[2];
        t[0] = h31 * f4; t[1] = h31; t[2] = h23 * f2; t[3] = h23;
        t[4] = h33 * f4; t[5] = h33; t[6] = h21 * f2; t[7] = h21;
      } else if (option == 1) {
        const double h21 = H(1, 0) / d.dph[1], h22 = H(1, 1) / d.dph[1];
        const double h31 = H(2, 0) / d.dph[2], h32 = H(2, 1) / d.dph[2];
        t[0] = h21 * f4; t[1] = h21; t[2] = h32 * f2; t[3] = h32;
        t[4] = h22 * f4; t[5] = h22; t[6] = h31 * f2; t[7] = h31;
      }
    } break;
    case NZ_PDTA: {
      const double lr = log(fr / refs[2]);
      const double h21 = H(1, 0) / d.dph[1], h23 = H(1, 3) / d.dph[1], h24 = H(1, 4) / d.dph[1];
      const double h41 = H(4, 0) / lr, h42 = H(4, 1) / lr, h43 = H(4, 3) / lr;
      t[0] = f2 * h21; t[1] = f2 * h23; t[2] = f2 * h24;
      t[3] = h21; t[4] = h23; t[5] = h24;
      t[6] = lnf * h41; t[7] = lnf * h42; t[8] = lnf * h43;
      t[9] = h41; t[10] = h42; t[11] = h43;
      t[12] = H(0, 0); t[13] = H(1, 1); t[14] = H(3, 3); t[15] = H(4, 4);
      t[16] = H(0, 1); t[17] = H(0, 3); t[18] = H(0, 4); t[19] = H(1, 3); t[20] = H(1, 4);
      t[21] = H(3, 4);
    } break;
    case NZ_PDGT: {
      const double g2 = f2 - 1.0 / (refs[0] * refs[0]);
      const double r1 = 1.0 / (refs[1] * refs[1]);
      const double g4 = f4 - r1 * r1;
      if (option == 0) {
        const double h21 = H(1, 0) / g2, h23 = H(1, 2) / g2, h24 = H(1, 3) / g2;
        const double h31 = H(2, 0) / g4, h33 = H(2, 2) / g4, h34 = H(2, 3) / g4;
        t[0] = f4 * h34; t[1] = h34; t[2] = f2 * h21; t[3] = h21; t[4] = f4 * h31; t[5] = h31;
        t[6] = f2 * h23; t[7] = h23; t[8] = f4 * h33; t[9] = h33; t[10] = f2 * h24; t[11] = h24;
      } else if (option == 1) {
        const double h21 = H(1, 0) / g2, h22 = H(1, 1) / g2, h24 = H(1, 3) / g2;
        const double h31 = H(2, 0) / g4, h32 = H(2, 1) / g4, h34 = H(2, 3) / g4;
        t[0] = f2 * h24; t[1] = h24; t[2] = f4 * h31; t[3] = h31; t[4] = f2 * h21; t[5] = h21;
        t[6] = f4 * h32; t[7] = h32; t[8] = f2 * h22; t[9] = h22; t[10] = f4 * h34; t[11] = h34;
      }
      t[12] = H(3, 0); t[13] = H(3, 3);
    } break;
    default: break;
  }
}

// number of channel sums nz_terms fills for a branch
__device__ __forceinline__ int nz_nsums(int br) {
  switch (br) {
    case NZ_PD: case NZ_PG: case NZ_TA: return 2;
    case NZ_PDT: return 6;
    case NZ_PDG: return 8;
    case NZ_PDGT: return 14;
    case NZ_PDTA: return 22;
    default: return 0;
  }
}

// block_sum_vec over the first N of 22 sums
template <int N>
__device__ __forceinline__ void block_sum_first(double (&v)[22], double (*red)[48]) {
  double u[N];
#pragma unroll
  for (int i = 0; i < N; ++i) u[i] = v[i];
  block_sum_vec(u, red);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = u[i];
}

// the positive root (sqrt of it when sq) closest to fmean
__device__ double closest_positive(const double* r, int nr, bool sq, double fmean) {
  double best = NAN, bd = INFINITY;
  for (int i = 0; i < nr; ++i) {
    if (!(r[i] > 0.0)) continue;
    const double x = sq ? sqrt(r[i]) : r[i];
    const double dd = fabs(fmean - x);
    if (dd < bd) { bd = dd; best = x; }
  }
  return best;
}

// Solve the branch from the channel sums t[22]; writes nz[3] (refs preset).
// The GM branches leave a polynomial in y = nu^2 in w.co and return its
// degree: the block's root finder and closest_positive finish them.
__device__ int nz_solve(int br, int option, const double* t, double* nz, PostWs& w) {
  switch (br) {
    case NZ_PD: nz[0] = pow(t[0] / t[1], -0.5); break;
    case NZ_PG: nz[1] = pow(t[0] / t[1], -0.25); break;
    case NZ_TA: nz[2] = exp(t[0] / t[1]); break;
    case NZ_PDT: {
      const double num = t[4] * t[0] - t[5] * t[1];
      const double den = t[4] * t[2] - t[5] * t[3];
      nz[0] = pow(num / den, -0.5);
    } break;
    case NZ_PDG: {
      if (option == 0 || option == 1) {
        const double A = t[0], B = t[1], C = t[2], D = t[3], E = t[4], F = t[5], G = t[6],
                     Hh = t[7];
        // coeffs [A C - E G, 0, E H - A D, 0, F G - B C, 0, B D - F H] in nu:
        // a cubic in y = nu^2 (pptoaslib.py:789-794)
        double* cy = w.co;
        cy[0] = A * C - E * G;
        cy[1] = E * Hh - A * D;
        cy[2] = F * G - B * C;
        cy[3] = B * D - F * Hh;
        return 3;
      }
    } break;
    case NZ_PDTA: {
      const double H11 = t[12], H22 = t[13], H33 = t[14], H44 = t[15], H12 = t[16], H13 = t[17],
                   H14 = t[18], H23 = t[19], H24 = t[20], H34 = t[21];
      const double a1 = H34 * H34 - H33 * H44, a2 = H13 * H44 - H14 * H34,
                   a3 = H14 * H33 - H13 * H34;
      nz[0] = pow((a1 * t[0] + a2 * t[1] + a3 * t[2]) / (a1 * t[3] + a2 * t[4] + a3 * t[5]), -0.5);
      const double b1 = H13 * H22 - H12 * H23, b2 = H11 * H23 - H12 * H13,
                   b3 = H12 * H12 - H11 * H22;
      nz[2] = exp((b1 * t[6] + b2 * t[7] + b3 * t[8]) / (b1 * t[9] + b2 * t[10] + b3 * t[11]));
    } break;
    case NZ_PDGT: {
      if (option == 0 || option == 1) {
        const double A = t[0], a = t[1], B = t[2], b = t[3], C = t[4], c = t[5], D = t[6],
                     d = t[7], E = t[8], e = t[9], F = t[10], f = t[11], H14 = t[12],
                     H44 = t[13];
        double* co = w.co;
        int deg;
        if (option == 0) {
          co[0] = A * A * B + H44 * C * D + H14 * E * F - H44 * B * E - A * C * F - H14 * A * D;
          co[1] = -A * A * b - H44 * C * d - H14 * E * f + H44 * b * E + A * C * f + H14 * A * d;
          co[2] = -2 * A * a * B - H44 * c * D - H14 * e * F + H44 * B * e + (A * c + a * C) * F +
                  H14 * a * D;
          co[3] = 2 * A * a * b + H44 * c * d + H14 * e * f - H44 * b * e - (A * c + a * C) * f -
                  H14 * a * d;
          co[4] = a * a * B - a * c * F;
          co[5] = -a * a * b + a * c * f;
          deg = 5;
        } else {
          co[0] = A * A * B + H44 * C * D + H14 * E * F - H44 * B * E - A * C * F - H14 * A * D;
          co[1] = -2 * A * a * B - H44 * c * D - H14 * e * F + H44 * B * e + (A * c + a * C) * F +
                  H14 * a * D;
          co[2] = -(A * A * b - a * a * B) - H44 * C * d - H14 * E * f + H44 * b * E +
                  (A * C * f - a * c * F) + H14 * A * d;
          co[3] = 2 * A * a * b + H44 * c * d + H14 * e * f - H44 * b * e - (A * c + a * C) * f -
                  H14 * a * d;
          co[4] = -a * a * b + a * c * f;
          deg = 4;
        }
        return deg;
      }
    } break;
    default: break;
  }
  return 0;
}

struct PostShared {
  PostWs ws;
  double lrow[kWaves * 8][48];  // with-scales sweep: one row per channel lane
  double prm[5], refs[3], nu[3];
  double out[48];
  double red[kWaves][48];
  double Xinv[25];
  double ifact[kMT];  // c_inv_fact for the Taylor sweep
  int ifit[5];
  int nfit, nok, bad;
  double fmean, Sd;
};

// zero-covariance frequencies, outputs at nu_out and the with-scales
// covariance of one subint (all threads of the block)
template <bool SCAT, bool W>  // W: one copy per k_post instantiation (its only caller)
__device__ void post_subint(const FitArgs& a, int c, int s, unsigned char* dyn, PostShared& sh) {
  const int tid = threadIdx.x;
  const int nchan = a.nchan;
  // diagnostic phase clock (ppf_phase_profile): thread 0 adds; the clock is
  // wave-uniform (scalar registers, see k_fit_taylor)
  const bool prof = a.ptime != nullptr;
  unsigned long long t0 = prof ? wall_clock64() : 0ull;
  auto mark = [&](int i) {
    if (prof) {
      const unsigned long long t1 = wall_clock64();
      if (tid == 0) atomicAdd(&a.ptime[i], t1 - t0);
      t0 = t1;
    }
  };
  const Meta m = load_meta(a, c, s, dyn, &sh.nok);
  const SolveState& st = a.st[c];
  const double P = a.P[s];
  const bool log10_tau = a.log10_tau != 0;
  // zero the per-channel outputs of masked channels
  if (a.mask) {
    for (int n = tid; n < nchan; n += kBlock) {
      if (a.mask[(size_t)s * nchan + n]) continue;
      const size_t o = (size_t)s * nchan + n;
      a.o_scales[o] = 0.0;
      a.o_scale_errs[o] = 0.0;
      a.o_channel_snrs[o] = 0.0;
    }
  }
  // Sd (pptoaslib.py:985) and mean frequency of the fitted channels
  {
    double v[2] = {0.0, 0.0};
    for (int j = tid; j < m.nok; j += kBlock) {
      v[0] += a.dsum[(size_t)c * nchan + m.chan[j]] * m.iw2[j];
      v[1] += m.fr[j];
    }
    block_sum_vec(v, sh.red);
    if (tid == 0) { sh.Sd = v[0]; sh.fmean = v[1] / (double)m.nok; }
  }
  if (tid == 0) {
    sh.nfit = 0;
    for (int i = 0; i < 5; ++i) if (a.flags[i]) sh.ifit[sh.nfit++] = i;
    for (int i = 0; i < 3; ++i) sh.refs[i] = st.refs[i];
    sh.bad = (m.nok == 0);
  }
  __syncthreads();
  mark(16);
  if (sh.bad) {
    if (tid == 0) {
      for (int i = 0; i < 5; ++i) {
        a.o_params[(size_t)s * 5 + i] = NAN;
        a.o_param_errs[(size_t)s * 5 + i] = NAN;
      }
      a.o_status[s] = -1;
      a.o_nfev[s] = 0;
    }
    return;
  }
  // ---- nu_out: given values, else zero-covariance frequencies ----
  const double* acc_fin = a.acc + ((size_t)c * 2 + st.slot) * nchan * NACC;
  bool need = false;
  double nuo[3];
  for (int i = 0; i < 3; ++i) {
    nuo[i] = a.nu_out[(size_t)s * 3 + i];
    if (isnan(nuo[i]) || nuo[i] == 0.0) need = true;
  }
  if (need) {
    int fl[5];
    for (int i = 0; i < 5; ++i) fl[i] = a.flags[i] ? 1 : 0;
    const int br = nz_branch(fl);
    if (br == NZ_PDTA) fl[2] = 0;  // [1,1,1,1,1] -> [1,1,0,1,1]
    double t[22];
    double sums[22];
    for (int i = 0; i < 22; ++i) sums[i] = 0.0;
    if (br != NZ_NONE) {
      const double tau_lin = log10_tau ? pow(10.0, st.x[3]) : st.x[3];
      const bool scat = SCAT && tau_lin != 0.0;
      for (int j = tid; j < m.nok; j += kBlock) {
        const ChanDeriv d = derive<SCAT>(acc_fin + (size_t)j * NACC, scat, m.pn[j], m.iw2[j], m.fr[j],
                                   st.x, tau_lin, sh.refs, P, log10_tau);
        nz_terms(br, a.option, d, m.fr[j], sh.refs, fl, t);
        for (int i = 0; i < 22; ++i) sums[i] += t[i];
      }
    }
    switch (nz_nsums(br)) {  // uniform across the block
      case 2: block_sum_first<2>(sums, sh.red); break;
      case 6: block_sum_first<6>(sums, sh.red); break;
      case 8: block_sum_first<8>(sums, sh.red); break;
      case 14: block_sum_first<14>(sums, sh.red); break;
      case 22: block_sum_first<22>(sums, sh.red); break;
      default: break;
    }
    double* nz = sh.ws.nz;  // thread 0's, in LDS: no registers live across the root finder
    if (tid == 0) {
      for (int i = 0; i < 3; ++i) nz[i] = sh.refs[i];
      sh.ws.deg = nz_solve(br, a.option, sums, nz, sh.ws);
    }
    __syncthreads();
    const int pdeg = sh.ws.deg;
    if (pdeg > 0) {
      const int nr = poly_real_roots(sh.ws.co, pdeg, sh.ws, tid);
      if (tid == 0) nz[0] = nz[1] = closest_positive(sh.ws.prev, nr, true, sh.fmean);
    }
    if (tid == 0)
      for (int i = 0; i < 3; ++i) if (isnan(nuo[i])) nuo[i] = nz[i];
  }
  mark(17);
  if (tid == 0) {
    if (a.is_toa) {  // pptoaslib.py:1048-1050
      if (a.flags[1]) nuo[1] = nuo[0];
      else if (a.flags[2]) nuo[0] = nuo[1];
    }
    const double* x = st.x;
    // phi at nu_out (pptoaslib.py:1052-1057)
    const double phi_inf = x[0] + kDconst * x[1] * (0.0 - 1.0 / (sh.refs[0] * sh.refs[0])) / P +
                           kDconst2 * x[2] *
                               (0.0 - 1.0 / (sh.refs[1] * sh.refs[1] * sh.refs[1] * sh.refs[1])) / P;
    double phi_out = phi_inf + ((kDconst / P) * x[1] * pow(nuo[0], -2.0)) +
                     ((kDconst2 / P) * x[2] * pow(nuo[1], -4.0));
    if (fabs(phi_out) >= 0.5) phi_out = pymod1(phi_out);
    if (phi_out >= 0.5) phi_out -= 1.0;
    // tau at nu_out (pptoaslib.py:1059-1065)
    const double tau_fit = log10_tau ? pow(10.0, x[3]) : x[3];
    double tau_out = tau_fit * pow(nuo[2] / sh.refs[2], x[4]);
    if (log10_tau) tau_out = log10(tau_out);
    sh.prm[0] = phi_out;
    sh.prm[1] = x[1];
    sh.prm[2] = x[2];
    sh.prm[3] = tau_out;
    sh.prm[4] = x[4];
    for (int i = 0; i < 3; ++i) sh.nu[i] = nuo[i];
  }
  __syncthreads();
  // ---- with-scales Hessian at the output parameters ----
  // Taylor-path subints: the output params give the same phi_n (mod 1) as the
  // accepted point, so the centre that evaluated it covers them too.
  TaylorSrc ts{};
  if (!SCAT && st.taylor) {
    const double Ks = 0.5 * (double)a.nbin;
    if (tid < kMT) sh.ifact[tid] = c_inv_fact[tid];  // published by taylor_reach's barriers
    int best = st.xslot;
    double by = INFINITY;
    for (int q = 0; q < 2; ++q) {
      if (!(st.mvalid & (1 << q))) continue;
      const TaylorSrc tq{a.T + ((size_t)c * 2 + q) * nchan * kMT, st.xc[q], st.refs};
      const double y = taylor_reach(m, sh.prm, sh.nu, tq, P, Ks, sh.red[0]);
      if (y < by) { by = y; best = q; }
    }
    ts = TaylorSrc{a.T + ((size_t)c * 2 + best) * nchan * kMT, st.xc[best], st.refs, false,
                   sh.ifact};
  }
  mark(18);
  sweep<1, SCAT>(a, m, c, s, sh.prm, sh.nu, P, nullptr, sh.out, sh.red, ts, sh.lrow);
  mark(19);
  if (tid == 0) {
    bool fit[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) fit[i] = a.flags[i] != 0;
    double A[5][5], Ai[5][5];
#pragma unroll
    for (int p = 0; p < 15; ++p) {
      const int pi = pair_i(p), pj = pair_j(p);
      A[pi][pj] = A[pj][pi] = sh.out[p] - sh.out[15 + p];  // A - U C^-1 V
    }
    const bool ok = invert5_fitted(A, fit, Ai);
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = 0; j < 5; ++j)
        sh.Xinv[i * 5 + j] = ok ? Ai[i][j] : ((fit[i] && fit[j]) ? NAN : 0.0);
    if (a.o_cov_nosc) {
#pragma unroll
      for (int p = 0; p < 15; ++p) {
        const int pi = pair_i(p), pj = pair_j(p);
        A[pi][pj] = A[pj][pi] = 0.5 * sh.out[30 + p];
      }
      const bool okc = invert5_fitted(A, fit, Ai);
      double* cn = a.o_cov_nosc + (size_t)s * 25;
      // compacted to the fitted block's leading nf x nf corner (as before)
      int q = 0;
#pragma unroll
      for (int i = 0; i < 25; ++i) cn[i] = 0.0;
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        if (!fit[i]) continue;
        int r = 0;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          if (!fit[j]) continue;
          cn[q * 5 + r] = okc ? Ai[i][j] : NAN;
          ++r;
        }
        ++q;
      }
    }
  }
  __syncthreads();
  mark(20);
  // ---- per-channel amplitude errors and S/N (pptoaslib.py:717-724, 1079-1082) ----
  const int nf = sh.nfit;
  double snr2 = 0.0;
  for (int j = tid; j < m.nok; j += kBlock) {
    const double* w = a.wsc + ((size_t)c * nchan + j) * 8;
    const double sc = w[0], S = w[1];
    const double ic = 1.0 / (2.0 * S);
    // fitted parameters in order; Xinv is 0 outside the fitted block, and
    // adding its zeros leaves the compact sums bitwise unchanged
    double LL[5], U[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) U[q] = a.flags[q] ? w[2 + q] : 0.0;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < 5; ++i)
        if (a.flags[i] && a.flags[q]) t += U[i] * sh.Xinv[i * 5 + q];
      LL[q] = -ic * t;
    }
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < 5; ++q)
      if (a.flags[q]) t += LL[q] * U[q];
    const double LR = -t * ic + ic;
    const double csnr = sc * sqrt(S);
    const int n = m.chan[j];
    const size_t o = (size_t)s * nchan + n;
    a.o_scales[o] = sc;
    a.o_scale_errs[o] = sqrt(2.0 * LR);
    a.o_channel_snrs[o] = csnr;
    snr2 += csnr * csnr;
  }
  snr2 = block_sum(snr2, sh.red[0]);
  if (tid == 0) {
    double* op = a.o_params + (size_t)s * 5;
    double* oe = a.o_param_errs + (size_t)s * 5;
    for (int i = 0; i < 5; ++i) { op[i] = sh.prm[i]; oe[i] = 0.0; }
    double* cv = a.o_cov + (size_t)s * 25;
    for (int i = 0; i < 25; ++i) cv[i] = 0.0;
    int q = 0;
    for (int i = 0; i < 5; ++i) {
      if (!a.flags[i]) continue;
      oe[i] = sqrt(2.0 * sh.Xinv[i * 5 + i]);
      int r = 0;
      for (int j = 0; j < 5; ++j) {
        if (!a.flags[j]) continue;
        cv[q * 5 + r] = 2.0 * sh.Xinv[i * 5 + j];
        ++r;
      }
      ++q;
    }
    for (int i = 0; i < 3; ++i) a.o_nu_out[(size_t)s * 3 + i] = sh.nu[i];
    const double dof = (double)a.nbin * (double)m.nok - (double)(nf + m.nok);
    const double chi2 = sh.Sd + st.fun;
    a.o_chi2[s] = chi2;
    a.o_red_chi2[s] = chi2 / dof;
    a.o_snr[s] = sqrt(snr2);
    a.o_nfev[s] = st.nfev;
    a.o_status[s] = st.status;
    if (a.o_init_used) for (int i = 0; i < 5; ++i) a.o_init_used[(size_t)s * 5 + i] = st.init[i];
    if (a.o_fun) a.o_fun[s] = st.fun;
  }
  mark(21);
  if (prof && tid == 0) atomicAdd(&a.ptime[22], 1ull);
}

// Phase-family post-fit: two workgroups per CU as the launch bound, which
// the compiler meets with 168 VGPRs (three waves per SIMD, no spills).  r04
// A/B at config 2: four per CU (128 VGPRs, 77 spilled) 0.47 -> 0.56 ms (r02's
// code had preferred the cap).  The scattering variant keeps its registers.
template <bool SCAT, bool WIDE>
#ifndef PPF_POST_SCAT_WG_PER_CU
// two workgroups per CU (256 VGPRs, 12 B/lane spilled) instead of one (256 +
// 7 AGPRs): config 3's k_post<true> 1.30 -> 1.09-1.10 ms, bitwise the same
// (a two-phase with-scales sweep, 236 VGPRs unspilled, measured the same
// and moved param_errs by an ulp: not kept)
#define PPF_POST_SCAT_WG_PER_CU 2
#endif
__global__ __launch_bounds__(kBlock, SCAT ? PPF_POST_SCAT_WG_PER_CU : PPF_POST_WG_PER_CU) void k_post(FitArgs a) {
  extern __shared__ __align__(16) unsigned char dyn[];
  __shared__ PostShared sh;
  const int c = blockIdx.x, s = a.sub0 + c;
  if ((a.st[c].scat_post != 0) != SCAT) return;
  post_subint<SCAT, WIDE>(a, c, s, chan_tables<WIDE>(a, dyn), sh);
}

}  // namespace ppf
