// ppfit_kernels.hpp -- kernel argument blocks and the shared FFTFIT search.
#pragma once
#include "ppfit.h"
#include "ppfit_device.hpp"

namespace ppf {

// ---------------------------------------------------------------------------
// Argument blocks (passed by value)
// ---------------------------------------------------------------------------
struct SpecArgs {
  int sub0, nchan, NHP, kc, guess;
  int log10_tau, fit_tau, exact;  // which subints the Taylor path fits (spec_taylor_sub)
  int spec_mode;           // PPF_SPEC_* (ppfit.h)
  const double* data;      // [nsub][nchan][nbin]
  const double2* M;        // [nmodel][nchan][NHP] DC-zeroed template spectra
  const int* model_idx;    // [nsub] or null
  const double* freqs;     // [nsub][nchan]
  const double* errs;      // [nsub][nchan] or null
  const uint8_t* mask;     // [nsub][nchan] or null
  const double* weights;   // [nsub][nchan] or null
  const double* P;         // [nsub]
  const double* init;      // [nsub][5]
  const double* guess_nu;  // [nsub] or null
  double2* X;              // chunk [c][nchan][NHP]
  double2* R;              // chunk [c][NHP]
  double* sig;             // chunk [c][nchan]
  double* dsum;            // chunk [c][nchan]
  const double2* tw;
  double2* D;              // chunk [c][nchan][NHP] data spectra (spec cache) or null
  unsigned char* gdyn;     // WIDE kernels: [block][gdyn_stride] per-channel tables in HBM
  size_t gdyn_stride;
};

// The per-channel tables a workgroup builds (Meta, the data pass's channel
// phases and flags) live in dynamic LDS up to PPF_LDS_NCHAN channels.  The
// WIDE instantiations, taken above that (or under PPF_OPT_HBM_TABLES), keep
// them in the block's slice of an HBM workspace instead: the same values and
// the same arithmetic, so the same fits, at any channel count up to
// PPF_MAX_NCHAN.  Block-local data either way (written, block barrier, read).
template <bool WIDE, class Args>
__device__ __forceinline__ unsigned char* chan_tables(const Args& a, unsigned char* lds) {
  if constexpr (WIDE) return a.gdyn + (size_t)blockIdx.x * a.gdyn_stride;
  else return lds;
}

// Subint s fitted by the Taylor path (fused_taylor's test, on the data
// pass's arguments): no scattering at the start and tau not fitted.
__device__ __forceinline__ bool spec_taylor_sub(const SpecArgs& a, int s) {
  const double t3 = a.init[(size_t)s * 5 + 3];
  const double tl = a.log10_tau ? pow(10.0, t3) : t3;
  return !a.exact && !a.fit_tau && tl == 0.0;
}

struct PhaseShiftArgs {
  int NHP, kc, Ns;
  double lo, hi;
  const double* data;      // [nprof][nbin]
  const double2* M;        // [nmodel][NHP] DC-zeroed
  const int* model_idx;
  const double* noise;     // [nprof] or null (NaN -> estimate)
  double* out;             // [nprof][6]
  const double2* tw;
};

// Taylor-moment cross-spectrum (phase-family fits, see ppfit_taylor.hip):
// kMT moments T_m = sum_k v_k^m W_k per channel, v_k = k / N in [0, 1]; an
// evaluation at per-channel offset y = 2 pi N delta uses terms m < kMTerm and
// is accepted while |y| <= kTaylorY, where the truncation
// kTaylorY^kMTerm / kMTerm! e^kTaylorY is < 2e-17 of sum_k |W_k|.
// Only one real part of each moment is ever used (Re T_m for even m, Im T_m
// for odd m: the sweep needs Re G_0, Im G_1, Re G_2 and i^m selects that part),
// so a channel's moments are kMT doubles ("compact moments", taylor_cells).
constexpr int kMT = 32;
// rows of the moment power table: every harmonic a moment block can touch
// (k <= N plus the zero-padded tail of the last block of steps)
__host__ __device__ constexpr int kVpowRows(int N) { return N + 1 + 4 * 64; }
constexpr int kMTerm = kMT - 2;
// k_fit_taylor keeps moments [0, tnl) of T slot 0 in LDS, tnl as large as
// lets kTaylorBlocksPerCU of its blocks share a CU's kLdsPerCU (the register
// limit is the same three blocks): all kMT up to 128 channels, 16 at 256
constexpr size_t kLdsPerCU = 160 * 1024;
constexpr int kTaylorBlocksPerCU = 3;
constexpr double kTaylorY = 3.0;

// Per-subint solver state handed from k_guess -> k_solve -> k_post (global).
struct SolveState {
  double x[5];     // current / final parameters
  double init[5];  // starting point (after the guess)
  double fun;
  double refs[3];  // nu_fit (resolved)
  // Taylor path: expansion centres (params at refs), and the trust-ncg state
  // saved when a proposal leaves both centres' radius (resumed after
  // k_moments recentres)
  double xc[2][5];
  double g[5], H[25], tr;
  int nfev, status, slot, scat, scat_post, taylor;
  int kit, phase, fin, mvalid, xslot, wslot;
  // split scattering solve (k_scat_sweep / k_scat_step): the proposal, its
  // step and predicted value, the Steihaug boundary flag, done
  double xp[5], pl[5], predv;
  int hits, sdone;
};

struct FitArgs {
  int sub0, nchan, nbin, NH, NHP, kc;
  int flags[5];
  int log10_tau, option, is_toa, guess, Ns, guess_wrap;
  int solver_flags;          // PPF_SOLVE_* / PPF_GUESS_* bits
  int method;                // PPF_METHOD_*
  int guess_wave;            // k_guess_w takes the subints it covers (guess_wave_ok)
  const double2* X;          // chunk [c][nchan][NHP]
  const double2* Dsp;        // chunk [c][nchan][NHP] data spectra (spec cache): the
                             // Taylor moment passes form X = D conj(M) from it
  const double2* R;          // chunk [c][NHP]
  const double2* M;          // [nmodel][nchan][NHP]
  const double* M2;          // [nmodel][nchan][NHP] |M|^2 (scattering sweeps)
  const double* pn;          // [nmodel][nchan]
  const int* model_idx;      // [nsub] or null
  const double* sig;         // chunk [c][nchan]
  const double* dsum;        // chunk [c][nchan]
  const double* freqs;       // [nsub][nchan]
  const uint8_t* mask;       // [nsub][nchan] or null
  const double* P;           // [nsub]
  const double* init;        // [nsub][5]
  const double* nu_fit;      // [nsub][3]
  const double* nu_out;      // [nsub][3]
  const double* guess_nu;    // [nsub] or null
  const double* guess_tau;   // [nsub] or null
  SolveState* st;            // chunk [c]
  double* T;                 // chunk [c][2][nchan][kMT] compact Taylor moments
  int tlds;                  // k_fit_taylor: byte offset of its LDS copy of T slot 0 in
                             // dynamic LDS (after the Meta arrays), 0 = read T from HBM
  int tnl;                   //   moments [0, tnl) of each channel in that copy: [nchan][tnl]
  const double2* tw;         // rfft twiddles e^{-2 pi i m / nbin}
  const double2* vpow;       // [kVpowRows(N)][16] (v^(2 col), v^(2 col + 1)), v = k / N
  const double2* Mmean;      // [nmodel][NHP] mean template spectrum or null
  unsigned long long* ptime; // [PPF_PHASE_N] k_fit_taylor phase clocks, or null
  double* trace;             // solver trace (ppf_set_trace): [nsub][trace_cap][kTraceRec]
  int trace_cap;             //   objective sweeps recorded per subint (0: off)
  double* acc;               // chunk [c][2][nchan][10]
  double* wsc;               // chunk [c][nchan][8]
  // outputs (global batch index sub0 + c)
  double* o_params;
  double* o_param_errs;
  double* o_nu_out;
  double* o_cov;
  double* o_scales;
  double* o_scale_errs;
  double* o_channel_snrs;
  double* o_chi2;
  double* o_red_chi2;
  double* o_snr;
  int* o_nfev;
  int* o_status;
  double* o_init_used;
  double* o_fun;
  double* o_cov_nosc;
  double* o_grad;            // [nsub][5] or null
  double* o_hess;            // [nsub][25] or null
  double bounds[5][2];       // TNC bounds (NaN = None)
  unsigned char* gdyn;       // WIDE kernels: [block][gdyn_stride] per-channel tables in HBM
  size_t gdyn_stride;
};

// One solver-trace record (diagnostic, ppf_set_trace): the point, f, the
// masked gradient and the 15 Hessian terms of one objective sweep, whether
// scipy counts it in nfev, and the sweep's index.  Written by thread 0.
constexpr int kTraceRec = 32;
__device__ __forceinline__ void trace_sweep(const FitArgs& a, int s, int isweep, const double* x,
                                            const double* out, int nout, bool counted) {
  if (!a.trace || threadIdx.x != 0 || isweep >= a.trace_cap) return;
  double* r = a.trace + ((size_t)s * a.trace_cap + isweep) * kTraceRec;
  for (int i = 0; i < 5; ++i) r[i] = x[i];
  for (int i = 0; i < 21; ++i) r[5 + i] = i < nout ? out[i] : NAN;
  r[26] = counted ? 1.0 : 0.0;
  r[27] = (double)isweep;
}

// ---------------------------------------------------------------------------
// FFTFIT search on a staged cross-spectrum rm_k = R_k conj(M_k), k < NH:
//   f(phi) = -Re sum_k rm_k e^{2 pi i k phi} / err^2      (pplib.py:1244-1256)
// scipy.optimize.brute on linspace(lo, hi, Ns) (first minimum), then
// scipy.optimize.fmin (Nelder-Mead, 1-D: nonzdelt 0.05, zdelt 2.5e-4,
// xatol = fatol = 1e-4, maxiter = maxfun = 200) from the grid minimum, as
// called by pplib.fit_phase_shift (pplib.py:2085-2086).
// ---------------------------------------------------------------------------
struct GuessShared {
  double red[kWaves];
  double bestv[kWaves];
  int besti[kWaves];
  double x0, x, fx;
  double out[8];
  double bf[kBlock];       // brute force: partial sums per (half, grid point)
  double2 fb[kBlock / 2];  // folded grid: b_j = sum_{k = j mod L} (-1)^k rm_k
  double2 fw[kBlock / 2];  //              w_m = e^{2 pi i m / L}
  double ev[2][kWaves];    // Nelder-Mead: per-wave partials, double-buffered
};

// np.argmin order: the first NaN wins, else the first smallest value.
__device__ __forceinline__ bool argmin_better(double v, int i, double bv, int bi) {
  if (i == 0x7fffffff) return false;
  if (bi == 0x7fffffff) return true;
  if (isnan(bv)) return isnan(v) && i < bi;
  if (isnan(v)) return true;
  return v < bv || (v == bv && i < bi);
}

// Sum over k in [k0, k1) of Re(rm_k e^{2 pi i k phi}) by one thread: the
// phasor advances by e^{2 pi i phi} per harmonic and is re-seeded exactly
// (turn_phasor) every 64 harmonics.
__device__ __forceinline__ double row_eval_phase(const double2* rm, int k0, int k1, double phi) {
  const double2 z = turn_phasor(1.0, phi);
  double acc = 0.0;
  for (int kb = k0; kb < k1; kb += 64) {
    double2 e = turn_phasor((double)kb, phi);
    const int ke = min(kb + 64, k1);
#pragma unroll 4
    for (int k = kb; k < ke; ++k) {
      const double2 r = rm[k];  // same address in every lane: LDS broadcast
      acc = fma(r.x, e.x, acc);
      acc = fma(-r.y, e.y, acc);
      e = cmul(e, z);
    }
  }
  return acc;
}

// All threads of the block evaluate sum_k Re(rm_k e^{2 pi i k phi}) together
// (thread t takes k = t, t + kBlock, ...); every thread returns the same
// value (fixed cross-wave order).  par: the LDS slot pair to use, alternated
// by the caller so that one barrier per evaluation suffices.
__device__ __forceinline__ double block_eval_phase(const double2* rm, int NH, double phi,
                                                   double* slot) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const double2 st = turn_phasor((double)kBlock, phi);
  double2 e = turn_phasor((double)tid, phi);
  double acc = 0.0;
  for (int k = tid; k < NH; k += kBlock) {
    const double2 r = rm[k];
    acc = fma(r.x, e.x, acc);
    acc = fma(-r.y, e.y, acc);
    e = cmul(e, st);
  }
  acc = wave_sum(acc);
  if (lane == 0) slot[w] = acc;
  __syncthreads();
  double t = slot[0];
#pragma unroll
  for (int q = 1; q < kWaves; ++q) t += slot[q];
  return t;
}

// One brute-force pass over the grid: FOLD evaluates the folded L-point DFT
// (gs.fb / gs.fw ready), else direct sums.  Leaves the argmin in
// gs.bestv[0] / gs.besti[0] and gs.x0; returns this thread's grid value for
// the single chunk of a FOLD pass (NaN otherwise).
template <bool FOLD>
__device__ __forceinline__ double brute_pass(const double2* rm, int NH, double ie2, int Ns,
                                             double lo, double hi, GuessShared& gs) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int GP = kBlock / 2;
  const double step = (hi - lo) / (double)(Ns - 1);
  const int half = tid / GP, gl = tid % GP;
  const int kmid = (NH + 1) / 2;
  const int L = Ns - 1;
  double bv = NAN, myf = NAN;
  int bi = 0x7fffffff;
  for (int g0 = 0; g0 < Ns; g0 += GP) {
    const int g = g0 + gl;
    double part = 0.0;
    if (g < Ns) {
      if constexpr (FOLD) {
        const int jm = (L + 1) / 2;
        const int j0 = half ? jm : 0, j1 = half ? L : jm;
        int mi = (j0 * g) % L;
        for (int j = j0; j < j1; ++j) {
          const double2 b = gs.fb[j], wv = gs.fw[mi];
          part = fma(b.x, wv.x, part);
          part = fma(-b.y, wv.y, part);
          mi += g;
          if (mi >= L) mi -= L;
        }
      } else {
        const double ph = (g == Ns - 1) ? hi : __dadd_rn(__dmul_rn((double)g, step), lo);
        part = half ? row_eval_phase(rm, kmid, NH, ph) : row_eval_phase(rm, 0, kmid, ph);
      }
    }
    gs.bf[tid] = part;
    __syncthreads();
    if (tid < GP && g < Ns) {
      const double f = -(gs.bf[tid] + gs.bf[GP + tid]) * ie2;
      myf = f;
      if (argmin_better(f, g, bv, bi)) { bv = f; bi = g; }
    }
    __syncthreads();
  }
  // argmin over the owning threads (ascending g within a thread)
  if (tid < GP) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double ov = __shfl_xor(bv, o);
      const int oi = __shfl_xor(bi, o);
      if (argmin_better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) { gs.bestv[w] = bv; gs.besti[w] = bi; }
  }
  __syncthreads();
  if (tid == 0) {
    double v = gs.bestv[0];
    int i = gs.besti[0];
    for (int q = 1; q < GP / 64; ++q)
      if (argmin_better(gs.bestv[q], gs.besti[q], v, i)) { v = gs.bestv[q]; i = gs.besti[q]; }
    gs.x0 = (i == Ns - 1) ? hi : __dadd_rn(__dmul_rn((double)i, step), lo);
    gs.bestv[0] = v;
    gs.besti[0] = i;
  }
  __syncthreads();
  return myf;
}

// Prime-factor split of the grid DFT length L = A B (A, B coprime, B <=
// kPfaMax, the most balanced such pair): the get_TOAs / ppalign grids with
// Ns = nbin (L = nbin - 1: 2047 = 23 x 89, 1023 = 31 x 33, 4095 = 63 x 65,
// 511 = 7 x 73, 255 = 15 x 17) take two passes of short DFTs instead of
// Ns x NH phasor terms.  false: no such split (L prime, or too long).
constexpr int kPfaMax = 256, kPfaPer = 16;  // <= kPfaPer grid values per thread
__host__ __device__ inline bool pfa_split(int L, int& A, int& B) {
  A = B = 0;
  if (L < 6 || L > kBlock * kPfaPer) return false;
  int best = 1 << 30;
  for (int a = 2; a * a <= L; ++a) {
    if (L % a) continue;
    const int b = L / a;
    int x = a, y = b;
    while (y) { const int t = x % y; x = y; y = t; }
    if (x != 1 || b > kPfaMax) continue;
    if (a + b < best) { best = a + b; A = a; B = b; }
  }
  return A > 0;
}
// LDS scratch (double2 slots) guess_search needs for the PFA grid of Ns
// points on (-1/2, 1/2): Y [L] plus the A- and B-point roots of unity; 0 when
// the grid is not taken that way
__host__ __device__ inline int pfa_scratch_slots(int Ns, int NH) {
  const int L = Ns - 1;
  int A, B;
  if (L <= kBlock / 2 && NH > 2 * L) return 0;  // the folded direct grid
  return pfa_split(L, A, B) ? L + A + B : 0;
}

// Brute-force grid on (-1/2, 1/2) by the prime-factor DFT: with phi_g =
// -1/2 + g / L, f(phi_g) = -Re sum_{j < L} b_j w^{j g} / err^2, b_j =
// sum_{k = j mod L} (-1)^k rm_k, w = e^{2 pi i / L}.  Good-Thomas: j = (B n1
// + A n2) mod L, g = (B (B^-1 mod A) k1 + A (A^-1 mod B) k2) mod L, so
// w^{j g} = W_A^{n1 k1} W_B^{n2 k2}: Y[n1][k2] = sum_n2 b_j W_B^{n2 k2}, then
// sum_n1 Y[n1][k2] W_A^{n1 k1}.  Each thread keeps its grid values; returns
// (via gs) the argmin as brute_pass does, and whether another grid point is
// within rounding (1e-12 relative) of it -- then the caller re-takes the grid
// by direct sums, as for the folded grid.
__device__ inline bool pfa_pass(const double2* rm, int NH, double ie2, int Ns, double lo,
                                double hi, GuessShared& gs, double2* scr, int A, int B,
                                unsigned long long* clk = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  unsigned long long tc = clk ? wall_clock64() : 0ull;
  auto tick = [&](int slot) {  // diagnostic: [13 + slot] phase clocks of this pass
    if (clk && tid == 0) {      // (ptime 23-25: clear of k_post's 16-22)
      const unsigned long long t = wall_clock64();
      atomicAdd(&clk[13 + slot], t - tc);
      tc = t;
    }
  };
  const int L = Ns - 1;
  double2* Y = scr;
  double2* wB = scr + L;
  double2* wA = wB + B;
  for (int m = tid; m < B; m += kBlock) {
    double sn, cs;
    sincospi(2.0 * (double)m / (double)B, &sn, &cs);
    wB[m] = cmk(cs, sn);
  }
  for (int m = tid; m < A; m += kBlock) {
    double sn, cs;
    sincospi(2.0 * (double)m / (double)A, &sn, &cs);
    wA[m] = cmk(cs, sn);
  }
  __syncthreads();
  tick(0);
  // stage 1: Y[n1][k2] = sum_{n2 < B} b_{(B n1 + A n2) mod L} W_B^{n2 k2}, the
  // terms in four independent running sums (n2 mod 4) so that four LDS reads
  // are in flight instead of one dependent chain; with NH <= L every folded
  // b_j is one signed harmonic or 0.  (Only the argmin is taken from these
  // values, and any grid point within 1e-12 of it sends the caller to the
  // direct sums: the order of the additions cannot change the result.)
  const bool one = NH <= L;
  // branch-free when every fold has at most one term (an unconditional LDS
  // read and a select): the loop below then stays one basic block, so its
  // four terms' reads overlap
  auto bj = [&](int j) {
    if (one) {
      const double2 r = rm[min(j, NH - 1)];
      const double sg = j < NH ? ((j & 1) ? -1.0 : 1.0) : 0.0;
      return cmk(sg * r.x, sg * r.y);
    }
    double2 b = cmk(0.0, 0.0);
    for (int k = j; k < NH; k += L) b = (k & 1) ? csub(b, rm[k]) : cadd(b, rm[k]);
    return b;
  };
  // The twiddles W_B^{n2 k2} of a lane's output run along its own chain
  // (times W_B^{4 k2} per block of four terms) instead of a table read per
  // term: the B-entry table is read by every lane at a different index, and
  // those bank-conflicted reads made this stage LDS-bound.  Each chain is
  // re-seeded exactly from the table every 32 terms.
  auto stage1 = [&](auto onec) {
  constexpr bool ONE = decltype(onec)::value;
  auto bj1 = [&](int j) {
    if constexpr (ONE) {
      const double2 r = rm[min(j, NH - 1)];
      const double sg = j < NH ? ((j & 1) ? -1.0 : 1.0) : 0.0;
      return cmk(sg * r.x, sg * r.y);
    } else {
      return bj(j);
    }
  };
  for (int q = tid; q < L; q += kBlock) {
    const int n1 = q / B, k2 = q - n1 * B;
    int j = (B * n1) % L;
    const double2 st4 = wB[(4 * k2) % B];
    double2 acc[4] = {cmk(0.0, 0.0), cmk(0.0, 0.0), cmk(0.0, 0.0), cmk(0.0, 0.0)};
    double2 tw[4];
    int n2 = 0;
    for (; n2 + 4 <= B; n2 += 4) {
      if ((n2 & 31) == 0) {
#pragma unroll
        for (int u = 0; u < 4; ++u) tw[u] = wB[((n2 + u) * k2) % B];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc[u] = cadd(acc[u], cmul(bj1(j), tw[u]));
        tw[u] = cmul(tw[u], st4);
        j += A;
        if (j >= L) j -= L;
      }
    }
#pragma unroll
    for (int u = 0; u < 3; ++u) {  // the B mod 4 last terms
      if (n2 + u < B) {
        acc[u] = cadd(acc[u], cmul(bj1(j), wB[((n2 + u) * k2) % B]));
        j += A;
        if (j >= L) j -= L;
      }
    }
    Y[q] = cadd(cadd(acc[0], acc[1]), cadd(acc[2], acc[3]));
  }
  };
  if (one) stage1(std::true_type{});
  else stage1(std::false_type{});
  __syncthreads();
  tick(1);
  // stage 2 and the per-thread grid values (int arithmetic: B Ai, A Bi <= L)
  int Ai = 1, Bi = 1;  // B^-1 mod A, A^-1 mod B
  while (B * Ai % A != 1) ++Ai;
  while (A * Bi % B != 1) ++Bi;
  const int cB = B * Ai % L, cA = A * Bi % L;
  double vals[kPfaPer];
  int gi[kPfaPer];
  double bv = NAN;
  int bi = 0x7fffffff;
#pragma unroll
  for (int r = 0; r < kPfaPer; ++r) {
    const int q = tid + r * kBlock;
    vals[r] = NAN;
    gi[r] = 0x7fffffff;
    if (q < L) {
      const int k1 = q / B, k2 = q - k1 * B;
      double rs[4] = {0.0, 0.0, 0.0, 0.0};
      int m = 0, n1 = 0;
      for (; n1 + 4 <= A; n1 += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const double2 y = Y[(n1 + u) * B + k2], t = wA[m];
          rs[u] = fma(y.x, t.x, rs[u]);
          rs[u] = fma(-y.y, t.y, rs[u]);
          m += k1;
          if (m >= A) m -= A;
        }
      }
#pragma unroll
      for (int u = 0; u < 3; ++u) {  // the A mod 4 last terms
        if (n1 + u < A) {
          const double2 y = Y[(n1 + u) * B + k2], t = wA[m];
          rs[u] = fma(y.x, t.x, rs[u]);
          rs[u] = fma(-y.y, t.y, rs[u]);
          m += k1;
          if (m >= A) m -= A;
        }
      }
      const double re = (rs[0] + rs[1]) + (rs[2] + rs[3]);
      const int g = (cB * k1 + cA * k2) % L;
      const double f = -re * ie2;
      vals[r] = f;
      gi[r] = g;
      if (argmin_better(f, g, bv, bi)) { bv = f; bi = g; }
    }
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double ov = __shfl_xor(bv, o);
    const int oi = __shfl_xor(bi, o);
    if (argmin_better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
  }
  tick(2);
  if (lane == 0) { gs.bestv[w] = bv; gs.besti[w] = bi; }
  __syncthreads();
  if (tid == 0) {
    double v = gs.bestv[0];
    int i = gs.besti[0];
    for (int q = 1; q < kWaves; ++q)
      if (argmin_better(gs.bestv[q], gs.besti[q], v, i)) { v = gs.bestv[q]; i = gs.besti[q]; }
    const double step = (hi - lo) / (double)(Ns - 1);
    gs.x0 = (i == Ns - 1) ? hi : __dadd_rn(__dmul_rn((double)i, step), lo);
    gs.bestv[0] = v;
    gs.besti[0] = i;
  }
  __syncthreads();
  const double v = gs.bestv[0];
  const int i = gs.besti[0];
  bool near = false;
#pragma unroll
  for (int r = 0; r < kPfaPer; ++r)
    if (gi[r] != 0x7fffffff && gi[r] != i && !(fabs(vals[r] - v) > 1e-12 * fabs(v))) near = true;
  return __syncthreads_or(near);
}

// scipy.optimize.fmin's simplex moves in one variable (guess_search's
// polish, maxiter 200, xtol = ftol = 1e-4): F(x) evaluates and counts (it
// sets stop instead once maxfun calls are spent); on return (s0, f0) is the
// best vertex and (s1, f1) the other.  Written as a state machine around ONE
// call of F, so the evaluation (a block- or wave-wide phasor sum) is inlined
// once instead of at each of the seven moves.  stt names the point xv being
// evaluated: 0 s0, 1 s1 (the start), 2 reflection, 3 expansion, 4 outside
// contraction, 5 inside contraction, 6 shrink.
template <class Eval>
__device__ __forceinline__ void nm_polish(Eval& F, const bool& stop, const int& fcalls,
                                          int maxfun, double x0, double& s0, double& f0,
                                          double& s1, double& f1) {
  const int maxiter = 200;
  s0 = x0;
  s1 = (s0 != 0.0) ? (1.0 + 0.05) * s0 : 0.00025;
  f0 = 0.0;
  f1 = 0.0;
  double fxr = 0.0, xr = 0.0, xv = s0;
  int it = 1;
  int stt = 0;
  for (;;) {
    const double fv = F(xv);
    if (stop) break;
    bool moved = false;  // an iteration's move is complete
    if (stt == 0) {
      f0 = fv;
      xv = s1;
      stt = 1;
      continue;
    } else if (stt == 1) {
      f1 = fv;
      if (f1 < f0) { double t = s0; s0 = s1; s1 = t; t = f0; f0 = f1; f1 = t; }
    } else if (stt == 2) {
      fxr = fv;
      xr = xv;
      const double xbar = s0;
      if (fxr < f0) {
        xv = __dsub_rn(__dmul_rn(3.0, xbar), __dmul_rn(2.0, s1));
        stt = 3;
      } else if (fxr < f1) {
        xv = __dsub_rn(__dmul_rn(1.5, xbar), __dmul_rn(0.5, s1));
        stt = 4;
      } else {
        xv = __dadd_rn(__dmul_rn(0.5, xbar), __dmul_rn(0.5, s1));
        stt = 5;
      }
      continue;
    } else if (stt == 3) {
      if (fv < fxr) { s1 = xv; f1 = fv; } else { s1 = xr; f1 = fxr; }
      moved = true;
    } else if (stt == 4 || stt == 5) {
      if (stt == 4 ? (fv <= fxr) : (fv < f1)) {
        s1 = xv;
        f1 = fv;
        moved = true;
      } else {  // shrink toward the best vertex
        s1 = __dadd_rn(s0, __dmul_rn(0.5, __dsub_rn(s1, s0)));
        xv = s1;
        stt = 6;
        continue;
      }
    } else {
      f1 = fv;
      moved = true;
    }
    if (moved) {
      ++it;
      if (f1 < f0) { double t = s0; s0 = s1; s1 = t; t = f0; f0 = f1; f1 = t; }
    }
    // the next iteration: loop condition, convergence test, reflection
    if (!(fcalls < maxfun && it < maxiter)) break;
    if (fabs(s1 - s0) <= 1e-4 && fabs(f0 - f1) <= 1e-4) break;
    xv = __dsub_rn(__dmul_rn(2.0, s0), s1);
    stt = 2;
  }
  if (f1 < f0) { double t = s0; s0 = s1; s1 = t; t = f0; f0 = f1; f1 = t; }
}

__device__ inline void guess_search(const double2* rm, int NH, double ie2, int Ns, double lo,
                                    double hi, GuessShared& gs, bool allow_fold = true,
                                    unsigned long long* clk = nullptr,
                                    double2* pfa_scr = nullptr) {
  const int tid = threadIdx.x;
  // diagnostic clocks (ppf_phase_profile): [0] brute force, [1] Nelder-Mead, [2] NM calls,
  // [3] prime-factor grids re-taken by direct sums
  const unsigned long long c0 = clk ? wall_clock64() : 0ull;
  // ---- brute force over the inclusive grid (np.mgrid[lo:hi:Ns*1j]) ----
  // grid and simplex arithmetic use explicit _rn ops: hipcc would otherwise
  // contract them into FMAs and move the points off numpy's values.
  // Threads own grid points (kBlock / 2 per chunk) and walk half of the
  // harmonics each; the halves meet in LDS.
  // On the get_TOAs grid (lo, hi) = (-0.5, 0.5) every grid phase is
  // -1/2 + g / L, L = Ns - 1, so f(phi_g) = Re sum_j b_j w^{j g} with the
  // spectrum folded mod L: an L-point DFT instead of Ns x NH phasor terms.
  // The end points phi = -0.5 and 0.5 get the same folded sum (w^0 and w^L):
  // their direct sums were already bitwise equal (turn_phasor is exact at
  // half turns), so argmin's tie rule still picks g = 0.  Every grid point
  // takes the folded path: a direct sum on any lane would hold its wave.
  // The folded values round differently from the direct sums, so when any
  // other grid point comes within 1e-12 (relative) of the minimum the grid
  // is re-taken by direct sums and np.argmin decides on those.
  constexpr int GP = kBlock / 2;
  const int L = Ns - 1;
  const bool fold = allow_fold && lo == -0.5 && hi == 0.5 && L >= 2 && L <= GP && NH > 2 * L;
  if (fold) {
    if (tid < L) {
      double2 b = cmk(0.0, 0.0);
      for (int k = tid; k < NH; k += L) {
        const double2 r = rm[k];
        b = (k & 1) ? csub(b, r) : cadd(b, r);
      }
      gs.fb[tid] = b;
      double sn, cs;
      sincospi(2.0 * (double)tid / (double)L, &sn, &cs);
      gs.fw[tid] = cmk(cs, sn);
    }
    __syncthreads();
    const double myf = brute_pass<true>(rm, NH, ie2, Ns, lo, hi, gs);
    // near tie on the folded grid (the end points -0.5 / 0.5 are one point)
    const double v = gs.bestv[0];
    const int i = gs.besti[0];
    const bool endpair = (i == 0 && tid == Ns - 1) || (i == Ns - 1 && tid == 0);
    const bool near = tid < Ns && tid != i && !endpair && !(fabs(myf - v) > 1e-12 * fabs(v));
    if (__syncthreads_or(near)) brute_pass<false>(rm, NH, ie2, Ns, lo, hi, gs);
  } else {
    int A = 0, B = 0;
    const bool pfa = pfa_scr && allow_fold && lo == -0.5 && hi == 0.5 &&
                     pfa_scratch_slots(Ns, NH) > 0 && pfa_split(L, A, B);
    if (!pfa || pfa_pass(rm, NH, ie2, Ns, lo, hi, gs, pfa_scr, A, B, clk)) {
      if (clk && pfa && tid == 0) atomicAdd(&clk[3], 1ull);  // [3] PFA near-tie re-takes
      brute_pass<false>(rm, NH, ie2, Ns, lo, hi, gs);
    }
  }
  const unsigned long long c1 = clk ? wall_clock64() : 0ull;
  // ---- Nelder-Mead polish: every thread runs the (uniform, scalar) simplex
  // logic; each evaluation is one block-wide sum ----
  {
    const int maxfun = 200;
    int fcalls = 0;
    bool stop = false;
    auto F = [&](double xv) -> double {
      if (fcalls >= maxfun) { stop = true; return 0.0; }
      ++fcalls;
      return -block_eval_phase(rm, NH, xv, gs.ev[fcalls & 1]) * ie2;
    };
    double s0, f0, s1, f1;
    nm_polish(F, stop, fcalls, maxfun, gs.x0, s0, f0, s1, f1);
    if (tid == 0) {
      gs.x = s0;
      gs.fx = fmin(f0, f1);
      if (clk) {
        atomicAdd(&clk[0], c1 - c0);
        atomicAdd(&clk[1], wall_clock64() - c1);
        atomicAdd(&clk[2], (unsigned long long)fcalls);
      }
    }
  }
  __syncthreads();
}

constexpr int kMaxGauss = 32;
struct GaussArgs {
  int nbin, ngauss;
  int code[3];              // evolution of loc / wid / amp: 0 power law, 1 linear
  double nu_ref, lnu;       // reference frequency and its log (host numpy)
  double fwhm, sqrt2pi;     // 2 sqrt(2 ln 2), sqrt(2 pi) as numpy forms them
  double params[2 + 6 * kMaxGauss];  // DC, TAU, then loc, dloc, wid, dwid, amp, damp
};

constexpr int kMaxSplineK = 5, kMaxEig = 64;
struct SplineArgs {
  int nbin, neig, n, k, ncoef;  // bins, eigenvectors, knots, degree, coefficients per dimension
  const double* t;              // [n] knots
  const double* c;              // [neig][ncoef] B-spline coefficients
  const double* mean;           // [nbin] mean profile
  const double* eigvec;         // [nbin][neig]
};

constexpr int kMaxIrf = 16;
struct IrArgs {
  int nw;                 // instrumental responses besides the DM smearing
  int type[kMaxIrf];      // 0 rect, 1 gauss
  double wid[kMaxIrf];    // [rot]
  double fwhm;            // 2 sqrt(2 ln 2) as numpy forms it
  double dm_wid_num;      // 8.3e-6 chan_bw (0: no DM smearing response)
  double P;               // period [s]
};

struct ResidArgs {
  const double* data;      // [nrow][nbin]
  const double* phase;     // [nrow] or NULL
  const double* model;     // [nmodel][nbin]
  const int* model_row;    // [nrow] or NULL (row r)
  const double* scale;     // [nrow]
  const double* tau;       // [nrow] scattering time [rot] or NULL
  const double* errs;      // [nrow]
  double dof;
  double* out;             // [nrow]
};

// ---------------------------------------------------------------------------
// kernel declarations
// ---------------------------------------------------------------------------
__global__ void k_twiddles(double2* tw, int nbin);
template <int LOGN>
__global__ void k_model_spec(const double* model, double2* M, double* pn, int NHP, int zero_dc,
                             const double2* tw, double* M2);
template <int LOGN, bool WIDE = false> __global__ void k_data_xspec(SpecArgs a);
template <int LOGN> __global__ void k_phase_shift(PhaseShiftArgs a);
template <int LOGN>
__global__ void k_rotate_rows(const double* in, const double* phase, const double* tau,
                              double* out, const double2* tw);
template <int LOGN>
__global__ void k_irfft_rows(const double2* spec, double* out, const double2* tw);
template <int LOGN>
__global__ void k_noise_rows(const double* in, double* out, int kc, const double2* tw);
template <int LOGN>
__global__ void k_synth(const double2* Mfull, const double* phase, double* data, int nchan,
                        int NHP, double sigma, uint64_t seed, int64_t sub0, const double2* tw);
template <int LOGN>
__global__ void k_rot_accum(const double* data, const double* phase, const double* weight,
                            double2* partial, int nsub, int nchan, int nsplit,
                            const double2* tw);
__global__ void k_rot_accum_w(const double* data, const double* phase, const double* weight,
                              double2* partial, int nsub, int nchan, int nsplit, const double2* tw);
__global__ void k_rot_accum_spec(const double2* spec, const double* phase, const double* weight,
                                 double2* partial, int nsub, int nchan, int nsplit, int N,
                                 int NHP);
__global__ void k_accum_reduce(const double2* partial, double2* accum, int nsplit, size_t count);
template <int LOGN> __global__ void k_resid_chi2(ResidArgs a, const double2* tw);
__global__ void k_vpow(double2* vp, int nbin, int rows);
// any nbin (ppfit_generic.hip)
__global__ void k_model_spec_gen(const double* model, double2* M, double* pn, int NHP, int zero_dc,
                                 const double2* tw, double* M2, int nbin);
__global__ void k_rotate_rows_gen(const double* in, const double* phase, const double* tau,
                                  double* out, const double2* tw, int nbin);
__global__ void k_phase_shift_gen(PhaseShiftArgs a, int nbin);
__global__ void k_rfft_rows_gen(const double* in, double2* spec, const double2* tw, int nbin);
__global__ void k_irfft_rows_gen(const double2* spec, double* out, const double2* tw, int nbin);
__global__ void k_noise_rows_gen(const double* in, double* out, int kc, const double2* tw, int nbin);
__global__ void k_rot_accum_gen(const double* data, const double* phase, const double* weight,
                                double2* partial, int nsub, int nchan, int nsplit,
                                const double2* tw, int nbin);
__global__ void k_resid_chi2_gen(ResidArgs a, const double2* tw, int nbin);
template <bool LTW>
__global__ void k_dft_rows_mfma(const double* rows, double2* D, int nrows, int nbin, int NHP,
                                const double2* tw);
__global__ void k_data_post_gen(SpecArgs a, int nbin);
__global__ void k_synth_gen(const double2* Mfull, const double* phase, double* data, int nchan,
                            int NHP, double sigma, uint64_t seed, int64_t sub0,
                            const double2* tw, int nbin);
__global__ void k_gauss_port(GaussArgs g, const double* freqs, double* out);
template <typename T>
__global__ void k_unpack(const T* raw, const double* scl, const double* offs, int nsub, int npol,
                         int nchan, int nbin, int pmode, double* out);
__global__ void k_remove_baseline(double* data, const double* w, int npol, int nchan, int nbin,
                                  int ntot, int width, int* win_out);
__global__ void k_profile_snr(const double* rows, int nbin, int width, double thr, double* out);
__global__ void k_scat_taus(const double* freqs, int n, double tau, double alpha, double nu_ref,
                            double* out);
__global__ void k_guess(FitArgs a);
constexpr int kScatPart = 24;  // split scattering sweep partial: f, g[5], H pairs[15], pad
constexpr int kScatAcc = 10;   // cell-loop accumulators per channel (NACC)
// k_scat_sweep's dynamic LDS: the Meta arrays, then (two-phase sweep) one row
// of kScatAcc group sums per channel a block can take at the given split
__host__ __device__ inline size_t scat_meta_lds(int nchan) {
  return ((size_t)nchan * (5 * sizeof(double) + sizeof(int)) + 255) & ~(size_t)255;
}
__host__ __device__ inline size_t scat_sweep_lds(int nchan, int split) {
  const int ng = (nchan + 7) >> 3;
  // rows of kScatAcc sums, then one (phase, tau_n) pair per row
  const size_t rows = (size_t)((ng + split - 1) / split) * 8;
  return scat_meta_lds(nchan) + rows * (kScatAcc * sizeof(double) + 2 * sizeof(double));
}
__global__ void k_scat_sweep(FitArgs a, double* part, int split, int init);
__global__ void k_scat_step(FitArgs a, const double* part, int init, int* ctrs, int par);
__global__ void k_model_mean(const double2* M, double2* Mmean, int nchan, int NHP);
template <bool MOM, bool DSP, bool WIDE = false>
__global__ void k_fit_taylor(FitArgs a);
template <int U, bool DSP>
__global__ void k_moments(FitArgs a);
__global__ void k_selftest(int* fails);
template <bool SCAT, bool WIDE = false> __global__ void k_solve(FitArgs a);
template <bool SCAT, bool WIDE = false> __global__ void k_tnc(FitArgs a);
template <bool SCAT, bool WIDE = false> __global__ void k_ncg(FitArgs a);
__global__ void k_guess_w(FitArgs a);
template <bool SCAT, bool WIDE = false> __global__ void k_post(FitArgs a);

}  // namespace ppf
