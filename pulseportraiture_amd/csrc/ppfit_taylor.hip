// ppfit_taylor.hip -- the cross-spectrum-free solver for phase-family fits.
//
// For fits whose channels differ only by a phase shift phi_n (fit flags over
// phi, DM, GM with tau = 0; the get_TOAs headline path and ppalign), every
// quantity the objective, gradient and Hessian need from a channel is
//   C_n(phi_n)   = Re  sum_k X_nk e^{2 pi i k phi_n}        (pptoaslib.py:431)
//   dC_n/dphi_n  ∝ Im  sum_k k X_nk e^{2 pi i k phi_n}      (pptoaslib.py:437-449)
//   d2C_n/dphi_n2 ∝ Re sum_k k^2 X_nk e^{2 pi i k phi_n}    (pptoaslib.py:451-461)
// with X_nk = D_nk conj(M_nk).  Instead of re-reading X (16 B per cell) on
// every trust-region evaluation, k_moments reads it once and reduces each
// channel to kMT Taylor moments about a centre phi_c,n:
//   T_nm = sum_k v_k^m X_nk e^{2 pi i k phi_c,n},   v_k = k / N,
// so that any later evaluation within |2 pi N (phi_n - phi_c,n)| <= kTaylorY
// is a kMTerm-term series (taylor_cells in ppfit_fit.hip) accurate to the
// fp64 rounding of the exact sums.  k_fit_taylor runs scipy's trust-ncg on
// those series; a proposal outside the radius of both stored centres gets a
// new centre (one more pass over the subint's X, moments_from_X) first.  Per
// subint X is written once (k_data_xspec) and read once (k_moments), plus
// once per recentring.
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

// ---------------------------------------------------------------------------
// Moments of the fitted channels of subint c about centre xc (at refs), from
// the cross-spectrum rows X written by k_data_xspec, into T[c][slot]:
//   T_nm = sum_k v_k^m W_nk,  v_k = k / N,  W_nk = X_nk e^{2 pi i k phi_c,n}.
// The k-contraction runs on the f64 matrix cores: each wave takes tiles of 16
// fitted channels; per step of 4 harmonics, v_mfma_f64_16x16x4 multiplies
// A = v^(2i) (the 16 even moments x 4 harmonics) by B = Re W, and A = v^(2i+1)
// (the 16 odd moments) by B = Im W (4 harmonics x 16 channels): the compact
// moments (kernels.hpp), Re T_m for even m and Im T_m for odd m, and nothing
// else -- two MFMAs per step.  Lane l supplies harmonic 4 s + (l >> 4) of
// channel l & 15 to B and v^(2 (l & 15)), v^(2 (l & 15) + 1) of that harmonic
// to A (v is exact when N is a power of two).  X rows stream through
// registers U steps ahead of the MFMAs.  All kMT moments are kept (cnt =
// kMT): the truncation bound then holds for any spectrum.
// ---------------------------------------------------------------------------
typedef double f64x4 __attribute__((ext_vector_type(4)));

// Steps (of 4 harmonics) between exact re-seeds of the phasor chains
// (turn_phasor is a sincospi: re-seeded every block it cost more vector
// issue than the chains); in between each chain advances by e^{2 pi i 8
// phi_c} per step pair.  A multiple of every tile's U, so the 16- and
// 8-channel tiles re-seed at the same harmonics (bitwise the same moments).
constexpr int kMomReseedSteps = 8;
// steps in flight of k_fit_taylor's fused first moment pass when it forms X
// from the data-spectrum cache (two load streams, D and M, per step)
#ifndef PPF_DSP_U
#define PPF_DSP_U 2
#endif
// ... and when it reads X (one load stream)
#ifndef PPF_MOM_U
#define PPF_MOM_U 4
#endif


// X rows: plain loads (the non-temporal hint measured slower here)
__device__ __forceinline__ double2 xload(const double2* p) { return *p; }

// v^m (m < 32) in one fixed order: v, v^2, v^4, v^8 by squaring, the
// factors of m & 15 multiplied in bit order, then v^16 = v^8 v^8 for m >= 16.
__device__ __forceinline__ double vpow_m(double v, double v2, double v4, double v8, int m) {
  double pc = (m & 1) ? v : 1.0;
  pc *= (m & 2) ? v2 : 1.0;
  pc *= (m & 4) ? v4 : 1.0;
  pc *= (m & 8) ? v8 : 1.0;
  return (m & 16) ? pc * (v8 * v8) : pc;
}

// v^(2 col) and v^(2 col + 1) of harmonic k (v = k iN), in the table's order.
__device__ __forceinline__ double2 vpow_inline(int k, double iN, int col) {
  const double v = (double)k * iN;
  const double v2 = v * v, v4 = v2 * v2, v8 = v4 * v4;
  return cmk(vpow_m(v, v2, v4, v8, 2 * col), vpow_m(v, v2, v4, v8, 2 * col + 1));
}

// The A operands, v^(2i) and v^(2i+1) for the harmonic k = 4 step + (l >> 4)
// of a lane and its row i = l & 15, come from a table built once per nbin
// (k_vpow): the powers are the same for every channel, so forming them per
// step (3 squarings and up to 5 selected products each, on every lane) would
// cost more vector issue than the two MFMAs they feed.
// v = k / (nbin / 2): 2 / nbin is 1 / N to the bit for even nbin, and keeps
// v y = 2 pi k d for odd nbin (taylor_cells' y = 2 pi (nbin / 2) d)
__global__ void k_vpow(double2* vp, int nbin, int rows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * 16) return;
  const int k = i >> 4, col = i & 15;
  vp[i] = vpow_inline(k, 2.0 / (double)nbin, col);
}

// One 16-channel tile by one wave: lane l handles channel n (column l & 15 of
// the B operand; ok = fitted) at harmonic offset l >> 4, with centre phase
// phic; U = steps in flight.  Each step is two MFMAs: Re W times the even
// moment rows of A and Im W times the odd ones, with even and odd steps in
// separate accumulators (independent chains).
// A lane rotates its own element and feeds it straight to the matrix core:
// no cross-lane trade, no select.  Its two phasor chains (even / odd steps)
// restart from turn_phasor every kMomReseedSteps steps.  The next block's X and power rows
// stream into each step's registers as soon as its MFMAs have issued, so U
// steps of loads stay in flight with one register set.
// DSP (data-spectrum cache, a.Dsp): the lane loads D_k and M_k instead and
// forms X_k = D_k conj(M_k) (0 at k = 0) -- k_data_xspec's arithmetic on the
// same operands, so the same X bit for bit.
template <int U, bool DSP>
__device__ __forceinline__ void moment_tile16(const FitArgs& a, int c, int slot, int n, bool ok,
                                              double phic) {
  static_assert(kMT == 32, "two 16-row MFMA tiles");
  static_assert(U % 2 == 0, "steps go in pairs");
  constexpr int UP = U / 2;
  const int lane = threadIdx.x & 63;
  const int N = a.nbin / 2;
  const int nblk = ((N + 1 + 3) / 4 + U - 1) / U;  // blocks of U 4-harmonic steps
  const int col = lane & 15, kk = lane >> 4;
  const size_t xrow = ((size_t)c * a.nchan + (ok ? n : 0)) * a.NHP;
  const double2* __restrict__ Xr = (DSP ? a.Dsp : a.X) + xrow;
  const double2* __restrict__ Mr = nullptr;
  if constexpr (DSP) {
    const int s = a.sub0 + c;
    const int midx = a.model_idx ? a.model_idx[s] : 0;
    Mr = a.M + ((size_t)midx * a.nchan + (ok ? n : 0)) * a.NHP;
  }
  // power row of step t for this lane: vpow[(4 t + kk) * 16 + col]
  const double2* __restrict__ vp = a.vpow + (size_t)kk * 16 + col;
  const double2 s8 = turn_phasor(8.0, phic);
  // Re T of the even moments (d) and Im T of the odd ones (g); even / odd steps
  f64x4 d0 = {0.0, 0.0, 0.0, 0.0}, d2 = d0;
  f64x4 g0 = d0, g2 = d0;
  // loads are unpredicated (X index clamped to N; the power table is padded
  // past the last block); cells k > N and idle lanes are zeroed at use
  double2 xb[U], pb[U], mb[DSP ? U : 1];
#pragma unroll
  for (int t = 0; t < U; ++t) {
    xb[t] = xload(Xr + min(4 * t + kk, N));
    if constexpr (DSP) mb[t] = Mr[min(4 * t + kk, N)];
    pb[t] = vp[(size_t)t * 64];
  }
  // step t's cell from register set i
  auto xcell = [&](int t, int i) {
    const int k = 4 * t + kk;
    if constexpr (DSP) {
      const double2 x = cmulc(xb[i], mb[i]);
      return (ok && k >= 1 && k <= N) ? x : cmk(0.0, 0.0);
    } else {
      return (ok && k <= N) ? xb[i] : cmk(0.0, 0.0);
    }
  };
  double2 e0 = cmk(1.0, 0.0), e1 = e0;
  for (int b = 0; b < nblk; ++b) {
    if ((b * U) % kMomReseedSteps == 0) {  // exact phasors; the chains carry them between
      e0 = turn_phasor((double)(4 * (b * U) + kk), phic);
      e1 = turn_phasor((double)(4 * (b * U + 1) + kk), phic);
    }
#pragma unroll
    for (int u = 0; u < UP; ++u) {
      const double2 W0 = cmul(xcell(b * U + 2 * u, 2 * u), e0);
      const double2 W1 = cmul(xcell(b * U + 2 * u + 1, 2 * u + 1), e1);
      const double2 p0 = pb[2 * u], p1 = pb[2 * u + 1];
      d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(p0.x, W0.x, d0, 0, 0, 0);
      g0 = __builtin_amdgcn_mfma_f64_16x16x4f64(p0.y, W0.y, g0, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f64_16x16x4f64(p1.x, W1.x, d2, 0, 0, 0);
      g2 = __builtin_amdgcn_mfma_f64_16x16x4f64(p1.y, W1.y, g2, 0, 0, 0);
      e0 = cmul(e0, s8);
      e1 = cmul(e1, s8);
      // rolling prefetch: this pair's registers take the next block's rows
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int t = 2 * u + h;
        xb[t] = xload(Xr + min(4 * ((b + 1) * U + t) + kk, N));
        if constexpr (DSP) mb[t] = Mr[min(4 * ((b + 1) * U + t) + kk, N)];
        pb[t] = vp[(size_t)((b + 1) * U + t) * 64];
      }
    }
  }
  d0 += d2;
  g0 += g2;
  // D[row i = (l >> 4) + 4 r][col = channel l & 15]: moments 2 i and 2 i + 1
  if (ok) {
    double2* Tn = reinterpret_cast<double2*>(a.T + (((size_t)c * 2 + slot) * a.nchan + n) * kMT);
#pragma unroll
    for (int r = 0; r < 4; ++r) Tn[kk + 4 * r] = cmk(d0[r], g0[r]);
  }
}

// The same moments from an 8-channel tile (recentring inside k_fit_taylor,
// whose registers leave room for four accumulators only): lane l holds
// channel (l & 15) >> 1, part p = l & 1; steps go in pairs, lane part p
// loads X at the harmonic of step 2u + p and rotates it on its own phasor
// chain (the p chain of moment_tile16), keeps the part it feeds to B and
// trades the other with its partner (DPP quad_perm [1,0,3,2]).  B's columns
// are (channel, Re W) and (channel, Im W): the even-row MFMA's Re columns and
// the odd-row MFMA's Im columns are the compact moments.  Powers are formed
// inline in the table's order, and every kept element sees the operands of
// moment_tile16: bitwise the same moments.  DSP: as moment_tile16's.
template <int U, bool DSP>
__device__ __forceinline__ void moment_tile8(const FitArgs& a, int c, int slot, int n, bool ok,
                                             double phic) {
  static_assert(kMT == 32, "two 16-row MFMA tiles");
  static_assert(U % 2 == 0, "steps go in pairs");
  constexpr int UP = U / 2;
  const int lane = threadIdx.x & 63;
  const int N = a.nbin / 2;
  const int nblk = ((N + 1 + 3) / 4 + U - 1) / U;
  const int col = lane & 15, part = col & 1, kk = lane >> 4;
  const size_t xrow = ((size_t)c * a.nchan + (ok ? n : 0)) * a.NHP;
  const double2* __restrict__ Xr = (DSP ? a.Dsp : a.X) + xrow;
  const double2* __restrict__ Mr = nullptr;
  if constexpr (DSP) {
    const int s = a.sub0 + c;
    const int midx = a.model_idx ? a.model_idx[s] : 0;
    Mr = a.M + ((size_t)midx * a.nchan + (ok ? n : 0)) * a.NHP;
  }
  // X_k of this lane (0 for k past N and idle lanes)
  auto xget = [&](bool on, int k) {
    if constexpr (DSP) return (on && k >= 1 && k <= N) ? cmulc(Xr[k], Mr[k]) : cmk(0.0, 0.0);
    else return (on && k <= N) ? Xr[k] : cmk(0.0, 0.0);
  };
  const double2 s8 = turn_phasor(8.0, phic);
  const double iN = 2.0 / (double)a.nbin;  // as k_vpow's
  f64x4 d0 = {0.0, 0.0, 0.0, 0.0}, d1 = d0, d2 = d0, d3 = d0;
  double2 xb[UP];
#pragma unroll
  for (int u = 0; u < UP; ++u) {
    const int k = 4 * (2 * u + part) + kk;
    xb[u] = xget(ok, k);
  }
  double2 e = cmk(1.0, 0.0);
  for (int b = 0; b < nblk; ++b) {
    const bool more = b + 1 < nblk;
    if ((b * U) % kMomReseedSteps == 0) e = turn_phasor((double)(4 * (b * U + part) + kk), phic);
#pragma unroll
    for (int u = 0; u < UP; ++u) {
      const double2 W = cmul(xb[u], e);
      const double recv = dpp_mov<0xB1>(part ? W.x : W.y);
      const double bv0 = part ? recv : W.x;  // step 2u: part p of the even harmonic
      const double bv1 = part ? W.y : recv;  // step 2u + 1
      const double2 p0 = vpow_inline(4 * (b * U + 2 * u) + kk, iN, col);
      const double2 p1 = vpow_inline(4 * (b * U + 2 * u + 1) + kk, iN, col);
      d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(p0.x, bv0, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(p0.y, bv0, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f64_16x16x4f64(p1.x, bv1, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f64_16x16x4f64(p1.y, bv1, d3, 0, 0, 0);
      e = cmul(e, s8);
      const int k = 4 * ((b + 1) * U + 2 * u + part) + kk;
      xb[u] = xget(more && ok, k);
    }
  }
  d0 += d2;
  d1 += d3;
  // D[row i = (l >> 4) + 4 r][col = l & 15]: the Re lanes (part 0) keep the
  // even moment 2 i from d0, the Im lanes (part 1) the odd one 2 i + 1 from d1
  if (ok) {
    double* Tn = a.T + (((size_t)c * 2 + slot) * a.nchan + n) * kMT;
#pragma unroll
    for (int r = 0; r < 4; ++r) Tn[2 * (kk + 4 * r) + part] = part ? d1[r] : d0[r];
  }
}

// All fitted channels of subint c, all threads of the block (recentring).
template <bool DSP>
__device__ void moments_from_X(const FitArgs& a, const Meta& m, int c, int s, int slot,
                               const double* xc, const double* refs, double P) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int chl = (lane & 15) >> 1;
  for (int t = w; t * 8 < m.nok; t += kWaves) {
    const int j = t * 8 + chl;
    const bool ok = j < m.nok;
    moment_tile8<DSP ? 4 : 8, DSP>(a, c, slot, ok ? m.chan[j] : 0, ok,
                    ok ? phase_frac(xc, m.fr[j], refs, P) : 0.0);
  }
}

// ---------------------------------------------------------------------------
// k_moments: the first moment pass of every phase-family subint, about its
// start point st.xc[0] (k_guess), into T slot 0 -- a pure stream over X at
// full occupancy.  Block (c, y): wave w takes channels 16 (4 y + w) .. + 15
// (masked channels idle in their lane).
// ---------------------------------------------------------------------------
template <int U, bool DSP>
__global__ __launch_bounds__(kBlock, 3) void k_moments(FitArgs a) {
  const int c = blockIdx.x, s = a.sub0 + c;
  if (!fused_taylor(a, s)) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n0 = 16 * (kWaves * (int)blockIdx.y + w);
  if (n0 >= a.nchan) return;  // whole wave
  const SolveState& st = a.st[c];
  const int n = n0 + (lane & 15);
  const bool ok = n < a.nchan && (!a.mask || a.mask[(size_t)s * a.nchan + n]);
  const double phic = ok ? phase_frac(st.xc[0], a.freqs[(size_t)s * a.nchan + n], st.refs, a.P[s])
                         : 0.0;
  moment_tile16<U, DSP>(a, c, 0, n, ok, phic);
}

template __global__ void k_moments<4, false>(FitArgs);
template __global__ void k_moments<4, true>(FitArgs);

// ---------------------------------------------------------------------------
// k_fit_taylor: one workgroup per phase-family subint, the whole fit:
//   guess_subint (get_TOAs initial phase, pptoas.py:420-456)
//   moments_from_X about the start point
//   scipy trust-ncg (k_solve<false>'s control flow, same nfev / status) with
//     every evaluation a Taylor series; a proposal outside the radius of
//     both stored centres gets its own centre (one more pass over X) first
//   post_subint<false> (nu_zero, outputs at nu_out, with-scales covariance)
// ---------------------------------------------------------------------------
struct TaylorShared {
  double x[5], xp[5];
  double xc[2][5];  // the two centres (st.xc), read by every sweep
  double out[48];
  double red[kWaves][48];
  double ifact[kMT];  // c_inv_fact for taylor_cells
  int done, nok, slot, tslot, q, mvalid;
  int same;  // the proposal repeats the last evaluated point (same_point8)
  // wave 0's solver state between its steps (per lane: gradient, point, last
  // evaluated point, step and Hessian row; uniform scalars once): parked here
  // across the sweeps every wave runs, so that those registers serve the
  // sweeps instead of spilling them
  double sv_g[64], sv_xl[64], sv_xe[64], sv_pl[64], sv_H[5][64];
  double sv_f, sv_tr, sv_predv;
  int sv_hits, sv_k, sv_status, sv_nfev;
};

// Moments [0, a.tnl) of T slot 0 of subint c into the kernel's LDS copy
// [nchan][tnl] (all threads; the caller syncs), kU loads in flight per thread.
__device__ __forceinline__ void stage_T0(const FitArgs& a, int c, double* tl) {
  const double* __restrict__ src = a.T + (size_t)c * 2 * a.nchan * kMT;
  const int nl = a.tnl;
  const int n = a.nchan * nl;
  constexpr int kU = 8;
  for (int i0 = 0; i0 < n; i0 += kBlock * kU) {
    double v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * kBlock + (int)threadIdx.x;
      const int ch = i / nl;
      v[u] = i < n ? src[(size_t)ch * kMT + (i - ch * nl)] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * kBlock + (int)threadIdx.x;
      if (i < n) tl[i] = v[u];
    }
  }
}

// taylor_reach for one wave (every lane gets it): the largest |y_n| over the
// fitted channels for evaluating (p0, p1, p2) from centre xc, refs = nu_fit.
__device__ __forceinline__ double wave_reach(const Meta& m, double p0, double p1, double p2,
                                             const double* xc, double Ks) {
  const double prm[3] = {p0, p1, p2};
  double mx = 0.0;
  for (int j = (int)threadIdx.x & 63; j < m.nok; j += 64)
    mx = fmax(mx, fabs(taylor_delta_lin(prm, xc, m.d1[j], m.d2[j])));
  return kTwoPi * Ks * wave_max(mx);
}


// MOM: the first moment pass (k_moments' tiles, wave w taking channels
// 16 (w + 4 t) .. + 15) runs at the top of this kernel instead of in its own
// launch, so that a CU's workgroups interleave the streaming moment pass of
// one subint with the latency-bound trust-region iterations of another
// (measured: 9.26 -> 9.03 ms per headline step; fusing the post-fit too
// spilled 784 B per lane and was slower, 10.0 ms).
template <bool MOM, bool DSP, bool WIDE>
__global__ __launch_bounds__(kBlock, 3) void k_fit_taylor(FitArgs a) {
  extern __shared__ __align__(16) unsigned char dyn[];
  __shared__ TaylorShared sh;
  __shared__ double refs[3];
  const int c = blockIdx.x, s = a.sub0 + c, tid = threadIdx.x;
  const int lane = tid & 63;
  if (!fused_taylor(a, s)) return;
  // diagnostic phase clock (ppf_phase_profile): thread 0 adds each phase's
  // time straight into ptime; the clock itself is wave-uniform (scalar
  // registers), so nothing of the profiler stays live in vector registers
  const bool prof = a.ptime != nullptr;
  unsigned long long t0 = prof ? wall_clock64() : 0ull;
  auto mark = [&](int i) {
    if (prof) {
      const unsigned long long t1 = wall_clock64();
      if (tid == 0) atomicAdd(&a.ptime[i], t1 - t0);
      t0 = t1;
    }
  };
  if constexpr (MOM) {
    const SolveState& st0 = a.st[c];
    const int w = tid >> 6;
    for (int t = w; 16 * t < a.nchan; t += kWaves) {
      const int n = 16 * t + (lane & 15);
      const bool ok = n < a.nchan && (!a.mask || a.mask[(size_t)s * a.nchan + n]);
      const double phic =
          ok ? phase_frac(st0.xc[0], a.freqs[(size_t)s * a.nchan + n], st0.refs, a.P[s]) : 0.0;
      moment_tile16<DSP ? PPF_DSP_U : PPF_MOM_U, DSP>(a, c, 0, n, ok, phic);
    }
    // T slot 0 is read back below by other waves of this workgroup
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  mark(0);  // slot 0: the fused first moment pass
  unsigned char* dmeta = chan_tables<WIDE>(a, dyn);
  SolveState& st = a.st[c];
  // T slot 0 (k_moments) read once into LDS: every sweep about centre 0 then
  // reads LDS instead of HBM.  load_meta's barrier publishes it.
  double* tl = a.tlds ? reinterpret_cast<double*>(dyn + a.tlds) : nullptr;
  if (tl) stage_T0(a, c, tl);
  const Meta m = load_meta(a, c, s, dmeta, &sh.nok);
  const double P = a.P[s];
  const double Ks = 0.5 * (double)a.nbin;
  if (tid < 5) sh.x[tid] = st.x[tid];
  if (tid < 5) sh.xc[0][tid] = st.xc[0][tid];
  if (tid < 3) refs[tid] = st.refs[tid];
  if (tid < kMT) sh.ifact[tid] = c_inv_fact[tid];
  if (tid == 0) {
    sh.done = (m.nok == 0);
    sh.slot = 0;
    sh.tslot = 0;
    sh.mvalid = 1;
    st.mvalid = 1;  // slot 0: k_moments, about st.xc[0]
  }
  __syncthreads();
  mark(1);
  double* acc0 = a.acc + (size_t)c * 2 * a.nchan * NACC;
  // wave-0 solver state (lane i < 5 owns component i; scalars are uniform)
  double f = 0.0, g = 0.0, xl = 0.0, Hrow[5] = {0, 0, 0, 0, 0};
  double tr = 1.0, predv = 0.0, pl = 0.0;
  int hits = 0, k = 0, status = (m.nok == 0) ? -1 : 0, nfev = 0;
  double xe = 0.0;  // lane i < 5: the last evaluated point
  auto save = [&] {  // wave 0
    sh.sv_g[lane] = g;
    sh.sv_xl[lane] = xl;
    sh.sv_xe[lane] = xe;
    sh.sv_pl[lane] = pl;
#pragma unroll
    for (int j = 0; j < 5; ++j) sh.sv_H[j][lane] = Hrow[j];
    if (lane == 0) {
      sh.sv_f = f;
      sh.sv_tr = tr;
      sh.sv_predv = predv;
      sh.sv_hits = hits;
      sh.sv_k = k;
      sh.sv_status = status;
      sh.sv_nfev = nfev;
    }
  };
  auto restore = [&] {  // wave 0, after the barrier that follows its save
    g = sh.sv_g[lane];
    xl = sh.sv_xl[lane];
    xe = sh.sv_xe[lane];
    pl = sh.sv_pl[lane];
#pragma unroll
    for (int j = 0; j < 5; ++j) Hrow[j] = sh.sv_H[j][lane];
    f = sh.sv_f;
    tr = sh.sv_tr;
    predv = sh.sv_predv;
    hits = sh.sv_hits;
    k = sh.sv_k;
    status = sh.sv_status;
    nfev = sh.sv_nfev;
  };
  if (tid < 64) save();
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
  // the stored centre nearest p within reach (taylor_reach <= kTaylorY, the
  // first of equals), or -1; wave 0 only, no barrier
  auto pick = [&](double p0, double p1, double p2) -> int {
    int best = -1;
    double by = INFINITY;
    for (int q = 0; q < 2; ++q) {
      if (!(sh.mvalid & (1 << q))) continue;
      const double y = wave_reach(m, p0, p1, p2, sh.xc[q], Ks);
      if (y <= kTaylorY && y < by) { by = y; best = q; }
    }
    return best;
  };
  auto source = [&](int q) {
    const bool l = q == 0 && tl;
    return TaylorSrc{a.T + ((size_t)c * 2 + q) * a.nchan * kMT, sh.xc[q], refs, true, sh.ifact,
                     l ? tl : nullptr, l ? a.tnl : 0};
  };
  // no stored centre covers p: p itself becomes one (one more X pass)
  auto recentre = [&](const double* p) -> int {
    const int wsl = sh.tslot ^ 1;
    if (prof && tid == 0) atomicAdd(&a.ptime[8], 1ull);  // recentres
    if (tid == 0) {
      st.mvalid &= ~(1 << wsl);
      sh.mvalid = st.mvalid;
      for (int i = 0; i < 5; ++i) st.xc[wsl][i] = p[i];
    }
    if (tid < 5) sh.xc[wsl][tid] = p[tid];
    __syncthreads();
    moments_from_X<DSP>(a, m, c, s, wsl, sh.xc[wsl], refs, P);
    __syncthreads();
    if (wsl == 0 && tl) stage_T0(a, c, tl);
    if (tid == 0) {
      st.mvalid |= 1 << wsl;
      sh.mvalid = st.mvalid;
    }
    __syncthreads();
    if (tid < 64) {
      const int q = pick(p[0], p[1], p[2]);
      if (lane == 0) sh.q = q;
    }
    __syncthreads();
    return sh.q;  // p is that centre: |y| = 0
  };
  if (!sh.done) {
    if (tid < 64) {
      const int q0 = pick(sh.x[0], sh.x[1], sh.x[2]);
      if (lane == 0) sh.q = q0;
    }
    __syncthreads();
    int q = sh.q;
    if (q < 0) q = recentre(sh.x);
    mark(2);
    sweep<0, false>(a, m, c, s, sh.x, refs, P, acc0, sh.out, sh.red, source(q));
    mark(3);
    if (tid < 64) {
      load_fgh(f, g, Hrow);
      xl = lane < 5 ? sh.x[lane] : 0.0;
      xe = xl;
      nfev = 1;
      trace_sweep(a, s, 0, sh.x, sh.out, 21, true);
      if (a.solver_flags & PPF_SOLVE_EVAL) {  // objective at init only
        status = 1;
        if (lane == 0) sh.done = 1;
      }
      save();
    }
    if (tid == 0) sh.tslot = q;
  }
  __syncthreads();
  while (!sh.done) {
    if (tid < 64) {
      restore();
      const double jm = sqrt(dot8(g, g));
      if (!(jm >= -1.0)) {  // NaN gradient: scipy's loop condition fails
        status = 0;
        if (lane == 0) sh.done = 1;
      } else {
        pl = steihaug(f, g, Hrow, tr, hits);
        predv = model_val(f, g, Hrow, pl);
        const double pv = xl + pl;  // lane i < 5: component i of the proposal
        if (lane < 5) sh.xp[lane] = pv;
        const bool same = same_point8(lane, pv, xe);
        const int qp = same ? sh.q : pick(__shfl(pv, 0), __shfl(pv, 1), __shfl(pv, 2));
        if (lane == 0) {
          sh.q = qp;
          sh.same = same;
        }
      }
      save();
    }
    __syncthreads();
    mark(4);
    if (sh.done) break;
    // a repeat of the last evaluated point reuses its sweep (sh.out, the
    // accumulator half and the centre are still its own)
    const bool fresh = !sh.same;
    int q = sh.q;
    if (fresh && q < 0) q = recentre(sh.xp);
    mark(2);
    double* sl = acc0 + (size_t)(sh.slot ^ 1) * a.nchan * NACC;
    if (fresh) sweep<0, false>(a, m, c, s, sh.xp, refs, P, sl, sh.out, sh.red, source(q));
    mark(3);
    if (tid < 64) {
      restore();
      double fp, gp, Hp[5] = {0, 0, 0, 0, 0};
      load_fgh(fp, gp, Hp);
      if (fresh) {
        nfev += 1;
        xe = xl + pl;
        trace_sweep(a, s, nfev - 1, sh.xp, sh.out, 21, true);
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
          if (lane == 0) { sh.slot ^= 1; sh.tslot = q; }
          if (lane < 5) sh.x[lane] = xl;
        }
        k += 1;
        if (k >= 1000) {
          status = 1;
          if (lane == 0) sh.done = 1;
        }
      }
      save();
    }
    __syncthreads();
  }
  if (tid < 64) restore();
  if (tid < 5) st.x[tid] = sh.x[tid];
  if (tid < 5) store_grad_hess(a, s, lane, m.nok > 0, g, Hrow);
  if (tid == 0) {
    st.fun = m.nok ? f : NAN;
    st.nfev = m.nok ? nfev : 0;
    st.status = status;
    st.slot = sh.slot;
    st.xslot = sh.tslot;
    st.fin = 1;
    st.scat_post = false;
    if (prof) atomicAdd(&a.ptime[9], 1ull);
  }
}

template __global__ void k_fit_taylor<false, false>(FitArgs);
template __global__ void k_fit_taylor<true, false>(FitArgs);
template __global__ void k_fit_taylor<false, true>(FitArgs);
template __global__ void k_fit_taylor<true, true>(FitArgs);
template __global__ void k_fit_taylor<false, false, true>(FitArgs);
template __global__ void k_fit_taylor<true, false, true>(FitArgs);
template __global__ void k_fit_taylor<false, true, true>(FitArgs);
template __global__ void k_fit_taylor<true, true, true>(FitArgs);

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
  // v_mfma_f64_16x16x4: A[i][k] = i + 1 + 16 k, B[k][j] = 2 j + 3 k + 1
  {
    const int i = l & 15, kq = l >> 4;
    f64x4 d = {0.0, 0.0, 0.0, 0.0};
    d = __builtin_amdgcn_mfma_f64_16x16x4f64((double)(i + 1 + 16 * kq),
                                             (double)(2 * i + 3 * kq + 1), d, 0, 0, 0);
    bool ok = true;
    for (int r = 0; r < 4; ++r) {
      const int row = kq + 4 * r;
      double ref = 0.0;
      for (int q = 0; q < 4; ++q) ref += (double)(row + 1 + 16 * q) * (double)(2 * i + 3 * q + 1);
      ok = ok && d[r] == ref;
    }
    chk(9, ok);
  }
}


}  // namespace ppf
