// ppfit_device.hpp -- device-side building blocks for libppfit (gfx950).
//
// Complex fp64 helpers, 64-lane wave reductions, a Philox4x32-10 counter RNG
// and the LDS-resident Stockham FFT used for every real<->complex transform
// on the hot path (numpy.fft.rfft / irfft in the reference: pplib.py:27).
#pragma once

#ifndef PPF_NT
// streaming (non-temporal) hint on the data pass's read-once portrait rows:
// with the write-once X stores, 5.57 -> 5.04 ms at config 2 (r02; the moment
// pass's X loads were slower with the hint and stay plain).  r04: the stores
// are plain again (PPF_NT_ST below); on the loads the hint is worth 0.15-0.27
// ms of the config-5 data pass (256-channel template blocks stay in L2) and
// is within box-to-box noise at config 2
#define PPF_NT 1
#endif
#ifndef PPF_EARLY_ROW
// wave-per-row streams (data pass, ppalign's rotate-and-sum) start the next
// row's load inside the register FFT, right after stage A (A/B knob)
#define PPF_EARLY_ROW 1
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

namespace ppf {

// Compile-time loop: f(std::integral_constant<int, i>) for i in [0, N), so
// register arrays indexed by i stay in registers.
template <int I, int N, class F>
__device__ __forceinline__ void static_for_impl(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for_impl<I + 1, N>(f);
  }
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) { static_for_impl<0, N>(f); }

// pplib.py:48-51: Dconst = 0.000241**-1 (bit-identical double)
constexpr double kDconst = 0x1.03560a9f560aap+12;
constexpr double kPi = 3.141592653589793116;
constexpr double kLn10 = 0x1.26bb1bbb55516p+1;
constexpr int kBlock = 256;   // threads per workgroup (4 waves)
constexpr int kWaves = kBlock / 64;

__device__ __forceinline__ double2 cmk(double x, double y) { return make_double2(x, y); }
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return cmk(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return cmk(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cscale(double2 a, double s) { return cmk(a.x * s, a.y * s); }
__device__ __forceinline__ double2 cconj(double2 a) { return cmk(a.x, -a.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return cmk(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
// a * conj(b)
__device__ __forceinline__ double2 cmulc(double2 a, double2 b) {
  return cmk(fma(a.x, b.x, a.y * b.y), fma(a.y, b.x, -a.x * b.y));
}
__device__ __forceinline__ double cabs2(double2 a) { return fma(a.x, a.x, a.y * a.y); }

// e^{2 pi i k phi} with the argument reduced exactly: k*phi is split into
// its rounded product and the FMA remainder, the integer part is dropped, and
// sincospi evaluates the fractional turn (no large-argument rounding, unlike
// exp(2j*pi*outer(phi,k)) in pptoaslib.py:237, which is within 1e-11 of this).
__device__ __forceinline__ double2 turn_phasor(double k, double phi) {
  double t = k * phi;
  double e = fma(k, phi, -t);
  double r = (t - rint(t)) + e;
  double s, c;
  sincospi(2.0 * r, &s, &c);
  return cmk(c, s);
}

// Cross-lane moves without the LDS crossbar: DPP within 16-lane rows and
// v_permlane16/32_swap across rows (gfx950), each on the two dwords of a double.
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
  const unsigned long long u = __double_as_longlong(v);
  // bound_ctrl: a lane whose source is out of the row reads 0 (row_shr);
  // every lane is written, so no old value has to be materialised first
  const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)u, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// value of the lane in the other 16-lane row of the pair (O = 16) / other half-wave (O = 32)
template <int O>
__device__ __forceinline__ double swap_rows(double v) {
  const unsigned long long u = __double_as_longlong(v);
  unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
  if constexpr (O == 16) {
    const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    // lanes of even rows receive in [1], odd rows in [0]
    const bool odd = (threadIdx.x & 16) != 0;
    lo = odd ? a[0] : a[1];
    hi = odd ? b[0] : b[1];
  } else {
    const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const bool up = (threadIdx.x & 32) != 0;
    lo = up ? a[0] : a[1];
    hi = up ? b[0] : b[1];
  }
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Sum over the 8 lanes that share (lane >> 3): quad xor 1, xor 2, then the
// half-row mirror pairs the two quads.  Every lane of the 8 gets the sum.
__device__ __forceinline__ double group8_sum(double v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  return v;
}

// Sum over the wave; every lane gets it.
__device__ __forceinline__ double wave_sum(double v) {
  v = group8_sum(v);
  v += dpp_mov<0x140>(v);  // row_mirror: the two 8-lane halves of a row
  v += swap_rows<16>(v);
  v += swap_rows<32>(v);
  return v;
}

// wave_sum of a value held only by the lanes with (lane & 7) == 0 (zero on
// the rest), without the group8_sum stage that only adds those zeros: row_shr
// 8 pairs the row's two holders, then the row and half-wave swaps.  Every
// addition meets the same two operands as in wave_sum (in commuted order),
// so the result is bitwise wave_sum's; it is valid on lanes (lane & 15) == 8.
__device__ __forceinline__ double chan8_sum(double v) {
  v += dpp_mov<0x118>(v);  // row_shr:8 (lanes 0-7 of a row receive 0)
  v += swap_rows<16>(v);
  v += swap_rows<32>(v);
  return v;
}

// Max over the wave; every lane gets it.
__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, dpp_mov<0xB1>(v));
  v = fmax(v, dpp_mov<0x4E>(v));
  v = fmax(v, dpp_mov<0x141>(v));
  v = fmax(v, dpp_mov<0x140>(v));
  v = fmax(v, swap_rows<16>(v));
  v = fmax(v, swap_rows<32>(v));
  return v;
}

// Lane 0's value as a wave-uniform (scalar) double.
__device__ __forceinline__ double lane0(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Lane J's value, wave-uniform.
template <int J>
__device__ __forceinline__ double lane_at(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, J);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), J);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Lane j's value (j wave-uniform, known at run time), wave-uniform.
__device__ __forceinline__ double lane_of(double v, int j) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, j);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), j);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Block-wide sum; `red` is >= kWaves doubles of LDS.  Every thread gets it.
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) s += red[i];
  __syncthreads();
  return s;
}

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. 2011): counter-based, so CPU and GPU can
// regenerate identical uniform streams for the synthetic inputs.
// ---------------------------------------------------------------------------
struct u32x4 { uint32_t v[4]; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c.v[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c.v[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    u32x4 n;
    n.v[0] = hi1 ^ c.v[1] ^ k0;
    n.v[1] = lo1;
    n.v[2] = hi0 ^ c.v[3] ^ k1;
    n.v[3] = lo0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Two N(0,1) deviates (Box-Muller) from one Philox block.
__device__ __forceinline__ double2 philox_normal2(u32x4 c, uint64_t seed) {
  u32x4 x = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const double inv53 = 1.1102230246251565404e-16;  // 2^-53
  double u1 = ((double)(x.v[0] >> 5) * 67108864.0 + (double)(x.v[1] >> 6) + 0.5) * inv53;
  double u2 = ((double)(x.v[2] >> 5) * 67108864.0 + (double)(x.v[3] >> 6)) * inv53;
  double r = sqrt(-2.0 * log(u1));
  double s, co;
  sincospi(2.0 * u2, &s, &co);
  return cmk(r * co, r * s);
}

// ---------------------------------------------------------------------------
// LDS Stockham autosort FFT of N = 2^LOGN complex points, all kBlock threads.
// tw[m] = exp(-2 pi i m / (2N)), m in [0, 2N), built by k_twiddles.
// Forward uses exp(-i...), INV the conjugate (unnormalised both ways).
// Radix-2 first pass when LOGN is odd, then radix-4 passes.
// ---------------------------------------------------------------------------
template <bool INV>
__device__ __forceinline__ void radix4(double2& a0, double2& a1, double2& a2, double2& a3) {
  double2 t0 = cadd(a0, a2), t1 = csub(a0, a2);
  double2 t2 = cadd(a1, a3), d = csub(a1, a3);
  double2 t3 = INV ? cmk(-d.y, d.x) : cmk(d.y, -d.x);  // (+/-i)(a1-a3)
  a0 = cadd(t0, t2);
  a1 = cadd(t1, t3);
  a2 = csub(t0, t2);
  a3 = csub(t1, t3);
}

template <int LOGN, bool INV>
__device__ void lds_fft(double2* buf, const double2* __restrict__ tw) {
  constexpr int N = 1 << LOGN;
  constexpr int Q = N / 4;
  constexpr int B4 = (Q + kBlock - 1) / kBlock;
  const int tid = threadIdx.x;
  int Ns = 1;
  if constexpr (LOGN & 1) {
    constexpr int H = N / 2;
    constexpr int B2 = (H + kBlock - 1) / kBlock;
    double2 a[B2], b[B2];
#pragma unroll
    for (int c = 0; c < B2; ++c) {
      const int j = tid + c * kBlock;
      if (j < H) { a[c] = buf[j]; b[c] = buf[j + H]; }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < B2; ++c) {
      const int j = tid + c * kBlock;
      if (j < H) { buf[2 * j] = cadd(a[c], b[c]); buf[2 * j + 1] = csub(a[c], b[c]); }
    }
    __syncthreads();
    Ns = 2;
  }
#pragma unroll
  for (int p = 0; p < LOGN / 2; ++p) {
    double2 v[B4][4];
#pragma unroll
    for (int c = 0; c < B4; ++c) {
      const int j = tid + c * kBlock;
      if (j < Q) {
        const int k = j & (Ns - 1);
        const int tstep = 2 * k * (N / (4 * Ns));
        v[c][0] = buf[j];
#pragma unroll
        for (int r = 1; r < 4; ++r) {
          double2 w = tw[r * tstep];
          if (INV) w.y = -w.y;
          v[c][r] = cmul(buf[j + r * Q], w);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < B4; ++c) {
      const int j = tid + c * kBlock;
      if (j < Q) {
        radix4<INV>(v[c][0], v[c][1], v[c][2], v[c][3]);
        const int k = j & (Ns - 1);
        const int d = (j - k) * 4 + k;
        buf[d] = v[c][0];
        buf[d + Ns] = v[c][1];
        buf[d + 2 * Ns] = v[c][2];
        buf[d + 3 * Ns] = v[c][3];
      }
    }
    __syncthreads();
    Ns *= 4;
  }
}

// Sync for the threads that share an LDS FFT buffer: the whole block, or one
// wave (LDS operations of a wave execute in order; the wave barrier and the
// fences only stop the compiler from moving LDS accesses across it).
template <bool WAVE>
__device__ __forceinline__ void fft_sync() {
  if constexpr (WAVE) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// Forward Stockham FFT of N = 2^LOGN points in buf by NT threads (t = 0..NT-1),
// twiddles from an LDS table twl[e] = e^{-2 pi i e / N}, e < 3N/4 (radix-4
// pass with span Ns needs exponents r k N / (4 Ns) < 3N/4).  WAVE: NT = 64
// and buf is private to the calling wave.
template <int LOGN, int NT, bool WAVE>
__device__ __forceinline__ void stockham_twl(double2* buf, const double2* twl, int t) {
  constexpr int N = 1 << LOGN;
  constexpr int Q = N / 4;
  constexpr int B4 = (Q + NT - 1) / NT;
  int Ns = 1;
  if constexpr (LOGN & 1) {
    constexpr int H = N / 2;
    constexpr int B2 = (H + NT - 1) / NT;
    double2 a[B2], b[B2];
#pragma unroll
    for (int c = 0; c < B2; ++c) {
      const int j = t + c * NT;
      if (j < H) { a[c] = buf[j]; b[c] = buf[j + H]; }
    }
    fft_sync<WAVE>();
#pragma unroll
    for (int c = 0; c < B2; ++c) {
      const int j = t + c * NT;
      if (j < H) { buf[2 * j] = cadd(a[c], b[c]); buf[2 * j + 1] = csub(a[c], b[c]); }
    }
    fft_sync<WAVE>();
    Ns = 2;
  }
#pragma unroll
  for (int p = 0; p < LOGN / 2; ++p) {
    double2 v[B4][4];
#pragma unroll
    for (int c = 0; c < B4; ++c) {
      const int j = t + c * NT;
      if (j < Q) {
        const int k = j & (Ns - 1);
        const int e = k * (N / (4 * Ns));
        v[c][0] = buf[j];
#pragma unroll
        for (int r = 1; r < 4; ++r) v[c][r] = cmul(buf[j + r * Q], twl[r * e]);
      }
    }
    fft_sync<WAVE>();
#pragma unroll
    for (int c = 0; c < B4; ++c) {
      const int j = t + c * NT;
      if (j < Q) {
        radix4<false>(v[c][0], v[c][1], v[c][2], v[c][3]);
        const int k = j & (Ns - 1);
        const int d = (j - k) * 4 + k;
        buf[d] = v[c][0];
        buf[d + Ns] = v[c][1];
        buf[d + 2 * Ns] = v[c][2];
        buf[d + 3 * Ns] = v[c][3];
      }
    }
    fft_sync<WAVE>();
    Ns *= 4;
  }
}

// Per-pass twiddle tables for the wave FFT.  A radix-4 pass of span Ns needs
// w^{r k}, w = e^{-2 pi i / (4 Ns)}, k < Ns, r = 1..3.  Read from one table of
// e^{-2 pi i e / N} they sit N / (4 Ns) entries apart, so the lanes of a pass
// hit one LDS bank (up to 16-way conflicts); here each pass has its own
// contiguous rows [r = 1][k], [r = 2][k] and w^{3k} = w^k w^{2k}.
template <int LOGN>
struct PassTw {
  static constexpr int NP = LOGN / 2;                 // radix-4 passes
  static constexpr int NS0 = (LOGN & 1) ? 2 : 1;      // span of the first one
  static constexpr int span(int p) { return NS0 << (2 * p); }
  static constexpr int off(int p) { return p == 0 ? 0 : off(p - 1) + 2 * span(p - 1); }
  static constexpr int SIZE = off(NP);
};

// tpt[off(p) + (r-1) Ns + k] = e^{-2 pi i r k / (4 Ns)} from tw[m] = e^{-2 pi i m / (2N)}
template <int LOGN>
__device__ __forceinline__ void fill_pass_tw(double2* tpt, const double2* __restrict__ tw, int t,
                                             int nt) {
  using T = PassTw<LOGN>;
  constexpr int N = 1 << LOGN;
  for (int e = t; e < T::SIZE; e += nt) {
    int p = 0;
    while (p + 1 < T::NP && e >= T::off(p + 1)) ++p;
    const int Ns = T::span(p);
    const int q = e - T::off(p);
    const int r = 1 + q / Ns, k = q % Ns;
    tpt[e] = tw[r * k * (N / (2 * Ns))];
  }
}

// Wave-synchronous forward Stockham FFT (64 lanes) with per-pass twiddles.
template <int LOGN>
__device__ __forceinline__ void wave_fft(double2* buf, const double2* tpt, int t) {
  using T = PassTw<LOGN>;
  constexpr int N = 1 << LOGN;
  constexpr int NT = 64;
  constexpr int Q = N / 4;
  constexpr int B4 = (Q + NT - 1) / NT;
  if constexpr (LOGN & 1) {
    constexpr int H = N / 2;
    constexpr int B2 = (H + NT - 1) / NT;
    double2 a[B2], b[B2];
#pragma unroll
    for (int c = 0; c < B2; ++c) {
      const int j = t + c * NT;
      if (j < H) { a[c] = buf[j]; b[c] = buf[j + H]; }
    }
    fft_sync<true>();
#pragma unroll
    for (int c = 0; c < B2; ++c) {
      const int j = t + c * NT;
      if (j < H) { buf[2 * j] = cadd(a[c], b[c]); buf[2 * j + 1] = csub(a[c], b[c]); }
    }
    fft_sync<true>();
  }
#pragma unroll
  for (int p = 0; p < T::NP; ++p) {
    const int Ns = T::span(p);
    const double2* tp = tpt + T::off(p);
    double2 v[B4][4];
#pragma unroll
    for (int c = 0; c < B4; ++c) {
      const int j = t + c * NT;
      if (j < Q) {
        const int k = j & (Ns - 1);
        v[c][0] = buf[j];
        if (Ns == 1) {
#pragma unroll
          for (int r = 1; r < 4; ++r) v[c][r] = buf[j + r * Q];
        } else {
          const double2 w1 = tp[k], w2 = tp[Ns + k];
          v[c][1] = cmul(buf[j + Q], w1);
          v[c][2] = cmul(buf[j + 2 * Q], w2);
          v[c][3] = cmul(buf[j + 3 * Q], cmul(w1, w2));
        }
      }
    }
    fft_sync<true>();
#pragma unroll
    for (int c = 0; c < B4; ++c) {
      const int j = t + c * NT;
      if (j < Q) {
        radix4<false>(v[c][0], v[c][1], v[c][2], v[c][3]);
        const int k = j & (Ns - 1);
        const int d = (j - k) * 4 + k;
        buf[d] = v[c][0];
        buf[d + Ns] = v[c][1];
        buf[d + 2 * Ns] = v[c][2];
        buf[d + 3 * Ns] = v[c][3];
      }
    }
    fft_sync<true>();
  }
}

// Block-wide forward FFT with LDS twiddles (all kBlock threads).
template <int LOGN>
__device__ __forceinline__ void lds_fft_twl(double2* buf, const double2* twl) {
  stockham_twl<LOGN, kBlock, false>(buf, twl, threadIdx.x);
}

// rfft_post with the twiddle e^{-2 pi i k / 2N} passed in (a register).
template <int LOGN>
__device__ __forceinline__ double2 rfft_post_w(const double2* buf, int k, double2 w) {
  constexpr int N = 1 << LOGN;
  const double2 zk = buf[k & (N - 1)];
  const double2 zc = cconj(buf[(N - k) & (N - 1)]);
  const double2 e = cscale(cadd(zk, zc), 0.5);
  const double2 dd = csub(zk, zc);
  const double2 o = cmk(0.5 * dd.y, -0.5 * dd.x);
  return cadd(e, cmul(w, o));
}

// Real-input spectrum X_k (k in [0, N]) of the 2N-point real row packed as
// buf[j] = (x_{2j}, x_{2j+1}) after a forward lds_fft (numpy rfft layout).
template <int LOGN>
__device__ __forceinline__ double2 rfft_post(const double2* buf, int k, const double2* __restrict__ tw) {
  constexpr int N = 1 << LOGN;
  const double2 zk = buf[k & (N - 1)];
  const double2 zc = cconj(buf[(N - k) & (N - 1)]);
  const double2 e = cscale(cadd(zk, zc), 0.5);
  const double2 dd = csub(zk, zc);
  const double2 o = cmk(0.5 * dd.y, -0.5 * dd.x);  // -i/2 (zk - zc)
  return cadd(e, cmul(tw[k], o));
}

// Packed spectrum Z_k (k in [0, N)) for the inverse: irfft(X) = (1/N) *
// unpack(IFFT_N(Z)).  Imaginary parts of X_0 and X_N are ignored (pocketfft c2r).
template <int LOGN>
__device__ __forceinline__ double2 irfft_pre(double2 xk, double2 xnk, int k, const double2* __restrict__ tw) {
  const double2 xc = cconj(xnk);
  const double2 e = cscale(cadd(xk, xc), 0.5);
  const double2 o = cmul(cscale(csub(xk, xc), 0.5), cconj(tw[k]));
  return cmk(e.x - o.y, e.y + o.x);  // e + i o
}

}  // namespace ppf

namespace ppf {

// Read-once / write-once rows: non-temporal when PPF_NT (streaming hint).
typedef double f64x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ld_stream(const double2* p) {
#if PPF_NT
  const f64x2v v = __builtin_nontemporal_load(reinterpret_cast<const f64x2v*>(p));
  return cmk(v.x, v.y);
#else
  return *p;
#endif
}
#ifndef PPF_NT_ST
// ... but the write-once X stores go through the caches: with the hint they
// measured 4.675 ms for the data pass, without it 4.556 ms (r04, same box;
// the moment pass that reads X back is unchanged within 1 %)
#define PPF_NT_ST 0
#endif
__device__ __forceinline__ void st_stream(double2 v, double2* p) {
#if PPF_NT_ST
  f64x2v w;
  w.x = v.x;
  w.y = v.y;
  __builtin_nontemporal_store(w, reinterpret_cast<f64x2v*>(p));
#else
  *p = v;
#endif
}

// ---------------------------------------------------------------------------
// Wave-per-row streaming (k_data_xspec, k_moments): each wave owns one LDS
// row buffer of N + 8 packed complex slots and walks its own channel list,
// so the channel loop has no workgroup barrier.  Rows of N <= 1024 points
// are prefetched into registers (16 doubles2 per lane) one channel ahead.
// ---------------------------------------------------------------------------
template <int LOGN>
struct WaveRow {
  static constexpr int N = 1 << LOGN;
  static constexpr int LI = N >= 64 ? N / 64 : 1;
  static constexpr bool kPrefetch = LOGN <= 10;
  static constexpr int PL = kPrefetch ? LI : 1;
  double x[PL], y[PL];
  // global -> registers (prefetch form)
  __device__ __forceinline__ void load(const double* __restrict__ src, int lane) {
    if constexpr (kPrefetch) {
      const double2* r2 = reinterpret_cast<const double2*>(src);
#pragma unroll
      for (int i = 0; i < LI; ++i) {
        const int j = lane + 64 * i;
        if (N >= 64 || j < N) {
          const double2 v = ld_stream(r2 + j);  // read once
          x[i] = v.x;
          y[i] = v.y;
        }
      }
    }
  }
  // registers -> LDS (prefetch form) or global -> LDS directly
  __device__ __forceinline__ void store(double2* buf, const double* __restrict__ src,
                                        int lane) const {
    if constexpr (kPrefetch) {
#pragma unroll
      for (int i = 0; i < LI; ++i) {
        const int j = lane + 64 * i;
        if (N >= 64 || j < N) buf[j] = cmk(x[i], y[i]);
      }
    } else {
      const double2* r2 = reinterpret_cast<const double2*>(src);
#pragma unroll 4
      for (int i = 0; i < LI; ++i) buf[lane + 64 * i] = r2[lane + 64 * i];
    }
  }
};

// Spectrum pair of a real 2N-point row from its packed forward FFT Z in buf
// (numpy rfft layout): for k in [0, N/2], w = e^{-i pi k / N},
//   X_k = E + w O,  X_{N-k} = conj(E - w O),
//   E = (Z_k + conj Z_{N-k}) / 2,  O = -i (Z_k - conj Z_{N-k}) / 2.
// (k = 0 gives X_0 and X_N from Z_0; at k = N/2 both are X_{N/2}.)
template <int LOGN>
__device__ __forceinline__ void rfft_pair(const double2* buf, int k, double2 w, double2& Xk,
                                          double2& Xnk) {
  constexpr int N = 1 << LOGN;
  const double2 zk = buf[k];
  const double2 zc = cconj(buf[(N - k) & (N - 1)]);
  const double2 E = cscale(cadd(zk, zc), 0.5);
  const double2 dd = csub(zk, zc);
  const double2 O = cmk(0.5 * dd.y, -0.5 * dd.x);
  const double2 P = cmul(w, O);
  Xk = cadd(E, P);
  Xnk = cconj(csub(E, P));
}

// Same, from the two packed values Z_k and Z_{(N-k) mod N} already loaded.
__device__ __forceinline__ void rfft_pair_v(double2 zk, double2 znk, double2 w, double2& Xk,
                                            double2& Xnk) {
  const double2 zc = cconj(znk);
  const double2 E = cscale(cadd(zk, zc), 0.5);
  const double2 dd = csub(zk, zc);
  const double2 O = cmk(0.5 * dd.y, -0.5 * dd.x);
  const double2 P = cmul(w, O);
  Xk = cadd(E, P);
  Xnk = cconj(csub(E, P));
}

// ---------------------------------------------------------------------------
// Register-resident 1024-point forward FFT of one packed row per wave
// (nbin = 2048, the headline shape).  N = 16 x 16 x 4:
//   A  lane j holds z[j + 64 m] (the coalesced row load), 16-point DFT over m
//      in registers, twiddle W_1024^{j r}, one LDS transpose;
//   B  lane (j0 = l & 3, r = l >> 2) takes Y_{j0 + 4 t}[r], 16-point DFT over
//      t in registers, twiddle W_64^{j0 s};
//   C  the twiddled values go through LDS once more (slot 64 s + 16 j0 +
//      (rr ^ 2 j0): conflict-free for the quad-strided writes and for the
//      reads), lane (rr = l & 15, q = l >> 4) takes the four j0 of s = 4 q + c
//      (c < 4) and does the 4-point DFTs over j0 in registers (radix4: the
//      -i is a component swap, no cross-lane moves or lane selects);
// then Z_k goes to LDS once, in the padded order P(k) = k + 4 (k >> 8) that
// keeps the writes (8 consecutive rr per group) and the (k, N - k) reads of
// the real-FFT post-processing free of bank conflicts.  Three LDS round trips
// per row instead of the Stockham path's six.  Twiddles are exact table
// values (W^{4a+b} = W^{4a} W^b: at most one rounding).  Stage C forms
// exactly the sums of the former DPP radix-2 pair (a0 + a2, a0 - a2, -i(a1 -
// a3), ...), so the spectrum is bitwise unchanged.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double2 mul_negi(double2 a) { return cmk(a.y, -a.x); }

// 16-point forward DFT in place; Y[c + 4 d] ends in v[4 c + d].
__device__ __forceinline__ void dft16(double2 (&v)[16]) {
  constexpr double C1 = 0.92387953251128675613, S1 = 0.38268343236508977173,
                   H = 0.70710678118654752440;
#pragma unroll
  for (int b = 0; b < 4; ++b) radix4<false>(v[b], v[4 + b], v[8 + b], v[12 + b]);
  v[5] = cmul(v[5], cmk(C1, -S1));
  v[9] = cmul(v[9], cmk(H, -H));
  v[13] = cmul(v[13], cmk(S1, -C1));
  v[6] = cmul(v[6], cmk(H, -H));
  v[10] = mul_negi(v[10]);
  v[14] = cmul(v[14], cmk(-H, -H));
  v[7] = cmul(v[7], cmk(S1, -C1));
  v[11] = cmul(v[11], cmk(-H, -H));
  v[15] = cmul(v[15], cmk(-C1, S1));
#pragma unroll
  for (int c = 0; c < 4; ++c) radix4<false>(v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]);
}
__device__ __forceinline__ constexpr int dft16_pos(int r) { return 4 * (r & 3) + (r >> 2); }

// Stage twiddles, one LDS table per workgroup (read per row, not held in
// registers across the channel loop).
struct Fft1024Tw {
  double2 a[3][64], b[3][64];  // W_1024^{j b}, W_1024^{4 j a}  (stage A, j = lane), b, a = 1..3
  double2 c[3][4], d[3][4];    // W_64^{j0 b}, W_64^{4 j0 a}    (stage B, j0 = lane & 3)
  // tw[m] = e^{-2 pi i m / 2048}
  __device__ __forceinline__ void fill(const double2* __restrict__ tw, int t, int nt) {
    for (int e = t; e < 3 * 64; e += nt) {
      const int i = 1 + e / 64, j = e % 64;
      a[i - 1][j] = tw[2 * j * i];
      b[i - 1][j] = tw[8 * j * i];
    }
    for (int e = t; e < 3 * 4; e += nt) {
      const int i = 1 + e / 4, j0 = e % 4;
      c[i - 1][j0] = tw[32 * j0 * i];
      d[i - 1][j0] = tw[128 * j0 * i];
    }
  }
};
__device__ __forceinline__ double2 tw_pow(int r, const double2 (&lo)[4], const double2 (&hi)[4]) {
  const int b = r & 3, a = r >> 2;
  if (a == 0) return lo[b];
  if (b == 0) return hi[a];
  return cmul(hi[a], lo[b]);
}
constexpr int kFftPadRow = 68;                // stage-A transpose row pitch
constexpr int kFft1024Slots = 16 * kFftPadRow;  // >= P(1024) + 1
__device__ __forceinline__ int fft1024_slot(int k) { return k + ((k >> 8) << 2); }

struct NoHook {
  __device__ __forceinline__ void operator()() const {}
};

// row: x[m], y[m] = packed sample j + 64 m of this lane (WaveRow<10>).
// after_a runs once stage A has left the row in LDS: the row registers are
// free from there, so a caller can start the next row's load in it and have
// stages B and C (not only its own post-processing) cover that load.
template <class Hook = NoHook>
__device__ __forceinline__ void fft1024_wave(const double (&x)[16], const double (&y)[16],
                                             double2* buf, const Fft1024Tw& t, int lane,
                                             Hook after_a = Hook{}) {
  double2 v[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) v[m] = cmk(x[m], y[m]);
  double2 lo[4], hi[4];
  lo[0] = hi[0] = cmk(1.0, 0.0);
#pragma unroll
  for (int i = 1; i < 4; ++i) { lo[i] = t.a[i - 1][lane]; hi[i] = t.b[i - 1][lane]; }
  dft16(v);
#pragma unroll
  for (int r = 0; r < 16; ++r)
    buf[r * kFftPadRow + lane] = r ? cmul(v[dft16_pos(r)], tw_pow(r, lo, hi)) : v[0];
  after_a();
  fft_sync<true>();
  const int j0 = lane & 3, rr = lane >> 2;
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = buf[rr * kFftPadRow + j0 + 4 * q];
#pragma unroll
  for (int i = 1; i < 4; ++i) { lo[i] = t.c[i - 1][j0]; hi[i] = t.d[i - 1][j0]; }
  dft16(v);
  fft_sync<true>();
#pragma unroll
  for (int s = 0; s < 16; ++s)
    buf[64 * s + 16 * j0 + (rr ^ (2 * j0))] = s ? cmul(v[dft16_pos(s)], tw_pow(s, lo, hi)) : v[0];
  fft_sync<true>();
  const int r2 = lane & 15, q4 = lane >> 4;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) v[4 * c + j] = buf[64 * (4 * q4 + c) + 16 * j + (r2 ^ (2 * j))];
  fft_sync<true>();  // all reads done before Z overwrites their slots
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    radix4<false>(v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]);
#pragma unroll
    for (int u = 0; u < 4; ++u) buf[r2 + 16 * (4 * q4 + c) + 260 * u] = v[4 * c + u];
  }
  fft_sync<true>();
}

// Channel walk of one wave: n = first, first + step, ... skipping masked.
__device__ __forceinline__ int next_chan(int n, int step, int nchan, const uint8_t* mask) {
  while (n < nchan && mask && !mask[n]) n += step;
  return n;
}

}  // namespace ppf
