// ppfit_kernels.hpp -- kernel argument blocks and the shared FFTFIT search.
#pragma once
#include "ppfit_device.hpp"

namespace ppf {

// ---------------------------------------------------------------------------
// Argument blocks (passed by value)
// ---------------------------------------------------------------------------
struct SpecArgs {
  int sub0, nchan, NHP, kc, guess;
  int log10_tau, fit_tau, exact;  // X is written only for subints that need it
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
};

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
constexpr int kMT = 32;
constexpr int kMTerm = kMT - 2;
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
};

struct FitArgs {
  int sub0, nchan, nbin, NH, NHP, kc;
  int flags[5];
  int log10_tau, option, is_toa, guess, Ns, guess_wrap;
  const double2* X;          // chunk [c][nchan][NHP]
  const double2* R;          // chunk [c][NHP]
  const double2* M;          // [nmodel][nchan][NHP]
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
  double2* T;                // chunk [c][2][nchan][kMT] Taylor moments
  int* Tcnt;                 // chunk [c][2][nchan] moments stored per row
  const double2* tw;         // rfft twiddles e^{-2 pi i m / nbin}
  const double2* Mmean;      // [nmodel][NHP] mean template spectrum or null
  unsigned long long* ptime; // [PPF_PHASE_N] k_fit_taylor phase clocks, or null
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
};

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
};

// One wave evaluates sum_k Re(rm_k e^{2 pi i k phi}); every lane gets it.
__device__ __forceinline__ double wave_eval_phase(const double2* rm, int NH, double phi) {
  const int lane = threadIdx.x & 63;
  const double2 step = turn_phasor(64.0, phi);
  double2 e = cmk(1.0, 0.0);
  double acc = 0.0;
  int j = 0;
  for (int k = lane; k < NH; k += 64, ++j) {
    if ((j & 15) == 0) e = turn_phasor((double)k, phi);
    else e = cmul(e, step);
    const double2 r = rm[k];
    acc = fma(r.x, e.x, acc);
    acc = fma(-r.y, e.y, acc);
  }
  return wave_sum(acc);
}

// np.argmin order: the first NaN wins, else the first smallest value.
__device__ __forceinline__ bool argmin_better(double v, int i, double bv, int bi) {
  if (i == 0x7fffffff) return false;
  if (bi == 0x7fffffff) return true;
  if (isnan(bv)) return isnan(v) && i < bi;
  if (isnan(v)) return true;
  return v < bv || (v == bv && i < bi);
}

__device__ inline void guess_search(const double2* rm, int NH, double ie2, int Ns, double lo,
                                    double hi, GuessShared& gs) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // ---- brute force over the inclusive grid (np.mgrid[lo:hi:Ns*1j]) ----
  // grid and simplex arithmetic use explicit _rn ops: hipcc would otherwise
  // contract them into FMAs and move the points off numpy's values.
  const double step = (hi - lo) / (double)(Ns - 1);
  double bv = NAN;
  int bi = 0x7fffffff;
  for (int g = w; g < Ns; g += kWaves) {  // ascending per wave
    const double ph = (g == Ns - 1) ? hi : __dadd_rn(__dmul_rn((double)g, step), lo);
    const double f = -wave_eval_phase(rm, NH, ph) * ie2;
    if (argmin_better(f, g, bv, bi)) { bv = f; bi = g; }
  }
  if (lane == 0) { gs.bestv[w] = bv; gs.besti[w] = bi; }
  __syncthreads();
  if (tid == 0) {
    double v = gs.bestv[0];
    int i = gs.besti[0];
    for (int q = 1; q < kWaves; ++q)
      if (argmin_better(gs.bestv[q], gs.besti[q], v, i)) { v = gs.bestv[q]; i = gs.besti[q]; }
    gs.x0 = (i == Ns - 1) ? hi : __dadd_rn(__dmul_rn((double)i, step), lo);
  }
  __syncthreads();
  // ---- Nelder-Mead polish, wave 0 (uniform scalar control flow) ----
  if (w == 0) {
    const int maxfun = 200, maxiter = 200;
    int fcalls = 0;
    bool stop = false;
    auto F = [&](double xv) -> double {
      if (fcalls >= maxfun) { stop = true; return 0.0; }
      ++fcalls;
      return -wave_eval_phase(rm, NH, xv) * ie2;
    };
    double s0 = gs.x0;
    double s1 = (s0 != 0.0) ? (1.0 + 0.05) * s0 : 0.00025;
    double f0 = F(s0), f1 = F(s1);
    if (f1 < f0) { double t = s0; s0 = s1; s1 = t; t = f0; f0 = f1; f1 = t; }
    int it = 1;
    while (fcalls < maxfun && it < maxiter) {
      if (fabs(s1 - s0) <= 1e-4 && fabs(f0 - f1) <= 1e-4) break;
      const double xbar = s0;
      const double xr = __dsub_rn(__dmul_rn(2.0, xbar), s1);
      const double fxr = F(xr);
      if (stop) break;
      bool shrink = false;
      if (fxr < f0) {
        const double xe = __dsub_rn(__dmul_rn(3.0, xbar), __dmul_rn(2.0, s1));
        const double fxe = F(xe);
        if (stop) break;
        if (fxe < fxr) { s1 = xe; f1 = fxe; } else { s1 = xr; f1 = fxr; }
      } else {
        if (fxr < f1) {
          const double xc = __dsub_rn(__dmul_rn(1.5, xbar), __dmul_rn(0.5, s1));
          const double fxc = F(xc);
          if (stop) break;
          if (fxc <= fxr) { s1 = xc; f1 = fxc; } else shrink = true;
        } else {
          const double xcc = __dadd_rn(__dmul_rn(0.5, xbar), __dmul_rn(0.5, s1));
          const double fxcc = F(xcc);
          if (stop) break;
          if (fxcc < f1) { s1 = xcc; f1 = fxcc; } else shrink = true;
        }
        if (shrink) {
          s1 = __dadd_rn(s0, __dmul_rn(0.5, __dsub_rn(s1, s0)));
          f1 = F(s1);
          if (stop) break;
        }
      }
      ++it;
      if (f1 < f0) { double t = s0; s0 = s1; s1 = t; t = f0; f0 = f1; f1 = t; }
    }
    if (f1 < f0) { double t = s0; s0 = s1; s1 = t; t = f0; f0 = f1; f1 = t; }
    if (lane == 0) { gs.x = s0; gs.fx = fmin(f0, f1); }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// kernel declarations
// ---------------------------------------------------------------------------
__global__ void k_twiddles(double2* tw, int nbin);
template <int LOGN>
__global__ void k_model_spec(const double* model, double2* M, double* pn, int NHP, int zero_dc,
                             const double2* tw);
template <int LOGN> __global__ void k_data_xspec(SpecArgs a);
template <int LOGN> __global__ void k_phase_shift(PhaseShiftArgs a);
template <int LOGN>
__global__ void k_rotate_rows(const double* in, const double* phase, double* out,
                              const double2* tw);
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
__global__ void k_accum_reduce(const double2* partial, double2* accum, int nsplit, size_t count);
__global__ void k_guess(FitArgs a);
__global__ void k_model_mean(const double2* M, double2* Mmean, int nchan, int NHP);
__global__ void k_fit_taylor(FitArgs a);
__global__ void k_selftest(int* fails);
template <bool SCAT> __global__ void k_solve(FitArgs a);
template <bool SCAT> __global__ void k_post(FitArgs a);

}  // namespace ppf
