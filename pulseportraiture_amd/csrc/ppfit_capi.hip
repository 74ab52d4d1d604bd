// ppfit_capi.hip -- host side of libppfit: context, workspace, launches.
// Implements include/ppfit.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ppfit.h"
#include "ppfit_kernels.hpp"

// Source hash of this build (pulseportraiture_amd/build.py compares it with
// today's sources before reusing a built library).
#ifndef PPF_SRC_HASH
#define PPF_SRC_HASH "unbuilt"
#endif
extern "C" __attribute__((visibility("default"), used)) const char ppf_build_tag[] =
    "PPF_SRC_HASH=" PPF_SRC_HASH;

using namespace ppf;

namespace {

struct TimedLaunch {
  int kid;
  hipEvent_t a, b;
};

struct Buffer {
  void* p = nullptr;
  size_t bytes = 0;
};

}  // namespace

struct ppf_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  int64_t ws_limit = (int64_t)32 << 30;
  double2* tw[16] = {nullptr};
  double2* vp[16] = {nullptr};  // moment power tables (k_vpow)
  // the same two tables for nbin that are not powers of two
  std::vector<std::pair<int, double2*>> tw_gen, vp_gen;
  Buffer ws;     // per-chunk fit workspace
  Buffer mspec;   // template spectra
  Buffer aux;     // misc (synth templates, partial sums)
  Buffer mmean;   // mean template spectra (guess)
  Buffer ptime;   // k_fit_taylor phase clocks (ppf_phase_profile)
  Buffer spart;   // split scattering solve: block partials + running count
  Buffer tmpl;    // template builders: knots / coefficients, rows and spectra
  int* active_h = nullptr;  // pinned host copies of the running count (two in flight)
  hipEvent_t scat_ev[2] = {nullptr, nullptr};  // their copies' completion
  hipStream_t stream2 = nullptr;        // second queue of the piece pipeline
  int pipe = 0;                         // pieces per chunk (0: default)
  std::vector<hipEvent_t> sync_events;  // ordering events (no timing)
  bool phase_prof = false;
  bool timing = false;
  std::vector<TimedLaunch> pending;
  std::vector<hipEvent_t> pool;
  double* trace = nullptr;  // solver trace buffer (ppf_set_trace), device
  int trace_cap = 0;
  // launch-schedule options (ppf_set_option; include/ppfit.h)
  int opt[PPF_NUM_OPTS] = {1, 1, 512, 1, 1, 0};
  double ktime[PPF_NUM_KERNELS] = {0};
  int64_t klaunch[PPF_NUM_KERNELS] = {0};
};

namespace {

int fail(ppf_ctx* ctx, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (ctx) ctx->err = buf;
  return code;
}

#define HIPCHK(ctx, expr)                                                              \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return fail(ctx, PPF_ERR_DEVICE, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

int ilog2_exact(int v) {
  if (v <= 0 || (v & (v - 1))) return -1;
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

// Any nbin in [16, 8192]: *logN = log2(nbin / 2) selects the FFT kernels of
// a power of two from 64 up, -1 the generic-length ones (ppfit_generic.hip)
// for every other length.
int check_nbin_any(ppf_ctx* ctx, int nbin, int* logN) {
  if (nbin < 16 || nbin > 8192)
    return fail(ctx, PPF_ERR_UNSUPPORTED, "nbin=%d: outside [16, 8192]", nbin);
  const int l = ilog2_exact(nbin);
  *logN = l < 6 ? -1 : l - 1;
  return PPF_OK;
}

// dynamic LDS of the generic-length kernels
size_t gen_row_lds(int nbin) { return (size_t)nbin * sizeof(double); }
size_t gen_rot_lds(int nbin) {
  return (((size_t)nbin * sizeof(double) + 15) & ~(size_t)15) + (size_t)(nbin / 2 + 1) * sizeof(double2);
}

// the generic-length data pass of n subints: every row's rfft on the matrix
// cores into the X rows, then the per-subint pass (ppfit_generic.hip)
// (data-spectrum cache: the spectra into the cache's rows under STORE; under
// USE they are there already)
void launch_data_gen(const SpecArgs& sa, int n, int nbin, hipStream_t st) {
  const int nrows = n * sa.nchan, NH = nbin / 2 + 1;
  const double* rows = sa.data + (size_t)sa.sub0 * sa.nchan * nbin;
  const dim3 g((nrows + kGenRows - 1) / kGenRows, (NH + 255) / 256);
  double2* dst = sa.D ? sa.D : sa.X;
  if (sa.spec_mode != PPF_SPEC_USE) {
    if (nbin <= kGenLdsTw)
      hipLaunchKernelGGL(k_dft_rows_mfma<true>, g, dim3(kBlock), dft_mfma_lds(nbin, true), st,
                         rows, dst, nrows, nbin, sa.NHP, sa.tw);
    else
      hipLaunchKernelGGL(k_dft_rows_mfma<false>, g, dim3(kBlock), dft_mfma_lds(nbin, false), st,
                         rows, dst, nrows, nbin, sa.NHP, sa.tw);
  }
  hipLaunchKernelGGL(k_data_post_gen, dim3(n), dim3(kBlock), 0, st, sa, nbin);
}

// the table of nbin in a generic-length cache (created by make on first use)
template <typename F>
int gen_table(ppf_ctx* ctx, std::vector<std::pair<int, double2*>>& cache, int nbin, size_t n,
              F&& make, const double2** out) {
  for (auto& p : cache)
    if (p.first == nbin) { *out = p.second; return PPF_OK; }
  double2* t = nullptr;
  HIPCHK(ctx, hipMalloc(&t, n * sizeof(double2)));
  make(t);
  if (hipGetLastError() != hipSuccess) {  // not cached: the next call builds it again
    (void)hipFree(t);
    return fail(ctx, PPF_ERR_DEVICE, "table launch for nbin=%d failed", nbin);
  }
  cache.push_back({nbin, t});
  *out = t;
  return PPF_OK;
}

// rows of 16 cells (256 B): measured faster than 8 or 32
int nharm_pad(int nbin) { return ((nbin / 2 + 1) + 15) & ~15; }

// get_noise_PS: kc = int((1 - 1/4) * nharm) (pplib.py:2245)
int noise_kc(int nbin) { return (int)(0.75 * (double)(nbin / 2 + 1)); }

int ensure(ppf_ctx* ctx, Buffer& b, size_t bytes) {
  if (b.bytes >= bytes) return PPF_OK;
  if (b.p) {
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    HIPCHK(ctx, hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
  }
  if (hipMalloc(&b.p, bytes) != hipSuccess)
    return fail(ctx, PPF_ERR_NOMEM, "hipMalloc(%zu) failed", bytes);
  b.bytes = bytes;
  return PPF_OK;
}

int twiddles(ppf_ctx* ctx, int nbin, const double2** out) {
  const int l = ilog2_exact(nbin);
  if (l < 0)
    return gen_table(ctx, ctx->tw_gen, nbin, (size_t)nbin, [&](double2* t) {
      hipLaunchKernelGGL(k_twiddles, dim3((nbin + 255) / 256), dim3(256), 0, ctx->stream, t, nbin);
    }, out);
  if (!ctx->tw[l]) {
    HIPCHK(ctx, hipMalloc(&ctx->tw[l], (size_t)nbin * sizeof(double2)));
    hipLaunchKernelGGL(k_twiddles, dim3((nbin + 255) / 256), dim3(256), 0, ctx->stream,
                       ctx->tw[l], nbin);
    HIPCHK(ctx, hipGetLastError());
  }
  *out = ctx->tw[l];
  return PPF_OK;
}

void launch_fit_taylor(const ppf_ctx* ctx, dim3 g, size_t lds, hipStream_t st, const FitArgs& fa);

// Moments per channel of T slot 0 that k_fit_taylor's LDS copy holds:
// kTaylorBlocksPerCU blocks of (static LDS + Meta + nchan * tnl doubles) in a
// CU's LDS, whole KB per block.
int taylor_lds_moments(int nchan, size_t lds_meta) {
  static size_t stat = 0;
  if (!stat) {
    size_t mx = 0;
    const void* ks[4] = {reinterpret_cast<const void*>(&k_fit_taylor<true, false>),
                         reinterpret_cast<const void*>(&k_fit_taylor<false, false>),
                         reinterpret_cast<const void*>(&k_fit_taylor<true, true>),
                         reinterpret_cast<const void*>(&k_fit_taylor<false, true>)};
    for (const void* k : ks) {
      hipFuncAttributes at;
      if (hipFuncGetAttributes(&at, k) != hipSuccess) return 0;
      mx = std::max(mx, at.sharedSizeBytes);
    }
    stat = mx;
  }
  const size_t per_block = (kLdsPerCU / kTaylorBlocksPerCU) & ~(size_t)1023;
  if (per_block <= stat + lds_meta) return 0;
  const size_t nl = (per_block - stat - lds_meta) / ((size_t)nchan * sizeof(double));
  return (int)std::min<size_t>(nl, kMT);
}

int vpow_table(ppf_ctx* ctx, int nbin, const double2** out) {
  const int l = ilog2_exact(nbin);
  const int rows = kVpowRows(nbin / 2);
  if (l < 0)
    return gen_table(ctx, ctx->vp_gen, nbin, (size_t)rows * 16, [&](double2* t) {
      hipLaunchKernelGGL(k_vpow, dim3((rows * 16 + 255) / 256), dim3(256), 0, ctx->stream, t,
                         nbin, rows);
    }, out);
  if (!ctx->vp[l]) {
    HIPCHK(ctx, hipMalloc(&ctx->vp[l], (size_t)rows * 16 * sizeof(double2)));
    hipLaunchKernelGGL(k_vpow, dim3((rows * 16 + 255) / 256), dim3(256), 0, ctx->stream,
                       ctx->vp[l], nbin, rows);
    HIPCHK(ctx, hipGetLastError());
  }
  *out = ctx->vp[l];
  return PPF_OK;
}

hipEvent_t ev_get(ppf_ctx* ctx) {
  if (!ctx->pool.empty()) {
    hipEvent_t e = ctx->pool.back();
    ctx->pool.pop_back();
    return e;
  }
  hipEvent_t e;
  (void)hipEventCreate(&e);
  return e;
}

// Launch helper: optional HIP-event bracket on the context stream.
template <typename F>
int timed_on(ppf_ctx* ctx, int kid, hipStream_t st, F&& launch) {
  hipEvent_t a = nullptr, b = nullptr;
  if (ctx->timing) {
    a = ev_get(ctx);
    b = ev_get(ctx);
    HIPCHK(ctx, hipEventRecord(a, st));
  }
  launch();
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(ctx, PPF_ERR_DEVICE, "kernel %d launch: %s", kid, hipGetErrorString(e));
  if (ctx->timing) {
    HIPCHK(ctx, hipEventRecord(b, st));
    ctx->pending.push_back({kid, a, b});
  }
  return PPF_OK;
}

template <typename F>
int timed(ppf_ctx* ctx, int kid, F&& launch) {
  return timed_on(ctx, kid, ctx->stream, launch);
}

// i-th ordering event of the context (created on first use)
int sync_event(ppf_ctx* ctx, size_t i, hipEvent_t* out) {
  while (ctx->sync_events.size() <= i) {
    hipEvent_t e;
    HIPCHK(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ctx->sync_events.push_back(e);
  }
  *out = ctx->sync_events[i];
  return PPF_OK;
}

int resolve_timing(ppf_ctx* ctx) {
  for (auto& t : ctx->pending) {
    HIPCHK(ctx, hipEventSynchronize(t.b));
    float ms = 0.f;
    HIPCHK(ctx, hipEventElapsedTime(&ms, t.a, t.b));
    ctx->ktime[t.kid] += (double)ms;
    ctx->klaunch[t.kid] += 1;
    ctx->pool.push_back(t.a);
    ctx->pool.push_back(t.b);
  }
  ctx->pending.clear();
  return PPF_OK;
}

#define LOGN_SWITCH(L, BODY)                          \
  switch (L) {                                        \
    case 5: { constexpr int LG = 5; BODY; } break;    \
    case 6: { constexpr int LG = 6; BODY; } break;    \
    case 7: { constexpr int LG = 7; BODY; } break;    \
    case 8: { constexpr int LG = 8; BODY; } break;    \
    case 9: { constexpr int LG = 9; BODY; } break;    \
    case 10: { constexpr int LG = 10; BODY; } break;  \
    case 11: { constexpr int LG = 11; BODY; } break;  \
    case 12: { constexpr int LG = 12; BODY; } break;  \
    default: break;                                   \
  }

// WD: the instantiation with the per-channel tables in HBM (chan_tables)
#define WIDE_SWITCH(W, ...)                                \
  do {                                                     \
    if (W) { constexpr bool WD = true; __VA_ARGS__; }      \
    else { constexpr bool WD = false; __VA_ARGS__; }       \
  } while (0)

// Template spectra for nrow rows of nbin (DC zeroed when zero_dc).
int model_spectra(ppf_ctx* ctx, int nrow, int nbin, const double* model, int zero_dc, Buffer& buf,
                  double2** M, double** pn, double** M2 = nullptr) {
  int logN;
  if (int r = check_nbin_any(ctx, nbin, &logN)) return r;
  const int NHP = nharm_pad(nbin);
  const size_t mbytes = (size_t)nrow * NHP * sizeof(double2);
  const size_t pbytes = ((size_t)nrow * sizeof(double) + 255) & ~(size_t)255;
  const size_t m2bytes = M2 ? (size_t)nrow * NHP * sizeof(double) : 0;
  if (int r = ensure(ctx, buf, mbytes + pbytes + m2bytes)) return r;
  *M = reinterpret_cast<double2*>(buf.p);
  *pn = reinterpret_cast<double*>(static_cast<char*>(buf.p) + mbytes);
  double* m2p = nullptr;
  if (M2) *M2 = m2p = reinterpret_cast<double*>(static_cast<char*>(buf.p) + mbytes + pbytes);
  const double2* tw;
  if (int r = twiddles(ctx, nbin, &tw)) return r;
  double2* Mp = *M;
  double* pp = *pn;
  return timed(ctx, PPF_K_MODEL_FFT, [&] {
    if (logN < 0)
      hipLaunchKernelGGL(k_model_spec_gen, dim3(nrow), dim3(kBlock), gen_row_lds(nbin),
                         ctx->stream, model, Mp, pp, NHP, zero_dc, tw, m2p, nbin);
    LOGN_SWITCH(logN, hipLaunchKernelGGL(k_model_spec<LG>, dim3(nrow), dim3(kBlock), 0,
                                         ctx->stream, model, Mp, pp, NHP, zero_dc, tw, m2p));
  });
}

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// the first moment pass inside k_fit_taylor (default) or its own k_moments
// launch (PPF_OPT_FUSE_MOMENTS = 0)
// launch; the moment passes form X from the data-spectrum cache when fa.Dsp is set
void launch_fit_taylor(const ppf_ctx* ctx, dim3 g, size_t lds, hipStream_t st, const FitArgs& fa) {
  const bool mom = ctx->opt[PPF_OPT_FUSE_MOMENTS] != 0;
  WIDE_SWITCH(fa.gdyn != nullptr, {
    if (fa.Dsp) {
      if (mom) hipLaunchKernelGGL((k_fit_taylor<true, true, WD>), g, dim3(kBlock), lds, st, fa);
      else hipLaunchKernelGGL((k_fit_taylor<false, true, WD>), g, dim3(kBlock), lds, st, fa);
    } else {
      if (mom) hipLaunchKernelGGL((k_fit_taylor<true, false, WD>), g, dim3(kBlock), lds, st, fa);
      else hipLaunchKernelGGL((k_fit_taylor<false, false, WD>), g, dim3(kBlock), lds, st, fa);
    }
  });
}

void launch_moments(dim3 g, hipStream_t st, const FitArgs& fa) {
  if (fa.Dsp) hipLaunchKernelGGL((k_moments<4, true>), g, dim3(kBlock), 0, st, fa);
  else hipLaunchKernelGGL((k_moments<4, false>), g, dim3(kBlock), 0, st, fa);
}

}  // namespace

extern "C" {

int ppf_version(void) { return PPF_VERSION; }

int ppf_ctx_create(int device, ppf_ctx** out) {
  if (!out) return PPF_ERR_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return PPF_ERR_DEVICE;
  if (device < 0 || device >= n) return PPF_ERR_INVALID;
  if (hipSetDevice(device) != hipSuccess) return PPF_ERR_DEVICE;
  ppf_ctx* c = new ppf_ctx();
  c->device = device;
  *out = c;
  return PPF_OK;
}

void ppf_ctx_destroy(ppf_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (auto& t : ctx->pending) { (void)hipEventDestroy(t.a); (void)hipEventDestroy(t.b); }
  for (auto e : ctx->pool) (void)hipEventDestroy(e);
  for (auto e : ctx->sync_events) (void)hipEventDestroy(e);
  if (ctx->stream2) {
    (void)hipStreamSynchronize(ctx->stream2);
    (void)hipStreamDestroy(ctx->stream2);
  }
  for (auto p : ctx->tw) if (p) (void)hipFree(p);
  for (auto p : ctx->vp) if (p) (void)hipFree(p);
  for (auto& p : ctx->tw_gen) (void)hipFree(p.second);
  for (auto& p : ctx->vp_gen) (void)hipFree(p.second);
  if (ctx->ptime.p) (void)hipFree(ctx->ptime.p);
  if (ctx->spart.p) (void)hipFree(ctx->spart.p);
  if (ctx->tmpl.p) (void)hipFree(ctx->tmpl.p);
  if (ctx->active_h) (void)hipHostFree(ctx->active_h);
  for (auto e : ctx->scat_ev) if (e) (void)hipEventDestroy(e);
  if (ctx->ws.p) (void)hipFree(ctx->ws.p);
  if (ctx->mspec.p) (void)hipFree(ctx->mspec.p);
  if (ctx->aux.p) (void)hipFree(ctx->aux.p);
  if (ctx->mmean.p) (void)hipFree(ctx->mmean.p);
  delete ctx;
}

const char* ppf_last_error(const ppf_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int ppf_set_stream(ppf_ctx* ctx, void* stream) {
  if (!ctx) return PPF_ERR_INVALID;
  ctx->stream = reinterpret_cast<hipStream_t>(stream);
  return PPF_OK;
}

int ppf_set_pipeline(ppf_ctx* ctx, int32_t pieces) {
  if (!ctx || pieces < 0 || pieces > 64) return PPF_ERR_INVALID;
  ctx->pipe = pieces;
  return PPF_OK;
}

int ppf_set_option(ppf_ctx* ctx, int32_t option, int32_t value) {
  if (!ctx) return PPF_ERR_INVALID;
  if (option < 0 || option >= PPF_NUM_OPTS)
    return fail(ctx, PPF_ERR_INVALID, "unknown option %d", option);
  if (option == PPF_OPT_SCAT_TAIL ? value < 0 : (value != 0 && value != 1))
    return fail(ctx, PPF_ERR_INVALID, "option %d: bad value %d", option, value);
  ctx->opt[option] = value;
  return PPF_OK;
}

int ppf_get_option(const ppf_ctx* ctx, int32_t option, int32_t* value) {
  if (!ctx || !value || option < 0 || option >= PPF_NUM_OPTS) return PPF_ERR_INVALID;
  *value = ctx->opt[option];
  return PPF_OK;
}

int ppf_synchronize(ppf_ctx* ctx) {
  if (!ctx) return PPF_ERR_INVALID;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return PPF_OK;
}

int ppf_set_workspace_limit(ppf_ctx* ctx, int64_t bytes) {
  if (!ctx || bytes <= 0) return PPF_ERR_INVALID;
  ctx->ws_limit = bytes;
  return PPF_OK;
}

int ppf_set_trace(ppf_ctx* ctx, double* buf, int32_t cap) {
  if (!ctx || cap < 0 || (cap > 0 && !buf)) return PPF_ERR_INVALID;
  ctx->trace = buf;
  ctx->trace_cap = cap;
  return PPF_OK;
}

int ppf_set_timing(ppf_ctx* ctx, int enable) {
  if (!ctx) return PPF_ERR_INVALID;
  ctx->timing = enable != 0;
  return PPF_OK;
}

int ppf_get_kernel_time(ppf_ctx* ctx, int kid, double* total_ms, int64_t* launches) {
  if (!ctx || kid < 0 || kid >= PPF_NUM_KERNELS) return PPF_ERR_INVALID;
  if (int r = resolve_timing(ctx)) return r;
  if (total_ms) *total_ms = ctx->ktime[kid];
  if (launches) *launches = ctx->klaunch[kid];
  return PPF_OK;
}

int ppf_reset_kernel_times(ppf_ctx* ctx) {
  if (!ctx) return PPF_ERR_INVALID;
  if (int r = resolve_timing(ctx)) return r;
  for (int i = 0; i < PPF_NUM_KERNELS; ++i) { ctx->ktime[i] = 0.0; ctx->klaunch[i] = 0; }
  return PPF_OK;
}

// ---------------------------------------------------------------------------
int ppf_fit_portrait_batch(ppf_ctx* ctx, const ppf_fit_desc* d, const ppf_fit_result* o) {
  if (!ctx || !d || !o) return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (d->nsub <= 0) return PPF_OK;
  if (d->nchan <= 0 || d->nchan > PPF_MAX_NCHAN)
    return fail(ctx, PPF_ERR_UNSUPPORTED, "nchan=%d outside [1, %d]", d->nchan, PPF_MAX_NCHAN);
  if (d->nmodel <= 0) return fail(ctx, PPF_ERR_INVALID, "nmodel must be >= 1");
  const bool tnc = d->method == PPF_METHOD_TNC || d->method == PPF_METHOD_TNC_LEGACY;
  const bool ncg = d->method == PPF_METHOD_NEWTON_CG;
  if (d->method != PPF_METHOD_TRUST_NCG && !tnc && !ncg)
    return fail(ctx, PPF_ERR_UNSUPPORTED, "Method %d is not implemented.", d->method);
  if (d->method == PPF_METHOD_TNC_LEGACY &&
      !(d->fit_flags[0] && d->fit_flags[1] && !d->fit_flags[2] && !d->fit_flags[3] &&
        !d->fit_flags[4]))
    return fail(ctx, PPF_ERR_INVALID, "legacy TNC fits phase and DM only (fit_flags [1,1,0,0,0])");
  if (d->solver_flags & ~(PPF_SOLVE_EXACT | PPF_SOLVE_EVAL | PPF_GUESS_DIRECT))
    return fail(ctx, PPF_ERR_INVALID, "unknown solver_flags bits 0x%x", d->solver_flags);
  if (!d->data || !d->model || !d->freqs || !d->P || !d->init || !d->nu_fit || !d->nu_out)
    return fail(ctx, PPF_ERR_INVALID, "missing required input pointer");
  if (!o->params || !o->param_errs || !o->nu_out || !o->cov || !o->scales || !o->scale_errs ||
      !o->channel_snrs || !o->chi2 || !o->red_chi2 || !o->snr || !o->nfev || !o->status)
    return fail(ctx, PPF_ERR_INVALID, "missing required output pointer");
  if (d->guess && d->guess_Ns < 2) return fail(ctx, PPF_ERR_INVALID, "guess_Ns must be >= 2");
  int logN;
  // nbin not a power of two: the generic-length data pass and template
  // spectra (ppfit_generic.hip); every solver kernel takes any nbin
  if (int r = check_nbin_any(ctx, d->nbin, &logN)) return r;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const int nchan = d->nchan, nbin = d->nbin;
  const int NH = nbin / 2 + 1, NHP = nharm_pad(nbin);
  const int kc = noise_kc(nbin);
  const double2* tw;
  if (int r = twiddles(ctx, nbin, &tw)) return r;
  double2* M;
  double* pn;
  double* M2;
  if (int r = model_spectra(ctx, d->nmodel * nchan, nbin, d->model, 1, ctx->mspec, &M, &pn, &M2))
    return r;

  // X, the cross-spectrum, is written once by k_data_xspec.  Phase-family
  // subints are fitted from Taylor moments of it (k_fit_taylor); scattering
  // fits, and every fit under PPF_SOLVE_EXACT, sweep it directly.
  const bool exact = (d->solver_flags & PPF_SOLVE_EXACT) != 0;
  const bool taylor = !exact && d->method == PPF_METHOD_TRUST_NCG;
  // data-spectrum cache: sig, dsum and R live in the caller's arrays, and
  // Taylor-path subints keep D instead of X (ppfit.h, PPF_SPEC_*)
  const int smode = d->spec_mode;
  if (smode != PPF_SPEC_NONE) {
    if (smode != PPF_SPEC_STORE && smode != PPF_SPEC_USE)
      return fail(ctx, PPF_ERR_INVALID, "spec_mode %d: PPF_SPEC_NONE, _STORE or _USE", smode);
    if (!d->spec || !d->spec_sig || !d->spec_dsum || !d->spec_R)
      return fail(ctx, PPF_ERR_INVALID, "spec_mode %d: spec, spec_sig, spec_dsum and spec_R "
                  "are required", smode);
    if (!taylor || d->fit_flags[3] || d->fit_flags[4])
      return fail(ctx, PPF_ERR_UNSUPPORTED, "the data-spectrum cache takes phase-family "
                  "trust-ncg fits only (tau and alpha not fitted, not PPF_SOLVE_EXACT)");
  }
  // mean template spectrum for the unmasked guess
  double2* Mmean = nullptr;
  if (d->guess) {
    if (int r = ensure(ctx, ctx->mmean, (size_t)d->nmodel * NHP * sizeof(double2))) return r;
    Mmean = reinterpret_cast<double2*>(ctx->mmean.p);
    if (int r = timed(ctx, PPF_K_MODEL_FFT, [&] {
          hipLaunchKernelGGL(k_model_mean, dim3((NHP + 255) / 256, d->nmodel), dim3(256), 0,
                             ctx->stream, M, Mmean, nchan, NHP);
        }))
      return r;
  }

  // per-subint workspace layout
  const size_t bX = (size_t)nchan * NHP * sizeof(double2);
  const size_t bT = taylor ? (size_t)2 * nchan * kMT * sizeof(double) : 0;
  const size_t bR = (size_t)NHP * sizeof(double2);
  const size_t bC = (size_t)nchan * sizeof(double);
  const size_t bAcc = (size_t)2 * nchan * 10 * sizeof(double);
  const size_t bW = (size_t)nchan * 8 * sizeof(double);
  // per-channel tables in HBM (the WIDE kernels, ppfit_kernels.hpp chan_tables)
  const bool wide = nchan > PPF_LDS_NCHAN || ctx->opt[PPF_OPT_HBM_TABLES] != 0;
  const size_t bG = wide ? align256(std::max(align256((size_t)nchan * (5 * sizeof(double) +
                                                                        sizeof(int))),
                                             xspec_dyn_lds(nchan)))
                         : 0;
  const size_t per_sub = bX + bT + 2 * bR + 2 * bC + sizeof(SolveState) + bAcc + bW + bG;
  int64_t chunk = ctx->ws_limit / (int64_t)(per_sub + 1024);
  if (chunk < 1) chunk = 1;
  if (chunk > d->nsub) chunk = d->nsub;
  const size_t cs = (size_t)chunk;
  const size_t offX = 0;
  const size_t offR = align256(offX + cs * bX);
  const size_t offMm = align256(offR + cs * bR);
  const size_t offSig = align256(offMm + cs * bR);
  const size_t offDs = align256(offSig + cs * bC);
  const size_t offSt = align256(offDs + cs * bC);
  const size_t offAcc = align256(offSt + cs * sizeof(SolveState));
  const size_t offW = align256(offAcc + cs * bAcc);
  const size_t offT = align256(offW + cs * bW);
  const size_t offG = align256(offT + cs * bT);
  const size_t total = align256(offG + cs * bG);
  if (int r = ensure(ctx, ctx->ws, total)) return r;
  char* base = static_cast<char*>(ctx->ws.p);

  SpecArgs sa;
  sa.nchan = nchan;
  sa.NHP = NHP;
  sa.kc = kc;
  sa.guess = d->guess;
  sa.data = d->data;
  sa.M = M;
  sa.model_idx = d->model_idx;
  sa.freqs = d->freqs;
  sa.errs = d->errs;
  sa.mask = d->chan_mask;
  sa.weights = d->weights;
  sa.P = d->P;
  sa.init = d->init;
  sa.guess_nu = d->guess_nu;
  sa.log10_tau = d->log10_tau;
  sa.fit_tau = d->fit_flags[3] ? 1 : 0;
  sa.exact = exact ? 1 : 0;
  sa.spec_mode = smode;
  sa.D = nullptr;
  sa.X = reinterpret_cast<double2*>(base + offX);
  sa.R = reinterpret_cast<double2*>(base + offR);
  sa.sig = reinterpret_cast<double*>(base + offSig);
  sa.dsum = reinterpret_cast<double*>(base + offDs);
  sa.tw = tw;
  sa.gdyn = wide ? reinterpret_cast<unsigned char*>(base + offG) : nullptr;
  sa.gdyn_stride = bG;

  FitArgs fa{};
  fa.nchan = nchan;
  fa.nbin = nbin;
  fa.NH = NH;
  fa.NHP = NHP;
  fa.kc = kc;
  for (int i = 0; i < 5; ++i) fa.flags[i] = d->fit_flags[i] ? 1 : 0;
  fa.log10_tau = d->log10_tau;
  fa.option = d->option;
  fa.is_toa = d->is_toa;
  fa.guess = d->guess;
  fa.Ns = d->guess_Ns;
  fa.guess_wrap = d->guess_wrap;
  fa.solver_flags = d->solver_flags;
  fa.method = d->method;
  fa.guess_wave = ctx->opt[PPF_OPT_GUESS_WAVE];
  for (int i = 0; i < 5; ++i)
    for (int j = 0; j < 2; ++j) fa.bounds[i][j] = d->bounds ? d->bounds[2 * i + j] : NAN;
  fa.X = sa.X;
  fa.Dsp = nullptr;
  fa.R = sa.R;
  fa.M = M;
  fa.M2 = M2;
  fa.pn = pn;
  fa.model_idx = d->model_idx;
  fa.sig = sa.sig;
  fa.dsum = sa.dsum;
  fa.freqs = d->freqs;
  fa.mask = d->chan_mask;
  fa.P = d->P;
  fa.init = d->init;
  fa.nu_fit = d->nu_fit;
  fa.nu_out = d->nu_out;
  fa.guess_nu = d->guess_nu;
  fa.guess_tau = d->guess_tau;
  fa.st = reinterpret_cast<SolveState*>(base + offSt);
  fa.acc = reinterpret_cast<double*>(base + offAcc);
  fa.wsc = reinterpret_cast<double*>(base + offW);
  fa.gdyn = sa.gdyn;
  fa.gdyn_stride = bG;
  fa.T = taylor ? reinterpret_cast<double*>(base + offT) : nullptr;
  fa.tw = tw;
  fa.vpow = nullptr;
  if (taylor)
    if (int r = vpow_table(ctx, nbin, &fa.vpow)) return r;
  fa.Mmean = Mmean;
  fa.ptime = ctx->phase_prof ? static_cast<unsigned long long*>(ctx->ptime.p) : nullptr;
  fa.trace = ctx->trace_cap > 0 ? ctx->trace : nullptr;
  fa.trace_cap = ctx->trace_cap;
  fa.o_params = o->params;
  fa.o_param_errs = o->param_errs;
  fa.o_nu_out = o->nu_out;
  fa.o_cov = o->cov;
  fa.o_scales = o->scales;
  fa.o_scale_errs = o->scale_errs;
  fa.o_channel_snrs = o->channel_snrs;
  fa.o_chi2 = o->chi2;
  fa.o_red_chi2 = o->red_chi2;
  fa.o_snr = o->snr;
  fa.o_nfev = o->nfev;
  fa.o_status = o->status;
  fa.o_init_used = o->init_used;
  fa.o_fun = o->fun;
  fa.o_cov_nosc = o->cov_nosc;
  fa.o_grad = o->grad;
  fa.o_hess = o->hess;

  // dynamic LDS of the Meta kernels (none for the WIDE ones)
  const size_t lds_meta =
      wide ? 0 : align256((size_t)nchan * (5 * sizeof(double) + sizeof(int)));
  const size_t lds_xspec = wide ? 0 : xspec_dyn_lds(nchan);
  // k_fit_taylor keeps moments [0, tnl) of T slot 0 in LDS (all of them when
  // they fit beside kTaylorBlocksPerCU - 1 other blocks; none when WIDE)
  fa.tnl = taylor && !wide ? taylor_lds_moments(nchan, lds_meta) : 0;
  fa.tlds = fa.tnl > 0 ? (int)lds_meta : 0;
  const size_t lds_taylor = lds_meta + (size_t)nchan * fa.tnl * sizeof(double);
  // trust-ncg scattering fits: every evaluation split over blocks of >= 64
  // fitted channels (k_scat_sweep / k_scat_step)
  // (PPF_OPT_SCAT_SPLIT = 0: one block per subint, k_solve<true>)
  const bool split_scat = ctx->opt[PPF_OPT_SCAT_SPLIT] && d->fit_flags[3] &&
                          d->method == PPF_METHOD_TRUST_NCG && !wide;
  const int split = std::max(1, std::min(16, nchan / 64));
  // the two-phase sweep's rows (any block's channel range at split or more)
  const size_t lds_scat = PPF_SCAT_TWO_PHASE ? scat_sweep_lds(nchan, split) : lds_meta;
  if (split_scat) {
    if (int r = ensure(ctx, ctx->spart,
                       (size_t)chunk * ((nchan + 7) / 8) * kScatPart * sizeof(double) +
                           64 * sizeof(int) + 256))
      return r;
    if (!ctx->active_h) HIPCHK(ctx, hipHostMalloc(&ctx->active_h, 2 * sizeof(int)));
    for (auto& e : ctx->scat_ev)
      if (!e) HIPCHK(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  const size_t lds_guess =
      (size_t)(NHP + (d->guess ? pfa_scratch_slots(d->guess_Ns, NH) : 0)) * sizeof(double2);
  // the cache rows of subints sub .. (spec_mode set): D, and sig / dsum / R in
  // place of the workspace's
  auto bind_spec = [&](SpecArgs& sp, FitArgs& fp, int64_t sub) {
    if (smode == PPF_SPEC_NONE) return;
    sp.D = reinterpret_cast<double2*>(d->spec) + (size_t)sub * nchan * NHP;
    fp.Dsp = sp.D;
    sp.sig = d->spec_sig + (size_t)sub * nchan;
    fp.sig = sp.sig;
    sp.dsum = d->spec_dsum + (size_t)sub * nchan;
    fp.dsum = sp.dsum;
    sp.R = reinterpret_cast<double2*>(d->spec_R) + (size_t)sub * NHP;
    fp.R = sp.R;
  };
  // Phase-family Taylor path, several pieces per chunk on two queues: piece
  // p's data pass starts when piece p-1's has finished, so the latency-bound
  // guess / fit / post-fit kernels of one piece run beside the HBM-bound
  // data pass of the next.  Each piece owns its slice of the workspace.
  const int pieces = ctx->pipe > 0 ? ctx->pipe : 1;
  const bool phase_family = !d->fit_flags[3] && !d->fit_flags[4];
  if (taylor && !tnc && phase_family && pieces > 1) {
    if (!ctx->stream2)
      HIPCHK(ctx, hipStreamCreateWithFlags(&ctx->stream2, hipStreamNonBlocking));
    hipEvent_t start, prev_x = nullptr;
    if (int r = sync_event(ctx, 0, &start)) return r;
    HIPCHK(ctx, hipEventRecord(start, ctx->stream));  // templates, tables, earlier calls
    HIPCHK(ctx, hipStreamWaitEvent(ctx->stream2, start, 0));
    size_t ev = 1;
    for (int64_t s0 = 0; s0 < d->nsub; s0 += chunk) {
      const int nc = (int)std::min<int64_t>(chunk, d->nsub - s0);
      const int np = std::min(pieces, nc);
      const int ps = (nc + np - 1) / np;
      for (int p = 0; p * ps < nc; ++p) {
        const int off = p * ps, n = std::min(ps, nc - off);
        hipStream_t st = (p & 1) ? ctx->stream2 : ctx->stream;
        SpecArgs sp = sa;
        FitArgs fp = fa;
        sp.sub0 = fp.sub0 = (int)s0 + off;
        sp.X = sa.X + (size_t)off * nchan * NHP;
        fp.X = sp.X;
        sp.R = sa.R + (size_t)off * NHP;
        fp.R = sp.R;
        sp.sig = sa.sig + (size_t)off * nchan;
        fp.sig = sp.sig;
        sp.dsum = sa.dsum + (size_t)off * nchan;
        fp.dsum = sp.dsum;
        fp.st = fa.st + off;
        fp.T = fa.T + (size_t)off * 2 * nchan * kMT;
        fp.acc = fa.acc + (size_t)off * 2 * nchan * 10;
        fp.wsc = fa.wsc + (size_t)off * nchan * 8;
        if (wide) {
          sp.gdyn = sa.gdyn + (size_t)off * bG;
          fp.gdyn = sp.gdyn;
        }
        bind_spec(sp, fp, s0 + off);
        if (prev_x) HIPCHK(ctx, hipStreamWaitEvent(st, prev_x, 0));
        if (int r = timed_on(ctx, PPF_K_DATA_XSPEC, st, [&] {
              if (logN < 0) launch_data_gen(sp, n, nbin, st);
              LOGN_SWITCH(logN, WIDE_SWITCH(wide, hipLaunchKernelGGL((k_data_xspec<LG, WD>), dim3(n),
                                                   dim3(XspecCfg<LG>::WPB * 64),
                                                   lds_xspec, st, sp)));
            }))
          return r;
        if (int r = sync_event(ctx, ev++, &prev_x)) return r;
        HIPCHK(ctx, hipEventRecord(prev_x, st));
        if (int r = timed_on(ctx, PPF_K_GUESS, st, [&] {
              if (d->guess && fp.guess_wave)
                hipLaunchKernelGGL(k_guess_w, dim3(n), dim3(64), 0, st, fp);
              hipLaunchKernelGGL(k_guess, dim3(n), dim3(kBlock), d->guess ? lds_guess : 0, st, fp);
            }))
          return r;
        if (!ctx->opt[PPF_OPT_FUSE_MOMENTS])
          if (int r = timed_on(ctx, PPF_K_MOMENTS, st, [&] {
                const dim3 g(n, (nchan + 16 * kWaves - 1) / (16 * kWaves));
                launch_moments(g, st, fp);
              }))
            return r;
        if (int r = timed_on(ctx, PPF_K_FIT_TAYLOR, st, [&] {
              launch_fit_taylor(ctx, dim3(n), lds_taylor, st, fp);
            }))
          return r;
        // subints the Taylor path does not take (tau != 0 at the start, not
        // fitted): the one-workgroup scattering solve and post-fit, as on
        // one queue (both exit at once for every other subint)
        if (int r = timed_on(ctx, PPF_K_SOLVE, st, [&] {
              WIDE_SWITCH(wide, hipLaunchKernelGGL((k_solve<true, WD>), dim3(n), dim3(kBlock),
                                                   lds_meta, st, fp));
            }))
          return r;
        if (int r = timed_on(ctx, PPF_K_POST, st, [&] {
              WIDE_SWITCH(wide, {
                hipLaunchKernelGGL((k_post<false, WD>), dim3(n), dim3(kBlock), lds_meta, st, fp);
                hipLaunchKernelGGL((k_post<true, WD>), dim3(n), dim3(kBlock), lds_meta, st, fp);
              });
            }))
          return r;
        if (o->errs_out)
          HIPCHK(ctx, hipMemcpyAsync(o->errs_out + (size_t)(s0 + off) * nchan, sp.sig,
                                     (size_t)n * nchan * sizeof(double),
                                     hipMemcpyDeviceToDevice, st));
      }
    }
    // join: the caller's stream sees every piece
    hipEvent_t done;
    if (int r = sync_event(ctx, ev++, &done)) return r;
    HIPCHK(ctx, hipEventRecord(done, ctx->stream2));
    HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, done, 0));
    return PPF_OK;
  }
  for (int64_t s0 = 0; s0 < d->nsub; s0 += chunk) {
    const int nc = (int)std::min<int64_t>(chunk, d->nsub - s0);
    sa.sub0 = (int)s0;
    fa.sub0 = (int)s0;
    bind_spec(sa, fa, s0);
    if (int r = timed(ctx, PPF_K_DATA_XSPEC, [&] {
          if (logN < 0) launch_data_gen(sa, nc, nbin, ctx->stream);
          LOGN_SWITCH(logN, WIDE_SWITCH(wide, hipLaunchKernelGGL((k_data_xspec<LG, WD>), dim3(nc),
                                                                 dim3(XspecCfg<LG>::WPB * 64),
                                                                 lds_xspec, ctx->stream, sa)));
        }))
      return r;
    if (int r = timed(ctx, PPF_K_GUESS, [&] {
          if (d->guess && fa.guess_wave)
            hipLaunchKernelGGL(k_guess_w, dim3(nc), dim3(64), 0, ctx->stream, fa);
          hipLaunchKernelGGL(k_guess, dim3(nc), dim3(kBlock), d->guess ? lds_guess : 0,
                             ctx->stream, fa);
        }))
      return r;
    // each subint runs in exactly one of the exact phase-only / scattering /
    // fused Taylor variants (the others exit at once)
    if (int r = timed(ctx, PPF_K_SOLVE, [&] {
          WIDE_SWITCH(wide, {
            if (tnc) {
              hipLaunchKernelGGL((k_tnc<false, WD>), dim3(nc), dim3(kBlock), lds_meta, ctx->stream,
                                 fa);
              hipLaunchKernelGGL((k_tnc<true, WD>), dim3(nc), dim3(kBlock), lds_meta, ctx->stream,
                                 fa);
              return;
            }
            if (ncg) {
              hipLaunchKernelGGL((k_ncg<false, WD>), dim3(nc), dim3(kBlock), lds_meta, ctx->stream,
                                 fa);
              hipLaunchKernelGGL((k_ncg<true, WD>), dim3(nc), dim3(kBlock), lds_meta, ctx->stream,
                                 fa);
              return;
            }
            if (exact)
              hipLaunchKernelGGL((k_solve<false, WD>), dim3(nc), dim3(kBlock), lds_meta,
                                 ctx->stream, fa);
            if (!split_scat)
              hipLaunchKernelGGL((k_solve<true, WD>), dim3(nc), dim3(kBlock), lds_meta,
                                 ctx->stream, fa);
          });
        }))
      return r;
    if (split_scat && !tnc && !ncg) {
      // k_solve<true> with each evaluation over `cur` blocks per subint
      // (k_scat_sweep) and then every subint's solver step (k_scat_step)
      double* part = static_cast<double*>(ctx->spart.p);
      int* ctrs = reinterpret_cast<int*>(part + (size_t)nc * ((nchan + 7) / 8) * kScatPart);
      HIPCHK(ctx, hipMemsetAsync(ctrs, 0, 2 * sizeof(int), ctx->stream));
      // iterations go in groups of kCheck launches; after each group its
      // running count is copied to pinned memory, and the host reads group
      // g's count only once group g + 1 is queued behind it, so the device
      // never waits for the host (a group launched after the last subint has
      // finished costs kCheck near-empty grids)
      constexpr int kCheck = 4;
      // once few subints are left (the tail of slow fits), each sweep is
      // spread over more blocks: one 8-channel group per wave.  The group
      // partials, and so every result, do not depend on the split.
      int cur = split;
      const int split_tail = std::max(split, std::min(32, (nchan + 31) / 32));
      // groups after the first are one hipGraph launch each (the same kernels
      // in the same order, captured once per call and split)
      hipGraphExec_t gx[2] = {nullptr, nullptr};
      auto graph_for = [&](int sp, hipGraphExec_t* ex) -> int {
        if (*ex) return PPF_OK;
        // captured on the context's second queue (the context stream may be
        // the legacy default stream, which cannot capture); launched on the
        // context stream
        if (!ctx->stream2)
          HIPCHK(ctx, hipStreamCreateWithFlags(&ctx->stream2, hipStreamNonBlocking));
        hipStream_t cs = ctx->stream2;
        hipGraph_t g = nullptr;
        HIPCHK(ctx, hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
        for (int k = 0; k < kCheck; ++k) {
          hipLaunchKernelGGL(k_scat_sweep, dim3(nc, sp), dim3(kBlock), lds_scat, cs, fa, part, sp,
                             0);
          hipLaunchKernelGGL(k_scat_step, dim3(nc), dim3(64), 0, cs, fa, part, 0, ctrs, k & 1);
        }
        HIPCHK(ctx, hipStreamEndCapture(cs, &g));
        const hipError_t e = hipGraphInstantiate(ex, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (e != hipSuccess)
          return fail(ctx, PPF_ERR_DEVICE, "scattering solve graph: %s", hipGetErrorString(e));
        return PPF_OK;
      };
      // the execs are destroyed on every way out of the loop, error returns
      // included, after the work launched from them has drained
      struct GraphFree {
        hipGraphExec_t* g;
        hipStream_t st;
        ~GraphFree() {
          if (!g[0] && !g[1]) return;
          (void)hipStreamSynchronize(st);
          for (int i = 0; i < 2; ++i)
            if (g[i]) (void)hipGraphExecDestroy(g[i]);
        }
      } gfree{gx, ctx->stream};
      // group gi: iterations kCheck * gi ... + kCheck - 1 (the first is the
      // init sweep); its count lands in active_h[gi & 1]
      auto issue = [&](int gi) -> int {
        const int it0 = kCheck * gi;
        if (gi > 0 && ctx->opt[PPF_OPT_SCAT_GRAPH]) {
          hipGraphExec_t* ex = &gx[cur == split ? 0 : 1];
          if (int r = graph_for(cur, ex)) return r;
          if (int r = timed(ctx, PPF_K_SOLVE, [&] { (void)hipGraphLaunch(*ex, ctx->stream); }))
            return r;
        } else {
          for (int k = 0; k < kCheck; ++k) {
            const int init = it0 + k == 0 ? 1 : 0;
            if (int r = timed(ctx, PPF_K_SOLVE, [&] {
                  hipLaunchKernelGGL(k_scat_sweep, dim3(nc, cur), dim3(kBlock), lds_scat,
                                     ctx->stream, fa, part, cur, init);
                }))
              return r;
            if (int r = timed(ctx, PPF_K_SOLVE, [&] {
                  hipLaunchKernelGGL(k_scat_step, dim3(nc), dim3(64), 0, ctx->stream, fa, part,
                                     init, ctrs, (it0 + k) & 1);
                }))
              return r;
          }
        }
        HIPCHK(ctx, hipMemcpyAsync(ctx->active_h + (gi & 1), ctrs + ((it0 + kCheck - 1) & 1),
                                   sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, hipEventRecord(ctx->scat_ev[gi & 1], ctx->stream));
        return PPF_OK;
      };
      // trust-ncg stops a fit at 1000 iterations (+ the init sweep)
      const int max_groups = (1001 + kCheck) / kCheck + 1;
      if (int r = issue(0)) return r;
      for (int gi = 0;; ++gi) {
        if (gi + 1 < max_groups)
          if (int r = issue(gi + 1)) return r;
        HIPCHK(ctx, hipEventSynchronize(ctx->scat_ev[gi & 1]));
        const int running = ctx->active_h[gi & 1];
        if (running == 0 || gi + 1 >= max_groups) break;
        if (running < ctx->opt[PPF_OPT_SCAT_TAIL]) cur = split_tail;
      }
    }
    if (taylor) {
      // the first moment pass inside k_fit_taylor (default), or its own
      // launch (PPF_OPT_FUSE_MOMENTS = 0)
      if (!ctx->opt[PPF_OPT_FUSE_MOMENTS])
        if (int r = timed(ctx, PPF_K_MOMENTS, [&] {
              const dim3 g(nc, (nchan + 16 * kWaves - 1) / (16 * kWaves));
              launch_moments(g, ctx->stream, fa);
            }))
          return r;
      if (int r = timed(ctx, PPF_K_FIT_TAYLOR, [&] {
            launch_fit_taylor(ctx, dim3(nc), lds_taylor, ctx->stream, fa);
          }))
        return r;
    }
    if (int r = timed(ctx, PPF_K_POST, [&] {
          WIDE_SWITCH(wide, {
            hipLaunchKernelGGL((k_post<false, WD>), dim3(nc), dim3(kBlock), lds_meta, ctx->stream,
                               fa);
            hipLaunchKernelGGL((k_post<true, WD>), dim3(nc), dim3(kBlock), lds_meta, ctx->stream,
                               fa);
          });
        }))
      return r;
    if (o->errs_out)  // the sigma each channel was fitted with (k_data_xspec)
      HIPCHK(ctx, hipMemcpyAsync(o->errs_out + (size_t)s0 * nchan, sa.sig,
                                 (size_t)nc * nchan * sizeof(double), hipMemcpyDeviceToDevice,
                                 ctx->stream));
  }
  return PPF_OK;
}

int ppf_phase_profile(ppf_ctx* ctx, int32_t enable, uint64_t* out) {
  if (!ctx) return fail(ctx, PPF_ERR_INVALID, "null context");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const size_t bytes = PPF_PHASE_N * sizeof(uint64_t);
  if (!ctx->ptime.p) {
    if (int r = ensure(ctx, ctx->ptime, bytes)) return r;
    HIPCHK(ctx, hipMemsetAsync(ctx->ptime.p, 0, bytes, ctx->stream));
  }
  if (out) HIPCHK(ctx, hipMemcpyAsync(out, ctx->ptime.p, bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipMemsetAsync(ctx->ptime.p, 0, bytes, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  ctx->phase_prof = enable != 0;
  return PPF_OK;
}

int ppf_selftest(ppf_ctx* ctx, int32_t* fails) {
  if (!ctx || !fails) return fail(ctx, PPF_ERR_INVALID, "null argument");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  int* d = nullptr;
  HIPCHK(ctx, hipMalloc(&d, PPF_SELFTEST_N * sizeof(int)));
  (void)hipMemsetAsync(d, 0, PPF_SELFTEST_N * sizeof(int), ctx->stream);
  hipLaunchKernelGGL(k_selftest, dim3(1), dim3(64), 0, ctx->stream, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess)
    e = hipMemcpyAsync(fails, d, PPF_SELFTEST_N * sizeof(int), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(ctx, PPF_ERR_DEVICE, "selftest: %s", hipGetErrorString(e));
  return PPF_OK;
}

int ppf_phase_shift_batch(ppf_ctx* ctx, int32_t nprof, int32_t nbin, const double* data,
                          const double* model, const int32_t* model_idx, const double* noise,
                          int32_t Ns, double lo, double hi, double* out) {
  if (!ctx || !data || !model || !out) return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nprof <= 0) return PPF_OK;
  if (Ns < 2) return fail(ctx, PPF_ERR_INVALID, "Ns must be >= 2");
  int logN;
  if (int r = check_nbin_any(ctx, nbin, &logN)) return r;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  // number of template rows = 1 + max(model_idx); the caller sizes model.
  int nmodel = 1;
  if (model_idx) {
    std::vector<int32_t> h(nprof);
    HIPCHK(ctx, hipMemcpyAsync(h.data(), model_idx, nprof * sizeof(int32_t), hipMemcpyDeviceToHost,
                               ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    for (int32_t v : h) {
      if (v < 0) return fail(ctx, PPF_ERR_INVALID, "negative model_idx");
      nmodel = std::max(nmodel, (int)v + 1);
    }
  }
  double2* M;
  double* pn;
  if (int r = model_spectra(ctx, nmodel, nbin, model, 1, ctx->aux, &M, &pn)) return r;
  const double2* tw;
  if (int r = twiddles(ctx, nbin, &tw)) return r;
  PhaseShiftArgs pa;
  pa.NHP = nharm_pad(nbin);
  pa.kc = noise_kc(nbin);
  pa.Ns = Ns;
  pa.lo = lo;
  pa.hi = hi;
  pa.data = data;
  pa.M = M;
  pa.model_idx = model_idx;
  pa.noise = noise;
  pa.out = out;
  pa.tw = tw;
  return timed(ctx, PPF_K_PHASE_SHIFT, [&] {
    if (logN < 0)
      hipLaunchKernelGGL(k_phase_shift_gen, dim3(nprof), dim3(kBlock), gen_rot_lds(nbin),
                         ctx->stream, pa, nbin);
    LOGN_SWITCH(logN, hipLaunchKernelGGL(k_phase_shift<LG>, dim3(nprof), dim3(kBlock), 0,
                                         ctx->stream, pa));
  });
}

int ppf_rotate_rows(ppf_ctx* ctx, int32_t nrow, int32_t nbin, const double* in,
                    const double* phase, double* out) {
  if (!ctx || !in || !phase || !out) return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nrow <= 0) return PPF_OK;
  int logN;
  if (int r = check_nbin_any(ctx, nbin, &logN)) return r;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const double2* tw;
  if (int r = twiddles(ctx, nbin, &tw)) return r;
  return timed(ctx, PPF_K_ROTATE, [&] {
    if (logN < 0)
      hipLaunchKernelGGL(k_rotate_rows_gen, dim3(nrow), dim3(kBlock), gen_rot_lds(nbin),
                         ctx->stream, in, phase, nullptr, out, tw, nbin);
    LOGN_SWITCH(logN, hipLaunchKernelGGL(k_rotate_rows<LG>, dim3(nrow), dim3(kBlock), 0,
                                         ctx->stream, in, phase, nullptr, out, tw));
  });
}

int ppf_scatter_rotate_rows(ppf_ctx* ctx, int32_t nrow, int32_t nbin, const double* in,
                            const double* phase, const double* tau, double* out) {
  if (!ctx || !in || !out) return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nrow <= 0) return PPF_OK;
  int logN;
  if (int r = check_nbin_any(ctx, nbin, &logN)) return r;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const double2* tw;
  if (int r = twiddles(ctx, nbin, &tw)) return r;
  if (!phase) return fail(ctx, PPF_ERR_INVALID, "phase must be given (zeros for none)");
  return timed(ctx, PPF_K_ROTATE, [&] {
    if (logN < 0)
      hipLaunchKernelGGL(k_rotate_rows_gen, dim3(nrow), dim3(kBlock), gen_rot_lds(nbin),
                         ctx->stream, in, phase, tau, out, tw, nbin);
    LOGN_SWITCH(logN, hipLaunchKernelGGL(k_rotate_rows<LG>, dim3(nrow), dim3(kBlock), 0,
                                         ctx->stream, in, phase, tau, out, tw));
  });
}

int ppf_spline_portraits(ppf_ctx* ctx, int32_t nrow, int32_t nbin_in, int32_t nbin, int32_t neig,
                         const double* mean_prof, const double* eigvec, int32_t nknot, int32_t k,
                         const double* t, const double* c, int32_t ncoef, const double* freqs,
                         double* out) {
  if (!ctx || !mean_prof || !freqs || !out || (neig > 0 && (!eigvec || !t || !c)))
    return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nrow <= 0) return PPF_OK;
  if (neig < 0 || neig > kMaxEig)
    return fail(ctx, PPF_ERR_UNSUPPORTED, "neig=%d: at most %d eigenvectors", neig, kMaxEig);
  if (neig > 0) {
    if (k < 1 || k > kMaxSplineK)
      return fail(ctx, PPF_ERR_UNSUPPORTED, "spline degree k=%d: 1..%d", k, kMaxSplineK);
    if (nknot < 2 * (k + 1) || ncoef < nknot - k - 1)
      return fail(ctx, PPF_ERR_INVALID, "nknot=%d, ncoef=%d: need nknot >= 2(k+1), ncoef >= nknot-k-1",
                  nknot, ncoef);
  }
  if (nbin_in <= 0) return fail(ctx, PPF_ERR_INVALID, "nbin_in=%d", nbin_in);
  int logI = 0, logO = 0;
  const bool resample = nbin_in != nbin;
  if (resample) {
    if (int r = check_nbin_any(ctx, nbin_in, &logI)) return r;
    if (int r = check_nbin_any(ctx, nbin, &logO)) return r;
  } else if (nbin <= 0) {
    return fail(ctx, PPF_ERR_INVALID, "nbin=%d", nbin);
  }
  HIPCHK(ctx, hipSetDevice(ctx->device));
  // device copies of the knots and coefficients, then (resampling) the rows
  // at nbin_in and both spectra
  const size_t ntc = neig > 0 ? (size_t)nknot + (size_t)neig * ncoef : 0;
  const size_t nrows_in = resample ? (size_t)nrow * nbin_in : 0;
  const size_t hin = (size_t)nbin_in / 2 + 1, hout = (size_t)nbin / 2 + 1;
  const size_t nspec = resample ? (size_t)nrow * (hin + hout) * 2 : 0;
  if (int r = ensure(ctx, ctx->tmpl, (ntc + nrows_in + nspec) * sizeof(double))) return r;
  double* base = static_cast<double*>(ctx->tmpl.p);
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));  // tmpl may still feed an earlier launch
  SplineArgs s;
  s.nbin = nbin_in;
  s.neig = neig;
  s.n = nknot;
  s.k = k;
  s.ncoef = ncoef;
  s.t = base;
  s.c = base + nknot;
  s.mean = mean_prof;
  s.eigvec = eigvec;
  if (neig > 0) {
    HIPCHK(ctx, hipMemcpy(base, t, (size_t)nknot * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(base + nknot, c, (size_t)neig * ncoef * sizeof(double),
                          hipMemcpyHostToDevice));
  }
  double* rows = resample ? base + ntc : out;
  if (int r = timed(ctx, PPF_K_MODEL_FFT, [&] {
        hipLaunchKernelGGL(k_spline_rows, dim3(nrow), dim3(256), 0, ctx->stream, s, freqs, rows);
      }))
    return r;
  if (!resample) return PPF_OK;
  double2* X = reinterpret_cast<double2*>(base + ntc + nrows_in);
  double2* Y = X + (size_t)nrow * hin;
  const double2 *twi, *two;
  if (int r = twiddles(ctx, nbin_in, &twi)) return r;
  if (int r = twiddles(ctx, nbin, &two)) return r;
  // ss.resample introduces a shift, undone by rotate_portrait (pplib.py:953-955)
  const double shift = 0.5 * (1.0 / (double)nbin - 1.0 / (double)nbin_in);
  const size_t ny = (size_t)nrow * hout;
  return timed(ctx, PPF_K_MODEL_FFT, [&] {
    if (logI < 0)
      hipLaunchKernelGGL(k_rfft_rows_gen, dim3(nrow), dim3(kBlock), gen_row_lds(nbin_in),
                         ctx->stream, rows, X, twi, nbin_in);
    LOGN_SWITCH(logI, hipLaunchKernelGGL(k_rfft_rows<LG>, dim3(nrow), dim3(kBlock), 0, ctx->stream,
                                         rows, X, twi));
    hipLaunchKernelGGL(k_resample_spec, dim3((unsigned)((ny + 255) / 256)), dim3(256), 0,
                       ctx->stream, X, nbin_in, nbin, shift, nrow, Y);
    if (logO < 0)
      hipLaunchKernelGGL(k_irfft_rows_gen, dim3(nrow), dim3(kBlock), hout * sizeof(double2),
                         ctx->stream, Y, out, two, nbin);
    LOGN_SWITCH(logO, hipLaunchKernelGGL(k_irfft_rows<LG>, dim3(nrow), dim3(kBlock), 0,
                                         ctx->stream, Y, out, two));
  });
}

int ppf_instrumental_response_rows(ppf_ctx* ctx, int32_t nrow, int32_t nbin, const double* in,
                                   int32_t nw, const double* wids, const int32_t* types,
                                   double DM, double chan_bw, double P, const double* freqs,
                                   double* out) {
  if (!ctx || !out || (nw > 0 && (!wids || !types)) || (DM != 0.0 && !freqs))
    return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nrow <= 0) return PPF_OK;
  if (nw < 0 || nw > kMaxIrf)
    return fail(ctx, PPF_ERR_UNSUPPORTED, "nw=%d: at most %d responses", nw, kMaxIrf);
  IrArgs g;
  g.nw = nw;
  g.fwhm = 2.0 * std::sqrt(2.0 * std::log(2.0));
  for (int w = 0; w < nw; ++w) {
    if (types[w] != 0 && types[w] != 1)
      return fail(ctx, PPF_ERR_INVALID, "irf type %d: 0 (rect) or 1 (gauss)", types[w]);
    if (!(wids[w] > 0.0))
      return fail(ctx, PPF_ERR_INVALID, "irf width %g: must be > 0", wids[w]);
    if (types[w] == 1) {
      // a = 1 / (2 sqrt 2 sigma_t) >= 6 keeps the dropped exp(-a^2) w(z) term below 2.4e-16
      const double st = wids[w] / g.fwhm;
      if (1.0 / (2.0 * M_SQRT2 * st) < 6.0)
        return fail(ctx, PPF_ERR_UNSUPPORTED,
                    "gauss irf FWHM %g rot: supported up to %.4f rot", wids[w],
                    g.fwhm / (12.0 * M_SQRT2));
    }
    g.type[w] = types[w];
    g.wid[w] = wids[w];
  }
  g.dm_wid_num = DM != 0.0 ? 8.3e-6 * chan_bw : 0.0;
  g.P = P;
  if (DM != 0.0 && !(P > 0.0)) return fail(ctx, PPF_ERR_INVALID, "P=%g", P);
  int logN;
  if (int r = check_nbin_any(ctx, nbin, &logN)) return r;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const size_t nh = (size_t)nbin / 2 + 1, n = (size_t)nrow * nh;
  const unsigned grid = (unsigned)((n + 255) / 256);
  if (!in)  // the response table R [nrow][nharm] itself
    return timed(ctx, PPF_K_MODEL_FFT, [&] {
      hipLaunchKernelGGL(k_ir_spec, dim3(grid), dim3(256), 0, ctx->stream, nullptr, out, nrow,
                         (int)nh, g, freqs);
    });
  if (int r = ensure(ctx, ctx->tmpl, n * sizeof(double2))) return r;
  double2* X = static_cast<double2*>(ctx->tmpl.p);
  const double2* tw;
  if (int r = twiddles(ctx, nbin, &tw)) return r;
  return timed(ctx, PPF_K_MODEL_FFT, [&] {
    if (logN < 0)
      hipLaunchKernelGGL(k_rfft_rows_gen, dim3(nrow), dim3(kBlock), gen_row_lds(nbin),
                         ctx->stream, in, X, tw, nbin);
    LOGN_SWITCH(logN, hipLaunchKernelGGL(k_rfft_rows<LG>, dim3(nrow), dim3(kBlock), 0, ctx->stream,
                                         in, X, tw));
    hipLaunchKernelGGL(k_ir_spec, dim3(grid), dim3(256), 0, ctx->stream, X, nullptr, nrow, (int)nh,
                       g, freqs);
    if (logN < 0)
      hipLaunchKernelGGL(k_irfft_rows_gen, dim3(nrow), dim3(kBlock), nh * sizeof(double2),
                         ctx->stream, X, out, tw, nbin);
    LOGN_SWITCH(logN, hipLaunchKernelGGL(k_irfft_rows<LG>, dim3(nrow), dim3(kBlock), 0,
                                         ctx->stream, X, out, tw));
  });
}

int ppf_tscrunch(ppf_ctx* ctx, int32_t nsub, int32_t npol, int32_t nchan, int32_t nbin,
                 const double* data, const double* weights, double* out, double* wsum) {
  if (!ctx || !data || !weights || !out) return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nsub <= 0 || npol <= 0 || nchan <= 0 || nbin <= 0)
    return fail(ctx, PPF_ERR_INVALID, "empty archive (%d, %d, %d, %d)", nsub, npol, nchan, nbin);
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const size_t total = (size_t)npol * nchan * nbin;
  return timed(ctx, PPF_K_MODEL_FFT, [&] {
    hipLaunchKernelGGL(k_tscrunch, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, ctx->stream,
                       data, weights, nsub, npol, nchan, nbin, out, wsum);
  });
}

int ppf_irfft_rows(ppf_ctx* ctx, int32_t nrow, int32_t nbin, const double* spec, double* out) {
  if (!ctx || !spec || !out) return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nrow <= 0) return PPF_OK;
  int logN;
  if (int r = check_nbin_any(ctx, nbin, &logN)) return r;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const double2* tw;
  if (int r = twiddles(ctx, nbin, &tw)) return r;
  const double2* sp = reinterpret_cast<const double2*>(spec);
  return timed(ctx, PPF_K_IRFFT, [&] {
    if (logN < 0)
      hipLaunchKernelGGL(k_irfft_rows_gen, dim3(nrow), dim3(kBlock),
                         (size_t)(nbin / 2 + 1) * sizeof(double2), ctx->stream, sp, out, tw, nbin);
    LOGN_SWITCH(logN, hipLaunchKernelGGL(k_irfft_rows<LG>, dim3(nrow), dim3(kBlock), 0,
                                         ctx->stream, sp, out, tw));
  });
}

int ppf_noise_rows(ppf_ctx* ctx, int32_t nrow, int32_t nbin, const double* in, double* out) {
  if (!ctx || !in || !out) return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nrow <= 0) return PPF_OK;
  int logN;
  if (int r = check_nbin_any(ctx, nbin, &logN)) return r;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const double2* tw;
  if (int r = twiddles(ctx, nbin, &tw)) return r;
  const int kc = noise_kc(nbin);
  return timed(ctx, PPF_K_NOISE, [&] {
    if (logN < 0)
      hipLaunchKernelGGL(k_noise_rows_gen, dim3(nrow), dim3(kBlock), gen_row_lds(nbin),
                         ctx->stream, in, out, kc, tw, nbin);
    LOGN_SWITCH(logN, hipLaunchKernelGGL(k_noise_rows<LG>, dim3(nrow), dim3(kBlock), 0,
                                         ctx->stream, in, out, kc, tw));
  });
}

int ppf_synth_portraits(ppf_ctx* ctx, int32_t nsub, int32_t nchan, int32_t nbin,
                        const double* model, const double* phase, double sigma, uint64_t seed,
                        int64_t sub0, double* data) {
  if (!ctx || !model || !phase || !data) return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nsub <= 0 || nchan <= 0) return PPF_OK;
  int logN;
  if (int r = check_nbin_any(ctx, nbin, &logN)) return r;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  double2* M;
  double* pn;
  if (int r = model_spectra(ctx, nchan, nbin, model, 0, ctx->aux, &M, &pn)) return r;
  const double2* tw;
  if (int r = twiddles(ctx, nbin, &tw)) return r;
  const int NHP = nharm_pad(nbin);
  const int64_t rows = (int64_t)nsub * nchan;
  if (rows > 0x7fffffff) return fail(ctx, PPF_ERR_INVALID, "too many rows");
  return timed(ctx, PPF_K_SYNTH, [&] {
    if (logN < 0)
      hipLaunchKernelGGL(k_synth_gen, dim3((unsigned)rows), dim3(kBlock),
                         (size_t)(nbin / 2 + 1) * sizeof(double2), ctx->stream, M, phase, data,
                         nchan, NHP, sigma, seed, sub0, tw, nbin);
    LOGN_SWITCH(logN, hipLaunchKernelGGL(k_synth<LG>, dim3((unsigned)rows), dim3(kBlock), 0,
                                         ctx->stream, M, phase, data, nchan, NHP, sigma, seed,
                                         sub0, tw));
  });
}

int ppf_rotate_accumulate(ppf_ctx* ctx, int32_t nsub, int32_t nchan, int32_t nbin,
                          const double* data, const double* phase, const double* weight,
                          double* accum) {
  if (!ctx || !data || !phase || !weight || !accum)
    return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nsub <= 0 || nchan <= 0) return PPF_OK;
  int logN;
  if (int r = check_nbin_any(ctx, nbin, &logN)) return r;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const double2* tw;
  if (int r = twiddles(ctx, nbin, &tw)) return r;
  const int NH = nbin / 2 + 1;
  // one workgroup per (slice, channel), about 2048 of them (8 per CU); nbin
  // 2048: four waves each streaming every fourth row of the slice (register
  // FFT), so a slice should hold a few groups of four
  const bool wave = logN == 10;
  int nsplit = (2048 + nchan - 1) / nchan;
  if (wave && nsplit > (nsub + 3) / 4) nsplit = (nsub + 3) / 4;
  if (nsplit > nsub) nsplit = nsub;
  if (nsplit < 1) nsplit = 1;
  const size_t count = (size_t)nchan * NH;
  if (int r = ensure(ctx, ctx->aux, (size_t)nsplit * count * sizeof(double2))) return r;
  double2* partial = reinterpret_cast<double2*>(ctx->aux.p);
  if (int r = timed(ctx, PPF_K_ROT_ACCUM, [&] {
        if (logN < 0)
          hipLaunchKernelGGL(k_rot_accum_gen, dim3(nsplit * nchan), dim3(kBlock),
                             gen_row_lds(nbin), ctx->stream, data, phase, weight, partial, nsub,
                             nchan, nsplit, tw, nbin);
        else if (wave)
          hipLaunchKernelGGL(k_rot_accum_w, dim3(nsplit * nchan), dim3(256), 0,
                             ctx->stream, data, phase, weight, partial, nsub, nchan, nsplit, tw);
        else
          LOGN_SWITCH(logN, hipLaunchKernelGGL(k_rot_accum<LG>, dim3(nsplit * nchan),
                                               dim3(kBlock), 0, ctx->stream, data, phase, weight,
                                               partial, nsub, nchan, nsplit, tw));
      }))
    return r;
  double2* acc = reinterpret_cast<double2*>(accum);
  return timed(ctx, PPF_K_ROT_ACCUM, [&] {
    hipLaunchKernelGGL(k_accum_reduce, dim3((unsigned)((count + 255) / 256)), dim3(256), 0,
                       ctx->stream, partial, acc, nsplit, count);
  });
}

int32_t ppf_spec_nhp(int32_t nbin) {
  int logN;
  if (check_nbin_any(nullptr, nbin, &logN)) return -1;
  return nharm_pad(nbin);
}

int ppf_rotate_accumulate_spec(ppf_ctx* ctx, int32_t nsub, int32_t nchan, int32_t nbin,
                               const double* spec, const double* phase, const double* weight,
                               double* accum) {
  if (!ctx || !spec || !phase || !weight || !accum)
    return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nsub <= 0 || nchan <= 0) return PPF_OK;
  int logN;
  if (int r = check_nbin_any(ctx, nbin, &logN)) return r;  // spectra of any length
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const int N = nbin / 2, NH = N + 1, NHP = nharm_pad(nbin);
  // one workgroup per (slice, channel), about 2048 of them (8 per CU)
  int nsplit = (2048 + nchan - 1) / nchan;
  if (nsplit > nsub) nsplit = nsub;
  if (nsplit < 1) nsplit = 1;
  const size_t count = (size_t)nchan * NH;
  if (int r = ensure(ctx, ctx->aux, (size_t)nsplit * count * sizeof(double2))) return r;
  double2* partial = reinterpret_cast<double2*>(ctx->aux.p);
  if (int r = timed(ctx, PPF_K_ROT_ACCUM, [&] {
        hipLaunchKernelGGL(k_rot_accum_spec, dim3(nsplit * nchan), dim3(256), 0, ctx->stream,
                           reinterpret_cast<const double2*>(spec), phase, weight, partial, nsub,
                           nchan, nsplit, N, NHP);
      }))
    return r;
  double2* acc = reinterpret_cast<double2*>(accum);
  return timed(ctx, PPF_K_ROT_ACCUM, [&] {
    hipLaunchKernelGGL(k_accum_reduce, dim3((unsigned)((count + 255) / 256)), dim3(256), 0,
                       ctx->stream, partial, acc, nsplit, count);
  });
}

int ppf_gaussian_portraits(ppf_ctx* ctx, int32_t nrow, int32_t nbin, int32_t ngauss,
                           const int32_t* code, const double* params, double nu_ref, double alpha,
                           const double* freqs, double* out) {
  if (!ctx || !code || !params || !freqs || !out) return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nrow <= 0) return PPF_OK;
  if (ngauss < 0 || ngauss > kMaxGauss)
    return fail(ctx, PPF_ERR_UNSUPPORTED, "ngauss=%d: at most %d components", ngauss, kMaxGauss);
  for (int i = 0; i < 3; ++i)
    if (code[i] != 0 && code[i] != 1)
      return fail(ctx, PPF_ERR_INVALID, "model code digit %d: 0 (power law) or 1 (linear)", code[i]);
  int logN;
  if (int r = check_nbin_any(ctx, nbin, &logN)) return r;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  GaussArgs g;
  g.nbin = nbin;
  g.ngauss = ngauss;
  for (int i = 0; i < 3; ++i) g.code[i] = code[i];
  // the constants numpy forms on the host (glibc log / sqrt, as numpy's)
  g.nu_ref = nu_ref;
  g.lnu = std::log(nu_ref);
  g.fwhm = 2.0 * std::sqrt(2.0 * std::log(2.0));
  g.sqrt2pi = std::sqrt(2.0 * M_PI);
  for (int i = 0; i < 2 + 6 * ngauss; ++i) g.params[i] = params[i];
  const bool scat = params[1] != 0.0;
  // gen_gaussian_portrait's scattering branch (pplib.py:915-922): unscattered
  // rows into a scratch buffer, then scattered into out
  double* rows = out;
  double* taus = nullptr;
  if (scat) {
    const size_t nb = (size_t)nrow * nbin;
    if (int r = ensure(ctx, ctx->aux, (nb + (size_t)nrow) * sizeof(double))) return r;
    rows = static_cast<double*>(ctx->aux.p);
    taus = rows + nb;
  }
  if (int r = timed(ctx, PPF_K_MODEL_FFT, [&] {
        hipLaunchKernelGGL(k_gauss_port, dim3(nrow), dim3(256), 0, ctx->stream, g, freqs, rows);
      }))
    return r;
  if (!scat) return PPF_OK;
  const double2* tw;
  if (int r = twiddles(ctx, nbin, &tw)) return r;
  return timed(ctx, PPF_K_MODEL_FFT, [&] {
    hipLaunchKernelGGL(k_scat_taus, dim3((nrow + 255) / 256), dim3(256), 0, ctx->stream, freqs,
                       nrow, params[1] / (double)nbin, alpha, nu_ref, taus);
    if (logN < 0)
      hipLaunchKernelGGL(k_rotate_rows_gen, dim3(nrow), dim3(kBlock), gen_rot_lds(nbin),
                         ctx->stream, rows, nullptr, taus, out, tw, nbin);
    LOGN_SWITCH(logN, hipLaunchKernelGGL(k_rotate_rows<LG>, dim3(nrow), dim3(kBlock), 0,
                                         ctx->stream, rows, nullptr, taus, out, tw));
  });
}

int ppf_unpack_subints(ppf_ctx* ctx, int32_t nsub, int32_t npol, int32_t nchan, int32_t nbin,
                       int32_t raw_type, const void* raw, const double* scl, const double* offs,
                       int32_t pmode, double* out) {
  if (!ctx || !raw || !scl || !offs || !out) return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nsub <= 0) return PPF_OK;
  if (npol <= 0 || nchan <= 0 || nbin <= 0) return fail(ctx, PPF_ERR_INVALID, "bad shape");
  if (raw_type < 1 || raw_type > 3) return fail(ctx, PPF_ERR_INVALID, "raw_type %d", raw_type);
  if (pmode < 0 || pmode > 2 || (pmode == 1 && npol < 2))
    return fail(ctx, PPF_ERR_INVALID, "pmode %d with npol %d", pmode, npol);
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const int npo = pmode ? 1 : npol;
  const size_t rows = (size_t)nsub * npo * nchan;
  if (rows > 0x7fffffffULL) return fail(ctx, PPF_ERR_INVALID, "%zu profiles in one call", rows);
  const dim3 g((unsigned)rows);
  return timed(ctx, PPF_K_UNPACK, [&] {
    switch (raw_type) {
      case 1:
        hipLaunchKernelGGL(k_unpack<uint8_t>, g, dim3(256), 0, ctx->stream,
                           static_cast<const uint8_t*>(raw), scl, offs, nsub, npol, nchan, nbin,
                           pmode, out);
        break;
      case 2:
        hipLaunchKernelGGL(k_unpack<int16_t>, g, dim3(256), 0, ctx->stream,
                           static_cast<const int16_t*>(raw), scl, offs, nsub, npol, nchan, nbin,
                           pmode, out);
        break;
      default:
        hipLaunchKernelGGL(k_unpack<float>, g, dim3(256), 0, ctx->stream,
                           static_cast<const float*>(raw), scl, offs, nsub, npol, nchan, nbin,
                           pmode, out);
    }
  });
}

int ppf_remove_baseline(ppf_ctx* ctx, int32_t nsub, int32_t npol, int32_t nchan, int32_t nbin,
                        int32_t ntot, int32_t width, double* data, const double* weights,
                        int32_t* window) {
  if (!ctx || !data || !weights) return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nsub <= 0) return PPF_OK;
  if (npol <= 0 || nchan <= 0 || nbin <= 0 || nbin > 8192)
    return fail(ctx, PPF_ERR_INVALID, "bad shape (%d, %d, %d)", npol, nchan, nbin);
  if (ntot < 1 || ntot > npol) return fail(ctx, PPF_ERR_INVALID, "ntot %d with npol %d", ntot, npol);
  if (width < 1 || width > nbin) return fail(ctx, PPF_ERR_INVALID, "width %d", width);
  HIPCHK(ctx, hipSetDevice(ctx->device));
  return timed(ctx, PPF_K_UNPACK, [&] {
    hipLaunchKernelGGL(k_remove_baseline, dim3(nsub), dim3(256), (size_t)nbin * sizeof(double),
                       ctx->stream, data, weights, npol, nchan, nbin, ntot, width, window);
  });
}

int ppf_profile_snr(ppf_ctx* ctx, int32_t nrow, int32_t nbin, const double* rows, int32_t width,
                    double threshold, double* out) {
  if (!ctx || !rows || !out) return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nrow <= 0) return PPF_OK;
  if (nbin <= 0 || nbin > 8192) return fail(ctx, PPF_ERR_INVALID, "nbin %d", nbin);
  if (width < 1 || width > nbin) return fail(ctx, PPF_ERR_INVALID, "width %d", width);
  if (!(threshold >= 0.0 && threshold < 0.5))
    return fail(ctx, PPF_ERR_INVALID, "threshold %g outside [0, 0.5)", threshold);
  HIPCHK(ctx, hipSetDevice(ctx->device));
  return timed(ctx, PPF_K_UNPACK, [&] {
    hipLaunchKernelGGL(k_profile_snr, dim3(nrow), dim3(64), (size_t)nbin * sizeof(double),
                       ctx->stream, rows, nbin, width, threshold, out);
  });
}

int ppf_resid_chi2_rows(ppf_ctx* ctx, int32_t nrow, int32_t nbin, const double* data,
                        const double* phase, const double* model, const int32_t* model_row,
                        const double* scale, const double* tau, const double* errs,
                        double dof, double* out) {
  if (!ctx || !data || !model || !scale || !errs || !out)
    return fail(ctx, PPF_ERR_INVALID, "null argument");
  if (nrow <= 0) return PPF_OK;
  if (!(dof > 0.0)) return fail(ctx, PPF_ERR_INVALID, "dof must be > 0");
  int logN;
  if (int r = check_nbin_any(ctx, nbin, &logN)) return r;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const double2* tw;
  if (int r = twiddles(ctx, nbin, &tw)) return r;
  ResidArgs ra{data, phase, model, model_row, scale, tau, errs, dof, out};
  return timed(ctx, PPF_K_RESID, [&] {
    if (logN < 0)
      hipLaunchKernelGGL(k_resid_chi2_gen, dim3(nrow), dim3(kBlock), gen_rot_lds(nbin),
                         ctx->stream, ra, tw, nbin);
    LOGN_SWITCH(logN, hipLaunchKernelGGL(k_resid_chi2<LG>, dim3(nrow), dim3(kBlock), 0,
                                         ctx->stream, ra, tw));
  });
}

}  // extern "C"
