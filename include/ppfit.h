/*
 * ppfit.h -- C ABI of libppfit.so, the MI355X (gfx950) implementation of the
 * PulsePortraiture wideband FFTFIT hot path.
 *
 * The reference (kmjc/PulsePortraiture) is pure Python; its "plugin surface"
 * is the set of Python call signatures listed in SURVEY.md §8(b).  Each entry
 * point below is what the Python drop-ins in pulseportraiture_amd/ bind via
 * ctypes in place of the reference's numpy/scipy code:
 *
 *   ppf_fit_portrait_batch  <- pptoaslib.fit_portrait_full   pptoaslib.py:928-1096
 *                              (+ the get_TOAs initial guess pptoas.py:420-456,
 *                               ppalign.py:180-185, batched over subints)
 *   ppf_phase_shift_batch   <- pplib.fit_phase_shift          pplib.py:2054-2100
 *   ppf_rotate_rows         <- pplib.rotate_data / rotate_portrait /
 *                              pptoaslib.rotate_portrait_full pplib.py:2338-2460,
 *                                                             pptoaslib.py:52-81
 *   ppf_rotate_accumulate   <- ppalign.align_archives' weighted sum
 *                              ppalign.py:202-208
 *   ppf_rotate_accumulate_spec <- the same sum over cached data spectra
 *                              (ppalign.py:202-208, iterations after the first)
 *   ppf_irfft_rows          <- numpy.fft.irfft (final step of ppalign.py:210-213)
 *   ppf_noise_rows          <- pplib.get_noise_PS(chans=True)  pplib.py:2227-2253
 *   ppf_unpack_subints      <- PSRCHIVE Archive_load + pscrunch in
 *                              pplib.load_data  pplib.py:2670-2732 (with
 *                              include/ppfits.h, the host PSRFITS reader)
 *   ppf_profile_snr         <- Profile::snr() for load_data's SNRs
 *                              pplib.py:2762-2770 (PSRCHIVE restated)
 *   ppf_gaussian_portraits  <- pplib.gen_gaussian_portrait / read_model
 *                              pplib.py:853-930, 2873-2959
 *   ppf_scatter_rotate_rows <- GetTOAs.show_fit port/model  pptoas.py:1389-1402
 *   ppf_resid_chi2_rows     <- pplib.get_red_chi2 per channel in
 *                              GetTOAs.get_channels_to_zap  pptoas.py:1201-1278
 *   ppf_synth_portraits     <- (test/bench input producer; pplib.make_fake_pulsar
 *                              math, pplib.py:3342-3377, on device)
 *
 * Conventions
 *  - Every array argument is a DEVICE pointer (hipMalloc'd or a torch CUDA
 *    tensor's data_ptr) unless documented otherwise; arrays are C-order fp64.
 *  - Calls are stream-ordered on the context's stream (ppf_set_stream); they
 *    do not synchronise unless stated.  One context per device per host
 *    thread; a context is not re-entrant.
 *  - Return codes: PPF_OK (0) or a negative PPF_ERR_*; ppf_last_error()
 *    describes the last failure.  Per-subint solver status follows scipy's
 *    trust-ncg codes (0 gradient small / NaN, 1 maxiter, 2 no predicted
 *    reduction, 3 linalg error), as returned by the reference's
 *    results.status (pptoaslib.py:1018).
 *  - Shapes (PPF_ERR_UNSUPPORTED with a message outside them, never a
 *    silent fallback): nbin in [16, 8192] and nchan <= PPF_MAX_NCHAN (the
 *    reference takes any; 16384 channels covers every receiver in use).
 *    The FFT kernels are built per power of two; for any other nbin (the
 *    reference's numpy rfft takes any length, pptoaslib.py:976-978)
 *    ppf_fit_portrait_batch, ppf_rotate_rows, ppf_scatter_rotate_rows,
 *    ppf_gaussian_portraits, ppf_spline_portraits,
 *    ppf_instrumental_response_rows, ppf_phase_shift_batch,
 *    ppf_rotate_accumulate, ppf_irfft_rows, ppf_noise_rows and
 *    ppf_resid_chi2_rows run direct-sum kernels instead (O(nbin^2) per row;
 *    tests/test_gpu_generic_nbin.py), and so do the data-spectrum cache
 *    (PPF_SPEC_*, ppf_spec_nhp, ppf_rotate_accumulate_spec) and
 *    ppf_synth_portraits: every entry point takes any nbin in [16, 8192]
 *    (powers of two below 64 take the generic kernels too).
 *  - Channel counts: up to PPF_LDS_NCHAN a fit workgroup keeps its subint's
 *    per-channel tables (frequencies, weights, dispersion derivatives, the
 *    fitted-channel list) in LDS; above it (or under PPF_OPT_HBM_TABLES) the
 *    same kernels, instantiated for it, keep them in an HBM workspace slice
 *    per workgroup, and scattering fits take one workgroup per subint
 *    (PPF_OPT_SCAT_SPLIT is not used).  The fits are bitwise the same either
 *    way (tests/test_gpu_wide.py); only their speed differs.
 */
#ifndef PPFIT_H
#define PPFIT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PPF_OK 0
#define PPF_ERR_INVALID -1
#define PPF_ERR_DEVICE -2
#define PPF_ERR_UNSUPPORTED -3
#define PPF_ERR_NOMEM -4

#define PPF_MAX_NCHAN 16384
#define PPF_LDS_NCHAN 2048
#define PPF_VERSION 1

/* kernel ids for ppf_get_kernel_time */
#define PPF_K_MODEL_FFT 0
#define PPF_K_DATA_XSPEC 1
#define PPF_K_SOLVE 2
#define PPF_K_PHASE_SHIFT 3
#define PPF_K_ROTATE 4
#define PPF_K_ROT_ACCUM 5
#define PPF_K_SYNTH 6
#define PPF_K_IRFFT 7
#define PPF_K_NOISE 8
#define PPF_K_GUESS 9
#define PPF_K_POST 10
#define PPF_K_FIT_TAYLOR 11
#define PPF_K_MOMENTS 12
#define PPF_K_RESID 13
#define PPF_K_UNPACK 14
#define PPF_NUM_KERNELS 15

typedef struct ppf_ctx ppf_ctx;

int ppf_version(void);
int ppf_ctx_create(int device, ppf_ctx** out);
void ppf_ctx_destroy(ppf_ctx* ctx);
const char* ppf_last_error(const ppf_ctx* ctx);
/* hip stream (hipStream_t cast to void*); NULL selects the null stream */
int ppf_set_stream(ppf_ctx* ctx, void* stream);
int ppf_synchronize(ppf_ctx* ctx);
/* Phase-family fits (trust-ncg, no tau/alpha) split each workspace chunk
 * into `pieces` launches alternating between the context stream and a
 * second internal queue, piece p's data pass ordered after piece p-1's, so
 * one piece's latency-bound solver kernels overlap the next one's HBM-bound
 * pass.  Results are bitwise those of pieces = 1.  0 = the library default
 * (1: measured no faster); at most 64.                        */
int ppf_set_pipeline(ppf_ctx* ctx, int32_t pieces);
/* Launch-schedule options of one context (diagnostic / A-B use; the
 * library reads no environment variables).  None of them changes a
 * result: every setting gives bitwise the same fits (tests/test_gpu_options.py).
 *   PPF_OPT_SCAT_GRAPH   1: the split scattering solve launches each group of
 *                        four iterations as one hipGraph (default); 0: one
 *                        launch per kernel.
 *   PPF_OPT_SCAT_SPLIT   1: trust-ncg scattering fits spread every evaluation
 *                        over several workgroups (k_scat_sweep/k_scat_step,
 *                        default); 0: one workgroup per subint (k_solve).
 *   PPF_OPT_SCAT_TAIL    running subints below which the split solve takes
 *                        one 8-channel group per wave (default 512; 0 never).
 *   PPF_OPT_FUSE_MOMENTS 1: the first Taylor moment pass runs inside
 *                        k_fit_taylor (default); 0: its own k_moments launch.
 *   PPF_OPT_GUESS_WAVE   1: the single-wave guess kernel takes the subints it
 *                        covers (default); 0: every guess in k_guess.
 *   PPF_OPT_HBM_TABLES   1: the per-channel tables in HBM at every channel
 *                        count (default 0: only above PPF_LDS_NCHAN).       */
#define PPF_OPT_SCAT_GRAPH 0
#define PPF_OPT_SCAT_SPLIT 1
#define PPF_OPT_SCAT_TAIL 2
#define PPF_OPT_FUSE_MOMENTS 3
#define PPF_OPT_GUESS_WAVE 4
#define PPF_OPT_HBM_TABLES 5
#define PPF_NUM_OPTS 6
int ppf_set_option(ppf_ctx* ctx, int32_t option, int32_t value);
int ppf_get_option(const ppf_ctx* ctx, int32_t option, int32_t* value);
/* Upper bound on workspace bytes the context may hold (default 32 GiB). */
int ppf_set_workspace_limit(ppf_ctx* ctx, int64_t bytes);
/* Per-kernel HIP-event timing on the context stream (off by default). */
int ppf_set_timing(ppf_ctx* ctx, int enable);
/* Diagnostic: record every objective sweep of the TNC and Newton-CG solvers
 * and of the split trust-ncg scattering solve (the point, f, gradient,
 * Hessian terms, whether it counts in nfev) into buf [nsub][cap][32]
 * doubles (device memory, caller-owned; batch subint index), at most cap
 * sweeps per subint.  cap 0 turns it off.  Split scattering records also
 * hold, in fields 28-31, the trust radius after the evaluation's update,
 * the predicted reduction and rho of the step that led to it, and its
 * Steihaug boundary flag.                                                 */
int ppf_set_trace(ppf_ctx* ctx, double* buf, int32_t cap);
int ppf_get_kernel_time(ppf_ctx* ctx, int kernel_id, double* total_ms,
                        int64_t* launches);
int ppf_reset_kernel_times(ppf_ctx* ctx);
/* Device self-test of the cross-lane primitives the kernels rely on
 * (DPP row/quad moves, permlane16/32 swaps, readlane).  fails[t] (t <
 * PPF_SELFTEST_N) = number of lanes where test t is wrong; all 0 = pass.   */
#define PPF_SELFTEST_N 10
int ppf_selftest(ppf_ctx* ctx, int32_t* fails);
/* Diagnostic phase clock of the Taylor fit kernel (off by default).  When
 * enabled, every k_fit_taylor workgroup adds its wall_clock64 ticks (100 MHz)
 * per phase into device counters: out[0] guess, [1] meta + first moments,
 * [2] centre selection incl. recentring, [3] objective sweeps, [4] trust-
 * region step, [8] recentring passes, [9] workgroups; every k_post
 * workgroup likewise: [16] meta + Sd, [17] nu_zero sums and solve, [18]
 * outputs at nu_out + centre pick, [19] with-scales sweep, [20] inverses,
 * [21] per-channel errors + stores, [22] workgroups.  The call copies the
 * counters to out (if non-null), zeroes them and sets the enable state.   */
#define PPF_PHASE_N 32
int ppf_phase_profile(ppf_ctx* ctx, int32_t enable, uint64_t* out);

/* ---------------------------------------------------------------------- */
/* Batched wideband fit: fit_portrait_full over nsub subints.              */
/* ---------------------------------------------------------------------- */
/* minimize() method of fit_portrait_full (pptoaslib.py:995-1014)          */
#define PPF_METHOD_TRUST_NCG 0   /* scipy trust-ncg, gtol = -1 (the default)  */
#define PPF_METHOD_TNC 1         /* scipy TNC with bounds, xtol 1e-10, minfev */
#define PPF_METHOD_NEWTON_CG 2   /* scipy Newton-CG, xtol = -1, maxiter 2000   */
#define PPF_METHOD_TNC_LEGACY 3  /* pplib.fit_portrait: TNC over (phase, DM) only,
                                    xtol 1e-10 (pplib.py:2144-2148); fit_flags
                                    must be [1,1,0,0,0]                        */

/* Phase-family fits (tau = 0 and not fitted) evaluate the objective from
 * per-channel Taylor moments of the cross-spectrum (no nchan x nharm
 * workspace).  PPF_SOLVE_EXACT forces the exact cross-spectrum sweeps
 * instead (same results to rounding; used to cross-check the two).
 * PPF_SOLVE_EVAL evaluates f, g, H and the post-fit at init without any
 * solver step (status 1, nfev 1): the objective-kernel parity hook for
 * fit_portrait_full_function{,_deriv,_2deriv} (pptoaslib.py:525-643).
 * PPF_GUESS_DIRECT takes the brute-force grid of the initial guess by
 * direct sums instead of the folded L-point DFT.                          */
#define PPF_SOLVE_EXACT 1
#define PPF_SOLVE_EVAL 2
#define PPF_GUESS_DIRECT 4

/* Data-spectrum cache (spec_mode; ppalign's iterations, ppalign.py:160-213,
 * refit the same subints against each new template).  The cache is the
 * caller's: spec [nsub][nchan][NHP] complex (interleaved re, im; NHP =
 * ppf_spec_nhp(nbin)), spec_sig and spec_dsum [nsub][nchan], spec_R
 * [nsub][NHP] complex.
 *   PPF_SPEC_STORE: the data pass also stores each subint's spectrum (rfft
 *     of the row, DC included), noise sigma, sum |D|^2 / sigma^2 and guess
 *     average in the cache (every other output as without the cache);
 *   PPF_SPEC_USE: no data pass -- those come from the cache, and the Taylor
 *     moment passes form the cross-spectrum D conj(M) from the cached
 *     spectrum as they stream it: the same X, bitwise, so the same fits.
 *     Only phase-family trust-ncg fits (tau = 0, not fitted; not
 *     PPF_SOLVE_EXACT) take it, with the data, freqs, errs, mask, weights, P
 *     and guess_nu of the STORE call.                                    */
#define PPF_SPEC_NONE 0
#define PPF_SPEC_STORE 1
#define PPF_SPEC_USE 2
int32_t ppf_spec_nhp(int32_t nbin);

typedef struct {
  int32_t nsub, nchan, nbin, nmodel;
  int32_t fit_flags[5];   /* phi, DM, GM, tau, alpha (pptoaslib.py:928)     */
  int32_t log10_tau;      /* fit log10(tau) instead of tau                 */
  int32_t option;         /* get_nu_zeros option (pptoaslib.py:733)        */
  int32_t method;         /* PPF_METHOD_*                                   */
  int32_t is_toa;         /* pptoaslib.py:1048-1050                         */
  int32_t guess;          /* 1: in-kernel initial phase guess (pptoas.py:420-456) */
  int32_t guess_Ns;       /* opt.brute grid size (100 in pptoas, nbin in ppalign) */
  int32_t guess_wrap;     /* 1: phase_transform(..., mod=True) to nu_fit_DM */
  int32_t solver_flags;   /* PPF_SOLVE_* bits (0 = default)                */
  const double* data;       /* [nsub][nchan][nbin]                          */
  const double* model;      /* [nmodel][nchan][nbin]                        */
  const int32_t* model_idx; /* [nsub] or NULL (all 0)                       */
  const double* freqs;      /* [nsub][nchan] MHz                            */
  const double* errs;       /* [nsub][nchan] time-domain sigma; NULL or a NaN
                               entry: estimated as get_noise_PS (pplib.py:2227) */
  const uint8_t* chan_mask; /* [nsub][nchan] 1 = fit channel, or NULL       */
  const double* weights;    /* [nsub][nchan] guess-average weights or NULL  */
  const double* P;          /* [nsub] period, s                             */
  const double* init;       /* [nsub][5] initial params                     */
  const double* nu_fit;     /* [nsub][3] NaN -> mean of fitted freqs        */
  const double* nu_out;     /* [nsub][3] NaN -> zero-covariance frequency   */
  const double* guess_nu;   /* [nsub] dedispersion ref of the guess; NaN ->
                               mean freq (pptoas) ; NULL -> NaN             */
  const double* guess_tau;  /* [nsub] linear tau [rot] at nu_fit_tau applied
                               to the guess template, or NULL (0)           */
  const double* bounds;     /* HOST pointer, [5][2] (low, high) per parameter
                               for the whole batch, NaN = None; read by
                               PPF_METHOD_TNC only (NULL = all None)        */
  int32_t spec_mode;        /* PPF_SPEC_* (data-spectrum cache, above)       */
  double* spec;             /* [nsub][nchan][NHP] complex, or NULL            */
  double* spec_sig;         /* [nsub][nchan]                                  */
  double* spec_dsum;        /* [nsub][nchan]                                  */
  double* spec_R;           /* [nsub][NHP] complex                            */
} ppf_fit_desc;

typedef struct {
  double* params;       /* [nsub][5] (phi at nu_DM, DM, GM, tau(log10?), alpha) */
  double* param_errs;   /* [nsub][5]                                        */
  double* nu_out;       /* [nsub][3] nu_DM, nu_GM, nu_tau                  */
  double* cov;          /* [nsub][5][5] nfit x nfit block top-left           */
  double* scales;       /* [nsub][nchan] (0 on masked channels)             */
  double* scale_errs;   /* [nsub][nchan]                                    */
  double* channel_snrs; /* [nsub][nchan]                                    */
  double* chi2;         /* [nsub]                                           */
  double* red_chi2;     /* [nsub]                                           */
  double* snr;          /* [nsub]                                           */
  int32_t* nfev;        /* [nsub]                                           */
  int32_t* status;      /* [nsub]                                           */
  double* init_used;    /* [nsub][5] or NULL: starting point after the guess */
  double* fun;          /* [nsub] or NULL: final objective value            */
  double* cov_nosc;     /* [nsub][5][5] or NULL: inv(0.5 H) of the curvature
                           without amplitude terms at the output params
                           (legacy pplib.fit_portrait errors, pplib.py:2184-2190) */
  double* grad;         /* [nsub][5] or NULL: gradient at the final point (jac) */
  double* hess;         /* [nsub][5][5] or NULL: Hessian at the final point     */
  double* errs_out;     /* [nsub][nchan] or NULL: the time-domain noise sigma
                           each channel was fitted with -- desc->errs, or
                           get_noise_PS of the row where that is NULL / NaN
                           (pplib.py:2227-2253); 0 for masked channels.  Lets
                           a caller weight by load_data's noise_stds without
                           a separate noise pass (ppalign.py:202-208)      */
} ppf_fit_result;

int ppf_fit_portrait_batch(ppf_ctx* ctx, const ppf_fit_desc* desc,
                           const ppf_fit_result* out);

/* ---------------------------------------------------------------------- */
/* fit_phase_shift over nprof profiles (pplib.py:2054-2100).              */
/* out[nprof][6] = phase, phase_err, scale, scale_err, snr, red_chi2       */
/* noise: [nprof] time-domain sigma or NaN/NULL -> get_noise (PS)          */
/* ---------------------------------------------------------------------- */
int ppf_phase_shift_batch(ppf_ctx* ctx, int32_t nprof, int32_t nbin,
                          const double* data, const double* model,
                          const int32_t* model_idx, const double* noise,
                          int32_t Ns, double lo, double hi, double* out);

/* out[r] = irfft(rfft(in[r]) * exp(2 pi i k phase[r]))  (rotate_data)     */
int ppf_rotate_rows(ppf_ctx* ctx, int32_t nrow, int32_t nbin, const double* in,
                    const double* phase, double* out);

/* accum[n][k] += sum_s weight[s][n] * rfft(data[s][n])[k] * e^{2 pi i k phase[s][n]}
 * accum is complex [nchan][nbin/2+1] interleaved (re, im); weight 0 skips.  */
int ppf_rotate_accumulate(ppf_ctx* ctx, int32_t nsub, int32_t nchan,
                          int32_t nbin, const double* data, const double* phase,
                          const double* weight, double* accum);
/* The same sum from cached spectra (PPF_SPEC_STORE's spec, [nsub][nchan][NHP]
 * complex): no FFT, one pass over the spectra.  Rows of channels the fit
 * masked hold zeros (give them weight 0, as ppalign does).               */
int ppf_rotate_accumulate_spec(ppf_ctx* ctx, int32_t nsub, int32_t nchan,
                               int32_t nbin, const double* spec, const double* phase,
                               const double* weight, double* accum);

/* Gaussian-component template rows (gen_gaussian_portrait, pplib.py:853-930,
 * as read_model calls it, pplib.py:2873-2959): out[r][:] at freqs[r] for
 * nrow rows (portraits x channels, any mix of frequencies).  code: HOST
 * int32[3], the evolution of loc / wid / amp (0 power law, 1 linear:
 * evolve_parameter, pplib.py:1030-1046); params: HOST double[2 + 6 ngauss],
 * DC, TAU [bin] (read_model's TAU * nbin / P), then per component loc,
 * dloc, wid, dwid, amp, damp; ngauss <= 32.  TAU != 0 scatters row r by
 * TAU / nbin (freqs[r] / nu_ref)^alpha.  out may not alias freqs.        */
int ppf_gaussian_portraits(ppf_ctx* ctx, int32_t nrow, int32_t nbin, int32_t ngauss,
                           const int32_t* code, const double* params, double nu_ref,
                           double alpha, const double* freqs, double* out);

/* B-spline (PCA) template rows (gen_spline_portrait, pplib.py:932-956, as
 * read_spline_model builds them, pplib.py:2961-2993): row r at freqs[r] is
 * mean_prof + sum_e splev(freqs[r], (t, c[e], k), ext=0) eigvec[:, e]
 * (FITPACK splev / fpbspl); neig == 0 tiles mean_prof.  When nbin_in !=
 * nbin the rows are resampled as scipy.signal.resample (rfft branch) and
 * rotated by 0.5 (1/nbin - 1/nbin_in) (rotate_portrait), both then in
 * [16, 8192].  t HOST [nknot], c HOST [neig][ncoef] (ncoef >=
 * nknot - k - 1), 1 <= k <= 5, neig <= 64; mean_prof [nbin_in], eigvec
 * [nbin_in][neig], freqs [nrow], out [nrow][nbin] on the device.          */
int ppf_spline_portraits(ppf_ctx* ctx, int32_t nrow, int32_t nbin_in, int32_t nbin, int32_t neig,
                         const double* mean_prof, const double* eigvec, int32_t nknot, int32_t k,
                         const double* t, const double* c, int32_t ncoef, const double* freqs,
                         double* out);

/* Instrumental-response convolution of template rows (get_TOAs with
 * add_instrumental_response, pptoas.py:387-393): out[r] = irfft(R_r *
 * rfft(in[r])) with R = instrumental_response_port_FT(nbin, freqs, DM, P,
 * wids, irf_types) (pptoaslib.py:145-179): the product over nw responses
 * (types HOST [nw]: 0 'rect' np.sinc(k wid), 1 'gauss' the normalised
 * Gaussian FT of FWHM wid [rot] <= 0.1388; wids HOST [nw], > 0) and, when
 * DM != 0, 'rect' of width 8.3e-6 chan_bw / (freqs[r] / 1e3)^3 / P (the
 * reference's formula: DM only switches it on).  chan_bw is the caller's
 * |freqs[1] - freqs[0]|.  in NULL: out receives R itself [nrow][nbin/2+1]. */
int ppf_instrumental_response_rows(ppf_ctx* ctx, int32_t nrow, int32_t nbin, const double* in,
                                   int32_t nw, const double* wids, const int32_t* types,
                                   double DM, double chan_bw, double P, const double* freqs,
                                   double* out);

/* tscrunch (load_data's arch.tscrunch(), pplib.py:2700) of fold-mode
 * subints: out[p][n][j] = sum_s w[s][n] data[s][p][n][j] / sum_s w[s][n]
 * (0 where the weights sum to 0), wsum[n] = sum_s w[s][n] (NULL: not
 * written).  data [nsub][npol][nchan][nbin], weights [nsub][nchan].      */
int ppf_tscrunch(ppf_ctx* ctx, int32_t nsub, int32_t npol, int32_t nchan, int32_t nbin,
                 const double* data, const double* weights, double* out, double* wsum);

/* PSRFITS samples to physical values (PSRCHIVE's load + pscrunch in
 * load_data, pplib.py:2670-2732): raw [nsub][npol][nchan][nbin] of
 * raw_type (ppfits.h PPFITS_RAW_*: 1 uint8, 2 int16, 3 float32), scl and
 * offs [nsub][npol][nchan] (DAT_SCL, DAT_OFFS); value = raw * scl + offs.
 * pmode 0 keeps every polarisation, 1 sums the first two (AA + BB), 2 takes
 * the first (Stokes I); out [nsub][pmode ? 1 : npol][nchan][nbin].        */
int ppf_unpack_subints(ppf_ctx* ctx, int32_t nsub, int32_t npol, int32_t nchan, int32_t nbin,
                       int32_t raw_type, const void* raw, const double* scl, const double* offs,
                       int32_t pmode, double* out);

/* remove_baseline in place (load_data's arch.remove_baseline(),
 * pplib.py:2691; PSRCHIVE Integration::remove_baseline with its default
 * estimator): per subint s the total-intensity profile
 *   t[j] = sum_{n: w[s][n] != 0} w[s][n] sum_{p < ntot} data[s][p][n][j]
 * gives the off-pulse window [j0, j0 + width) (circular) of smallest sum,
 * first on ties; every profile data[s][p][n] then has its mean over that
 * window subtracted.  data [nsub][npol][nchan][nbin] (nbin <= 8192),
 * weights [nsub][nchan]; window [nsub] receives j0 (NULL: not written).
 * Callers pass width = floor(0.15 nbin), PSRCHIVE's default duty cycle.   */
int ppf_remove_baseline(ppf_ctx* ctx, int32_t nsub, int32_t npol, int32_t nchan, int32_t nbin,
                        int32_t ntot, int32_t width, double* data, const double* weights,
                        int32_t* window);

/* Per-profile S/N, load_data's SNRs[isub, ipol, ichan] =
 * Profile::snr() (pplib.py:2762-2770; get_TOAs weights guess_fit_freq with
 * them, pptoas.py:401).  Restated from PSRCHIVE's default "phase" S/N
 * estimator (PSRCHIVE is not in this image: PARITY UNPINNED):
 *   off-pulse window: the circular run of `width` bins with the smallest
 *     sum (first on ties; windows summed bin by bin from their start);
 *   m, v: mean and sample variance (n - 1) over that window;
 *   edges (cumulative-power peak): with y the profile minus m read
 *     circularly from the bin after the window, c its running sum and
 *     C = c[nbin - 1], rise = the first bin with c >= threshold C, fall =
 *     the first with c >= (1 - threshold) C;
 *   snr = (c[fall] - c[rise] + y[rise]) / sqrt(fall - rise + 1) / sqrt(v),
 *     0 when C <= 0 or v <= 0.
 * rows [nrow][nbin] (nbin <= 8192), out [nrow].  Callers pass width =
 * floor(0.15 nbin) and threshold 0.1.                                      */
int ppf_profile_snr(ppf_ctx* ctx, int32_t nrow, int32_t nbin, const double* rows, int32_t width,
                    double threshold, double* out);

/* out[r] = irfft(rfft(in[r]) e^{2 pi i k phase[r]} / (1 + 2 pi i k tau[r]))
 * (rotate_portrait_full of a scattered template, pptoas.py:1389-1397);
 * tau NULL = no scattering.                                              */
int ppf_scatter_rotate_rows(ppf_ctx* ctx, int32_t nrow, int32_t nbin, const double* in,
                            const double* phase, const double* tau, double* out);

/* Per-channel reduced chi2 of a fitted portrait, get_red_chi2 as
 * GetTOAs.get_channels_to_zap calls it (pplib.py:727-749, pptoas.py:1233):
 *   port  = irfft(rfft(data[r]) e^{2 pi i k phase[r]})
 *   model = scale[r] irfft(rfft(model[mrow]) / (1 + 2 pi i k tau[r]))
 *   out[r] = sum_j ((port_j - model_j) / errs[r])^2 / dof
 * evaluated in the Fourier domain (Parseval); mrow = model_row[r] (or r
 * when NULL), phase NULL = 0, tau NULL = no scattering.                  */
int ppf_resid_chi2_rows(ppf_ctx* ctx, int32_t nrow, int32_t nbin, const double* data,
                        const double* phase, const double* model, const int32_t* model_row,
                        const double* scale, const double* tau, const double* errs,
                        double dof, double* out);

/* out[r] = irfft(spec[r]) where spec is complex [nrow][nbin/2+1]           */
int ppf_irfft_rows(ppf_ctx* ctx, int32_t nrow, int32_t nbin, const double* spec,
                   double* out);

/* out[r] = get_noise_PS(in[r]) (frac=4)                                   */
int ppf_noise_rows(ppf_ctx* ctx, int32_t nrow, int32_t nbin, const double* in,
                   double* out);

/* data[s][n] = irfft(rfft(model[n]) * e^{2 pi i k phase[s][n]})
 *              + sigma * N(0,1)[Philox4x32-10(seed; bin pair, n, s + sub0)] */
int ppf_synth_portraits(ppf_ctx* ctx, int32_t nsub, int32_t nchan, int32_t nbin,
                        const double* model, const double* phase, double sigma,
                        uint64_t seed, int64_t sub0, double* data);

#ifdef __cplusplus
}
#endif
#endif /* PPFIT_H */
