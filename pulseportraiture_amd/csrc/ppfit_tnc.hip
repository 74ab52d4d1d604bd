// ppfit_tnc.hip -- scipy's TNC (truncated-Newton, bound-constrained) on the device.
//
// fit_portrait_full(method='TNC') minimizes the wideband objective with
// scipy.optimize.minimize(..., method='TNC', jac=..., bounds=bounds,
// options={'xtol': 1e-10, 'minfev': dof - Sd}) (pptoaslib.py:995-1014), and
// the legacy pplib.fit_portrait minimizes the phase+DM objective the same way
// with xtol 1e-10 (pplib.py:2144-2148).  scipy's TNC is J.-S. Roy's tnc.c
// (v1.3, after S. Nash's TN); tools/tnc_model.py restates it and
// tests/test_tnc_model.py holds that restatement to scipy's compiled module
// point for point.  This file follows tools/tnc_model.py function for
// function, with the same operations in the same order (FP contraction off),
// so a trajectory driven by the same f and g values is the same.
//
// One workgroup per subint.  Every thread runs the (scalar, uniform) TNC
// control flow on its own register copy of the state; each objective
// evaluation is one block-wide sweep over the subint's cross-spectrum
// (sweep<0, SCAT> in ppfit_fit.hip: f and the masked gradient, as
// fit_portrait_full_function{,_deriv}, pptoaslib.py:525-574).  scipy's
// ScalarFunction re-evaluates only when x changes, and nfev counts those
// evaluations; the device does the same.
#include "ppfit_kernels.hpp"

namespace ppf {

namespace tnc {

constexpr int NMAX = 5;
constexpr double EPSM = 2.220446049250313e-16;  // DBL_EPSILON
enum { GETPTC_OK = 0, GETPTC_EVAL = 1, GETPTC_EINVAL = 2, GETPTC_FAIL = 3 };
enum { LS_OK = 0, LS_MAXFUN = 1, LS_FAIL = 2 };

__device__ __forceinline__ double dnrm2(int n, const double* v) {
#pragma clang fp contract(off)
  double dssq = 1.0, scale = 0.0;
#pragma unroll
  for (int i = 0; i < NMAX; ++i) {
    if (i >= n) break;
    const double x = v[i];
    if (x != 0.0) {
      const double ax = fabs(x);
      if (scale < ax) {
        const double ratio = scale / ax;
        dssq = 1.0 + dssq * ratio * ratio;
        scale = ax;
      } else {
        const double ratio = ax / scale;
        dssq += ratio * ratio;
      }
    }
  }
  return scale * sqrt(dssq);
}

__device__ __forceinline__ double ddot(int n, const double* a, const double* b) {
#pragma clang fp contract(off)
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NMAX; ++i)
    if (i < n) s += a[i] * b[i];
  return s;
}

// getptc state (linearSearch / getptcInit / getptcIter)
struct Ptc {
  double reltol, abstol, u, fu, gu, xmin, fmin, gmin, xw, fw, gw, a, b, oldf, b1, scxbnd, e,
      step, factor, gtest1, gtest2, tol, rmu;
  bool braktd;
};

__device__ int getptc_init(Ptc& S, double tnytol, double eta, double xbnd) {
#pragma clang fp contract(off)
  if (S.u <= 0.0 || xbnd <= tnytol || S.gu > 0.0) return GETPTC_EINVAL;
  if (xbnd < S.abstol) S.abstol = xbnd;
  S.tol = S.abstol;
  S.a = 0.0;
  S.xw = 0.0;
  S.xmin = 0.0;
  S.oldf = S.fu;
  S.fmin = S.fu;
  S.fw = S.fu;
  S.gw = S.gu;
  S.gmin = S.gu;
  S.step = S.u;
  S.factor = 5.0;
  S.braktd = false;
  S.scxbnd = xbnd;
  S.b = S.scxbnd + S.reltol * fabs(S.scxbnd) + S.abstol;
  S.e = S.b + S.b;
  S.b1 = S.b;
  S.gtest1 = -S.rmu * S.gu;
  S.gtest2 = -eta * S.gu;
  if (S.step >= S.scxbnd) {
    S.step = S.scxbnd;
    S.scxbnd -= (S.reltol * fabs(xbnd) + S.abstol) / (1.0 + S.reltol);
  }
  S.u = S.step;
  if (fabs(S.step) < S.tol && S.step < 0.0) S.u = -S.tol;
  if (fabs(S.step) < S.tol && S.step >= 0.0) S.u = S.tol;
  return GETPTC_EVAL;
}

__device__ int getptc_iter(Ptc& S, double big, double rtsmll, double tnytol, double fpresn,
                           double xbnd) {
#pragma clang fp contract(off)
  double u = S.u, fu = S.fu, gu = S.gu;
  bool to_conv = false;
  if (fu <= S.fmin) {
    const double chordu = S.oldf - (S.xmin + u) * S.gtest1;
    if (!(fu <= chordu)) {
      const double chordm = S.oldf - S.xmin * S.gtest1;
      gu = -S.gmin;
      double denom = chordm - S.fmin;
      if (fabs(denom) < 1e-15) {
        denom = 1e-15;
        if (chordm - S.fmin < 0.0) denom = -denom;
      }
      if (S.xmin != 0.0) gu = S.gmin * (chordu - fu) / denom;
      fu = 0.5 * u * (S.gmin + gu) + S.fmin;
      if (fu < S.fmin) fu = S.fmin;
    } else {
      S.fw = S.fmin;
      S.fmin = fu;
      S.gw = S.gmin;
      S.gmin = gu;
      S.xmin += u;
      S.a -= u;
      S.b -= u;
      S.xw = -u;
      S.scxbnd -= u;
      if (gu <= 0.0) {
        S.a = 0.0;
      } else {
        S.b = 0.0;
        S.braktd = true;
      }
      S.tol = fabs(S.xmin) * S.reltol + S.abstol;
      to_conv = true;
    }
  }
  if (!to_conv) {
    if (u < 0.0) {
      S.a = u;
    } else {
      S.b = u;
      S.braktd = true;
    }
    S.xw = u;
    S.fw = fu;
    S.gw = gu;
  }
  S.u = u;
  S.fu = fu;
  S.gu = gu;
  // ConvergenceCheck
  double twotol = S.tol + S.tol;
  const double xmidpt = 0.5 * (S.a + S.b);
  const bool convrg = (fabs(xmidpt) <= twotol - 0.5 * (S.b - S.a)) ||
                      (fabs(S.gmin) <= S.gtest2 && S.fmin < S.oldf &&
                       ((fabs(S.xmin - xbnd) > S.tol) || !S.braktd));
  if (convrg) {
    if (S.xmin != 0.0) return GETPTC_OK;
    if (fabs(S.oldf - S.fw) <= fpresn) return GETPTC_FAIL;
    S.tol = 0.1 * S.tol;
    if (S.tol < tnytol) return GETPTC_FAIL;
    S.reltol = 0.1 * S.reltol;
    S.abstol = 0.1 * S.abstol;
    twotol = 0.1 * twotol;
  }
  double r = 0.0, q = 0.0, s = 0.0;
  bool minimum_found = false;
  if (fabs(S.e) > S.tol) {
    r = 3.0 * (S.fmin - S.fw) / S.xw + S.gmin + S.gw;
    const double absr = fabs(r);
    q = absr;
    if (S.gw != 0.0 && S.gmin != 0.0) {
      const double abgw = fabs(S.gw);
      const double abgmin = fabs(S.gmin);
      s = sqrt(abgmin) * sqrt(abgw);
      if ((S.gw / abgw) * S.gmin > 0.0) {
        if (r >= s || r <= -s) {
          q = sqrt(fabs(r + s)) * sqrt(fabs(r - s));
        } else {
          r = 0.0;
          q = 0.0;
          minimum_found = true;
        }
      } else {
        double sumsq = 1.0, p = 0.0, scale;
        if (absr >= s) {
          if (absr > rtsmll) p = absr * rtsmll;
          if (s >= p) {
            const double value = s / absr;
            sumsq = 1.0 + value * value;
          }
          scale = absr;
        } else {
          if (s > rtsmll) p = s * rtsmll;
          if (absr >= p) {
            const double value = absr / s;
            sumsq = 1.0 + value * value;
          }
          scale = s;
        }
        sumsq = sqrt(sumsq);
        q = big;
        if (scale < big / sumsq) q = scale * sumsq;
      }
    }
    if (!minimum_found) {
      if (S.xw < 0.0) q = -q;
      s = S.xw * (S.gmin - r - q);
      q = S.gw - S.gmin + q + q;
      if (q > 0.0) s = -s;
      if (q <= 0.0) q = -q;
      r = S.e;
      if (S.b1 != S.step || S.braktd) S.e = S.step;
    }
  }
  // MinimumFound
  double a1 = S.a;
  S.b1 = S.b;
  S.step = xmidpt;
  if (!S.braktd || ((S.a == 0.0 && S.xw < 0.0) || (S.b == 0.0 && S.xw > 0.0))) {
    if (S.braktd) {
      const double d1 = S.xw;
      double d2 = S.a;
      if (S.a == 0.0) d2 = S.b;
      S.u = -d1 / d2;
      S.step = 5.0 * d2 * (0.1 + 1.0 / S.u) / 11.0;
      if (S.u < 1.0) S.step = 0.5 * d2 * sqrt(S.u);
    } else {
      S.step = -S.factor * S.xw;
      if (S.step > S.scxbnd) S.step = S.scxbnd;
      if (S.step != S.scxbnd) S.factor = 5.0 * S.factor;
    }
    if (S.step <= 0.0) a1 = S.step;
    if (S.step > 0.0) S.b1 = S.step;
  }
  if (fabs(s) <= fabs(0.5 * q * r) || s <= q * a1 || s >= q * S.b1) {
    S.e = S.b - S.a;
  } else {
    S.step = s / q;
    if (S.step - S.a < twotol || S.b - S.step < twotol) {
      if (xmidpt <= 0.0) S.step = -S.tol;
      else S.step = S.tol;
    }
  }
  if (S.step >= S.scxbnd) {
    S.step = S.scxbnd;
    S.scxbnd -= (S.reltol * fabs(xbnd) + S.abstol) / (1.0 + S.reltol);
  }
  S.u = S.step;
  if (fabs(S.step) < S.tol && S.step < 0.0) S.u = -S.tol;
  if (fabs(S.step) < S.tol && S.step >= 0.0) S.u = S.tol;
  return GETPTC_EVAL;
}

__device__ __forceinline__ double initial_step(double fnew, double fmin, double gtp,
                                               double smax) {
#pragma clang fp contract(off)
  const double d = fabs(fnew - fmin);
  double alpha = 1.0;
  if (d * 2.0 <= -gtp && d >= EPSM) alpha = d * 2.0 / -gtp;
  if (alpha >= smax) alpha = smax;
  return alpha;
}

__device__ __forceinline__ void ssbfgs(int n, double gamma, const double* sj, const double* hjv,
                                       const double* hjyj, double yjsj, double yjhyj, double vsj,
                                       double vhyj, double* out) {
#pragma clang fp contract(off)
  double delta, beta;
  if (yjsj == 0.0) {
    delta = 0.0;
    beta = 0.0;
  } else {
    delta = (gamma * yjhyj / yjsj + 1.0) * vsj / yjsj - gamma * vhyj / yjsj;
    beta = -gamma * vsj / yjsj;
  }
  double t[NMAX];
#pragma unroll
  for (int i = 0; i < NMAX; ++i)
    if (i < n) t[i] = gamma * hjv[i] + delta * sj[i] + beta * hjyj[i];
#pragma unroll
  for (int i = 0; i < NMAX; ++i)
    if (i < n) out[i] = t[i];
}

}  // namespace tnc

// The whole TNC state of one subint (every thread holds an identical copy).
struct TncState {
  int n;
  double low[5], up[5], xscale[5], xoffset[5];
  int pivot[5];
  double diagb[5], sk[5], yk[5], sr[5], yr[5];
  double yksk, yrsr, fscale, accuracy;
  int maxCGit, maxfun, nfeval;
  bool upd1, lreset;
};

// Objective at an unscaled point: a block-wide sweep, skipped (and not
// counted) when the point equals the previous one, as scipy's
// ScalarFunction does.
struct TncObjective {
  const FitArgs* a;
  const Meta* m;
  int c, s;
  const double* refs;
  double P;
  double* acc_slot;
  double (*red)[48];
  double* out;   // LDS, >= 6 doubles
  double lastx[5], lastf, lastg[5];
  bool have;
  int nfev;      // scipy's nfev (distinct consecutive points)
  template <bool SCAT>
  __device__ void eval(int n, const double* x, double& f, double* g) {
    bool same = have;
#pragma unroll
    for (int i = 0; i < 5; ++i)
      if (i < n && x[i] != lastx[i]) same = false;
    if (!same) {
      double pr[5];  // identical in every thread
#pragma unroll
      for (int i = 0; i < 5; ++i) pr[i] = i < n ? x[i] : lastx[i];
      sweep<0, SCAT>(*a, *m, c, s, pr, refs, P, acc_slot, out, red, TaylorSrc{});
      trace_sweep(*a, s, nfev, pr, out, 6, true);
      lastf = out[0];
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        lastg[i] = out[1 + i];
        if (i < n) lastx[i] = x[i];
      }
      have = true;
      ++nfev;
      __syncthreads();  // out / prm are reused by the next evaluation
    }
    f = lastf;
#pragma unroll
    for (int i = 0; i < 5; ++i)
      if (i < n) g[i] = lastg[i];
  }
};

struct TncShared {
  double out[48];
  double red[kWaves][48];
  int nok;
};

template <bool SCAT, bool W>  // W: one copy per k_tnc instantiation (its only caller)
__device__ int tnc_run(TncState& T, TncObjective& O, double* x, double& f_out, double fmin,
                       double xtol) {
#pragma clang fp contract(off)
  using namespace tnc;
  const int n = T.n;
  auto project = [&](double* v) {
#pragma unroll
    for (int i = 0; i < NMAX; ++i)
      if (i < n && T.pivot[i] != 0) v[i] = 0.0;
  };
  auto unscalex = [&](double* v) {
#pragma unroll
    for (int i = 0; i < NMAX; ++i)
      if (i < n) v[i] = v[i] * T.xscale[i] + T.xoffset[i];
  };
  auto coercex = [&](double* v) {
#pragma unroll
    for (int i = 0; i < NMAX; ++i) {
      if (i >= n) continue;
      if (v[i] < T.low[i]) v[i] = T.low[i];
      else if (v[i] > T.up[i]) v[i] = T.up[i];
    }
  };
  auto scaleg = [&](double* v) {
#pragma unroll
    for (int i = 0; i < NMAX; ++i)
      if (i < n) v[i] *= T.xscale[i] * T.fscale;
  };
  auto fg = [&](const double* xu, double& fv, double* gv) {
    ++T.nfeval;
    O.template eval<SCAT>(n, xu, fv, gv);
  };
  // ---- tnc(): coherency, coercion, first evaluation, scaling ----
#pragma unroll
  for (int i = 0; i < NMAX; ++i)
    if (i < n && T.low[i] > T.up[i]) { f_out = NAN; return -1; }
  coercex(x);
  double f, gfull[5] = {0, 0, 0, 0, 0};
  fg(x, f, gfull);
  int nc = 0;
#pragma unroll
  for (int i = 0; i < NMAX; ++i)
    if (i < n && T.low[i] == T.up[i]) { x[i] = T.low[i]; ++nc; }
  if (nc == n) { f_out = f; return 5; }
#pragma unroll
  for (int i = 0; i < NMAX; ++i) {
    if (i >= n) continue;
    if (T.low[i] != -INFINITY && T.up[i] != INFINITY) {
      T.xscale[i] = T.up[i] - T.low[i];
      T.xoffset[i] = (T.up[i] + T.low[i]) * 0.5;
    } else {
      T.xscale[i] = 1.0 + fabs(x[i]);
      T.xoffset[i] = x[i];
    }
  }
  const double rteps = sqrt(EPSM);
  double stepmx = 1.0e1;  // stepmx 0 < rteps * 10
  const double eta = 0.25, rescale = 1.3;
  int maxCGit = n / 2;
  if (maxCGit < 1) maxCGit = 1;
  if (maxCGit > n) maxCGit = n;
  T.maxCGit = maxCGit;
  const double accuracy = rteps;
  T.accuracy = accuracy;
  const double ftol = accuracy;
  const double pgtol = 1e-2 * sqrt(accuracy);
  if (xtol < 0.0) xtol = rteps;
  // ---- tnc_minimize ----
  T.fscale = 1.0;
  double difnew = 0.0, epsred = 0.05;
  T.upd1 = true;
  int icycle = n - 1;
  bool newcon = true;
  T.lreset = false;
  T.yrsr = 0.0;
  T.yksk = 0.0;
#pragma unroll
  for (int i = 0; i < NMAX; ++i) {
    T.sk[i] = T.yk[i] = T.sr[i] = T.yr[i] = 0.0;
    T.pivot[i] = 0;
  }
  double alpha = 0.0;
#pragma unroll
  for (int i = 0; i < NMAX; ++i)  // scalex
    if (i < n && T.xscale[i] > 0.0) x[i] = (x[i] - T.xoffset[i]) / T.xscale[i];
  f *= T.fscale;
#pragma unroll
  for (int i = 0; i < NMAX; ++i) {  // setConstraints
    if (i >= n) continue;
    if (T.xscale[i] == 0.0) {
      T.pivot[i] = 2;
    } else if (T.low[i] != -INFINITY &&
               (x[i] * T.xscale[i] + T.xoffset[i] - T.low[i] <= EPSM * 10.0 * (fabs(T.low[i]) + 1.0))) {
      T.pivot[i] = -1;
    } else if (T.up[i] != INFINITY &&
               (x[i] * T.xscale[i] + T.xoffset[i] - T.up[i] >= EPSM * 10.0 * (fabs(T.up[i]) + 1.0))) {
      T.pivot[i] = 1;
    } else {
      T.pivot[i] = 0;
    }
  }
  double g[5];
#pragma unroll
  for (int i = 0; i < NMAX; ++i) g[i] = gfull[i];
  scaleg(g);
#pragma unroll
  for (int i = 0; i < NMAX; ++i)
    if (i < n && -(double)T.pivot[i] * g[i] < 0.0) T.pivot[i] = 0;
  project(g);
  double gnorm = dnrm2(n, g);
  double flast_con = f, flast_reset = f;
#pragma unroll
  for (int i = 0; i < NMAX; ++i) T.diagb[i] = 1.0;
  int rc;
  double pk[5];
  for (;;) {
    if (dnrm2(n, g) <= pgtol * T.fscale) { rc = 0; break; }
    if (T.nfeval >= T.maxfun) { rc = 3; break; }
    double newscale = dnrm2(n, g);
    if (newscale > EPSM && fabs(log10(newscale)) > rescale) {
      newscale = 1.0 / newscale;
      f *= newscale;
      T.fscale *= newscale;
      gnorm *= newscale;
      flast_con *= newscale;
      flast_reset *= newscale;
      difnew *= newscale;
#pragma unroll
      for (int i = 0; i < NMAX; ++i) {
        if (i < n) g[i] *= newscale;
        T.diagb[i] = 1.0;
      }
      T.upd1 = true;
      icycle = n - 1;
      newcon = true;
    }
    double temp[5];
#pragma unroll
    for (int i = 0; i < NMAX; ++i) temp[i] = x[i];
    project(temp);
    const double xnorm = dnrm2(n, temp);
    const int oldnfeval = T.nfeval;
    // ---- tnc_direction: preconditioned truncated CG ----
    {
      auto msolve = [&](const double* gin, double* y) {
        if (T.upd1) {
#pragma unroll
          for (int i = 0; i < NMAX; ++i)
            if (i < n) y[i] = gin[i] / T.diagb[i];
          return;
        }
        const double gsk = ddot(n, gin, T.sk);
        double hg[5], hyk[5], hyr[5];
        if (T.lreset) {
#pragma unroll
          for (int i = 0; i < NMAX; ++i) {
            if (i >= n) continue;
            const double rdiagb = 1.0 / T.diagb[i];
            hg[i] = gin[i] * rdiagb;
            hyk[i] = T.yk[i] * rdiagb;
          }
          const double ykhyk = ddot(n, T.yk, hyk);
          const double ghyk = ddot(n, gin, hyk);
          ssbfgs(n, 1.0, T.sk, hg, hyk, T.yksk, ykhyk, gsk, ghyk, y);
          return;
        }
#pragma unroll
        for (int i = 0; i < NMAX; ++i) {
          if (i >= n) continue;
          const double rdiagb = 1.0 / T.diagb[i];
          hg[i] = gin[i] * rdiagb;
          hyk[i] = T.yk[i] * rdiagb;
          hyr[i] = T.yr[i] * rdiagb;
        }
        const double gsr = ddot(n, gin, T.sr);
        const double ghyr = ddot(n, gin, hyr);
        const double yrhyr = ddot(n, T.yr, hyr);
        ssbfgs(n, 1.0, T.sr, hg, hyr, T.yrsr, yrhyr, gsr, ghyr, hg);
        const double yksr = ddot(n, T.yk, T.sr);
        const double ykhyr = ddot(n, T.yk, hyr);
        ssbfgs(n, 1.0, T.sr, hyk, hyr, T.yrsr, yrhyr, yksr, ykhyr, hyk);
        const double ykhyk = ddot(n, hyk, T.yk);
        const double ghyk = ddot(n, hyk, gin);
        ssbfgs(n, 1.0, T.sk, hg, hyk, T.yksk, ykhyk, gsk, ghyk, y);
      };
      double zsol[5] = {0, 0, 0, 0, 0};
      const double rhsnrm = gnorm;
      const double ctol = 1e-12;
      double qold = 0.0, rzold = 0.0;
      double r[5], v[5] = {0, 0, 0, 0, 0}, emat[5], zk[5], gv[5];
#pragma unroll
      for (int i = 0; i < NMAX; ++i) r[i] = -g[i];
      project(r);
      // initPreconditioner
      if (T.upd1) {
#pragma unroll
        for (int i = 0; i < NMAX; ++i) emat[i] = T.diagb[i];
      } else {
        double bsk[5];
        if (T.lreset) {
#pragma unroll
          for (int i = 0; i < NMAX; ++i)
            if (i < n) bsk[i] = T.diagb[i] * T.sk[i];
          double sds = ddot(n, T.sk, bsk);
          const double yksk = T.yksk != 0.0 ? T.yksk : 1.0;
          if (sds == 0.0) sds = 1.0;
#pragma unroll
          for (int i = 0; i < NMAX; ++i) {
            if (i >= n) continue;
            const double td = T.diagb[i];
            emat[i] = td - td * td * T.sk[i] * T.sk[i] / sds + T.yk[i] * T.yk[i] / yksk;
          }
        } else {
#pragma unroll
          for (int i = 0; i < NMAX; ++i)
            if (i < n) bsk[i] = T.diagb[i] * T.sr[i];
          double sds = ddot(n, T.sr, bsk);
          const double srds = ddot(n, T.sk, bsk);
          const double yrsk = ddot(n, T.yr, T.sk);
          const double yrsr = T.yrsr != 0.0 ? T.yrsr : 1.0;
          if (sds == 0.0) sds = 1.0;
#pragma unroll
          for (int i = 0; i < NMAX; ++i) {
            if (i >= n) continue;
            const double td = T.diagb[i];
            bsk[i] = td * T.sk[i] - bsk[i] * srds / sds + T.yr[i] * yrsk / yrsr;
            emat[i] = td - td * td * T.sr[i] * T.sr[i] / sds + T.yr[i] * T.yr[i] / yrsr;
          }
          sds = ddot(n, T.sk, bsk);
          const double yksk = T.yksk != 0.0 ? T.yksk : 1.0;
          if (sds == 0.0) sds = 1.0;
#pragma unroll
          for (int i = 0; i < NMAX; ++i)
            if (i < n) emat[i] = emat[i] - bsk[i] * bsk[i] / sds + T.yk[i] * T.yk[i] / yksk;
        }
      }
      for (int k = 0; k < T.maxCGit; ++k) {
        project(r);
        msolve(r, zk);
        project(zk);
        const double rz = ddot(n, r, zk);
        if (rz / rhsnrm < ctol || T.nfeval >= T.maxfun - 1) {
          if (k == 0) {
#pragma unroll
            for (int i = 0; i < NMAX; ++i) zsol[i] = -g[i];
            project(zsol);
          }
          break;
        }
        const double beta = k == 0 ? 0.0 : rz / rzold;
#pragma unroll
        for (int i = 0; i < NMAX; ++i)
          if (i < n) v[i] = zk[i] + beta * v[i];
        project(v);
        // hessianTimesVector: gradient difference along v
        {
          const double delta = T.accuracy * (xnorm + 1.0);
          double xv[5];
#pragma unroll
          for (int i = 0; i < NMAX; ++i) xv[i] = x[i] + delta * v[i];
          unscalex(xv);
          coercex(xv);
          double fv;
          fg(xv, fv, gv);
          scaleg(gv);
          const double dinv = 1.0 / delta;
#pragma unroll
          for (int i = 0; i < NMAX; ++i)
            if (i < n) gv[i] = (gv[i] - g[i]) * dinv;
#pragma unroll
          for (int i = 0; i < NMAX; ++i)  // projectConstants
            if (i < n && T.xscale[i] == 0.0) gv[i] = 0.0;
        }
        project(gv);
        const double vgv = ddot(n, v, gv);
        if (vgv / rhsnrm < ctol) {
          if (k == 0) {
            msolve(g, zsol);
#pragma unroll
            for (int i = 0; i < NMAX; ++i) zsol[i] = -zsol[i];
            project(zsol);
          }
          break;
        }
        {  // diagonalScaling
          const double vr = 1.0 / ddot(n, v, r);
          const double ivgv = 1.0 / ddot(n, v, gv);
#pragma unroll
          for (int i = 0; i < NMAX; ++i) {
            if (i >= n) continue;
            emat[i] += -r[i] * r[i] * vr + gv[i] * gv[i] * ivgv;
            if (emat[i] <= 1e-6) emat[i] = 1.0;
          }
        }
        const double calpha = rz / vgv;
#pragma unroll
        for (int i = 0; i < NMAX; ++i)
          if (i < n) zsol[i] += calpha * v[i];
#pragma unroll
        for (int i = 0; i < NMAX; ++i)
          if (i < n) r[i] += -calpha * gv[i];
        const double gtp = ddot(n, zsol, g);
        const double pr = ddot(n, r, zsol);
        const double qnew = (gtp + pr) * 0.5;
        const double qtest = (double)(k + 1) * (1.0 - qnew / qold);
        if (qtest <= 0.5) break;
        if (gtp > 0.0) {
#pragma unroll
          for (int i = 0; i < NMAX; ++i)
            if (i < n) zsol[i] += -calpha * v[i];
          break;
        }
        qold = qnew;
        rzold = rz;
      }
#pragma unroll
      for (int i = 0; i < NMAX; ++i) {
        T.diagb[i] = i < n ? emat[i] : 1.0;
        pk[i] = i < n ? zsol[i] : 0.0;
      }
    }
    if (!newcon) {
      if (!T.lreset) {
#pragma unroll
        for (int i = 0; i < NMAX; ++i) {
          T.sr[i] += T.sk[i];
          T.yr[i] += T.yk[i];
        }
        ++icycle;
      } else {
#pragma unroll
        for (int i = 0; i < NMAX; ++i) {
          T.sr[i] = T.sk[i];
          T.yr[i] = T.yk[i];
        }
        flast_reset = f;
        icycle = 1;
      }
    }
    double oldg[5];
#pragma unroll
    for (int i = 0; i < NMAX; ++i) oldg[i] = g[i];
    const double oldf = f;
    const double oldgtp = ddot(n, pk, g);
    const double ustpmax = stepmx / (dnrm2(n, pk) + EPSM);
    double spe = ustpmax;  // stepMax
#pragma unroll
    for (int i = 0; i < NMAX; ++i) {
      if (i >= n || T.pivot[i] != 0 || pk[i] == 0.0) continue;
      if (pk[i] < 0.0) {
        const double t = (T.low[i] - T.xoffset[i]) / T.xscale[i] - x[i];
        if (t > spe * pk[i]) spe = t / pk[i];
      } else {
        const double t = (T.up[i] - T.xoffset[i]) / T.xscale[i] - x[i];
        if (t < spe * pk[i]) spe = t / pk[i];
      }
    }
    bool stop = false;
    if (spe > 0.0) {
      alpha = initial_step(f, fmin / T.fscale, oldgtp, spe);
      // ---- linearSearch ----
      int lsrc;
      {
        double tmp[5];
#pragma unroll
        for (int i = 0; i < NMAX; ++i) tmp[i] = gfull[i];
        scaleg(tmp);
        Ptc S;
        S.gu = ddot(n, tmp, pk);
#pragma unroll
        for (int i = 0; i < NMAX; ++i) tmp[i] = x[i];
        project(tmp);
        const double lxnorm = dnrm2(n, tmp);
        const double pe = dnrm2(n, pk) + EPSM;
        S.reltol = rteps * (lxnorm + 1.0) / pe;
        S.abstol = -EPSM * (1.0 + fabs(f)) / (S.gu - EPSM);
        const double tnytol = EPSM * (lxnorm + 1.0) / pe;
        const double rtsmll = EPSM;
        const double big = 1.0 / (EPSM * EPSM);
        S.u = alpha;
        S.fu = f;
        S.fmin = f;
        S.rmu = 1e-4;
        int itest = getptc_init(S, tnytol, eta, spe);
        if (itest == GETPTC_EINVAL) {
          lsrc = LS_FAIL;
        } else {
          while (itest == GETPTC_EVAL && T.nfeval < T.maxfun) {
            const double ualpha = S.xmin + S.u;
            double xt[5], tg[5], fu;
#pragma unroll
            for (int i = 0; i < NMAX; ++i) xt[i] = x[i] + ualpha * pk[i];
            unscalex(xt);
            coercex(xt);
            fg(xt, fu, tg);
            fu *= T.fscale;
            double ng[5];
#pragma unroll
            for (int i = 0; i < NMAX; ++i) ng[i] = tg[i];
            scaleg(ng);
            S.fu = fu;
            S.gu = ddot(n, ng, pk);
            itest = getptc_iter(S, big, rtsmll, tnytol, ftol, spe);
            if (S.xmin == ualpha) {
#pragma unroll
              for (int i = 0; i < NMAX; ++i) gfull[i] = tg[i];
            }
          }
          if (itest == GETPTC_OK) {
#pragma unroll
            for (int i = 0; i < NMAX; ++i)
              if (i < n) x[i] = x[i] + S.xmin * pk[i];
            f = S.fmin;
            lsrc = LS_OK;
          } else {
            lsrc = T.nfeval >= T.maxfun ? LS_MAXFUN : LS_FAIL;
          }
        }
        if (itest != GETPTC_EINVAL) alpha = S.xmin;  // EINVAL keeps the initial step
      }
      if (alpha >= 0.9 * ustpmax) stepmx *= 1e2;
      if (alpha - spe >= -EPSM * 10.0) {
        newcon = true;
      } else {
        if (lsrc != LS_OK) {
          rc = lsrc == LS_MAXFUN ? 3 : 4;
          stop = true;
        }
        newcon = false;
      }
    } else {
      newcon = true;
    }
    if (stop) break;
    if (newcon) {
      bool added = false;  // addConstraint
#pragma unroll
      for (int i = 0; i < NMAX; ++i) {
        if (i >= n || T.pivot[i] != 0 || pk[i] == 0.0) continue;
        if (pk[i] < 0.0 && T.low[i] != -INFINITY) {
          const double tl = EPSM * 10.0 * (fabs(T.low[i]) + 1.0);
          if (x[i] * T.xscale[i] + T.xoffset[i] - T.low[i] <= tl) {
            T.pivot[i] = -1;
            x[i] = (T.low[i] - T.xoffset[i]) / T.xscale[i];
            added = true;
          }
        } else if (pk[i] > 0.0 && T.up[i] != INFINITY) {
          const double tl = EPSM * 10.0 * (fabs(T.up[i]) + 1.0);
          if (T.up[i] - (x[i] * T.xscale[i] + T.xoffset[i]) <= tl) {
            T.pivot[i] = 1;
            x[i] = (T.up[i] - T.xoffset[i]) / T.xscale[i];
            added = true;
          }
        }
      }
      if (!added && T.nfeval == oldnfeval) { rc = 6; break; }
      flast_con = f;
    }
    const double difold = difnew;
    difnew = oldf - f;
    if (icycle == 1) {
      if (difnew > difold * 2.0) epsred += epsred;
      if (difnew < difold * 0.5) epsred *= 0.5;
    }
#pragma unroll
    for (int i = 0; i < NMAX; ++i) g[i] = gfull[i];
    scaleg(g);
#pragma unroll
    for (int i = 0; i < NMAX; ++i) temp[i] = g[i];
    project(temp);
    gnorm = dnrm2(n, temp);
    bool remcon = false;  // removeConstraint
    if (!(((flast_con - f) <= (oldgtp * -0.5)) && gnorm > pgtol * T.fscale)) {
      int imax = -1;
      double cmax = 0.0;
#pragma unroll
      for (int i = 0; i < NMAX; ++i) {
        if (i >= n || T.pivot[i] == 2) continue;
        const double t = -(double)T.pivot[i] * g[i];
        if (t < cmax) { cmax = t; imax = i; }
      }
      if (imax != -1) {
#pragma unroll
        for (int i = 0; i < NMAX; ++i)
          if (i == imax) T.pivot[i] = 0;
        remcon = true;
      }
    }
    if (remcon) {
#pragma unroll
      for (int i = 0; i < NMAX; ++i) temp[i] = g[i];
      project(temp);
      gnorm = dnrm2(n, temp);
    }
    if (!remcon && !newcon) {
      if (fabs(difnew) <= ftol * T.fscale) { rc = 1; break; }
      if (alpha * dnrm2(n, pk) <= xtol) { rc = 2; break; }
    }
    project(g);
    if (!newcon) {
#pragma unroll
      for (int i = 0; i < NMAX; ++i) {
        if (i >= n) continue;
        T.yk[i] = g[i] - oldg[i];
        T.sk[i] = alpha * pk[i];
      }
      T.yksk = ddot(n, T.yk, T.sk);
      if (icycle == n - 1 || difnew < epsred * (flast_reset - f)) {
        T.lreset = true;
      } else {
        T.yrsr = ddot(n, T.yr, T.sr);
        T.lreset = T.yrsr <= 0.0;
      }
      T.upd1 = false;
    }
  }
  unscalex(x);
  coercex(x);
  f_out = f / T.fscale;
  return rc;
}

// fit_portrait_full(method='TNC') / legacy fit_portrait on one subint.
template <bool SCAT, bool WIDE>
__global__ __launch_bounds__(kBlock, 1) void k_tnc(FitArgs a) {
  extern __shared__ __align__(16) unsigned char dyn[];
  __shared__ TncShared sh;
  __shared__ double refs[3];
  const int c = blockIdx.x, s = a.sub0 + c, tid = threadIdx.x;
  if (a.method != PPF_METHOD_TNC && a.method != PPF_METHOD_TNC_LEGACY) return;
  if ((a.st[c].scat != 0) != SCAT) return;  // the other variant owns this subint
  const Meta m = load_meta(a, c, s, chan_tables<WIDE>(a, dyn), &sh.nok);
  SolveState& st = a.st[c];
  const double P = a.P[s];
  if (tid < 3) refs[tid] = st.refs[tid];
  __syncthreads();
  const int n = a.method == PPF_METHOD_TNC_LEGACY ? 2 : 5;
  double x[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) x[i] = st.x[i];
  double* acc0 = a.acc + (size_t)c * 2 * a.nchan * NACC;
  TncObjective O;
  O.a = &a;
  O.m = &m;
  O.c = c;
  O.s = s;
  O.refs = refs;
  O.P = P;
  O.acc_slot = acc0;
  O.red = sh.red;
  O.out = sh.out;
  O.have = false;
  O.nfev = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) { O.lastx[i] = x[i]; O.lastg[i] = 0.0; }
  O.lastf = NAN;
  int status = -1;
  double f = NAN;
  if (m.nok > 0) {
    // minfev = dof - Sd for fit_portrait_full (pptoaslib.py:1005-1007); the
    // legacy fit passes none (0)
    double fmin = 0.0;
    if (n == 5) {
      double sd = 0.0;
      for (int j = tid; j < m.nok; j += kBlock) sd += a.dsum[(size_t)c * a.nchan + m.chan[j]] * m.iw2[j];
      sd = block_sum(sd, sh.red[0]);
      int nfit = 0;
      for (int i = 0; i < 5; ++i) nfit += a.flags[i] ? 1 : 0;
      const double dof = (double)a.nbin * (double)m.nok - (double)(nfit + m.nok);
      fmin = dof - sd;
    }
    // the trace's record 0 carries the minfev TNC was given (field 29)
    if (a.trace && tid == 0 && a.trace_cap > 0)
      a.trace[(size_t)s * a.trace_cap * kTraceRec + 29] = fmin;
    TncState T;
    T.n = n;
    T.maxfun = 100;  // max(100, 10 n), n <= 5
    T.nfeval = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const double lo = a.bounds[i][0], hi = a.bounds[i][1];
      T.low[i] = isnan(lo) ? -INFINITY : lo;
      T.up[i] = isnan(hi) ? INFINITY : hi;
      T.xscale[i] = 1.0;
      T.xoffset[i] = 0.0;
    }
    status = tnc_run<SCAT, WIDE>(T, O, x, f, fmin, 1e-10);
    // scipy's _minimize_tnc ends with func_and_grad(x): the result's fun and
    // jac, and one more nfev when x is not the last evaluated point.  Every
    // sweep writes acc slot 0, so it then holds x's per-channel sums (k_post).
    double fx, gx[5];
    O.template eval<SCAT>(n, x, fx, gx);
    f = fx;
  }
  if (tid < 5) st.x[tid] = x[tid];
  if (tid < 5 && a.o_grad) a.o_grad[(size_t)s * 5 + tid] = m.nok ? O.lastg[tid] : NAN;
  if (tid < 25 && a.o_hess) a.o_hess[(size_t)s * 25 + tid] = NAN;  // TNC has no Hessian
  if (tid == 0) {
    st.fun = m.nok ? f : NAN;
    st.nfev = m.nok ? O.nfev : 0;
    st.status = status;
    st.slot = 0;
    const double tl = a.log10_tau ? pow(10.0, x[3]) : x[3];
    st.scat_post = SCAT && tl != 0.0;
  }
}

template __global__ void k_tnc<false, false>(FitArgs);
template __global__ void k_tnc<true, false>(FitArgs);
template __global__ void k_tnc<false, true>(FitArgs);
template __global__ void k_tnc<true, true>(FitArgs);

}  // namespace ppf
