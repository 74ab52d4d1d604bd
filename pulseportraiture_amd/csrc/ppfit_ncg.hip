// ppfit_ncg.hip -- scipy's Newton-CG on the device.
//
// fit_portrait_full(method='Newton-CG') minimizes the wideband objective
// with scipy.optimize.minimize(..., method='Newton-CG', jac=..., hess=...,
// options={'maxiter': 2000, 'xtol': -1}) (pptoaslib.py:995-1014).  scipy
// 1.15's _minimize_newtoncg: a truncated CG solve of H p = -g per iteration,
// then _line_search_wolfe12 -- MINPACK-2's dcsrch / dcstep (line_search_
// wolfe1) and, when it fails, line_search_wolfe2's bracketing and zoom.
// tools/ncg_model.py restates that control flow in scalar Python and
// tests/test_ncg_model.py holds it to scipy; this file follows the model
// statement for statement (FP contraction off).  With xtol = -1 the loop ends
// only when both line searches fail (status 2), at maxiter (1), on a
// non-positive-definite CG (3) or a NaN (3).
//
// One workgroup per subint.  Every thread runs the uniform scalar control
// flow on its own registers; each objective evaluation is one block-wide
// sweep over the subint's cross-spectrum (sweep<0, SCAT>: f, the masked
// gradient and Hessian, pptoaslib.py:525-643), cached at the last point as
// scipy's ScalarFunction caches it, nfev counting the distinct points.
#include "ppfit_kernels.hpp"

namespace ppf {

namespace ncg {

constexpr int N = 5;
constexpr double EPS = 2.220446049250313e-16;

struct Obj {
  const FitArgs* a;
  const Meta* m;
  int c, s;
  const double* refs;
  double P;
  double* acc_slot;
  double (*red)[48];
  double* out;  // LDS, >= 21 doubles
  double lx[N], lf, lg[N], lH[N][N];
  bool have;
  int nfev;
  int nsweep;  // sweeps so far (the trace index)
  // f, g, H at x (a sweep unless x is the cached point); count: scipy
  // evaluates f there (nfev)
  template <bool SCAT>
  __device__ void at(const double* x, bool count = true) {
    bool same = have;
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (x[i] != lx[i]) same = false;
    if (same) return;
    double pr[N];
#pragma unroll
    for (int i = 0; i < N; ++i) pr[i] = x[i];
    sweep<0, SCAT>(*a, *m, c, s, pr, refs, P, acc_slot, out, red, TaylorSrc{});
    trace_sweep(*a, s, nsweep++, pr, out, 21, count);
    lf = out[0];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      lg[i] = out[1 + i];
      lx[i] = x[i];
    }
#pragma unroll
    for (int p = 0; p < 15; ++p) {
      lH[pair_i(p)][pair_j(p)] = out[6 + p];
      lH[pair_j(p)][pair_i(p)] = out[6 + p];
    }
    have = true;
    if (count) ++nfev;
    __syncthreads();  // out / red are reused by the next evaluation
  }
};

__device__ __forceinline__ double dot(const double* u, const double* v) {
#pragma clang fp contract(off)
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) s += u[i] * v[i];
  return s;
}

__device__ __forceinline__ double l1(const double* u) {
#pragma clang fp contract(off)
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) s += fabs(u[i]);
  return s;
}

// Python's builtin min / max (first argument kept unless the other compares
// strictly better: NaN-propagation as there) and np.sign
__device__ __forceinline__ double py_max(double a, double b) { return b > a ? b : a; }
__device__ __forceinline__ double py_min(double a, double b) { return b < a ? b : a; }
__device__ __forceinline__ double np_sign(double v) {
  return v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : (v == 0.0 ? 0.0 : v));
}
// np.clip (NaN passes through)
__device__ __forceinline__ double np_clip(double v, double lo, double hi) {
  if (v < lo) v = lo;
  if (v > hi) v = hi;
  return v;
}

struct Step {
  double stx, fx, dx, sty, fy, dy, stp;
  bool brackt;
};

// MINPACK-2 dcstep (scipy/optimize/_dcsrch.py)
__device__ void dcstep(Step& S, double fp, double dp, double stpmin, double stpmax) {
#pragma clang fp contract(off)
  const double stx = S.stx, fx = S.fx, dx = S.dx, sty = S.sty, fy = S.fy, dy = S.dy;
  const double stp = S.stp;
  const double sgnd = np_sign(dp) * np_sign(dx);
  double stpf;
  if (fp > fx) {
    const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    const double s = py_max(py_max(fabs(theta), fabs(dx)), fabs(dp));
    double gamma = s * sqrt((theta / s) * (theta / s) - (dx / s) * (dp / s));
    if (stp < stx) gamma = -gamma;
    const double p = (gamma - dx) + theta;
    const double q = ((gamma - dx) + gamma) + dp;
    const double r = p / q;
    const double stpc = stx + r * (stp - stx);
    const double stpq = stx + ((dx / ((fx - fp) / (stp - stx) + dx)) / 2.0) * (stp - stx);
    if (fabs(stpc - stx) <= fabs(stpq - stx)) stpf = stpc;
    else stpf = stpc + (stpq - stpc) / 2.0;
    S.brackt = true;
  } else if (sgnd < 0.0) {
    const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    const double s = py_max(py_max(fabs(theta), fabs(dx)), fabs(dp));
    double gamma = s * sqrt((theta / s) * (theta / s) - (dx / s) * (dp / s));
    if (stp > stx) gamma = -gamma;
    const double p = (gamma - dp) + theta;
    const double q = ((gamma - dp) + gamma) + dx;
    const double r = p / q;
    const double stpc = stp + r * (stx - stp);
    const double stpq = stp + (dp / (dp - dx)) * (stx - stp);
    stpf = (fabs(stpc - stp) > fabs(stpq - stp)) ? stpc : stpq;
    S.brackt = true;
  } else if (fabs(dp) < fabs(dx)) {
    const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
    const double s = py_max(py_max(fabs(theta), fabs(dx)), fabs(dp));
    double gamma = s * sqrt(py_max(0.0, (theta / s) * (theta / s) - (dx / s) * (dp / s)));
    if (stp > stx) gamma = -gamma;
    const double p = (gamma - dp) + theta;
    const double q = (gamma + (dx - dp)) + gamma;
    const double r = p / q;
    double stpc;
    if (r < 0.0 && gamma != 0.0) stpc = stp + r * (stx - stp);
    else if (stp > stx) stpc = stpmax;
    else stpc = stpmin;
    const double stpq = stp + (dp / (dp - dx)) * (stx - stp);
    if (S.brackt) {
      stpf = (fabs(stpc - stp) < fabs(stpq - stp)) ? stpc : stpq;
      if (stp > stx) stpf = py_min(stp + 0.66 * (sty - stp), stpf);
      else stpf = py_max(stp + 0.66 * (sty - stp), stpf);
    } else {
      stpf = (fabs(stpc - stp) > fabs(stpq - stp)) ? stpc : stpq;
      stpf = py_min(py_max(stpf, stpmin), stpmax);
    }
  } else {
    if (S.brackt) {
      const double theta = 3.0 * (fp - fy) / (sty - stp) + dy + dp;
      const double s = py_max(py_max(fabs(theta), fabs(dy)), fabs(dp));
      double gamma = s * sqrt((theta / s) * (theta / s) - (dy / s) * (dp / s));
      if (stp > sty) gamma = -gamma;
      const double p = (gamma - dp) + theta;
      const double q = ((gamma - dp) + gamma) + dy;
      const double r = p / q;
      stpf = stp + r * (sty - stp);
    } else if (stp > stx) {
      stpf = stpmax;
    } else {
      stpf = stpmin;
    }
  }
  if (fp > fx) {
    S.sty = stp;
    S.fy = fp;
    S.dy = dp;
  } else {
    if (sgnd < 0.0) {
      S.sty = stx;
      S.fy = fx;
      S.dy = dx;
    }
    S.stx = stp;
    S.fx = fp;
    S.dx = dp;
  }
  S.stp = stpf;
}

// The line-search functions of _minimize_newtoncg at the point xk + s pk.
struct Line {
  const double* xk;
  const double* pk;
  __device__ void point(double s, double* x) const {
#pragma clang fp contract(off)
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = xk[i] + s * pk[i];
  }
  template <bool SCAT>
  __device__ double phi(Obj& O, double s) const {
    double x[N];
    point(s, x);
    O.template at<SCAT>(x);
    return O.lf;
  }
  template <bool SCAT>
  __device__ double derphi(Obj& O, double s) const {
    double x[N];
    point(s, x);
    O.template at<SCAT>(x);
    return dot(O.lg, pk);
  }
};

// DCSRCH.__call__ / _iterate (scalar_search_wolfe1: ftol c1, gtol c2,
// xtol 1e-14, stpmin 1e-8, stpmax 50, maxiter 100).  ok = a step was found.
template <bool SCAT>
__device__ bool dcsrch(Obj& O, const Line& L, double alpha1, double phi0, double derphi0,
                       double ftol, double gtol, double& stp_out, double& phi1_out) {
#pragma clang fp contract(off)
  const double xtol = 1e-14, stpmin = 1e-8, stpmax = 50.0;
  const double p5 = 0.5, p66 = 0.66, xtrapl = 1.1, xtrapu = 4.0;
  double stp = alpha1, f = phi0, g = derphi0;
  phi1_out = phi0;
  if (stp < stpmin || stp > stpmax || g >= 0.0 || stpmax < stpmin) return false;  // ERROR
  bool stage2 = false;
  const double finit = f, ginit = g;
  const double gtest = ftol * ginit;
  double width = stpmax - stpmin;
  double width1 = width / p5;
  Step S{0.0, finit, ginit, 0.0, finit, ginit, stp, false};
  double stmin = 0.0, stmax = stp + xtrapu * stp;
  if (!isfinite(stp)) return false;
  f = L.template phi<SCAT>(O, stp);
  g = L.template derphi<SCAT>(O, stp);
  phi1_out = f;
  for (int it = 1; it < 100; ++it) {
    const double ftest = finit + stp * gtest;
    if (!stage2 && f <= ftest && g >= 0.0) stage2 = true;
    bool warn = false;
    if (S.brackt && (stp <= stmin || stp >= stmax)) warn = true;
    if (S.brackt && stmax - stmin <= xtol * stmax) warn = true;
    if (stp == stpmax && f <= ftest && g <= gtest) warn = true;
    if (stp == stpmin && (f > ftest || g >= gtest)) warn = true;
    if (f <= ftest && fabs(g) <= gtol * -ginit) {  // CONVERGENCE
      stp_out = stp;
      return true;
    }
    if (warn) return false;
    S.stp = stp;
    if (!stage2 && f <= S.fx && f > ftest) {
      // modified function (psi) values
      const double fm = f - stp * gtest;
      S.fx = S.fx - S.stx * gtest;
      S.fy = S.fy - S.sty * gtest;
      const double gm = g - gtest;
      S.dx = S.dx - gtest;
      S.dy = S.dy - gtest;
      dcstep(S, fm, gm, stmin, stmax);
      S.fx = S.fx + S.stx * gtest;
      S.fy = S.fy + S.sty * gtest;
      S.dx = S.dx + gtest;
      S.dy = S.dy + gtest;
    } else {
      dcstep(S, f, g, stmin, stmax);
    }
    stp = S.stp;
    if (S.brackt) {
      if (fabs(S.sty - S.stx) >= p66 * width1) stp = S.stx + p5 * (S.sty - S.stx);
      width1 = width;
      width = fabs(S.sty - S.stx);
    }
    if (S.brackt) {
      stmin = py_min(S.stx, S.sty);
      stmax = py_max(S.stx, S.sty);
    } else {
      stmin = stp + xtrapl * (stp - S.stx);
      stmax = stp + xtrapu * (stp - S.stx);
    }
    stp = np_clip(stp, stpmin, stpmax);
    if ((S.brackt && (stp <= stmin || stp >= stmax)) ||
        (S.brackt && stmax - stmin <= xtol * stmax))
      stp = S.stx;
    if (!isfinite(stp)) return false;
    f = L.template phi<SCAT>(O, stp);
    g = L.template derphi<SCAT>(O, stp);
    phi1_out = f;
  }
  return false;  // maxiter
}

// _cubicmin / _quadmin: false where numpy would raise (any non-finite
// intermediate of finite inputs)
__device__ bool cubicmin(double a, double fa, double fpa, double b, double fb, double c,
                         double fc, double& xmin) {
#pragma clang fp contract(off)
  const double C = fpa;
  const double db = b - a, dc = c - a;
  const double denom = (db * dc) * (db * dc) * (db - dc);
  const double d00 = dc * dc, d01 = -(db * db), d10 = -pow(dc, 3.0), d11 = pow(db, 3.0);
  const double v0 = fb - fa - C * db, v1 = fc - fa - C * dc;
  double A = d00 * v0 + d01 * v1;
  double B = d10 * v0 + d11 * v1;
  if (!isfinite(denom) || !isfinite(A) || !isfinite(B) || denom == 0.0) return false;
  A /= denom;
  B /= denom;
  const double radical = B * B - 3.0 * A * C;
  if (!isfinite(A) || !isfinite(B) || !isfinite(radical) || radical < 0.0 || A == 0.0)
    return false;
  xmin = a + (-B + sqrt(radical)) / (3.0 * A);
  return isfinite(xmin);
}

__device__ bool quadmin(double a, double fa, double fpa, double b, double fb, double& xmin) {
#pragma clang fp contract(off)
  const double D = fa, C = fpa;
  const double db = b - a * 1.0;
  const double dd = db * db;
  if (!isfinite(dd) || dd == 0.0) return false;
  const double B = (fb - D - C * db) / dd;
  if (!isfinite(B) || B == 0.0) return false;
  xmin = a - C / (2.0 * B);
  return isfinite(xmin);
}

template <bool SCAT>
__device__ bool zoom(Obj& O, const Line& L, double a_lo, double a_hi, double phi_lo,
                     double phi_hi, double derphi_lo, double phi0, double derphi0, double c1,
                     double c2, double& a_star, double& val_star) {
#pragma clang fp contract(off)
  const double delta1 = 0.2, delta2 = 0.1;
  double phi_rec = phi0, a_rec = 0.0;
  double a_j = 0.0;
  bool have_j = false;
  for (int i = 0;; ++i) {
    const double dalpha = a_hi - a_lo;
    double a, b;
    if (dalpha < 0.0) { a = a_hi; b = a_lo; }
    else { a = a_lo; b = a_hi; }
    double cchk = 0.0;
    if (i > 0) {
      cchk = delta1 * dalpha;
      have_j = cubicmin(a_lo, phi_lo, derphi_lo, a_hi, phi_hi, a_rec, phi_rec, a_j);
    }
    if (i == 0 || !have_j || a_j > b - cchk || a_j < a + cchk) {
      const double qchk = delta2 * dalpha;
      have_j = quadmin(a_lo, phi_lo, derphi_lo, a_hi, phi_hi, a_j);
      if (!have_j || a_j > b - qchk || a_j < a + qchk) a_j = a_lo + 0.5 * dalpha;
    }
    const double phi_aj = L.template phi<SCAT>(O, a_j);
    if (phi_aj > phi0 + c1 * a_j * derphi0 || phi_aj >= phi_lo) {
      phi_rec = phi_hi;
      a_rec = a_hi;
      a_hi = a_j;
      phi_hi = phi_aj;
    } else {
      const double derphi_aj = L.template derphi<SCAT>(O, a_j);
      if (fabs(derphi_aj) <= -c2 * derphi0) {
        a_star = a_j;
        val_star = phi_aj;
        return true;
      }
      if (derphi_aj * (a_hi - a_lo) >= 0.0) {
        phi_rec = phi_hi;
        a_rec = a_hi;
        a_hi = a_lo;
        phi_hi = phi_lo;
      } else {
        phi_rec = phi_lo;
        a_rec = a_lo;
      }
      a_lo = a_j;
      phi_lo = phi_aj;
      derphi_lo = derphi_aj;
    }
    if (i + 1 > 10) return false;
  }
}

// scalar_search_wolfe2 (amax None, maxiter 10); phi0_io: the old_fval handed
// in, returned as the new old_old_fval
template <bool SCAT>
__device__ bool wolfe2(Obj& O, const Line& L, double phi0, bool have_old, double old_phi0,
                       double derphi0, double c1, double c2, double& alpha_star,
                       double& phi_star) {
#pragma clang fp contract(off)
  double alpha0 = 0.0, alpha1;
  if (have_old && derphi0 != 0.0) alpha1 = py_min(1.0, 1.01 * 2.0 * (phi0 - old_phi0) / derphi0);
  else alpha1 = 1.0;
  if (alpha1 < 0.0) alpha1 = 1.0;
  double phi_a1 = L.template phi<SCAT>(O, alpha1);
  double phi_a0 = phi0, derphi_a0 = derphi0;
  for (int i = 0; i < 10; ++i) {
    if (alpha1 == 0.0) return false;
    if (phi_a1 > phi0 + c1 * alpha1 * derphi0 || (phi_a1 >= phi_a0 && i > 0))
      return zoom<SCAT>(O, L, alpha0, alpha1, phi_a0, phi_a1, derphi_a0, phi0, derphi0, c1, c2,
                        alpha_star, phi_star);
    const double derphi_a1 = L.template derphi<SCAT>(O, alpha1);
    if (fabs(derphi_a1) <= -c2 * derphi0) {
      alpha_star = alpha1;
      phi_star = phi_a1;
      return true;
    }
    if (derphi_a1 >= 0.0)
      return zoom<SCAT>(O, L, alpha1, alpha0, phi_a1, phi_a0, derphi_a1, phi0, derphi0, c1, c2,
                        alpha_star, phi_star);
    const double alpha2 = 2.0 * alpha1;
    alpha0 = alpha1;
    alpha1 = alpha2;
    phi_a0 = phi_a1;
    phi_a1 = L.template phi<SCAT>(O, alpha1);
    derphi_a0 = derphi_a1;
  }
  alpha_star = alpha1;  // maxiter: accepted, with no derivative
  phi_star = phi_a1;
  return true;
}

// _minimize_newtoncg (maxiter 2000, xtol -1, c1 1e-4, c2 0.9): status as scipy
template <bool SCAT, bool W>  // W: one copy per k_ncg instantiation (its only caller)
__device__ int run(Obj& O, double* xk, double& fval) {
#pragma clang fp contract(off)
  const double c1 = 1e-4, c2 = 0.9;
  const int maxiter = 2000, cg_maxiter = 20 * N;
  const double xtol = N * -1.0;
  double update_l1norm = 1.7976931348623157e308;
  O.template at<SCAT>(xk);  // ScalarFunction(x0): f and g at the start (nfev 1)
  double old_fval = O.lf, old_old_fval = 0.0;
  bool have_old_old = false;
  int k = 0;
  while (update_l1norm > xtol) {
    if (k >= maxiter) {
      fval = old_fval;
      return 1;
    }
    O.template at<SCAT>(xk);
    double b[N], gfk[N], A[N][N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      gfk[i] = O.lg[i];
      b[i] = -O.lg[i];
#pragma unroll
      for (int j = 0; j < N; ++j) A[i][j] = O.lH[i][j];
    }
    const double maggrad = l1(b);
    const double eta = py_min(0.5, sqrt(maggrad));
    const double termcond = eta * maggrad;
    double xsupi[N], ri[N], psupi[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      xsupi[i] = 0.0;
      ri[i] = -b[i];
      psupi[i] = -ri[i];
    }
    int icg = 0;
    double dri0 = dot(ri, ri);
    bool cg_done = false;
    for (int k2 = 0; k2 < cg_maxiter; ++k2) {
      if (l1(ri) <= termcond) { cg_done = true; break; }
      double Ap[N];
#pragma unroll
      for (int r = 0; r < N; ++r) Ap[r] = dot(A[r], psupi);
      const double curv = dot(psupi, Ap);
      if (0.0 <= curv && curv <= 3.0 * EPS) { cg_done = true; break; }
      if (curv < 0.0) {
        if (icg == 0) {  // steepest descent
#pragma unroll
          for (int i = 0; i < N; ++i) xsupi[i] = dri0 / (-curv) * b[i];
        }
        cg_done = true;
        break;
      }
      const double alphai = dri0 / curv;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        xsupi[i] = xsupi[i] + alphai * psupi[i];
        ri[i] = ri[i] + alphai * Ap[i];
      }
      const double dri1 = dot(ri, ri);
      const double betai = dri1 / dri0;
#pragma unroll
      for (int i = 0; i < N; ++i) psupi[i] = -ri[i] + betai * psupi[i];
      icg += 1;
      dri0 = dri1;
    }
    if (!cg_done) {  // "CG iterations didn't converge"
      fval = old_fval;
      return 3;
    }
    Line L{xk, xsupi};
    const double derphi0 = dot(gfk, xsupi);
    // line_search_wolfe1 -> scalar_search_wolfe1
    double alpha1;
    if (have_old_old && derphi0 != 0.0) {
      alpha1 = py_min(1.0, 1.01 * 2.0 * (old_fval - old_old_fval) / derphi0);
      if (alpha1 < 0.0) alpha1 = 1.0;
    } else {
      alpha1 = 1.0;
    }
    double stp = 0.0, fnew = 0.0;
    bool ok = dcsrch<SCAT>(O, L, alpha1, old_fval, derphi0, c1, c2, stp, fnew);
    if (!ok) ok = wolfe2<SCAT>(O, L, old_fval, have_old_old, old_old_fval, derphi0, c1, c2, stp,
                               fnew);
    if (!ok) {  // _LineSearchError: "Desired error not necessarily achieved"
      fval = old_fval;
      return 2;
    }
    old_old_fval = old_fval;
    have_old_old = true;
    old_fval = fnew;
    double update[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      update[i] = stp * xsupi[i];
      xk[i] = xk[i] + update[i];
    }
    k += 1;
    update_l1norm = l1(update);
  }
  fval = old_fval;
  if (isnan(old_fval) || isnan(update_l1norm)) return 3;
  return 0;
}

struct Shared {
  double out[48];
  double red[kWaves][48];
  int nok;
};

}  // namespace ncg

// fit_portrait_full(method='Newton-CG') on one subint.
template <bool SCAT, bool WIDE>
__global__ __launch_bounds__(kBlock, 1) void k_ncg(FitArgs a) {
  extern __shared__ __align__(16) unsigned char dyn[];
  __shared__ ncg::Shared sh;
  __shared__ double refs[3];
  const int c = blockIdx.x, s = a.sub0 + c, tid = threadIdx.x;
  if (a.method != PPF_METHOD_NEWTON_CG) return;
  if ((a.st[c].scat != 0) != SCAT) return;  // the other variant owns this subint
  const Meta m = load_meta(a, c, s, chan_tables<WIDE>(a, dyn), &sh.nok);
  SolveState& st = a.st[c];
  if (tid < 3) refs[tid] = st.refs[tid];
  __syncthreads();
  double x[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) x[i] = st.x[i];
  ncg::Obj O;
  O.a = &a;
  O.m = &m;
  O.c = c;
  O.s = s;
  O.refs = refs;
  O.P = a.P[s];
  O.acc_slot = a.acc + (size_t)c * 2 * a.nchan * NACC;
  O.red = sh.red;
  O.out = sh.out;
  O.have = false;
  O.nfev = 0;
  O.nsweep = 0;
  int status = -1;
  double f = NAN;
  if (m.nok > 0) {
    status = ncg::run<SCAT, WIDE>(O, x, f);
    // k_post reads the per-channel sums of x from acc slot 0: refresh them
    // when the last sweep was a rejected trial point (scipy does not
    // evaluate there: not counted)
    O.template at<SCAT>(x, false);
  }
  if (tid < 5) st.x[tid] = x[tid];
  if (tid < 5 && a.o_grad) a.o_grad[(size_t)s * 5 + tid] = m.nok ? O.lg[tid] : NAN;
  if (tid < 25 && a.o_hess) a.o_hess[(size_t)s * 25 + tid] = m.nok ? O.lH[tid / 5][tid % 5] : NAN;
  if (tid == 0) {
    st.fun = m.nok ? f : NAN;
    st.nfev = m.nok ? O.nfev : 0;
    st.status = status;
    st.slot = 0;
    const double tl = a.log10_tau ? pow(10.0, x[3]) : x[3];
    st.scat_post = SCAT && tl != 0.0;
  }
}

template __global__ void k_ncg<false, false>(FitArgs);
template __global__ void k_ncg<true, false>(FitArgs);
template __global__ void k_ncg<false, true>(FitArgs);
template __global__ void k_ncg<true, true>(FitArgs);

}  // namespace ppf
