"""Scalar restatement of scipy.optimize.minimize(method='Newton-CG') as
fit_portrait_full calls it (pptoaslib.py:1003-1004: jac, hess, maxiter 2000,
xtol -1) -- the model ppfit_ncg.hip follows statement for statement.

scipy 1.15: _minimize_newtoncg (optimize/_optimize.py), _line_search_wolfe12,
line_search_wolfe1 -> scalar_search_wolfe1 -> DCSRCH / dcstep
(optimize/_dcsrch.py), and the fallback line_search_wolfe2 ->
scalar_search_wolfe2 / _zoom / _cubicmin / _quadmin (optimize/_linesearch.py).
ScalarFunction semantics: f, g and H are cached at the last point; nfev
counts f evaluations at distinct points (the constructor evaluates f at x0).

Dot products and norms are plain sequential sums (numpy's BLAS may order
them differently: trajectories then differ in the last bits only).
tests/test_ncg_model.py holds this model to scipy on the oracle objective.
"""
import math

import numpy as np

EPS = 2.220446049250313e-16


class Objective:
    """ScalarFunction-like cache over fgh(x) -> (f, g[5], H[5][5])."""

    def __init__(self, fgh, x0):
        self.fgh = fgh
        self.x = None
        self.nfev = 0
        self._eval(x0)

    def _eval(self, x):
        if self.x is None or any(a != b for a, b in zip(x, self.x)):
            self.f, self.g, self.H = self.fgh(list(x))
            self.x = list(x)
            self.nfev += 1

    def fun(self, x):
        self._eval(x)
        return self.f

    def grad(self, x):
        self._eval(x)
        return list(self.g)

    def hess(self, x):
        self._eval(x)
        return [list(r) for r in self.H]


def dot(a, b):
    s = 0.0
    for u, v in zip(a, b):
        s += u * v
    return s


def l1(a):
    s = 0.0
    for u in a:
        s += abs(u)
    return s


def axpy_point(xk, s, pk):
    return [xk[i] + s * pk[i] for i in range(len(xk))]


# ---- MINPACK-2 dcstep (scipy/optimize/_dcsrch.py) ------------------------
def sign(v):
    return 1.0 if v > 0 else (-1.0 if v < 0 else (0.0 if v == 0 else v))


def dcstep(*args):
    with np.errstate(all="ignore"):
        return _dcstep(*[np.float64(a) if not isinstance(a, bool) else a for a in args])


def _dcstep(stx, fx, dx, sty, fy, dy, stp, fp, dp, brackt, stpmin, stpmax):
    sgnd = sign(dp) * sign(dx)
    if fp > fx:
        theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp
        s = max(abs(theta), abs(dx), abs(dp))
        gamma = s * np.sqrt((theta / s) ** 2 - (dx / s) * (dp / s))
        if stp < stx:
            gamma = -gamma
        p = (gamma - dx) + theta
        q = ((gamma - dx) + gamma) + dp
        r = p / q
        stpc = stx + r * (stp - stx)
        stpq = stx + ((dx / ((fx - fp) / (stp - stx) + dx)) / 2.0) * (stp - stx)
        if abs(stpc - stx) <= abs(stpq - stx):
            stpf = stpc
        else:
            stpf = stpc + (stpq - stpc) / 2.0
        brackt = True
    elif sgnd < 0.0:
        theta = 3 * (fx - fp) / (stp - stx) + dx + dp
        s = max(abs(theta), abs(dx), abs(dp))
        gamma = s * np.sqrt((theta / s) ** 2 - (dx / s) * (dp / s))
        if stp > stx:
            gamma = -gamma
        p = (gamma - dp) + theta
        q = ((gamma - dp) + gamma) + dx
        r = p / q
        stpc = stp + r * (stx - stp)
        stpq = stp + (dp / (dp - dx)) * (stx - stp)
        stpf = stpc if abs(stpc - stp) > abs(stpq - stp) else stpq
        brackt = True
    elif abs(dp) < abs(dx):
        theta = 3 * (fx - fp) / (stp - stx) + dx + dp
        s = max(abs(theta), abs(dx), abs(dp))
        gamma = s * np.sqrt(max(0, (theta / s) ** 2 - (dx / s) * (dp / s)))
        if stp > stx:
            gamma = -gamma
        p = (gamma - dp) + theta
        q = (gamma + (dx - dp)) + gamma
        r = p / q
        if r < 0 and gamma != 0:
            stpc = stp + r * (stx - stp)
        elif stp > stx:
            stpc = stpmax
        else:
            stpc = stpmin
        stpq = stp + (dp / (dp - dx)) * (stx - stp)
        if brackt:
            stpf = stpc if abs(stpc - stp) < abs(stpq - stp) else stpq
            if stp > stx:
                stpf = min(stp + 0.66 * (sty - stp), stpf)
            else:
                stpf = max(stp + 0.66 * (sty - stp), stpf)
        else:
            stpf = stpc if abs(stpc - stp) > abs(stpq - stp) else stpq
            stpf = min(max(stpf, stpmin), stpmax)
    else:
        if brackt:
            theta = 3.0 * (fp - fy) / (sty - stp) + dy + dp
            s = max(abs(theta), abs(dy), abs(dp))
            gamma = s * np.sqrt((theta / s) ** 2 - (dy / s) * (dp / s))
            if stp > sty:
                gamma = -gamma
            p = (gamma - dp) + theta
            q = ((gamma - dp) + gamma) + dy
            r = p / q
            stpf = stp + r * (sty - stp)
        elif stp > stx:
            stpf = stpmax
        else:
            stpf = stpmin
    if fp > fx:
        sty, fy, dy = stp, fp, dp
    else:
        if sgnd < 0:
            sty, fy, dy = stx, fx, dx
        stx, fx, dx = stp, fp, dp
    return stx, fx, dx, sty, fy, dy, stpf, brackt


def dcsrch(phi, derphi, alpha1, phi0, derphi0, ftol, gtol, xtol, stpmin, stpmax, maxiter=100):
    """DCSRCH.__call__ + _iterate: (stp or None, phi1, phi0)."""
    p5, p66, xtrapl, xtrapu = 0.5, 0.66, 1.1, 4.0
    stp, f, g = alpha1, phi0, derphi0
    # iteration 0: START
    if stp < stpmin or stp > stpmax or g >= 0 or stpmax < stpmin:
        return None, phi0, phi0
    brackt = False
    stage = 1
    finit, ginit = f, g
    gtest = ftol * ginit
    width = stpmax - stpmin
    width1 = width / p5
    stx, fx, gx = 0.0, finit, ginit
    sty, fy, gy = 0.0, finit, ginit
    stmin, stmax = 0.0, stp + xtrapu * stp
    if not math.isfinite(stp):
        return None, phi0, phi0
    f = phi(stp)
    g = derphi(stp)
    for it in range(1, maxiter):
        ftest = finit + stp * gtest
        if stage == 1 and f <= ftest and g >= 0:
            stage = 2
        warn = False
        if brackt and (stp <= stmin or stp >= stmax):
            warn = True
        if brackt and stmax - stmin <= xtol * stmax:
            warn = True
        if stp == stpmax and f <= ftest and g <= gtest:
            warn = True
        if stp == stpmin and (f > ftest or g >= gtest):
            warn = True
        if f <= ftest and abs(g) <= gtol * -ginit:
            return stp, f, phi0  # CONVERGENCE
        if warn:
            return None, f, phi0
        if stage == 1 and f <= fx and f > ftest:
            fm = f - stp * gtest
            fxm = fx - stx * gtest
            fym = fy - sty * gtest
            gm = g - gtest
            gxm = gx - gtest
            gym = gy - gtest
            stx, fxm, gxm, sty, fym, gym, stp, brackt = dcstep(
                stx, fxm, gxm, sty, fym, gym, stp, fm, gm, brackt, stmin, stmax)
            fx = fxm + stx * gtest
            fy = fym + sty * gtest
            gx = gxm + gtest
            gy = gym + gtest
        else:
            stx, fx, gx, sty, fy, gy, stp, brackt = dcstep(
                stx, fx, gx, sty, fy, gy, stp, f, g, brackt, stmin, stmax)
        if brackt:
            if abs(sty - stx) >= p66 * width1:
                stp = stx + p5 * (sty - stx)
            width1 = width
            width = abs(sty - stx)
        if brackt:
            stmin = min(stx, sty)
            stmax = max(stx, sty)
        else:
            stmin = stp + xtrapl * (stp - stx)
            stmax = stp + xtrapu * (stp - stx)
        stp = float(np.clip(stp, stpmin, stpmax))
        if (brackt and (stp <= stmin or stp >= stmax)) or \
                (brackt and stmax - stmin <= xtol * stmax):
            stp = stx
        if not math.isfinite(stp):
            return None, f, phi0
        f = phi(stp)
        g = derphi(stp)
    return None, f, phi0  # maxiter


# ---- wolfe2 (scipy/optimize/_linesearch.py) ------------------------------
def _fin(*v):
    return all(math.isfinite(u) for u in v)


def cubicmin(a, fa, fpa, b, fb, c, fc):
    """_cubicmin: None where numpy would raise (divide / overflow / invalid):
    any non-finite intermediate (the inputs are finite)."""
    C = fpa
    db = b - a
    dc = c - a
    denom = (db * dc) ** 2 * (db - dc)
    d00, d01, d10, d11 = dc ** 2, -db ** 2, -dc ** 3, db ** 3
    v0, v1 = fb - fa - C * db, fc - fa - C * dc
    A = d00 * v0 + d01 * v1
    B = d10 * v0 + d11 * v1
    if not _fin(denom, A, B) or denom == 0:
        return None
    A /= denom
    B /= denom
    radical = B * B - 3 * A * C
    if not _fin(A, B, radical) or radical < 0 or A == 0:
        return None
    xmin = a + (-B + math.sqrt(radical)) / (3 * A)
    return xmin if math.isfinite(xmin) else None


def quadmin(a, fa, fpa, b, fb):
    D = fa
    C = fpa
    db = b - a * 1.0
    dd = db * db
    if not _fin(dd) or dd == 0:
        return None
    B = (fb - D - C * db) / dd
    if not _fin(B) or B == 0:
        return None
    xmin = a - C / (2.0 * B)
    return xmin if math.isfinite(xmin) else None


def zoom(a_lo, a_hi, phi_lo, phi_hi, derphi_lo, phi, derphi, phi0, derphi0, c1, c2):
    maxiter, i = 10, 0
    delta1, delta2 = 0.2, 0.1
    phi_rec, a_rec = phi0, 0
    a_j = None
    while True:
        dalpha = a_hi - a_lo
        a, b = (a_hi, a_lo) if dalpha < 0 else (a_lo, a_hi)
        cchk = None
        if i > 0:
            cchk = delta1 * dalpha
            a_j = cubicmin(a_lo, phi_lo, derphi_lo, a_hi, phi_hi, a_rec, phi_rec)
        if i == 0 or a_j is None or a_j > b - cchk or a_j < a + cchk:
            qchk = delta2 * dalpha
            a_j = quadmin(a_lo, phi_lo, derphi_lo, a_hi, phi_hi)
            if a_j is None or a_j > b - qchk or a_j < a + qchk:
                a_j = a_lo + 0.5 * dalpha
        phi_aj = phi(a_j)
        if phi_aj > phi0 + c1 * a_j * derphi0 or phi_aj >= phi_lo:
            phi_rec, a_rec = phi_hi, a_hi
            a_hi, phi_hi = a_j, phi_aj
        else:
            derphi_aj = derphi(a_j)
            if abs(derphi_aj) <= -c2 * derphi0:
                return a_j, phi_aj
            if derphi_aj * (a_hi - a_lo) >= 0:
                phi_rec, a_rec = phi_hi, a_hi
                a_hi, phi_hi = a_lo, phi_lo
            else:
                phi_rec, a_rec = phi_lo, a_lo
            a_lo, phi_lo, derphi_lo = a_j, phi_aj, derphi_aj
        i += 1
        if i > maxiter:
            return None, None


def wolfe2(phi, derphi, phi0, old_phi0, derphi0, c1, c2, maxiter=10):
    """scalar_search_wolfe2 with amax None: (alpha or None, phi_star, phi0)."""
    alpha0 = 0
    if old_phi0 is not None and derphi0 != 0:
        alpha1 = min(1.0, 1.01 * 2 * (phi0 - old_phi0) / derphi0)
    else:
        alpha1 = 1.0
    if alpha1 < 0:
        alpha1 = 1.0
    phi_a1 = phi(alpha1)
    phi_a0, derphi_a0 = phi0, derphi0
    for i in range(maxiter):
        if alpha1 == 0:
            return None, phi0, old_phi0
        if phi_a1 > phi0 + c1 * alpha1 * derphi0 or (phi_a1 >= phi_a0 and i > 0):
            a, ps = zoom(alpha0, alpha1, phi_a0, phi_a1, derphi_a0, phi, derphi, phi0,
                         derphi0, c1, c2)
            return a, ps, phi0
        derphi_a1 = derphi(alpha1)
        if abs(derphi_a1) <= -c2 * derphi0:
            return alpha1, phi_a1, phi0
        if derphi_a1 >= 0:
            a, ps = zoom(alpha1, alpha0, phi_a1, phi_a0, derphi_a1, phi, derphi, phi0,
                         derphi0, c1, c2)
            return a, ps, phi0
        alpha2 = 2 * alpha1
        alpha0, alpha1 = alpha1, alpha2
        phi_a0 = phi_a1
        phi_a1 = phi(alpha1)
        derphi_a0 = derphi_a1
    return alpha1, phi_a1, phi0


# ---- _minimize_newtoncg ----------------------------------------------------
def newton_cg(fgh, x0, maxiter=2000, xtol_opt=-1.0, c1=1e-4, c2=0.9):
    """(x, f, nfev, status) as scipy's Newton-CG with hess given."""
    n = len(x0)
    obj = Objective(fgh, x0)
    cg_maxiter = 20 * n
    xtol = n * xtol_opt
    update_l1norm = 1.7976931348623157e308
    xk = list(x0)
    k = 0
    old_fval = obj.fun(xk)
    old_old_fval = None
    while update_l1norm > xtol:
        if k >= maxiter:
            return xk, old_fval, obj.nfev, 1
        gk = obj.grad(xk)
        b = [-v for v in gk]
        maggrad = l1(b)
        eta = min(0.5, math.sqrt(maggrad))
        termcond = eta * maggrad
        xsupi = [0.0] * n
        ri = [-v for v in b]
        psupi = [-v for v in ri]
        i = 0
        dri0 = dot(ri, ri)
        A = obj.hess(xk)
        for k2 in range(cg_maxiter):
            if l1(ri) <= termcond:
                break
            Ap = [dot(A[r], psupi) for r in range(n)]
            curv = dot(psupi, Ap)
            if 0 <= curv <= 3 * EPS:
                break
            elif curv < 0:
                if i > 0:
                    break
                xsupi = [dri0 / (-curv) * v for v in b]
                break
            alphai = dri0 / curv
            xsupi = [xsupi[j] + alphai * psupi[j] for j in range(n)]
            ri = [ri[j] + alphai * Ap[j] for j in range(n)]
            dri1 = dot(ri, ri)
            betai = dri1 / dri0
            psupi = [-ri[j] + betai * psupi[j] for j in range(n)]
            i += 1
            dri0 = dri1
        else:
            return xk, old_fval, obj.nfev, 3
        pk = xsupi
        gfk = gk

        def phi(s):
            return obj.fun(axpy_point(xk, s, pk))

        def derphi(s):
            return dot(obj.grad(axpy_point(xk, s, pk)), pk)

        derphi0 = dot(gfk, pk)
        # line_search_wolfe1 -> scalar_search_wolfe1 (amax 50, amin 1e-8, xtol 1e-14)
        if old_old_fval is not None and derphi0 != 0:
            alpha1 = min(1.0, 1.01 * 2 * (old_fval - old_old_fval) / derphi0)
            if alpha1 < 0:
                alpha1 = 1.0
        else:
            alpha1 = 1.0
        stp, fval, phi0 = dcsrch(phi, derphi, alpha1, old_fval, derphi0, c1, c2, 1e-14,
                                 1e-8, 50.0)
        if stp is None:
            stp, fval, phi0 = wolfe2(phi, derphi, old_fval, old_old_fval, derphi0, c1, c2)
            if stp is None:
                return xk, old_fval, obj.nfev, 2
        old_fval, old_old_fval = fval, phi0
        update = [stp * v for v in pk]
        xk = [xk[j] + update[j] for j in range(n)]
        k += 1
        update_l1norm = l1(update)
    if math.isnan(old_fval) or math.isnan(update_l1norm):
        return xk, old_fval, obj.nfev, 3
    return xk, old_fval, obj.nfev, 0
