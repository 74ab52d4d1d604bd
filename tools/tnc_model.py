"""Scalar model of scipy's TNC (scipy/optimize/tnc/tnc.c, J.-S. Roy's C port of
S. Nash's truncated-Newton bound-constrained optimizer) -- DESIGN AID.

This is the specification the device solver (ppfit_tnc.hip) follows line for
line: the same operations in the same order, so that a trajectory computed
from the same f/g values is bitwise the same.  tests/test_tnc_model.py holds
it to scipy's compiled TNC by comparing the full sequence of points at which
the objective is evaluated.  Defaults are those scipy.optimize.minimize
(method='TNC') passes: scale/offset None, maxCGit -1, eta -1, stepmx 0,
accuracy 0, rescale -1, maxfun max(100, 10 n).
"""
import math

import numpy as np

EPS = np.finfo(float).eps
HUGE = math.inf

RC = {-1: "INFEASIBLE", 0: "LOCALMINIMUM", 1: "FCONVERGED", 2: "XCONVERGED", 3: "MAXFUN",
      4: "LSFAIL", 5: "CONSTANT", 6: "NOPROGRESS", 7: "USERABORT"}
GETPTC_OK, GETPTC_EVAL, GETPTC_EINVAL, GETPTC_FAIL = 0, 1, 2, 3
LS_OK, LS_MAXFUN, LS_FAIL = 0, 1, 2


def dnrm2(v):
    # tnc.c dnrm21: scaled sum of squares (BLAS dnrm2 style)
    dssq, scale = 1.0, 0.0
    for x in v:
        if x != 0.0:
            ax = abs(x)
            if scale < ax:
                dssq = 1.0 + dssq * (scale / ax) * (scale / ax)
                scale = ax
            else:
                dssq += (ax / scale) * (ax / scale)
    return scale * math.sqrt(dssq)


def ddot(a, b):
    s = 0.0
    for x, y in zip(a, b):
        s += x * y
    return s


class Counter:
    """scipy's ScalarFunction: a point equal to the previous one is not
    re-evaluated (nfev counts changes of x)."""

    def __init__(self, fg, x0):
        self.fg = fg
        self.x = np.array(x0, dtype=float)
        self.f, self.g = fg(self.x)
        self.nfev = 1
        self.points = [self.x.copy()]

    def __call__(self, x):
        x = np.array(x, dtype=float)
        if not np.array_equal(x, self.x):
            self.x = x
            self.f, self.g = self.fg(x)
            self.nfev += 1
            self.points.append(x.copy())
        return float(self.f), [float(v) for v in self.g]


class TNC:
    def __init__(self, fg, x0, bounds=None, maxfun=None, xtol=-1.0, ftol=-1.0, pgtol=-1.0,
                 fmin=0.0, eta=-1.0, stepmx=0.0, accuracy=0.0, rescale=-1.0, maxCGit=-1):
        n = len(x0)
        self.n = n
        self.fun = Counter(fg, x0)
        self.low = [(-HUGE if b is None or b[0] is None else float(b[0]))
                    for b in (bounds or [None] * n)]
        self.up = [(HUGE if b is None or b[1] is None else float(b[1]))
                   for b in (bounds or [None] * n)]
        self.maxfun = max(100, 10 * n) if maxfun is None else maxfun
        self.opts = dict(xtol=xtol, ftol=ftol, pgtol=pgtol, fmin=fmin, eta=eta, stepmx=stepmx,
                         accuracy=accuracy, rescale=rescale, maxCGit=maxCGit)
        self.x0 = [float(v) for v in x0]

    # --- helpers (tnc.c) -------------------------------------------------
    def f_g(self, x_unscaled):
        self.nfeval += 1
        return self.fun(x_unscaled)

    def coercex(self, x):
        for i in range(self.n):
            if x[i] < self.low[i]:
                x[i] = self.low[i]
            elif x[i] > self.up[i]:
                x[i] = self.up[i]

    def unscalex(self, x):
        for i in range(self.n):
            x[i] = x[i] * self.xscale[i] + self.xoffset[i]

    def scalex(self, x):
        for i in range(self.n):
            if self.xscale[i] > 0.0:
                x[i] = (x[i] - self.xoffset[i]) / self.xscale[i]

    def scaleg(self, g, fscale):
        for i in range(self.n):
            g[i] *= self.xscale[i] * fscale

    def project(self, v):
        for i in range(self.n):
            if self.pivot[i] != 0:
                v[i] = 0.0

    def project_constants(self, v):
        for i in range(self.n):
            if self.xscale[i] == 0.0:
                v[i] = 0.0

    def set_constraints(self, x):
        for i in range(self.n):
            if self.xscale[i] == 0.0:
                self.pivot[i] = 2
            elif self.low[i] != -HUGE and (x[i] * self.xscale[i] + self.xoffset[i] - self.low[i]
                                           <= EPS * 10.0 * (abs(self.low[i]) + 1.0)):
                self.pivot[i] = -1
            elif self.up[i] != HUGE and (x[i] * self.xscale[i] + self.xoffset[i] - self.up[i]
                                         >= EPS * 10.0 * (abs(self.up[i]) + 1.0)):
                self.pivot[i] = 1
            else:
                self.pivot[i] = 0

    def step_max(self, step, x, p):
        for i in range(self.n):
            if self.pivot[i] == 0 and p[i] != 0.0:
                if p[i] < 0.0:
                    t = (self.low[i] - self.xoffset[i]) / self.xscale[i] - x[i]
                    if t > step * p[i]:
                        step = t / p[i]
                else:
                    t = (self.up[i] - self.xoffset[i]) / self.xscale[i] - x[i]
                    if t < step * p[i]:
                        step = t / p[i]
        return step

    def add_constraint(self, x, p):
        newcon = False
        for i in range(self.n):
            if self.pivot[i] == 0 and p[i] != 0.0:
                if p[i] < 0.0 and self.low[i] != -HUGE:
                    tol = EPS * 10.0 * (abs(self.low[i]) + 1.0)
                    if x[i] * self.xscale[i] + self.xoffset[i] - self.low[i] <= tol:
                        self.pivot[i] = -1
                        x[i] = (self.low[i] - self.xoffset[i]) / self.xscale[i]
                        newcon = True
                elif p[i] > 0.0 and self.up[i] != HUGE:
                    tol = EPS * 10.0 * (abs(self.up[i]) + 1.0)
                    if self.up[i] - (x[i] * self.xscale[i] + self.xoffset[i]) <= tol:
                        self.pivot[i] = 1
                        x[i] = (self.up[i] - self.xoffset[i]) / self.xscale[i]
                        newcon = True
        return newcon

    def remove_constraint(self, gtpnew, gnorm, pgtolfs, f, flast, g):
        if (flast - f) <= (gtpnew * -0.5) and gnorm > pgtolfs:
            return False
        imax, cmax = -1, 0.0
        for i in range(self.n):
            if self.pivot[i] == 2:
                continue
            t = -self.pivot[i] * g[i]
            if t < cmax:
                cmax, imax = t, i
        if imax != -1:
            self.pivot[imax] = 0
            return True
        return False

    # --- preconditioner (msolve / initPreconditioner / ssbfgs) ------------
    @staticmethod
    def ssbfgs(n, gamma, sj, hjv, hjyj, yjsj, yjhyj, vsj, vhyj):
        if yjsj == 0.0:
            delta = beta = 0.0
        else:
            delta = (gamma * yjhyj / yjsj + 1.0) * vsj / yjsj - gamma * vhyj / yjsj
            beta = -gamma * vsj / yjsj
        return [gamma * hjv[i] + delta * sj[i] + beta * hjyj[i] for i in range(n)]

    def msolve(self, g):
        n = self.n
        diagb = self.diagb
        if self.upd1:
            return [g[i] / diagb[i] for i in range(n)]
        gsk = ddot(g, self.sk)
        if self.lreset:
            hg = [0.0] * n
            hyk = [0.0] * n
            for i in range(n):
                rdiagb = 1.0 / diagb[i]
                hg[i] = g[i] * rdiagb
                hyk[i] = self.yk[i] * rdiagb
            ykhyk = ddot(self.yk, hyk)
            ghyk = ddot(g, hyk)
            return self.ssbfgs(n, 1.0, self.sk, hg, hyk, self.yksk, ykhyk, gsk, ghyk)
        hg, hyk, hyr = [0.0] * n, [0.0] * n, [0.0] * n
        for i in range(n):
            rdiagb = 1.0 / diagb[i]
            hg[i] = g[i] * rdiagb
            hyk[i] = self.yk[i] * rdiagb
            hyr[i] = self.yr[i] * rdiagb
        gsr = ddot(g, self.sr)
        ghyr = ddot(g, hyr)
        yrhyr = ddot(self.yr, hyr)
        hg = self.ssbfgs(n, 1.0, self.sr, hg, hyr, self.yrsr, yrhyr, gsr, ghyr)
        yksr = ddot(self.yk, self.sr)
        ykhyr = ddot(self.yk, hyr)
        hyk = self.ssbfgs(n, 1.0, self.sr, hyk, hyr, self.yrsr, yrhyr, yksr, ykhyr)
        ykhyk = ddot(hyk, self.yk)
        ghyk = ddot(hyk, g)
        return self.ssbfgs(n, 1.0, self.sk, hg, hyk, self.yksk, ykhyk, gsk, ghyk)

    def init_preconditioner(self):
        n = self.n
        diagb = self.diagb
        if self.upd1:
            return list(diagb)
        emat = [0.0] * n
        bsk = [0.0] * n
        if self.lreset:
            for i in range(n):
                bsk[i] = diagb[i] * self.sk[i]
            sds = ddot(self.sk, bsk)
            yksk = self.yksk if self.yksk != 0.0 else 1.0
            if sds == 0.0:
                sds = 1.0
            for i in range(n):
                td = diagb[i]
                emat[i] = td - td * td * self.sk[i] * self.sk[i] / sds + \
                    self.yk[i] * self.yk[i] / yksk
        else:
            for i in range(n):
                bsk[i] = diagb[i] * self.sr[i]
            sds = ddot(self.sr, bsk)
            srds = ddot(self.sk, bsk)
            yrsk = ddot(self.yr, self.sk)
            yrsr = self.yrsr if self.yrsr != 0.0 else 1.0
            if sds == 0.0:
                sds = 1.0
            for i in range(n):
                td = diagb[i]
                bsk[i] = td * self.sk[i] - bsk[i] * srds / sds + self.yr[i] * yrsk / yrsr
                emat[i] = td - td * td * self.sr[i] * self.sr[i] / sds + \
                    self.yr[i] * self.yr[i] / yrsr
            sds = ddot(self.sk, bsk)
            yksk = self.yksk if self.yksk != 0.0 else 1.0
            if sds == 0.0:
                sds = 1.0
            for i in range(n):
                emat[i] = emat[i] - bsk[i] * bsk[i] / sds + self.yk[i] * self.yk[i] / yksk
        return emat

    def hessian_times_vector(self, v, x, g, xnorm):
        n = self.n
        delta = self.accuracy * (xnorm + 1.0)
        xv = [x[i] + delta * v[i] for i in range(n)]
        self.unscalex(xv)
        self.coercex(xv)
        _, gv = self.f_g(xv)
        gv = list(gv)
        self.scaleg(gv, self.fscale)
        dinv = 1.0 / delta
        for i in range(n):
            gv[i] = (gv[i] - g[i]) * dinv
        self.project_constants(gv)
        return gv

    def direction(self, x, g, gnorm, xnorm):
        """tnc_direction: preconditioned truncated CG for the Newton step."""
        n = self.n
        zsol = [0.0] * n
        if self.maxCGit == 0:
            zsol = [-v for v in g]
            self.project(zsol)
            return zsol
        rhsnrm = gnorm
        tol = 1e-12
        qold = 0.0
        rzold = 0.0
        r = [-v for v in g]
        self.project(r)
        emat = self.init_preconditioner()
        v = [0.0] * n
        for k in range(self.maxCGit):
            self.project(r)
            zk = self.msolve(r)
            self.project(zk)
            rz = ddot(r, zk)
            if rz / rhsnrm < tol or self.nfeval >= self.maxfun - 1:
                if k == 0:
                    zsol = [-vv for vv in g]
                    self.project(zsol)
                break
            beta = 0.0 if k == 0 else rz / rzold
            for i in range(n):
                v[i] = zk[i] + beta * v[i]
            self.project(v)
            gv = self.hessian_times_vector(v, x, g, xnorm)
            self.project(gv)
            vgv = ddot(v, gv)
            if vgv / rhsnrm < tol:
                if k == 0:
                    zsol = self.msolve(g)
                    zsol = [-vv for vv in zsol]
                    self.project(zsol)
                break
            self.diagonal_scaling(emat, v, gv, r)
            alpha = rz / vgv
            for i in range(n):
                zsol[i] += alpha * v[i]
            for i in range(n):
                r[i] += -alpha * gv[i]
            gtp = ddot(zsol, g)
            pr = ddot(r, zsol)
            qnew = (gtp + pr) * 0.5
            qtest = _qtest(k, qnew, qold)  # C double division: qold = 0 gives +-inf
            if qtest <= 0.5:
                break
            if gtp > 0.0:
                for i in range(n):
                    zsol[i] += -alpha * v[i]
                break
            qold = qnew
            rzold = rz
        self.diagb = list(emat)
        return zsol

    @staticmethod
    def diagonal_scaling(e, v, gv, r):
        vr = 1.0 / ddot(v, r)
        vgv = 1.0 / ddot(v, gv)
        for i in range(len(e)):
            e[i] += -r[i] * r[i] * vr + gv[i] * gv[i] * vgv
            if e[i] <= 1e-6:
                e[i] = 1.0

    # --- line search (linearSearch / getptcInit / getptcIter) --------------
    def linear_search(self, x, f, p, alpha, gfull, xbnd, eta, ftol):
        n = self.n
        temp = list(gfull)
        self.scaleg(temp, self.fscale)
        gu = ddot(temp, p)
        temp = list(x)
        self.project(temp)
        xnorm = dnrm2(temp)
        rteps = math.sqrt(EPS)
        pe = dnrm2(p) + EPS
        S = dict(reltol=rteps * (xnorm + 1.0) / pe,
                 abstol=-EPS * (1.0 + abs(f)) / (gu - EPS))
        tnytol = EPS * (xnorm + 1.0) / pe
        rtsmll = EPS
        big = 1.0 / (EPS * EPS)
        itcnt = 0
        fpresn = ftol
        S.update(u=alpha, fu=f, gu=gu, fmin=f, rmu=1e-4)
        itest = getptc_init(S, tnytol, eta, xbnd)
        if itest == GETPTC_EINVAL:
            return LS_FAIL, x, f, alpha, gfull
        gbest = list(gfull)
        while itest == GETPTC_EVAL and self.nfeval < self.maxfun:
            itcnt += 1
            ualpha = S["xmin"] + S["u"]
            temp = [x[i] + ualpha * p[i] for i in range(n)]
            self.unscalex(temp)
            self.coercex(temp)
            fu, tg = self.f_g(temp)
            fu *= self.fscale
            newg = list(tg)
            self.scaleg(newg, self.fscale)
            S["fu"] = fu
            S["gu"] = ddot(newg, p)
            itest = getptc_iter(S, big, rtsmll, tnytol, fpresn, xbnd)
            if S["xmin"] == ualpha:
                gbest = list(tg)
        if itest == GETPTC_OK:
            xn = [x[i] + S["xmin"] * p[i] for i in range(n)]
            return LS_OK, xn, S["fmin"], S["xmin"], gbest
        if self.nfeval >= self.maxfun:
            return LS_MAXFUN, x, f, S["xmin"], gbest
        return LS_FAIL, x, f, S["xmin"], gbest

    # --- driver (tnc + tnc_minimize) ----------------------------------------
    def run(self):
        n = self.n
        o = self.opts
        x = list(self.x0)
        self.nfeval = 0
        for i in range(n):
            if self.low[i] > self.up[i]:
                return self.result(x, None, -1)
        self.coercex(x)
        if self.maxfun < 1:
            return self.result(x, None, 3)
        f, g = self.f_g(list(x))
        gfull = list(g)
        nc = 0
        for i in range(n):
            if self.low[i] == self.up[i]:
                x[i] = self.low[i]
                nc += 1
        if nc == n:
            return self.result(x, f, 5)
        self.xscale = [0.0] * n
        self.xoffset = [0.0] * n
        for i in range(n):
            if self.low[i] != -HUGE and self.up[i] != HUGE:
                self.xscale[i] = self.up[i] - self.low[i]
                self.xoffset[i] = (self.up[i] + self.low[i]) * 0.5
            else:
                self.xscale[i] = 1.0 + abs(x[i])
                self.xoffset[i] = x[i]
        rteps = math.sqrt(EPS)
        stepmx = o["stepmx"]
        if stepmx < rteps * 10.0:
            stepmx = 1.0e1
        eta = o["eta"]
        if eta < 0.0 or eta >= 1.0:
            eta = 0.25
        rescale = o["rescale"]
        if rescale < 0.0:
            rescale = 1.3
        maxCGit = o["maxCGit"]
        if maxCGit < 0:
            maxCGit = n // 2
            if maxCGit < 1:
                maxCGit = 1
            elif maxCGit > 50:
                maxCGit = 50
        if maxCGit > n:
            maxCGit = n
        self.maxCGit = maxCGit
        accuracy = o["accuracy"]
        if accuracy <= EPS:
            accuracy = rteps
        self.accuracy = accuracy
        ftol = o["ftol"]
        if ftol < 0.0:
            ftol = accuracy
        pgtol = o["pgtol"]
        if pgtol < 0.0:
            pgtol = 1e-2 * math.sqrt(accuracy)
        xtol = o["xtol"]
        if xtol < 0.0:
            xtol = rteps
        rc, x, f = self.minimize(x, f, gfull, eta, stepmx, accuracy, o["fmin"], ftol, xtol,
                                 pgtol, rescale)
        return self.result(x, f, rc)

    def minimize(self, x, f, gfull, eta, stepmx, accuracy, fmin, ftol, xtol, pgtol, rescale):
        n = self.n
        self.fscale = 1.0
        difnew = 0.0
        epsred = 0.05
        self.upd1 = True
        icycle = n - 1
        newcon = True
        self.lreset = False
        self.yrsr = 0.0
        self.yksk = 0.0
        self.sk = [0.0] * n
        self.yk = [0.0] * n
        self.sr = [0.0] * n
        self.yr = [0.0] * n
        self.pivot = [0] * n
        alpha = 0.0
        self.scalex(x)
        f *= self.fscale
        self.set_constraints(x)
        g = list(gfull)
        self.scaleg(g, self.fscale)
        for i in range(n):
            if -self.pivot[i] * g[i] < 0.0:
                self.pivot[i] = 0
        self.project(g)
        gnorm = dnrm2(g)
        flast_con = f
        flast_reset = f
        self.diagb = [1.0] * n
        while True:
            if dnrm2(g) <= pgtol * self.fscale:
                rc = 0
                break
            if self.nfeval >= self.maxfun:
                rc = 3
                break
            newscale = dnrm2(g)
            if newscale > EPS and abs(math.log10(newscale)) > rescale:
                newscale = 1.0 / newscale
                f *= newscale
                self.fscale *= newscale
                gnorm *= newscale
                flast_con *= newscale
                flast_reset *= newscale
                difnew *= newscale
                for i in range(n):
                    g[i] *= newscale
                self.diagb = [1.0] * n
                self.upd1 = True
                icycle = n - 1
                newcon = True
            temp = list(x)
            self.project(temp)
            xnorm = dnrm2(temp)
            oldnfeval = self.nfeval
            pk = self.direction(x, g, gnorm, xnorm)
            if not newcon:
                if not self.lreset:
                    for i in range(n):
                        self.sr[i] += self.sk[i]
                        self.yr[i] += self.yk[i]
                    icycle += 1
                else:
                    self.sr = list(self.sk)
                    self.yr = list(self.yk)
                    flast_reset = f
                    icycle = 1
            oldg = list(g)
            oldf = f
            oldgtp = ddot(pk, g)
            ustpmax = stepmx / (dnrm2(pk) + EPS)
            spe = self.step_max(ustpmax, x, pk)
            if spe > 0.0:
                alpha = initial_step(f, fmin / self.fscale, oldgtp, spe)
                lsrc, x, f, alpha, gfull = self.linear_search(x, f, pk, alpha, gfull, spe, eta,
                                                              ftol)
                if alpha >= 0.9 * ustpmax:
                    stepmx *= 1e2
                if alpha - spe >= -EPS * 10.0:
                    newcon = True
                else:
                    if lsrc != LS_OK:
                        rc = 3 if lsrc == LS_MAXFUN else 4
                        break
                    newcon = False
            else:
                newcon = True
            if newcon:
                if not self.add_constraint(x, pk):
                    if self.nfeval == oldnfeval:
                        rc = 6
                        break
                flast_con = f
            difold = difnew
            difnew = oldf - f
            if icycle == 1:
                if difnew > difold * 2.0:
                    epsred += epsred
                if difnew < difold * 0.5:
                    epsred *= 0.5
            g = list(gfull)
            self.scaleg(g, self.fscale)
            temp = list(g)
            self.project(temp)
            gnorm = dnrm2(temp)
            remcon = self.remove_constraint(oldgtp, gnorm, pgtol * self.fscale, f, flast_con, g)
            if remcon:
                temp = list(g)
                self.project(temp)
                gnorm = dnrm2(temp)
            if not remcon and not newcon:
                if abs(difnew) <= ftol * self.fscale:
                    rc = 1
                    break
                if alpha * dnrm2(pk) <= xtol:
                    rc = 2
                    break
            self.project(g)
            if not newcon:
                for i in range(n):
                    self.yk[i] = g[i] - oldg[i]
                    self.sk[i] = alpha * pk[i]
                self.yksk = ddot(self.yk, self.sk)
                if icycle == n - 1 or difnew < epsred * (flast_reset - f):
                    self.lreset = True
                else:
                    self.yrsr = ddot(self.yr, self.sr)
                    self.lreset = self.yrsr <= 0.0
                self.upd1 = False
        self.unscalex(x)
        self.coercex(x)
        f /= self.fscale
        return rc, x, f

    def result(self, x, f, rc):
        # scipy's _minimize_tnc evaluates func_and_grad(x) once more
        fv, gv = self.fun(x)
        return dict(x=np.array(x), fun=fv, jac=np.array(gv), status=rc, nfev=self.fun.nfev,
                    points=self.fun.points)


def _qtest(k, qnew, qold):
    with np.errstate(all="ignore"):
        return (k + 1) * (1.0 - np.float64(qnew) / np.float64(qold))


def initial_step(fnew, fmin, gtp, smax):
    d = abs(fnew - fmin)
    alpha = 1.0
    if d * 2.0 <= -gtp and d >= EPS:
        alpha = d * 2.0 / -gtp
    if alpha >= smax:
        alpha = smax
    return alpha


def getptc_init(S, tnytol, eta, xbnd):
    u, gu = S["u"], S["gu"]
    if u <= 0.0 or xbnd <= tnytol or gu > 0.0:
        return GETPTC_EINVAL
    if xbnd < S["abstol"]:
        S["abstol"] = xbnd
    S["tol"] = S["abstol"]
    S["a"] = 0.0
    S["xw"] = 0.0
    S["xmin"] = 0.0
    S["oldf"] = S["fu"]
    S["fmin"] = S["fu"]
    S["fw"] = S["fu"]
    S["gw"] = gu
    S["gmin"] = gu
    S["step"] = u
    S["factor"] = 5.0
    S["braktd"] = False
    S["scxbnd"] = xbnd
    S["b"] = S["scxbnd"] + S["reltol"] * abs(S["scxbnd"]) + S["abstol"]
    S["e"] = S["b"] + S["b"]
    S["b1"] = S["b"]
    S["gtest1"] = -S["rmu"] * gu
    S["gtest2"] = -eta * gu
    if S["step"] >= S["scxbnd"]:
        S["step"] = S["scxbnd"]
        S["scxbnd"] -= (S["reltol"] * abs(xbnd) + S["abstol"]) / (1.0 + S["reltol"])
    S["u"] = S["step"]
    if abs(S["step"]) < S["tol"] and S["step"] < 0.0:
        S["u"] = -S["tol"]
    if abs(S["step"]) < S["tol"] and S["step"] >= 0.0:
        S["u"] = S["tol"]
    return GETPTC_EVAL


def getptc_iter(S, big, rtsmll, tnytol, fpresn, xbnd):
    u, fu, gu = S["u"], S["fu"], S["gu"]
    to_conv = False
    if fu <= S["fmin"]:
        chordu = S["oldf"] - (S["xmin"] + u) * S["gtest1"]
        if not (fu <= chordu):
            chordm = S["oldf"] - S["xmin"] * S["gtest1"]
            gu = -S["gmin"]
            denom = chordm - S["fmin"]
            if abs(denom) < 1e-15:
                denom = 1e-15
                if chordm - S["fmin"] < 0.0:
                    denom = -denom
            if S["xmin"] != 0.0:
                gu = S["gmin"] * (chordu - fu) / denom
            fu = 0.5 * u * (S["gmin"] + gu) + S["fmin"]
            if fu < S["fmin"]:
                fu = S["fmin"]
        else:
            S["fw"] = S["fmin"]
            S["fmin"] = fu
            S["gw"] = S["gmin"]
            S["gmin"] = gu
            S["xmin"] += u
            S["a"] -= u
            S["b"] -= u
            S["xw"] = -u
            S["scxbnd"] -= u
            if gu <= 0.0:
                S["a"] = 0.0
            else:
                S["b"] = 0.0
                S["braktd"] = True
            S["tol"] = abs(S["xmin"]) * S["reltol"] + S["abstol"]
            to_conv = True
    if not to_conv:
        if u < 0.0:
            S["a"] = u
        else:
            S["b"] = u
            S["braktd"] = True
        S["xw"] = u
        S["fw"] = fu
        S["gw"] = gu
    S["u"], S["fu"], S["gu"] = u, fu, gu
    # ConvergenceCheck
    twotol = S["tol"] + S["tol"]
    xmidpt = 0.5 * (S["a"] + S["b"])
    convrg = (abs(xmidpt) <= twotol - 0.5 * (S["b"] - S["a"])) or (
        abs(S["gmin"]) <= S["gtest2"] and S["fmin"] < S["oldf"] and
        ((abs(S["xmin"] - xbnd) > S["tol"]) or (not S["braktd"])))
    if convrg:
        if S["xmin"] != 0.0:
            return GETPTC_OK
        if abs(S["oldf"] - S["fw"]) <= fpresn:
            return GETPTC_FAIL
        S["tol"] = 0.1 * S["tol"]
        if S["tol"] < tnytol:
            return GETPTC_FAIL
        S["reltol"] = 0.1 * S["reltol"]
        S["abstol"] = 0.1 * S["abstol"]
        twotol = 0.1 * twotol
    r = q = s = 0.0
    minimum_found = False
    if abs(S["e"]) > S["tol"]:
        r = 3.0 * (S["fmin"] - S["fw"]) / S["xw"] + S["gmin"] + S["gw"]
        absr = abs(r)
        q = absr
        if S["gw"] != 0.0 and S["gmin"] != 0.0:
            abgw = abs(S["gw"])
            abgmin = abs(S["gmin"])
            s = math.sqrt(abgmin) * math.sqrt(abgw)
            if (S["gw"] / abgw) * S["gmin"] > 0.0:
                if r >= s or r <= -s:
                    q = math.sqrt(abs(r + s)) * math.sqrt(abs(r - s))
                else:
                    r = 0.0
                    q = 0.0
                    minimum_found = True
            else:
                sumsq = 1.0
                p = 0.0
                if absr >= s:
                    if absr > rtsmll:
                        p = absr * rtsmll
                    if s >= p:
                        value = s / absr
                        sumsq = 1.0 + value * value
                    scale = absr
                else:
                    if s > rtsmll:
                        p = s * rtsmll
                    if absr >= p:
                        value = absr / s
                        sumsq = 1.0 + value * value
                    scale = s
                sumsq = math.sqrt(sumsq)
                q = big
                if scale < big / sumsq:
                    q = scale * sumsq
        if not minimum_found:
            if S["xw"] < 0.0:
                q = -q
            s = S["xw"] * (S["gmin"] - r - q)
            q = S["gw"] - S["gmin"] + q + q
            if q > 0.0:
                s = -s
            if q <= 0.0:
                q = -q
            r = S["e"]
            if S["b1"] != S["step"] or S["braktd"]:
                S["e"] = S["step"]
    # MinimumFound
    a1 = S["a"]
    S["b1"] = S["b"]
    S["step"] = xmidpt
    if (not S["braktd"]) or ((S["a"] == 0.0 and S["xw"] < 0.0) or
                             (S["b"] == 0.0 and S["xw"] > 0.0)):
        if S["braktd"]:
            d1 = S["xw"]
            d2 = S["a"]
            if S["a"] == 0.0:
                d2 = S["b"]
            S["u"] = -d1 / d2
            S["step"] = 5.0 * d2 * (0.1 + 1.0 / S["u"]) / 11.0
            if S["u"] < 1.0:
                S["step"] = 0.5 * d2 * math.sqrt(S["u"])
        else:
            S["step"] = -S["factor"] * S["xw"]
            if S["step"] > S["scxbnd"]:
                S["step"] = S["scxbnd"]
            if S["step"] != S["scxbnd"]:
                S["factor"] = 5.0 * S["factor"]
        if S["step"] <= 0.0:
            a1 = S["step"]
        if S["step"] > 0.0:
            S["b1"] = S["step"]
    if abs(s) <= abs(0.5 * q * r) or s <= q * a1 or s >= q * S["b1"]:
        S["e"] = S["b"] - S["a"]
    else:
        S["step"] = s / q
        if S["step"] - S["a"] < twotol or S["b"] - S["step"] < twotol:
            if xmidpt <= 0.0:
                S["step"] = -S["tol"]
            else:
                S["step"] = S["tol"]
    if S["step"] >= S["scxbnd"]:
        S["step"] = S["scxbnd"]
        S["scxbnd"] -= (S["reltol"] * abs(xbnd) + S["abstol"]) / (1.0 + S["reltol"])
    S["u"] = S["step"]
    if abs(S["step"]) < S["tol"] and S["step"] < 0.0:
        S["u"] = -S["tol"]
    if abs(S["step"]) < S["tol"] and S["step"] >= 0.0:
        S["u"] = S["tol"]
    return GETPTC_EVAL


def minimize_tnc(fg, x0, bounds=None, **kw):
    return TNC(fg, x0, bounds, **kw).run()
