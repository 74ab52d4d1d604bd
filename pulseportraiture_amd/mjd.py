"""MJD epoch with PSRCHIVE's representation: integer days, integer seconds
and fractional seconds (pr.MJD as used by pptoas.py:527-530 and write_TOAs,
pplib.py:3473-3479).  Adding a float adds *seconds* (pplib.py:3322)."""
import math

import numpy as np


class MJD(object):
    __slots__ = ("days", "secs", "fracsec")

    def __init__(self, *args):
        if len(args) == 0:
            d, s, f = 0, 0, 0.0
        elif len(args) == 1:
            dd = float(args[0])
            d = int(dd)
            fd = dd - d
            s = int(fd * 86400.0)
            f = fd * 86400.0 - s
        else:
            d, s, f = int(args[0]), int(args[1]), float(args[2])
        self.days, self.secs, self.fracsec = d, s, f
        self._settle()

    def _settle(self):
        isec = int(math.floor(self.fracsec))
        self.secs += isec
        self.fracsec -= isec
        iday = self.secs // 86400
        self.days += iday
        self.secs -= iday * 86400

    def __add__(self, other):
        if not isinstance(other, MJD):
            other = MJD(0, 0, float(other))
        return MJD(self.days + other.days, self.secs + other.secs,
                   self.fracsec + other.fracsec)

    __radd__ = __add__

    def in_days(self):
        return self.days + (self.secs + self.fracsec) / 86400.0

    def intday(self):
        return self.days

    def fracday(self):
        return (self.secs + self.fracsec) / 86400.0

    def as_tuple(self):
        return (self.days, self.secs, self.fracsec)

    def __repr__(self):
        return "MJD(%d, %d, %.17g)" % (self.days, self.secs, self.fracsec)

    @classmethod
    def _settled(cls, d, s, f):
        """An MJD from already-settled parts (no normalisation)."""
        m = object.__new__(cls)
        m.days, m.secs, m.fracsec = d, s, f
        return m


def epoch_parts(epochs):
    """(days, secs, fracsec) arrays of a list of MJDs."""
    n = len(epochs)
    d = np.fromiter((e.days for e in epochs), dtype=np.int64, count=n)
    s = np.fromiter((e.secs for e in epochs), dtype=np.int64, count=n)
    f = np.fromiter((e.fracsec for e in epochs), dtype=np.float64, count=n)
    return d, s, f


def _settle_arrays(d, s, f):
    """MJD._settle on arrays: the same integer / float operations elementwise."""
    isec = np.floor(f).astype(np.int64)
    s = s + isec
    f = f - isec
    iday = s // 86400
    return d + iday, s - iday * 86400, f


def add_days_parts(epochs_parts, x):
    """epochs[i] + MJD(x[i]) for float day offsets x, as MJD(x) then __add__
    compute them (every step elementwise with the same rounding), as
    (days, secs, fracsec) arrays."""
    d0, s0, f0 = epochs_parts
    x = np.asarray(x, dtype=np.float64)
    d = np.trunc(x).astype(np.int64)         # int(dd)
    fd = x - d
    s = np.trunc(fd * 86400.0).astype(np.int64)  # int(fd * 86400.0)
    f = fd * 86400.0 - s
    d, s, f = _settle_arrays(d, s, f)
    return _settle_arrays(d0 + d, s0 + s, f0 + f)


def add_days(epochs_parts, x):
    """add_days_parts as a list of MJDs."""
    d, s, f = add_days_parts(epochs_parts, x)
    mk = MJD._settled
    return [mk(a, b, c) for a, b, c in zip(d.tolist(), s.tolist(), f.tolist())]
