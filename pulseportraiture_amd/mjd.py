"""MJD epoch with PSRCHIVE's representation: integer days, integer seconds
and fractional seconds (pr.MJD as used by pptoas.py:527-530 and write_TOAs,
pplib.py:3473-3479).  Adding a float adds *seconds* (pplib.py:3322)."""
import math


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
