"""TOA records held as columns (the get_TOAs output side, pptoas.py:31-73,
606-661 and pplib.py:3451-3509).

The reference builds one ``TOA`` object per subint, each with a flag dict,
and write_TOAs %-formats every flag of every TOA in Python.  Here get_TOAs
builds one ``TOABlock`` per archive shard: the TOA fields and every flag as
columns (numpy arrays, constants, or per-row presence masks where a flag is
carried by some rows only).  ``TOAList`` -- the type of ``GetTOAs.TOA_list``
-- is a mutable sequence over such blocks and plain TOA objects:

- indexing or iterating builds the ``TOA`` objects of a block on access,
  with the reference's attributes and flag dict (insertion order as
  pptoas.py:606-661 sets it), and keeps them, so a TOA modified by the
  caller (pptoas.py:1593-1602's one-DM rewrite) is written as modified;
- ``write_TOAs`` (pplib.py) formats the rows never built as objects in one
  call of the native .tim writer (libpptim.so, include/pptim.h), and the
  built ones one by one as before -- the same text either way.

``MJDArray`` is the per-archive ``TOAs`` entry: the fitted MJDs of an
archive as integer-day / second / fractional-second columns, indexed like
the reference's object array (an unfitted subint reads 0).
"""
import bisect
import ctypes
import os
from collections.abc import MutableSequence

import numpy as np

from .mjd import MJD

_HERE = os.path.dirname(os.path.abspath(__file__))
TIM_LIB_PATH = os.path.join(_HERE, "libpptim.so")


class TOA:
    """TOA record, pptoas.py:31-73.  The reference sets every flag as an
    attribute (pptoas.py:70-72); here the base fields are slots and a flag
    attribute reads through to ``flags`` (attributes set later live in the
    instance dict, which shadows a flag of the same name)."""
    __slots__ = ("archive", "frequency", "MJD", "TOA_error", "telescope", "telescope_code",
                 "DM", "DM_error", "flags", "__dict__")

    def __init__(self, archive, frequency, MJD, TOA_error, telescope, telescope_code,
                 DM=None, DM_error=None, flags={}):
        self.archive = archive
        self.frequency = frequency
        self.MJD = MJD
        self.TOA_error = TOA_error
        self.telescope = telescope
        self.telescope_code = telescope_code
        self.DM = DM
        self.DM_error = DM_error
        self.flags = flags

    def __getattr__(self, name):  # only when no slot / instance attribute has it
        if name != "flags":
            try:
                return self.flags[name]
            except (KeyError, AttributeError):
                pass
        raise AttributeError("'TOA' object has no attribute %r" % name)

    def write_TOA(self, inf_is_zero=True, outfile=None):
        from .pplib import write_TOAs
        return write_TOAs(self, inf_is_zero=inf_is_zero, outfile=outfile, append=True)


# ---------------------------------------------------------------------------
# native .tim writer (include/pptim.h)
# ---------------------------------------------------------------------------
PPT_TEXT, PPT_I64, PPT_F64_FIXED, PPT_F64_EXP, PPT_F64_FRAC, PPT_STRS = range(6)


class _Field(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("prec", ctypes.c_int32), ("data", ctypes.c_void_p),
                ("offs", ctypes.c_void_p), ("present", ctypes.c_void_p)]


_tim = None


def load_tim_library():
    """libpptim.so (host C++); raises if it is not built -- there is no
    Python fallback for the bulk writer."""
    global _tim
    if _tim is not None:
        return _tim
    if not os.path.exists(TIM_LIB_PATH):
        raise RuntimeError("libpptim.so not found at %s: build it with "
                           "`python -c 'import __graft_entry__ as g; g.build()'`" % TIM_LIB_PATH)
    lib = ctypes.CDLL(TIM_LIB_PATH)
    vp = ctypes.c_void_p
    lib.ppt_format_rows.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(_Field), vp,
                                    ctypes.c_int32, ctypes.POINTER(vp)]
    lib.ppt_format_rows.restype = ctypes.c_int
    lib.ppt_text_nparts.argtypes = [vp]
    lib.ppt_text_nparts.restype = ctypes.c_int64
    lib.ppt_text_part.argtypes = [vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    lib.ppt_text_part.restype = vp
    lib.ppt_text_size.argtypes = [vp]
    lib.ppt_text_size.restype = ctypes.c_int64
    lib.ppt_text_rows.argtypes = [vp]
    lib.ppt_text_rows.restype = ctypes.c_int64
    lib.ppt_text_free.argtypes = [vp]
    lib.ppt_text_free.restype = None
    _tim = lib
    return lib


def _host_threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(8, n))


class TimText:
    """Text from the native writer: owns the library's buffers (freed with
    this object); ``chunks()`` are zero-copy memoryviews of them."""

    def __init__(self, handle):
        self._h = handle
        lib = load_tim_library()
        self.rows = lib.ppt_text_rows(handle)
        self.size = lib.ppt_text_size(handle)

    def chunks(self):
        lib = load_tim_library()
        out = []
        for i in range(lib.ppt_text_nparts(self._h)):
            sz = ctypes.c_int64()
            ptr = lib.ppt_text_part(self._h, i, ctypes.byref(sz))
            if sz.value:
                out.append(memoryview((ctypes.c_char * sz.value).from_address(ptr)).cast("B"))
        return out

    def to_bytes(self):
        return b"".join(bytes(c) for c in self.chunks())

    def __str__(self):
        return self.to_bytes().decode("utf-8", "surrogateescape")

    def __del__(self):
        if getattr(self, "_h", None) is not None and _tim is not None:
            _tim.ppt_text_free(self._h)
            self._h = None


def format_rows(n, fields, keep=None):
    """Run the native writer over n rows.  fields: list of (kind, prec, data,
    offs, present) with numpy arrays / bytes; returns a TimText."""
    lib = load_tim_library()
    arr = (_Field * max(1, len(fields)))()
    hold = []

    def ptr(a):
        if a is None:
            return None
        if isinstance(a, bytes):
            b = ctypes.create_string_buffer(a, len(a) + 1)
            hold.append(b)
            return ctypes.cast(b, ctypes.c_void_p)
        hold.append(a)
        return a.ctypes.data

    for i, (kind, prec, data, offs, present) in enumerate(fields):
        arr[i].kind, arr[i].prec = kind, prec
        arr[i].data, arr[i].offs, arr[i].present = ptr(data), ptr(offs), ptr(present)
    h = ctypes.c_void_p()
    kp = None if keep is None else np.ascontiguousarray(keep, dtype=np.uint8)
    rc = lib.ppt_format_rows(int(n), len(fields), arr, None if kp is None else kp.ctypes.data,
                             _host_threads(), ctypes.byref(h))
    if rc != 0:
        raise RuntimeError("ppt_format_rows failed (%d)" % rc)
    return TimText(h)


def _flag_kind(key, kind):
    """(PPT kind, precision) of a numeric flag column as write_TOAs formats
    it (pplib.py:3488-3503): int %d, '_cov' %.1e, 'phs' %.8f, 'flux' %.5f,
    else %.3f."""
    if kind == "i64":
        return PPT_I64, 0
    if key.find("_cov") >= 0:
        return PPT_F64_EXP, 1
    if key.find("phs") >= 0:
        return PPT_F64_FIXED, 8
    if key.find("flux") >= 0:
        return PPT_F64_FIXED, 5
    return PPT_F64_FIXED, 3


def _strs_field(texts):
    """A PPT_STRS field from per-row strings."""
    enc = [t.encode("utf-8", "surrogateescape") for t in texts]
    offs = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum([len(b) for b in enc], out=offs[1:])
    return (PPT_STRS, 0, b"".join(enc) or b"\0", offs, None)


# ---------------------------------------------------------------------------
# columns
# ---------------------------------------------------------------------------
class FlagColumn:
    """One flag of a block: ``kind`` "const" (``values`` is the one value),
    "f64" / "i64" (numpy arrays; the TOA objects get Python floats / ints),
    or "obj" (a list of Python objects).  ``present`` is None (every row
    carries the flag) or a bool array."""
    __slots__ = ("key", "kind", "values", "present")

    def __init__(self, key, kind, values, present=None):
        self.key, self.kind, self.values, self.present = key, kind, values, present

    @classmethod
    def of(cls, key, values, n, present=None):
        """A column from a constant, a numpy array or a list: float / int
        arrays are kept typed, anything else as objects."""
        if not isinstance(values, (list, tuple, np.ndarray)):
            return cls(key, "const", values, present)
        a = np.asarray(values) if not isinstance(values, np.ndarray) else values
        if a.dtype.kind == "f":
            return cls(key, "f64", np.ascontiguousarray(a, dtype=np.float64), present)
        if a.dtype.kind in "iu":
            return cls(key, "i64", np.ascontiguousarray(a, dtype=np.int64), present)
        vals = list(values)
        if vals and all(type(v) is float for v in vals):
            return cls(key, "f64", np.array(vals, dtype=np.float64), present)
        if vals and all(type(v) is int for v in vals):
            return cls(key, "i64", np.array(vals, dtype=np.int64), present)
        return cls(key, "obj", vals, present)

    def take(self, idx):
        p = None if self.present is None else self.present[idx]
        if self.kind == "const":
            return FlagColumn(self.key, "const", self.values, p)
        if self.kind == "obj":
            return FlagColumn(self.key, "obj", [self.values[i] for i in idx], p)
        return FlagColumn(self.key, self.kind, self.values[idx], p)

    def row_values(self):
        """Per-row Python values (tolist: Python floats / ints)."""
        if self.kind in ("f64", "i64"):
            return self.values.tolist()
        return self.values

    def value(self, r):
        if self.kind == "const":
            return self.values
        if self.kind == "f64":
            return float(self.values[r])
        if self.kind == "i64":
            return int(self.values[r])
        return self.values[r]


class TOABlock:
    """The TOA records of one archive shard as columns (pptoas.py:606-661).

    ``freq``, ``err`` float64 [n]; ``mjd`` (days int64, secs int64, fracsec
    float64) [n]; ``dm``, ``dme`` float64 [n] or None with ``dm_present``
    (rows whose TOA carries DM / DM_error; the others carry None); ``cols``
    the flags in insertion order.  ``cache`` holds the TOA objects built so
    far (None: none built)."""

    def __init__(self, archive, telescope, telescope_code, freq, mjd, err, dm=None, dme=None,
                 dm_present=None, cols=()):
        self.archive, self.telescope, self.telescope_code = archive, telescope, telescope_code
        self.freq = np.ascontiguousarray(freq, dtype=np.float64)
        self.n = len(self.freq)
        self.mjd = tuple(np.ascontiguousarray(a) for a in mjd)
        self.err = np.ascontiguousarray(err, dtype=np.float64)
        self.dm = None if dm is None else np.ascontiguousarray(dm, dtype=np.float64)
        self.dme = None if dme is None else np.ascontiguousarray(dme, dtype=np.float64)
        self.dm_present = dm_present
        self.cols = list(cols)
        self.cache = None
        self.text = None  # (inf_is_zero, text) pre-formatted by the shard's rank

    def __len__(self):
        return self.n

    def add_flags(self, items):
        """flags.update(items) on every row (pptoas.py:649-650): a key the
        block already has keeps its place where a row carries it and is
        appended where it does not."""
        for k, v in items:
            hit = [c for c in self.cols if c.key == k]
            if not hit:
                self.cols.append(FlagColumn(k, "const", v))
                continue
            have = np.zeros(self.n, dtype=bool)
            for c in hit:
                i = self.cols.index(c)
                self.cols[i] = FlagColumn(k, "const", v, c.present)
                have |= True if c.present is None else c.present
            if not have.all():
                self.cols.append(FlagColumn(k, "const", v, ~have))

    # -- TOA objects ---------------------------------------------------------
    def _build(self, rows):
        new = object.__new__
        mk = MJD._settled
        d, s, f = (a[rows].tolist() for a in self.mjd)
        fr, er = self.freq[rows].tolist(), self.err[rows].tolist()
        if self.dm is not None:
            dm, dme = self.dm[rows].tolist(), self.dme[rows].tolist()
            dp = [True] * len(rows) if self.dm_present is None else \
                self.dm_present[rows].tolist()
        cols = []
        for c in self.cols:
            cc = c.take(rows) if len(rows) != self.n else c
            cols.append((cc.key, cc.kind == "const", cc.values if cc.kind == "const"
                         else cc.row_values(),
                         None if cc.present is None else cc.present.tolist()))
        plain = all(p is None for _, _, _, p in cols)
        keys = [k for k, _, _, _ in cols]
        out = []
        for j in range(len(rows)):
            if plain:
                flags = dict(zip(keys, [v if const else v[j] for _, const, v, _ in cols]))
            else:
                flags = {}
                for k, const, v, p in cols:
                    if p is None or p[j]:
                        flags[k] = v if const else v[j]
            t = new(TOA)
            t.archive = self.archive
            t.frequency = fr[j]
            t.MJD = mk(d[j], s[j], f[j])
            t.TOA_error = er[j]
            t.telescope = self.telescope
            t.telescope_code = self.telescope_code
            if self.dm is not None and dp[j]:
                t.DM, t.DM_error = dm[j], dme[j]
            else:
                t.DM = t.DM_error = None
            t.flags = flags
            out.append(t)
        return out

    def toa(self, r):
        if self.cache is None:
            self.cache = [None] * self.n
        t = self.cache[r]
        if t is None:
            t = self.cache[r] = self._build([r])[0]
        return t

    def toas(self):
        """Every row's TOA object (built once, then kept)."""
        if self.cache is None:
            self.cache = self._build(np.arange(self.n))
        elif any(t is None for t in self.cache):
            miss = [r for r, t in enumerate(self.cache) if t is None]
            for r, t in zip(miss, self._build(np.asarray(miss))):
                self.cache[r] = t
        return self.cache

    # -- .tim text -------------------------------------------------------------
    def _fields(self, inf_is_zero):
        """The native writer's fields of one line (pplib.py:3471-3503)."""
        freq = self.freq
        if inf_is_zero:
            freq = np.where(freq == np.inf, 0.0, freq)
        days, secs, frac = self.mjd
        fracday = (secs.astype(np.float64) + frac) / 86400.0  # MJD.fracday
        f = [(PPT_TEXT, 0, ("%s " % (self.archive,)).encode("utf-8", "surrogateescape"),
              None, None),
             (PPT_F64_FIXED, 8, np.ascontiguousarray(freq), None, None),
             (PPT_TEXT, 0, b" ", None, None),
             (PPT_I64, 0, np.ascontiguousarray(days, dtype=np.int64), None, None),
             (PPT_F64_FRAC, 15, fracday, None, None),
             (PPT_TEXT, 0, b"   ", None, None),
             (PPT_F64_FIXED, 3, self.err, None, None),
             (PPT_TEXT, 0, ("  %s" % (self.telescope_code,)).encode("utf-8", "surrogateescape"),
              None, None)]
        if self.dm is not None:
            dp = None if self.dm_present is None else \
                np.ascontiguousarray(self.dm_present, dtype=np.uint8)
            f += [(PPT_TEXT, 0, b" -pp_dm ", None, dp), (PPT_F64_FIXED, 7, self.dm, None, dp),
                  (PPT_TEXT, 0, b" -pp_dme ", None, dp), (PPT_F64_FIXED, 7, self.dme, None, dp)]
        from .pplib import _flag_text
        for c in self.cols:
            p = None if c.present is None else np.ascontiguousarray(c.present, dtype=np.uint8)
            if c.kind == "const":
                if c.values is None:
                    continue
                f.append((PPT_TEXT, 0, _flag_text(c.key, c.values).encode(
                    "utf-8", "surrogateescape"), None, p))
            elif c.kind == "obj":
                kind, prec, data, offs, _ = _strs_field(
                    ["" if v is None else _flag_text(c.key, v) for v in c.values])
                f.append((kind, prec, data, offs, p))
            else:
                kind, prec = _flag_kind(c.key, c.kind)
                f.append((PPT_TEXT, 0, (" -%s " % c.key).encode("utf-8", "surrogateescape"),
                          None, p))
                f.append((kind, prec, c.values, None, p))
        return f

    def snr_keep(self, cutoff):
        """filter_TOAs(toas, "snr", cutoff, ">=", pass_unflagged=False) on the
        rows (pplib.py:3466): rows without an snr flag are dropped."""
        keep = np.zeros(self.n, dtype=bool)
        for c in self.cols:
            if c.key != "snr":
                continue
            p = np.ones(self.n, dtype=bool) if c.present is None else c.present
            if c.kind == "const":
                ok = np.full(self.n, _ge(c.values, cutoff))
            elif c.kind == "obj":
                ok = np.array([_ge(v, cutoff) for v in c.values], dtype=bool)
            else:
                ok = c.values >= cutoff
            keep = np.where(p, ok, keep)
        return keep

    def format(self, inf_is_zero=True, keep=None):
        """.tim text of the rows (keep: bool mask), '\\n'-terminated lines:
        bytes, or a TimText holding the native writer's buffers."""
        if keep is None and self.text is not None and self.text[0] == bool(inf_is_zero):
            return self.text[1]
        return format_rows(self.n, self._fields(inf_is_zero), keep)

    def preformat(self, inf_is_zero=True):
        """Format every row now and keep the text (get_TOAs does, for each
        shard as its fits complete, so write_TOAs only writes; a rank's
        shard travels to the gathering rank with its text)."""
        self.text = (bool(inf_is_zero), self.format(inf_is_zero))

    def __getstate__(self):
        st = dict(self.__dict__)
        if st.get("text") is not None:  # the native buffers travel as bytes
            st["text"] = (st["text"][0], _as_bytes(st["text"][1]))
        return st

    def __setstate__(self, st):
        self.__dict__.update(st)


def _as_bytes(piece):
    return piece.to_bytes() if isinstance(piece, TimText) else piece


def write_pieces(f, pieces):
    """Write tim_chunks' pieces to a binary file object."""
    for p in pieces:
        if isinstance(p, TimText):
            for c in p.chunks():
                f.write(c)
        else:
            f.write(p)


def _ge(v, cutoff):
    try:
        return bool(v >= cutoff)
    except TypeError:
        return False


class TOAList(MutableSequence):
    """GetTOAs.TOA_list: a list of TOA records whose get_TOAs part is held
    as TOABlocks (objects built on access) -- see the module docstring."""

    def __init__(self, iterable=()):
        self._segs = []
        self._starts = None
        if iterable:
            self.extend(iterable)

    # -- segments ----------------------------------------------------------
    def _index(self):
        if self._starts is None:
            st, n = [], 0
            for s in self._segs:
                st.append(n)
                n += len(s)
            self._starts, self._n = st, n
        return self._starts

    def _flat(self):
        """Collapse to one plain list segment (for arbitrary mutation)."""
        out = []
        for s in self._segs:
            out.extend(s.toas() if isinstance(s, TOABlock) else s)
        self._segs = [out] if out else []
        self._starts = None
        return out

    def add_block(self, block):
        if block.n:
            self._segs.append(block)
            self._starts = None

    def blocks(self):
        return [s for s in self._segs if isinstance(s, TOABlock)]

    # -- sequence protocol -----------------------------------------------------
    def __len__(self):
        self._index()
        return self._n

    def _locate(self, i):
        n = len(self)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError("list index out of range")
        k = bisect.bisect_right(self._starts, i) - 1
        return self._segs[k], i - self._starts[k]

    def __getitem__(self, i):
        if isinstance(i, slice):
            return list(self)[i]
        seg, j = self._locate(int(i))
        return seg.toa(j) if isinstance(seg, TOABlock) else seg[j]

    def __iter__(self):
        for s in self._segs:
            yield from (s.toas() if isinstance(s, TOABlock) else list(s))

    def __setitem__(self, i, v):
        flat = self._flat()
        flat[i] = v
        self._starts = None

    def __delitem__(self, i):
        flat = self._flat()
        del flat[i]
        self._segs = [flat] if flat else []
        self._starts = None

    def insert(self, i, v):
        if i >= len(self):
            self.append(v)
            return
        self._flat().insert(i, v)
        self._starts = None

    def append(self, v):
        if self._segs and isinstance(self._segs[-1], list):
            self._segs[-1].append(v)
        else:
            self._segs.append([v])
        self._starts = None

    def extend(self, vals):
        if isinstance(vals, TOAList):
            for s in list(vals._segs):
                if isinstance(s, TOABlock):
                    self._segs.append(s)
                else:
                    self._segs.append(list(s))
            self._starts = None
        elif isinstance(vals, TOABlock):
            self.add_block(vals)
        else:
            for v in vals:
                self.append(v)

    def __iadd__(self, vals):
        self.extend(vals)
        return self

    def __add__(self, other):
        return list(self) + list(other)

    def __radd__(self, other):
        return list(other) + list(self)

    def __eq__(self, other):
        if isinstance(other, (list, TOAList)):
            return len(self) == len(other) and all(a is b or a == b
                                                   for a, b in zip(self, other))
        return NotImplemented

    def __repr__(self):
        return "TOAList(%d TOAs)" % len(self)

    def clear(self):
        self._segs, self._starts = [], None

    def copy(self):
        return list(self)

    def sort(self, key=None, reverse=False):
        self._flat().sort(key=key, reverse=reverse)

    # -- .tim text ---------------------------------------------------------
    def tim_chunks(self, inf_is_zero=True, SNR_cutoff=0.0):
        """write_TOAs' text of every TOA (pplib.py:3464-3509) as a list of
        pieces, each bytes or a TimText (write its .chunks() while it is
        alive): rows of blocks whose objects were never built go through the
        native writer, built TOA objects through pplib.toa_line."""
        from .pplib import toa_line
        out = []

        def enc(lines):
            return "".join(ln + "\n" for ln in lines).encode("utf-8", "surrogateescape")

        for s in self._segs:
            if isinstance(s, TOABlock):
                keep = s.snr_keep(SNR_cutoff)
                if s.cache is None or all(t is None for t in s.cache):
                    out.append(s.format(inf_is_zero, None if keep.all() else keep))
                    continue
                built = np.array([t is not None for t in s.cache])
                fast = _as_bytes(s.format(inf_is_zero, keep & ~built))
                fi = iter(fast.decode("utf-8", "surrogateescape").split("\n"))
                lines = []
                for r in range(s.n):
                    if built[r]:
                        t = s.cache[r]
                        if hasattr(t, "snr") and _ge(t.snr, SNR_cutoff):
                            lines.append(toa_line(t, inf_is_zero))
                    elif keep[r]:
                        lines.append(next(fi))
                out.append(enc(lines))
            else:
                out.append(enc([toa_line(t, inf_is_zero) for t in s
                                if hasattr(t, "snr") and _ge(t.snr, SNR_cutoff)]))
        return out

    def tim_text(self, inf_is_zero=True, SNR_cutoff=0.0):
        """tim_chunks as one str."""
        return b"".join(_as_bytes(c) for c in self.tim_chunks(inf_is_zero, SNR_cutoff)).decode(
            "utf-8", "surrogateescape")


class MJDArray:
    """The fitted MJDs of one archive (get_TOAs' ``TOAs[iarch]``,
    pptoas.py:522-530, 694): days / secs / fracsec columns over nsub
    subints, ``valid`` marking the fitted ones.  Indexing gives an MJD (0 for
    an unfitted subint, as the reference's np.zeros(nsub, dtype=object)),
    slices and index arrays another MJDArray; np.asarray gives the
    reference's object array."""
    __slots__ = ("days", "secs", "fracsec", "valid")

    def __init__(self, days, secs, fracsec, valid=None):
        self.days = np.asarray(days, dtype=np.int64)
        self.secs = np.asarray(secs, dtype=np.int64)
        self.fracsec = np.asarray(fracsec, dtype=np.float64)
        self.valid = np.ones(len(self.days), dtype=bool) if valid is None else \
            np.asarray(valid, dtype=bool)

    @property
    def shape(self):
        return (len(self.days),)

    ndim = 1
    dtype = np.dtype(object)

    def __len__(self):
        return len(self.days)

    def __getitem__(self, i):
        if isinstance(i, (int, np.integer)):
            if not self.valid[i]:
                return 0
            return MJD._settled(int(self.days[i]), int(self.secs[i]), float(self.fracsec[i]))
        return MJDArray(self.days[i], self.secs[i], self.fracsec[i], self.valid[i])

    def __iter__(self):
        mk = MJD._settled
        for d, s, f, v in zip(self.days.tolist(), self.secs.tolist(), self.fracsec.tolist(),
                              self.valid.tolist()):
            yield mk(d, s, f) if v else 0

    def tolist(self):
        return list(self)

    def ravel(self):
        return self

    def __array__(self, dtype=None, copy=None):
        a = np.empty(len(self), dtype=object)
        a[:] = self.tolist()
        return a if dtype is None else a.astype(dtype)

    def in_days(self):
        """MJD.in_days of every entry (NaN where unfitted)."""
        x = self.days + (self.secs + self.fracsec) / 86400.0
        return np.where(self.valid, x, np.nan)

    def __repr__(self):
        return "MJDArray(%d)" % len(self)
