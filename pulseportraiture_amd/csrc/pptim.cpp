// pptim.cpp -- bulk .tim text (include/pptim.h): the line building of
// pplib.write_TOAs (/root/reference/pplib.py:3471-3503) over TOA records held
// as columns.  Host-only C++17; no GPU.
//
// Every number goes through std::to_chars with an explicit precision, which
// prints the correctly rounded decimal of the binary value -- the same digits
// as Python's '%.Nf' / '%.Ne' (both exact, ties to even on the exact binary
// value).  Rows are split over host threads in contiguous ranges and the
// per-thread texts joined in row order, so the output does not depend on the
// thread count.
#include "pptim.h"

#include <charconv>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <algorithm>
#include <new>
#include <string>
#include <thread>

#ifndef PPT_MIN_ROWS_PER_THREAD
#define PPT_MIN_ROWS_PER_THREAD 2048
#endif
#include <vector>

// Source hash of this build (pulseportraiture_amd/build.py compares it with
// today's sources before reusing a built library).
#ifndef PPF_SRC_HASH
#define PPF_SRC_HASH "unbuilt"
#endif
extern "C" __attribute__((visibility("default"), used)) const char ppt_build_tag[] =
    "PPF_SRC_HASH=" PPF_SRC_HASH;

namespace {

const uint64_t kPow10[20] = {1ull,
                             10ull,
                             100ull,
                             1000ull,
                             10000ull,
                             100000ull,
                             1000000ull,
                             10000000ull,
                             100000000ull,
                             1000000000ull,
                             10000000000ull,
                             100000000000ull,
                             1000000000000ull,
                             10000000000000ull,
                             100000000000000ull,
                             1000000000000000ull,
                             10000000000000000ull,
                             100000000000000000ull,
                             1000000000000000000ull,
                             10000000000000000000ull};

// '%.<prec>f' of a finite x with |x| < 2^53 and prec <= 19 by exact integer
// arithmetic: |x| = m 2^-s, so round(|x| 10^prec) = (m 10^prec) >> s rounded
// half to even on the exact remainder -- the correctly rounded decimal, as
// to_chars / Python give it, at a fraction of to_chars' cost.  Returns false
// (nothing written) outside that range.
inline bool put_fixed_fast(char* out, size_t& len, double x, int prec) {
  if (prec > 19) return false;
  uint64_t bits;
  std::memcpy(&bits, &x, 8);
  const bool neg = bits >> 63;
  const int be = static_cast<int>((bits >> 52) & 0x7ff);
  uint64_t m = bits & ((1ull << 52) - 1);
  int e2;  // |x| = m 2^e2
  if (be == 0) {
    e2 = -1074;  // zero or subnormal
  } else {
    m |= 1ull << 52;
    e2 = be - 1075;
  }
  unsigned __int128 q;
  if (m == 0) {
    q = 0;
  } else if (e2 >= 0) {
    if (e2 > 10) return false;  // |x| >= 2^63: leave it to to_chars
    q = static_cast<unsigned __int128>(m << e2) * kPow10[prec];
  } else {
    const int s = -e2;
    const unsigned __int128 n = static_cast<unsigned __int128>(m) * kPow10[prec];  // < 2^117
    if (s >= 118) {
      q = 0;  // |x| 10^prec < 2^-1: rounds to 0
    } else {
      q = n >> s;
      const unsigned __int128 r = n - (q << s), half = static_cast<unsigned __int128>(1) << (s - 1);
      if (r > half || (r == half && (q & 1))) ++q;
    }
  }
  // digits of q, right-aligned in tmp, at least prec + 1 of them
  static const char kPairs[] =
      "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
      "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
      "8081828384858687888990919293949596979899";
  char tmp[64];
  char* e = tmp + sizeof(tmp);
  char* p = e;
  auto u64_digits = [&](uint64_t c, bool full19) {
    char* stop = p - 19;
    while (c >= 100) {
      const uint64_t r = c % 100;
      c /= 100;
      p -= 2;
      std::memcpy(p, kPairs + 2 * r, 2);
    }
    if (c >= 10) {
      p -= 2;
      std::memcpy(p, kPairs + 2 * c, 2);
    } else if (c > 0) {
      *--p = static_cast<char>('0' + c);
    }
    if (full19)
      while (p > stop) *--p = '0';  // a middle chunk keeps its zeros
  };
  if ((q >> 64) == 0) {
    u64_digits(static_cast<uint64_t>(q), false);
  } else {
    while (q > 0) {
      const uint64_t chunk = static_cast<uint64_t>(q % 10000000000000000000ull);
      q /= 10000000000000000000ull;
      u64_digits(chunk, q > 0);
    }
  }
  while (e - p < prec + 1) *--p = '0';
  size_t k = 0;
  if (neg) out[k++] = '-';
  const size_t ni = static_cast<size_t>(e - p) - prec;
  std::memcpy(out + k, p, ni);
  k += ni;
  if (prec > 0) {
    out[k++] = '.';
    std::memcpy(out + k, p + ni, prec);
    k += prec;
  }
  len = k;
  return true;
}

// A row-text buffer: raw pointer appends with one capacity check per field.
// Text buffer: malloc'd, never zero-filled (a fresh page is touched once,
// by the text written into it); grown with realloc.
struct Buf {
  char* p = nullptr;
  size_t cap = 0;
  ~Buf() { std::free(p); }
  void reserve(size_t k) {
    if (k <= cap) return;
    char* q = static_cast<char*>(std::realloc(p, k));
    if (!q) throw std::bad_alloc();
    p = q;
    cap = k;
  }
};

struct Out {
  Buf* v;
  size_t n = 0;
  explicit Out(Buf* vv) : v(vv) {}
  char* room(size_t k) {  // k writable bytes at the end
    if (v->cap < n + k) v->reserve(std::max(v->cap + v->cap / 2, n + k + (1 << 16)));
    return v->p + n;
  }
  void put(const char* b, size_t k) {
    std::memcpy(room(k), b, k);
    n += k;
  }
};

inline void put_f64(Out& o, double x, int prec, std::chars_format fmt, bool drop1) {
  if (std::isnan(x)) {  // Python prints 'nan' for either sign
    o.put(drop1 ? "an" : "nan", drop1 ? 2 : 3);
    return;
  }
  char* buf = o.room(400);
  size_t len = 0;
  if (!(fmt == std::chars_format::fixed && std::isfinite(x) && put_fixed_fast(buf, len, x, prec))) {
    auto r = std::to_chars(buf, buf + 400, x, fmt, prec);
    len = r.ec == std::errc() ? static_cast<size_t>(r.ptr - buf) : 0;  // prec <= 40: fits
  }
  if (drop1 && len) {
    std::memmove(buf, buf + 1, len - 1);
    --len;
  }
  o.n += len;
}

inline void put_i64(Out& o, int64_t v) {
  char* buf = o.room(24);
  auto r = std::to_chars(buf, buf + 24, v);
  o.n += static_cast<size_t>(r.ptr - buf);
}

struct Field {
  int32_t kind, prec;
  const void* data;
  const int64_t* offs;
  const uint8_t* present;
  size_t tlen;  // PPT_TEXT length
};

void format_range(const std::vector<Field>& f, int64_t r0, int64_t r1, const uint8_t* keep,
                  Out& o, int64_t& rows) {
  for (int64_t r = r0; r < r1; ++r) {
    if (keep && !keep[r]) continue;
    for (const Field& x : f) {
      if (x.present && !x.present[r]) continue;
      switch (x.kind) {
        case PPT_TEXT:
          o.put(static_cast<const char*>(x.data), x.tlen);
          break;
        case PPT_I64:
          put_i64(o, static_cast<const int64_t*>(x.data)[r]);
          break;
        case PPT_F64_FIXED:
          put_f64(o, static_cast<const double*>(x.data)[r], x.prec, std::chars_format::fixed,
                  false);
          break;
        case PPT_F64_EXP:
          put_f64(o, static_cast<const double*>(x.data)[r], x.prec,
                  std::chars_format::scientific, false);
          break;
        case PPT_F64_FRAC:
          put_f64(o, static_cast<const double*>(x.data)[r], x.prec, std::chars_format::fixed,
                  true);
          break;
        case PPT_STRS: {
          const char* blob = static_cast<const char*>(x.data);
          o.put(blob + x.offs[r], static_cast<size_t>(x.offs[r + 1] - x.offs[r]));
          break;
        }
      }
    }
    o.put("\n", 1);
    ++rows;
  }
}

// Part buffers are recycled between calls: a fresh multi-MB buffer costs a
// page fault per 4 KB, more than the formatting itself.
std::mutex g_pool_mu;
std::vector<Buf*> g_pool;

Buf* pool_get() {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if (g_pool.empty()) return new Buf();
  auto* v = g_pool.back();
  g_pool.pop_back();
  return v;
}

void pool_put(Buf* v) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if (g_pool.size() < 32 && v->cap <= (size_t(256) << 20)) {
    g_pool.push_back(v);
  } else {
    delete v;
  }
}

}  // namespace

struct ppt_text {
  std::vector<Buf*> parts;
  std::vector<size_t> sizes;
  int64_t rows = 0;
  ~ppt_text() {
    for (auto* v : parts) pool_put(v);
  }
};

extern "C" int ppt_format_rows(int64_t n, int32_t nfield, const ppt_field* fields,
                               const uint8_t* keep, int32_t nthreads, ppt_text** out) {
  if (!out || n < 0 || nfield < 0 || (nfield > 0 && !fields)) return PPT_ERR_ARG;
  *out = nullptr;
  std::vector<Field> f;
  f.reserve(nfield);
  size_t est = 1;  // bytes per row, for the first reserve
  for (int32_t i = 0; i < nfield; ++i) {
    const ppt_field& g = fields[i];
    if (!g.data || g.kind < PPT_TEXT || g.kind > PPT_STRS) return PPT_ERR_ARG;
    if (g.kind >= PPT_F64_FIXED && g.kind <= PPT_F64_FRAC && (g.prec < 0 || g.prec > 40))
      return PPT_ERR_ARG;
    if (g.kind == PPT_STRS && !g.offs) return PPT_ERR_ARG;
    Field x{g.kind, g.prec, g.data, g.offs, g.present, 0};
    if (g.kind == PPT_TEXT) {
      x.tlen = std::strlen(static_cast<const char*>(g.data));
      est += x.tlen;
    } else if (g.kind == PPT_STRS) {
      est += static_cast<size_t>(n ? (g.offs[n] - g.offs[0]) / n + 1 : 1);
    } else {
      est += 12 + static_cast<size_t>(g.prec);
    }
    f.push_back(x);
  }
  unsigned hw = std::thread::hardware_concurrency();
  int64_t nt = nthreads > 0 ? nthreads : static_cast<int64_t>(hw ? (hw < 8 ? hw : 8) : 1);
  // rows per thread at least: below this a thread's start costs more than it
  // saves (r06, on the GPU box: 7,000 / 3,000-row pieces of a get_TOAs call)
  const int64_t min_rows = PPT_MIN_ROWS_PER_THREAD;
  if (nt > (n + min_rows - 1) / min_rows) nt = (n + min_rows - 1) / min_rows;
  if (nt < 1) nt = 1;
  auto* t = new (std::nothrow) ppt_text;
  if (!t) return PPT_ERR_NOMEM;
  try {
    t->parts.resize(nt, nullptr);
    t->sizes.assign(nt, 0);
    for (auto& v : t->parts) v = pool_get();
    std::vector<int64_t> rows(nt, 0);
    auto work = [&](int64_t i) {
      int64_t r0 = n * i / nt, r1 = n * (i + 1) / nt;
      t->parts[i]->reserve(static_cast<size_t>(r1 - r0) * est + 1024);
      Out o(t->parts[i]);
      format_range(f, r0, r1, keep, o, rows[i]);
      t->sizes[i] = o.n;
    };
    if (nt == 1) {
      work(0);
    } else {
      std::vector<std::thread> th;
      th.reserve(nt - 1);
      for (int64_t i = 1; i < nt; ++i) th.emplace_back(work, i);
      work(0);
      for (auto& x : th) x.join();
    }
    for (auto r : rows) t->rows += r;
  } catch (const std::bad_alloc&) {
    delete t;
    return PPT_ERR_NOMEM;
  }
  *out = t;
  return PPT_OK;
}

extern "C" int64_t ppt_text_nparts(const ppt_text* t) {
  return t ? static_cast<int64_t>(t->parts.size()) : 0;
}

extern "C" const char* ppt_text_part(const ppt_text* t, int64_t i, int64_t* size) {
  if (!t || i < 0 || i >= static_cast<int64_t>(t->parts.size())) {
    if (size) *size = 0;
    return nullptr;
  }
  if (size) *size = static_cast<int64_t>(t->sizes[i]);
  return t->parts[i]->p;
}

extern "C" int64_t ppt_text_size(const ppt_text* t) {
  int64_t s = 0;
  if (t)
    for (auto z : t->sizes) s += static_cast<int64_t>(z);
  return s;
}

extern "C" int64_t ppt_text_rows(const ppt_text* t) { return t ? t->rows : 0; }

extern "C" void ppt_text_free(ppt_text* t) { delete t; }
