// psrfits.cpp -- fold-mode PSRFITS reader behind include/ppfits.h.
//
// FITS (NOST 100-2.0 / FITS 4.0) is a sequence of HDUs, each an ASCII header
// of 80-character cards in 2880-byte blocks ending with END, followed by the
// data padded to 2880 bytes.  PSRFITS (the ATNF definition PSRCHIVE writes)
// puts the observation in the primary header and the folded profiles in the
// SUBINT binary table: per row TSUBINT, OFFS_SUB, optional PERIOD / PAR_ANG,
// DAT_FREQ[nchan], DAT_WTS[nchan], DAT_OFFS / DAT_SCL[npol][nchan] and
// DATA[npol][nchan][nbin] (TDIM (NBIN,NCHAN,NPOL), big-endian integers),
// the physical value being DATA * DAT_SCL + DAT_OFFS.  The predictor for the
// folding period is the POLYCO table; the HISTORY table's last row says
// whether the data were dedispersed.  Only what pplib.load_data reads from
// PSRCHIVE (pplib.py:2670-2735) is parsed.
#include "ppfits.h"

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

// Source hash of this build (pulseportraiture_amd/build.py compares it with
// today's sources before reusing a built library).
#ifndef PPF_SRC_HASH
#define PPF_SRC_HASH "unbuilt"
#endif
extern "C" __attribute__((visibility("default"), used)) const char ppfits_build_tag[] =
    "PPF_SRC_HASH=" PPF_SRC_HASH;

namespace {

constexpr size_t kBlock = 2880;
constexpr size_t kCard = 80;

struct Column {
  std::string name;
  char type = 0;       // FITS TFORM letter
  long repeat = 1;
  size_t width = 0;    // bytes per element
  size_t offset = 0;   // byte offset in the row
};

struct Hdu {
  std::map<std::string, std::string> kv;  // keyword -> raw value text
  size_t data_off = 0, data_bytes = 0;
  size_t row_bytes = 0, nrows = 0;
  std::vector<Column> cols;
  std::string extname;
};

size_t type_width(char t) {
  switch (t) {
    case 'L': case 'B': case 'A': return 1;
    case 'I': return 2;
    case 'J': case 'E': return 4;
    case 'K': case 'D': case 'C': case 'P': return 8;
    case 'M': case 'Q': return 16;
    default: return 0;
  }
}

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(' '), b = s.find_last_not_of(' ');
  return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

// value text of a card: a quoted string (quotes removed, '' -> ') or the
// token before any comment
std::string card_value(const char* c) {
  std::string v(c + 10, kCard - 10);
  size_t i = v.find_first_not_of(' ');
  if (i == std::string::npos) return "";
  if (v[i] == '\'') {
    std::string out;
    for (size_t j = i + 1; j < v.size(); ++j) {
      if (v[j] == '\'') {
        if (j + 1 < v.size() && v[j + 1] == '\'') { out += '\''; ++j; continue; }
        break;
      }
      out += v[j];
    }
    return trim(out);
  }
  size_t slash = v.find('/', i);
  return trim(v.substr(i, slash == std::string::npos ? std::string::npos : slash - i));
}

bool be_host() {
  const uint16_t x = 1;
  return *reinterpret_cast<const uint8_t*>(&x) == 0;
}

void swap_bytes(uint8_t* p, size_t width, size_t n) {
  if (width <= 1 || be_host()) return;
  for (size_t i = 0; i < n; ++i, p += width)
    for (size_t a = 0, b = width - 1; a < b; ++a, --b) { const uint8_t t = p[a]; p[a] = p[b]; p[b] = t; }
}

double elem_to_double(const uint8_t* p, char t) {  // p: native byte order
  switch (t) {
    case 'B': return (double)*p;
    case 'I': { int16_t v; memcpy(&v, p, 2); return (double)v; }
    case 'J': { int32_t v; memcpy(&v, p, 4); return (double)v; }
    case 'K': { int64_t v; memcpy(&v, p, 8); return (double)v; }
    case 'E': { float v; memcpy(&v, p, 4); return (double)v; }
    case 'D': { double v; memcpy(&v, p, 8); return v; }
    case 'L': return (*p == 'T') ? 1.0 : 0.0;
    case 'A': return (*p == 'T' || *p == '1') ? 1.0 : 0.0;
    default: return NAN;
  }
}

}  // namespace

struct ppfits_file {
  FILE* fp = nullptr;
  std::string err;
  std::vector<Hdu> hdus;
  int subint = -1, polyco = -1, history = -1;
  ppfits_info info{};

  ~ppfits_file() { if (fp) fclose(fp); }

  int fail(int code, const std::string& msg) { err = msg; return code; }

  bool read_at(size_t off, void* dst, size_t n) {
    if (fseeko(fp, (off_t)off, SEEK_SET) != 0) return false;
    return fread(dst, 1, n, fp) == n;
  }

  const std::string* get(const Hdu& h, const char* key) const {
    auto it = h.kv.find(key);
    return it == h.kv.end() ? nullptr : &it->second;
  }
  double num(const Hdu& h, const char* key, double dflt) const {
    const std::string* v = get(h, key);
    if (!v || v->empty()) return dflt;
    std::string s = *v;
    for (char& ch : s) if (ch == 'D' || ch == 'd') ch = 'E';  // Fortran exponents
    char* end = nullptr;
    const double x = strtod(s.c_str(), &end);
    return end == s.c_str() ? dflt : x;
  }
  std::string str(const Hdu& h, const char* key) const {
    const std::string* v = get(h, key);
    return v ? *v : std::string();
  }
  const Column* col(const Hdu& h, const char* name) const {
    for (const auto& c : h.cols) if (c.name == name) return &c;
    return nullptr;
  }

  int parse() {
    size_t off = 0;
    std::vector<char> blk(kBlock);
    for (int ih = 0;; ++ih) {
      Hdu h;
      bool end = false;
      size_t hdr = 0;
      while (!end) {
        if (!read_at(off + hdr, blk.data(), kBlock)) {
          if (ih > 0 && hdr == 0) return PPFITS_OK;  // clean end of file
          return fail(PPFITS_ERR_FORMAT, "truncated FITS header");
        }
        hdr += kBlock;
        for (size_t c = 0; c < kBlock; c += kCard) {
          const char* card = blk.data() + c;
          const std::string key = trim(std::string(card, 8));
          if (key == "END") { end = true; break; }
          if (ih == 0 && hdr == kBlock && c == 0 && key != "SIMPLE")
            return fail(PPFITS_ERR_FORMAT, "not a FITS file (no SIMPLE card)");
          if (card[8] == '=' && !key.empty()) h.kv[key] = card_value(card);
        }
      }
      h.data_off = off + hdr;
      // data size: |BITPIX|/8 * GCOUNT * (PCOUNT + NAXIS1 * ... * NAXISn)
      const long naxis = (long)num(h, "NAXIS", 0);
      size_t n = naxis > 0 ? 1 : 0;
      for (long a = 1; a <= naxis; ++a) {
        char k[32];
        snprintf(k, sizeof k, "NAXIS%ld", a);
        n *= (size_t)num(h, k, 0);
      }
      const size_t bitpix = (size_t)std::fabs(num(h, "BITPIX", 8));
      const size_t pcount = (size_t)num(h, "PCOUNT", 0), gcount = (size_t)num(h, "GCOUNT", 1);
      h.data_bytes = (bitpix / 8) * gcount * (pcount + n);
      h.extname = str(h, "EXTNAME");
      if (str(h, "XTENSION") == "BINTABLE") {
        h.row_bytes = (size_t)num(h, "NAXIS1", 0);
        h.nrows = (size_t)num(h, "NAXIS2", 0);
        const long nf = (long)num(h, "TFIELDS", 0);
        size_t co = 0;
        for (long i = 1; i <= nf; ++i) {
          char kt[32], kf[32];
          snprintf(kt, sizeof kt, "TTYPE%ld", i);
          snprintf(kf, sizeof kf, "TFORM%ld", i);
          Column c;
          c.name = str(h, kt);
          const std::string form = str(h, kf);
          size_t p = 0;
          while (p < form.size() && form[p] >= '0' && form[p] <= '9') ++p;
          c.repeat = p ? atol(form.substr(0, p).c_str()) : 1;
          if (p >= form.size()) return fail(PPFITS_ERR_FORMAT, "bad TFORM " + form);
          c.type = form[p];
          c.width = type_width(c.type);
          if (c.type == 'X') { c.width = 1; c.repeat = (c.repeat + 7) / 8; }
          if (!c.width) return fail(PPFITS_ERR_FORMAT, "unsupported TFORM " + form);
          c.offset = co;
          co += c.width * (size_t)c.repeat;
          h.cols.push_back(c);
        }
        if (co != h.row_bytes) return fail(PPFITS_ERR_FORMAT, "column widths != NAXIS1 in " + h.extname);
      }
      hdus.push_back(h);
      if (h.extname == "SUBINT") subint = ih;
      if (h.extname == "POLYCO") polyco = ih;
      if (h.extname == "HISTORY") history = ih;
      off = h.data_off + (h.data_bytes + kBlock - 1) / kBlock * kBlock;
    }
  }

  // one column of one row, elements converted to native order
  bool cell(const Hdu& h, const Column& c, size_t row, std::vector<uint8_t>& buf) {
    buf.resize(c.width * (size_t)c.repeat);
    if (!read_at(h.data_off + row * h.row_bytes + c.offset, buf.data(), buf.size())) return false;
    swap_bytes(buf.data(), c.width, (size_t)c.repeat);
    return true;
  }

  int fill_info() {
    if (subint < 0) return fail(PPFITS_ERR_MISSING, "no SUBINT table (not a PSRFITS fold-mode archive)");
    const Hdu& p = hdus[0];
    const Hdu& s = hdus[subint];
    ppfits_info& I = info;
    I.nsub = (int32_t)s.nrows;
    I.npol = (int32_t)num(s, "NPOL", 1);
    I.nchan = (int32_t)num(s, "NCHAN", 0);
    I.nbin = (int32_t)num(s, "NBIN", 0);
    const Column* d = col(s, "DATA");
    if (!d) return fail(PPFITS_ERR_MISSING, "SUBINT has no DATA column");
    if ((long)I.npol * I.nchan * I.nbin != d->repeat)
      return fail(PPFITS_ERR_FORMAT, "DATA length != NPOL * NCHAN * NBIN");
    I.raw_type = d->type == 'B' ? PPFITS_RAW_U8 : d->type == 'I' ? PPFITS_RAW_I16
                 : d->type == 'E' ? PPFITS_RAW_F32 : 0;
    if (!I.raw_type) return fail(PPFITS_ERR_FORMAT, "DATA type must be B, I or E");
    for (const char* need : {"DAT_FREQ", "DAT_WTS", "DAT_OFFS", "DAT_SCL"})
      if (!col(s, need)) return fail(PPFITS_ERR_MISSING, std::string("SUBINT has no ") + need);
    I.has_period = col(s, "PERIOD") != nullptr;
    I.has_par_ang = col(s, "PAR_ANG") != nullptr;
    I.stt_imjd = (int32_t)num(p, "STT_IMJD", 0);
    I.stt_smjd = num(p, "STT_SMJD", 0);
    I.stt_offs = num(p, "STT_OFFS", 0);
    I.obsfreq = num(p, "OBSFREQ", NAN);
    I.obsbw = num(p, "OBSBW", NAN);
    I.chan_dm = num(p, "CHAN_DM", NAN);
    I.be_delay = num(p, "BE_DELAY", 0.0);
    I.dm = num(s, "DM", NAN);
    I.chan_bw = num(s, "CHAN_BW", NAN);
    auto cp = [](char* dst, size_t n, const std::string& v) { snprintf(dst, n, "%s", v.c_str()); };
    cp(I.telescope, sizeof I.telescope, str(p, "TELESCOP"));
    cp(I.frontend, sizeof I.frontend, str(p, "FRONTEND"));
    cp(I.backend, sizeof I.backend, str(p, "BACKEND"));
    cp(I.source, sizeof I.source, str(p, "SRC_NAME"));
    cp(I.obs_mode, sizeof I.obs_mode, str(p, "OBS_MODE"));
    cp(I.pol_type, sizeof I.pol_type, str(s, "POL_TYPE"));
    if (polyco >= 0) {
      const Hdu& h = hdus[polyco];
      const Column* cc = col(h, "COEFF");
      I.npolyco = (int32_t)h.nrows;
      I.ncoef = cc ? (int32_t)cc->repeat : 0;
    }
    if (history >= 0) {
      const Hdu& h = hdus[history];
      const Column* c = col(h, "DEDISP");
      if (c && h.nrows) {
        std::vector<uint8_t> b;
        if (!cell(h, *c, h.nrows - 1, b)) return fail(PPFITS_ERR_IO, "HISTORY read failed");
        I.dedispersed = elem_to_double(b.data(), c->type) != 0.0;
      }
    }
    return PPFITS_OK;
  }
};

extern "C" {

int ppfits_open(const char* path, ppfits_file** out) {
  if (!path || !out) return PPFITS_ERR_IO;
  *out = nullptr;
  ppfits_file* f = new ppfits_file();
  f->fp = fopen(path, "rb");
  if (!f->fp) {
    f->err = std::string("cannot open ") + path + ": " + strerror(errno);
    *out = f;
    return PPFITS_ERR_IO;
  }
  int r = f->parse();
  if (r == PPFITS_OK) r = f->fill_info();
  *out = f;  // the caller reads the error and closes
  return r;
}

void ppfits_close(ppfits_file* f) { delete f; }

const char* ppfits_error(const ppfits_file* f) { return f ? f->err.c_str() : "null file"; }

int ppfits_get_info(const ppfits_file* f, ppfits_info* out) {
  if (!f || !out) return PPFITS_ERR_IO;
  if (f->subint < 0) return PPFITS_ERR_MISSING;
  *out = f->info;
  return PPFITS_OK;
}

int ppfits_read_meta(const ppfits_file* cf, double* freqs, double* wts, double* offs,
                     double* scl, double* tsubint, double* offs_sub, double* period,
                     double* par_ang) {
  ppfits_file* f = const_cast<ppfits_file*>(cf);
  if (!f || f->subint < 0) return PPFITS_ERR_MISSING;
  const Hdu& s = f->hdus[f->subint];
  const ppfits_info& I = f->info;
  struct Want { const char* name; double* dst; long n; };
  const Want wants[] = {{"DAT_FREQ", freqs, I.nchan}, {"DAT_WTS", wts, I.nchan},
                        {"DAT_OFFS", offs, (long)I.npol * I.nchan},
                        {"DAT_SCL", scl, (long)I.npol * I.nchan}, {"TSUBINT", tsubint, 1},
                        {"OFFS_SUB", offs_sub, 1}, {"PERIOD", period, 1}, {"PAR_ANG", par_ang, 1}};
  std::vector<uint8_t> b;
  for (const Want& w : wants) {
    if (!w.dst) continue;
    const Column* c = f->col(s, w.name);
    for (int32_t r = 0; r < I.nsub; ++r) {
      double* o = w.dst + (size_t)r * w.n;
      if (!c) {
        for (long i = 0; i < w.n; ++i) o[i] = NAN;
        continue;
      }
      if (c->repeat < w.n) return f->fail(PPFITS_ERR_FORMAT, std::string("short column ") + w.name);
      if (!f->cell(s, *c, (size_t)r, b)) return f->fail(PPFITS_ERR_IO, "SUBINT read failed");
      for (long i = 0; i < w.n; ++i) o[i] = elem_to_double(b.data() + i * c->width, c->type);
    }
  }
  return PPFITS_OK;
}

int ppfits_read_raw(const ppfits_file* cf, int32_t isub0, int32_t n, void* out) {
  ppfits_file* f = const_cast<ppfits_file*>(cf);
  if (!f || f->subint < 0 || !out) return PPFITS_ERR_MISSING;
  const ppfits_info& I = f->info;
  if (isub0 < 0 || n < 0 || isub0 + n > I.nsub)
    return f->fail(PPFITS_ERR_RANGE, "subint range outside the SUBINT table");
  const Hdu& s = f->hdus[f->subint];
  const Column* d = f->col(s, "DATA");
  const size_t bytes = d->width * (size_t)d->repeat;
  uint8_t* o = static_cast<uint8_t*>(out);
  for (int32_t r = 0; r < n; ++r, o += bytes) {
    if (!f->read_at(s.data_off + (size_t)(isub0 + r) * s.row_bytes + d->offset, o, bytes))
      return f->fail(PPFITS_ERR_IO, "DATA read failed");
    swap_bytes(o, d->width, (size_t)d->repeat);
  }
  return PPFITS_OK;
}

int ppfits_read_polyco(const ppfits_file* cf, double* ref_mjd, double* ref_f0, double* ref_phs,
                       double* nspan, double* coeff) {
  ppfits_file* f = const_cast<ppfits_file*>(cf);
  if (!f || f->polyco < 0) return f ? f->fail(PPFITS_ERR_MISSING, "no POLYCO table") : PPFITS_ERR_MISSING;
  const Hdu& h = f->hdus[f->polyco];
  const long nc = f->info.ncoef;
  struct Want { const char* name; double* dst; long n; };
  const Want wants[] = {{"REF_MJD", ref_mjd, 1}, {"REF_F0", ref_f0, 1}, {"REF_PHS", ref_phs, 1},
                        {"NSPAN", nspan, 1}, {"COEFF", coeff, nc}};
  std::vector<uint8_t> b;
  for (const Want& w : wants) {
    if (!w.dst) continue;
    const Column* c = f->col(h, w.name);
    if (!c) return f->fail(PPFITS_ERR_MISSING, std::string("POLYCO has no ") + w.name);
    for (size_t r = 0; r < h.nrows; ++r) {
      if (!f->cell(h, *c, r, b)) return f->fail(PPFITS_ERR_IO, "POLYCO read failed");
      for (long i = 0; i < w.n; ++i)
        w.dst[r * w.n + i] = i < c->repeat ? elem_to_double(b.data() + i * c->width, c->type) : 0.0;
    }
  }
  return PPFITS_OK;
}

}  // extern "C"
