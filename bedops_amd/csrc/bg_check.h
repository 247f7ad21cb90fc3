// bg_check.h — the reference's --ec row grammar (Bed::bed_check_iterator::check,
// interfaces/general-headers/data/bed/BedCheckIterator.hpp:326-634) as one branchy
// per-line function shared by the GPU validation kernel (bg_check.hip, one thread per
// line) and the host code that words the error message for the first failing line.
// Lines are Ext::ByLine lines (utility/ByLine.hpp: std::getline, '\n' only; a '\r' is part
// of the line). Codes name the reference's messages (bg_check_message() in bg_check.hip).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define BGC_HD __host__ __device__ __forceinline__
#else
#define BGC_HD static inline
#endif

enum {
  BGC_OK = 0, BGC_HEADER = 1,  // fine / a header line (allowed only at the top)
  BGC_EMPTY = 10, BGC_CHR_SPACE, BGC_CHR_TAB0, BGC_NO_TABS, BGC_CHR_LONG,
  BGC_S_TABS, BGC_S_NEG, BGC_S_SPACE, BGC_S_CHAR, BGC_S_NOTAB, BGC_S_DIGITS, BGC_S_MAX,
  BGC_E_TABS, BGC_E_NEG, BGC_E_SPACE, BGC_E_CHAR, BGC_ONLY3, BGC_E_DIGITS, BGC_E_MAX,
  BGC_ID_TABS, BGC_ID_SPACE, BGC_ONLY4, BGC_ID_EMPTY, BGC_ID_LONG,
  BGC_M_TABS, BGC_M_DOTS, BGC_M_DOTEXP, BGC_M_EXPS, BGC_M_SPACE, BGC_M_SIGNPOS, BGC_M_SIGNS,
  BGC_M_SIGNEXP, BGC_M_CHAR, BGC_ONLY5, BGC_M_EMPTY, BGC_M_ENDMINUS,
  BGC_ST_TABS, BGC_ST_CHAR, BGC_ST_TWO, BGC_ST_EMPTY, BGC_REST_LONG,
  BGC_UNSORTED_CHR, BGC_UNSORTED_START, BGC_UNSORTED_END, BGC_UNSORTED_REST, BGC_END_LE_START,
  BGC_HEADER_LATE, BGC_NESTED
};

#define BGC_MAXCHROMSIZE 127u          // TOKEN_CHR_MAX_LENGTH (BEDOPS.Constants.hpp:32)
#define BGC_MAXIDSIZE 16383u           // TOKEN_ID_MAX_LENGTH
#define BGC_MAXRESTSIZE (8u * 131072u) // TOKEN_REST_MAX_LENGTH
#define BGC_MAX_DEC_INTEGERS 12u
#define BGC_MAX_COORD_VALUE 999999999999ull

struct BgcRow {
  uint32_t chrom_len;   // chromosome = line[0, chrom_len)
  uint64_t start, end;  // as Bed::BasicCoords(string) reads them
  uint32_t rest_at;     // restMarker: where the end coordinate starts (:414)
  uint32_t bad;         // offending byte / size for the message
};

BGC_HD int bgc_isdigit(char c) { return c >= '0' && c <= '9'; }
BGC_HD char bgc_lower(char c) { return (c >= 'A' && c <= 'Z') ? (char)(c + 32) : c; }
// isUCSCheader: the (prefix of the) line is "browser" or "track", any case (:318-321)
BGC_HD int bgc_ucsc(const char* l, uint32_t n) {
  const char* b = "browser";
  const char* t = "track";
  if (n == 7) {
    for (uint32_t i = 0; i < 7; ++i) if (bgc_lower(l[i]) != b[i]) return 0;
    return 1;
  }
  if (n == 5) {
    for (uint32_t i = 0; i < 5; ++i) if (bgc_lower(l[i]) != t[i]) return 0;
    return 1;
  }
  return 0;
}
// digits [p, q) as a value (<= 12 digits after the length check; "" reads 0)
BGC_HD uint64_t bgc_value(const char* l, uint32_t p, uint32_t q) {
  uint64_t v = 0;
  for (uint32_t i = p; i < q && i < p + 19; ++i) v = v * 10 + (uint64_t)(l[i] - '0');
  return v;
}

// One coordinate field starting at `marker` (:379-410 start, :416-447 end). `first` = start.
BGC_HD int bgc_coord(const char* l, uint32_t sz, uint32_t& marker, int first, int nfields,
                     uint64_t& val, uint32_t& bad) {
  const uint32_t pos = marker;
  int msg = 0;
  while (!msg && marker < sz) {
    const char c = l[marker];
    if (!bgc_isdigit(c)) {
      if (c == '\t' && pos != marker) break;
      else if (c == '\t') msg = first ? BGC_S_TABS : BGC_E_TABS;
      else if (c == '-' && marker == pos) msg = first ? BGC_S_NEG : BGC_E_NEG;
      else if (c == ' ') msg = first ? BGC_S_SPACE : BGC_E_SPACE;
      else { msg = first ? BGC_S_CHAR : BGC_E_CHAR; bad = (uint8_t)c; }
    }
    ++marker;
  }
  if (msg) return msg;
  if (sz <= marker && first) return BGC_S_NOTAB;
  if (sz <= marker && !first && nfields > 3) return BGC_ONLY3;
  if (marker - pos > BGC_MAX_DEC_INTEGERS) return first ? BGC_S_DIGITS : BGC_E_DIGITS;
  val = bgc_value(l, pos, marker < sz ? marker : sz);
  if (val > BGC_MAX_COORD_VALUE) return first ? BGC_S_MAX : BGC_E_MAX;
  ++marker;  // past the tab
  return 0;
}

// check(bl) up to the row's own fields (:326-593): BGC_OK, BGC_HEADER or an error code
BGC_HD int bgc_line(const char* l, uint32_t sz, int nfields, int has_rest, BgcRow& R) {
  R.bad = 0;
  R.start = R.end = 0;
  if (sz == 0) return BGC_EMPTY;
  if (sz == 7 || sz == 5) if (bgc_ucsc(l, sz)) return BGC_HEADER;
  uint32_t marker = 0;
  int msg = 0;
  while (!msg && marker < sz) {  // chromosome
    const char c = l[marker];
    if (c == ' ') {
      if (bgc_ucsc(l, marker)) return BGC_HEADER;
      msg = BGC_CHR_SPACE;
    } else if (marker == 0 && (c == '@' || c == '#')) {
      return BGC_HEADER;  // SAM / VCF headers
    } else if (c == '\t') {
      if (marker == 0) msg = BGC_CHR_TAB0;
      else {
        if (bgc_ucsc(l, marker)) return BGC_HEADER;
        break;
      }
    }
    ++marker;
  }
  if (msg) return msg;
  if (sz <= marker) return BGC_NO_TABS;
  if (marker > BGC_MAXCHROMSIZE) { R.bad = marker; return BGC_CHR_LONG; }
  R.chrom_len = marker;
  ++marker;
  int rc = bgc_coord(l, sz, marker, 1, nfields, R.start, R.bad);
  if (rc) return rc;
  R.rest_at = marker;
  rc = bgc_coord(l, sz, marker, 0, nfields, R.end, R.bad);
  if (rc) return rc;
  if (nfields > 3) {  // id (:450-480)
    uint32_t pos = marker;
    while (!msg && marker < sz) {
      const char c = l[marker];
      if (c == '\t' && pos != marker) break;
      else if (c == '\t') msg = BGC_ID_TABS;
      else if (c == ' ') msg = BGC_ID_SPACE;
      ++marker;
    }
    if (msg) return msg;
    if (sz <= marker && nfields > 4) return BGC_ONLY4;
    if (pos == marker) return BGC_ID_EMPTY;
    if (marker - pos > BGC_MAXIDSIZE) { R.bad = marker - pos; return BGC_ID_LONG; }
    ++marker;
    if (nfields > 4) {  // measurement (:482-545)
      pos = marker;
      int dots = 0, exps = 0, signs = 0;
      uint32_t exp_pos = 0, sign_pos = 0;
      while (!msg && marker < sz) {
        const char c = l[marker];
        if (!bgc_isdigit(c)) {
          if (c == '\t' && pos != marker) break;
          else if (c == '\t') msg = BGC_M_TABS;
          else if (c == '.') {
            if (++dots > 1) msg = BGC_M_DOTS;
            else if (exps > 0) msg = BGC_M_DOTEXP;
          } else if (c == 'e' || c == 'E') {
            if (++exps > 1) msg = BGC_M_EXPS;
            exp_pos = marker;
          } else if (c == ' ') {
            msg = BGC_M_SPACE;
          } else if (c == '-' || c == '+') {
            if (marker != pos && exps < 1) msg = BGC_M_SIGNPOS;
            if (!msg && marker != pos) {
              if (++signs > 1) msg = BGC_M_SIGNS;
              else if (exp_pos + 1 != marker) msg = BGC_M_SIGNEXP;
              sign_pos = marker;
            }
          } else {
            msg = BGC_M_CHAR;
            R.bad = (uint8_t)c;
          }
        }
        ++marker;
      }
      if (msg) return msg;
      if (sz <= marker && nfields > 5) return BGC_ONLY5;
      if (pos == marker) return BGC_M_EMPTY;
      if (sign_pos > 0 && sign_pos + 1 == marker) return BGC_M_ENDMINUS;
      ++marker;
      if (nfields > 5) {  // strand (:548-575)
        pos = marker;
        while (!msg && marker < sz) {
          const char c = l[marker];
          if (c != '+' && c != '-') {
            if (c == '\t' && pos != marker) break;
            else if (c == '\t') msg = BGC_ST_TABS;
            else { msg = BGC_ST_CHAR; R.bad = (uint8_t)c; }
          } else if (marker != pos) {
            msg = BGC_ST_TWO;
          }
          ++marker;
        }
        if (msg) return msg;
      }
      // (:568-573: outside the strand block, so also with 5 fields, where it only steps)
      if (pos == marker) return BGC_ST_EMPTY;
      ++marker;
    }
  }
  if (has_rest && marker < sz && sz - marker > BGC_MAXRESTSIZE) { R.bad = sz - marker; return BGC_REST_LONG; }
  return BGC_OK;
}

// the order checks against the previous data row, then end > start (:594-624)
// (nest: bedmap --faster's nestCheck, :612-615: an end below the previous row's end on the
// same chromosome, after the sort checks)
BGC_HD int bgc_order(const char* p, uint32_t pn, const BgcRow& P, const char* l, uint32_t n,
                     const BgcRow& R, int has_rest, int nest = 0) {
  int cmp = 0;
  {  // strcmp of the chromosome names
    const uint32_t m = P.chrom_len < R.chrom_len ? P.chrom_len : R.chrom_len;
    for (uint32_t i = 0; i < m && !cmp; ++i)
      if (l[i] != p[i]) cmp = (uint8_t)l[i] < (uint8_t)p[i] ? -1 : 1;
    if (!cmp && R.chrom_len != P.chrom_len) cmp = R.chrom_len < P.chrom_len ? -1 : 1;
  }
  if (cmp < 0) return BGC_UNSORTED_CHR;
  if (cmp == 0) {
    if (R.start < P.start) return BGC_UNSORTED_START;
    if (R.start == P.start) {
      if (R.end < P.end) return BGC_UNSORTED_END;
      if (has_rest && R.end == P.end) {  // strcmp(bl.substr(restMarker), lastRest_) < 0
        const char* a = l + R.rest_at;
        const char* b = p + P.rest_at;
        const uint32_t la = n - R.rest_at, lb = pn - P.rest_at;
        const uint32_t m = la < lb ? la : lb;
        int c2 = 0;
        for (uint32_t i = 0; i < m && !c2; ++i)
          if (a[i] != b[i]) c2 = (uint8_t)a[i] < (uint8_t)b[i] ? -1 : 1;
        if (!c2 && la < lb) c2 = -1;
        if (c2 < 0) return BGC_UNSORTED_REST;
      }
    }
    if (nest && R.end < P.end) return BGC_NESTED;
  }
  (void)pn;
  if (R.end <= R.start) return BGC_END_LE_START;
  return BGC_OK;
}
