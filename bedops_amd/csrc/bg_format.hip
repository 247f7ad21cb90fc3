// bg_format.hip — K7: device-side rendering of results as BED / bedmap text.
//
// Replaces the reference's per-row printf calls:
//   intervals  "%s\t%lu\t%lu\n"        record() Bedops.cpp:148-152 -> Bed.hpp:228-232
//   rows+rest  "%s\t%lu\t%lu%s\n"      element-of / everything, Bed.hpp:321-325 (rest = verbatim
//                                     remainder)
//   bedmap     "%d" / "%.{p}lf" / "NAN" joined by --delim, '\n' per ref row
//              (MultiVisitor.hpp:83-98, CountVisitor.hpp:55-57, AverageVisitor.hpp:56-62,
//               Formats.hpp:42-50, NaN.cpp:26)
// Two passes over tiles of 1024 rows: (1) bytes per tile, scan; (2) each thread renders
// its rows into an LDS staging buffer at scanned offsets, then the workgroup streams the
// tile to HBM with 16-byte stores (byte stores only at the two unaligned edges).
// %.{p}lf is rendered exactly: the double's binary value times 10^p is rounded half-to-
// even in 128-bit integer arithmetic, which is what glibc printf does.
#include <climits>
#include <cstdlib>
#include <cstring>

#include "bg_internal.h"
#include "bg_decfmt.h"

#define FT_ROWS 2
#define FT_TILE (BG_NT * FT_ROWS)
#define FT_LDS 16384

struct FmtArgs {
  int kind;
  bg_dstatus* st;   // the write pass's checks (BG_FMT_MISMATCH)
  uint64_t total;   // bytes of the whole text (the write pass's bound)
  // intervals / rows
  const int64_t* s;
  const int64_t* e;
  const uint64_t* rows;
  const uint32_t* rlen;  // RES_MULTI: rows[k] = remainder address, rlen[k] its length
  int rest_tab;          // RES_MULTI: '\t' before a non-empty remainder (sort-bed)
  const char* text;
  const uint64_t* rest_off;
  const uint32_t* rest_len;
  // names
  const char* names;
  const uint32_t* name_off;
  const uint32_t* name_len;
  // map
  const int32_t* cnt;
  const int64_t* isum;
  const double* vmin;
  const double* vmax;
  const uint64_t* bases;
  const uint32_t* uniq;
  // --echo-map*: the map table (s2/e2/text2/rest_off2/rest_len2 below), its scores, each
  // row's candidate range and the overlap criterion
  const int64_t* isq;
  const double* dsum;  // decimal scores: running sums (else isum / isq)
  const double* dsq;
  const uint64_t* rrank;  // --echo-ref-row-id under --skip-unmapped (else the row index)
  int nrid;               // --echo-ref-row-id operations per line
  double op_arg[16];
  const double* score2;
  const uint64_t* wlo;
  const uint64_t* whi;
  LongRows lrows;      // long map rows by length class (bg_map_cands)
  const int64_t* zin;  // zero-length rows: sweep-window membership (bg_map_live)
  const int64_t* zout;
  const int64_t* maddr;  // map rows' heap addresses (bg_heap.hip), null: row order
  const uint32_t* maord;  // each tie run of equal (start, end) by increasing address (after maddr)
  uint64_t n2;           // map rows
  int crit, mapfields, mdlen;
  int64_t ovr, range;
  double perc;
  char mdelim[16];
  int nops;
  int ops[16];
  int prec;
  int sci;  // --sci
  int skip_unmapped;
  int dlen;
  char delim[16];
  uint64_t n;
  // closest-features: second table + chosen rows
  const int64_t* s2;
  const int64_t* e2;
  const char* text2;
  const uint64_t* rest_off2;
  const uint32_t* rest_len2;
  const int64_t* left;
  const int64_t* right;
  int shortest, print_dist, no_ref;
  // bedmap: --tmean values per operation; single-file mode; the row where the reference
  // throws (an element operation with nothing mapped) and where its text ends
  const double* tmv[16];
  int single, has_elem;
  uint64_t stop_row;
  uint64_t* stop_out;
  // each line's length from the count pass (RES_MAP / RES_CLOSEST): the write pass places
  // the lines without rendering them once more just to measure them
  uint32_t* rowlen;
};

__device__ __forceinline__ int dec_len_i32(int32_t v) {
  return v < 0 ? 1 + dec_len_u64((uint64_t)(-(int64_t)v)) : dec_len_u64((uint64_t)v);
}

// v as exactly `len` digits; 32-bit division by 10 when v fits (the common case)
template <typename Out>
__device__ __forceinline__ void put_u64(Out& o, uint64_t v, int len) {
  int k = len - 1;
  for (; k >= 0 && (v >> 32) != 0; --k) {
    o.put_at(k, (char)('0' + v % 10));
    v /= 10;
  }
  uint32_t w = (uint32_t)v;
  for (; k >= 0; --k) {
    const uint32_t q = w / 10u;
    o.put_at(k, (char)('0' + (w - 10u * q)));
    w = q;
  }
  o.adv(len);
}

// 4 ASCII digits of x (< 10000) as a little-endian dword, first digit in the low byte:
// x/100 and x%100 into the two 16-bit halves, then /10 and %10 on both halves at once
// (24-bit multiplies; the quotients are exact for these ranges)
__device__ __forceinline__ uint32_t dig4_ascii(uint32_t x) {
  const uint32_t h = __umul24(x, 5243u) >> 19;              // x / 100
  const uint32_t v = h | ((x - 100u * h) << 16);             // pairs: hi | lo << 16
  const uint32_t t = (__umul24(v, 103u) >> 10) & 0x000F000Fu;  // tens of both pairs
  const uint32_t u = v - 10u * t;                            // units of both pairs
  return (t | (u << 8)) + 0x30303030u;
}

// v (< 10^13, coordinates are < 2^40) as exactly len digits into LDS: three 4-digit groups,
// then byte stores (a 13th leading digit separately)
__device__ __forceinline__ void put_u64_lds(char* p, uint64_t v, int len) {
  if (len > 12) {
    const uint64_t top = v / 1000000000000ull;
    *p++ = (char)('0' + top);
    v -= top * 1000000000000ull;
    len = 12;
  }
  uint32_t hi, mid, lo;
  if ((v >> 32) == 0) {
    const uint32_t w = (uint32_t)v;
    const uint32_t q = w / 10000u;
    lo = w - q * 10000u;
    hi = q / 10000u;
    mid = q - hi * 10000u;
  } else {
    const uint64_t q = v / 10000u;
    lo = (uint32_t)(v - q * 10000u);
    hi = (uint32_t)(q / 10000u);
    mid = (uint32_t)(q - (uint64_t)hi * 10000u);
  }
  const uint32_t g[3] = {dig4_ascii(hi), dig4_ascii(mid), dig4_ascii(lo)};
  const int sk = 12 - len;  // leading zero characters to skip
#pragma unroll
  for (int i = 0; i < 12; ++i)
    if (i >= sk) p[i - sk] = (char)(g[i >> 2] >> (8 * (i & 3)));
}

// exact %.{prec}f of |v| split as integer N = round_half_even(|v| * 10^prec) (< 2^64);
// returns false if out of this path's range
__device__ __forceinline__ bool fixed_digits(double v, int prec, uint64_t& N, bool& neg) {
  uint64_t bits = __double_as_longlong(v);
  neg = (bits >> 63) != 0;
  const int bexp = (int)((bits >> 52) & 0x7ff);
  uint64_t m = bits & ((1ULL << 52) - 1);
  if (bexp == 0x7ff) return false;
  int ex;
  if (bexp == 0) { ex = -1074; }
  else { m |= 1ULL << 52; ex = bexp - 1075; }
  uint64_t P = 1;
  for (int k = 0; k < prec; ++k) P *= 10;
  typedef unsigned __int128 u128;
  const u128 X = (u128)m * P;  // < 2^110
  if (ex >= 0) {
    if (ex >= 64) return false;
    if ((X >> (64 - ex)) != 0) return false;  // result would not fit 64 bits
    N = (uint64_t)(X << ex);
    return true;
  }
  const int sh = -ex;
  if (sh >= 128) { N = 0; return true; }  // |v| * 10^prec < 2^-17: rounds to 0
  const u128 q = X >> sh;
  if ((q >> 64) != 0) return false;
  const u128 rem = X - (q << sh);
  const u128 half = (u128)1 << (sh - 1);
  uint64_t qq = (uint64_t)q;
  if (rem > half || (rem == half && (qq & 1))) ++qq;
  N = qq;
  return true;
}

// exact "%.{prec}e" of v (glibc: the binary value rounded half-to-even at prec+1
// significant digits), for 1e-16 <= |v| < 2^128 (and 0); false outside that range.
// N = round(|v| * 10^s) with s = prec - E must land in [10^prec, 10^(prec+1)); E starts
// from log10 and is corrected by one step when the rounding says so.
__device__ __forceinline__ bool sci_digits(double v, int prec, uint64_t& N, int& E, bool& neg) {
  typedef unsigned __int128 u128;
  uint64_t bits = __double_as_longlong(v);
  neg = (bits >> 63) != 0;
  const int bexp = (int)((bits >> 52) & 0x7ff);
  uint64_t m = bits & ((1ULL << 52) - 1);
  if (bexp == 0x7ff) return false;
  if (bexp == 0 && m == 0) { N = 0; E = 0; return true; }
  int ex;
  if (bexp == 0) ex = -1074;
  else { m |= 1ULL << 52; ex = bexp - 1075; }
  const double a = neg ? -v : v;
  if (a < 1e-16) return false;
  uint64_t P = 1;
  for (int k = 0; k < prec; ++k) P *= 10;
  E = (int)floor(log10(a));
  for (int attempt = 0; attempt < 3; ++attempt) {
    const int sc = prec - E;  // N = round(m * 2^ex * 10^sc)
    u128 num = m, den = 1;
    if (sc >= 0) {
      for (int k = 0; k < sc; ++k) {
        if (num > (~(u128)0) / 10) return false;
        num *= 10;
      }
    } else {
      for (int k = 0; k < -sc; ++k) den *= 10;  // -sc <= 38 + prec: fits while |v| < 2^128
      if (-sc > 38) return false;
    }
    if (ex >= 0) {
      for (int k = 0; k < ex; ++k) {
        if (num >> 127) return false;
        num <<= 1;
      }
    } else {
      if (-ex >= 128) return false;
      if ((den >> (127 + ex)) != 0) return false;
      den <<= -ex;
    }
    const u128 q = num / den, r = num - q * den;
    u128 qq = q;
    if (r * 2 > den || (r * 2 == den && (q & 1))) ++qq;
    if (qq >= (u128)P * 10) { ++E; continue; }
    if (qq < (u128)P) { --E; continue; }
    N = (uint64_t)qq;
    return true;
  }
  return false;
}

// N / 10^prec with the divisor a compile-time constant per case (a multiply-high sequence
// instead of the generic 64-bit division, ~100 instructions, the formatter's hot spot for
// bedmap's "%.{p}lf" columns); prec <= 17 (bg_map), uniform across the launch
template <uint64_t P>
__device__ __forceinline__ uint64_t div_c(uint64_t N) {
  return N / P;
}
__device__ __forceinline__ uint64_t div_pow10(uint64_t N, int prec) {
  switch (prec) {
    case 0: return N;
    case 1: return div_c<10ull>(N);
    case 2: return div_c<100ull>(N);
    case 3: return div_c<1000ull>(N);
    case 4: return div_c<10000ull>(N);
    case 5: return div_c<100000ull>(N);
    case 6: return div_c<1000000ull>(N);
    case 7: return div_c<10000000ull>(N);
    case 8: return div_c<100000000ull>(N);
    case 9: return div_c<1000000000ull>(N);
    case 10: return div_c<10000000000ull>(N);
    case 11: return div_c<100000000000ull>(N);
    case 12: return div_c<1000000000000ull>(N);
    case 13: return div_c<10000000000000ull>(N);
    case 14: return div_c<100000000000000ull>(N);
    case 15: return div_c<1000000000000000ull>(N);
    case 16: return div_c<10000000000000000ull>(N);
    default: {
      uint64_t P = 1;
      for (int k = 0; k < prec; ++k) P *= 10;
      return N / P;
    }
  }
}

__device__ __forceinline__ int fixed_len(uint64_t N, bool neg, int prec) {
  const uint64_t ip = div_pow10(N, prec);
  return (neg ? 1 : 0) + dec_len_u64(ip) + (prec > 0 ? 1 + prec : 0);
}

template <typename Out>
__device__ __forceinline__ void put_fixed(Out& o, uint64_t N, bool neg, int prec) {
  uint64_t P = 1;
  for (int k = 0; k < prec; ++k) P *= 10;
  const uint64_t ip = div_pow10(N, prec), fp = N - ip * P;
  if (neg) { o.put_at(0, '-'); o.adv(1); }
  put_u64(o, ip, dec_len_u64(ip));
  if (prec > 0) {
    o.put_at(0, '.');
    o.adv(1);
    put_u64(o, fp, prec);
  }
}

// "%.{prec}e": d[.ddd]e±XX (at least two exponent digits)
template <typename Out>
__device__ __forceinline__ void put_sci(Out& o, uint64_t N, int E, bool neg, int prec) {
  uint64_t P = 1;
  for (int k = 0; k < prec; ++k) P *= 10;
  if (neg) o.put('-');
  o.put((char)('0' + N / P));
  if (prec > 0) {
    o.put('.');
    put_u64(o, N % P, prec);
  }
  o.put('e');
  o.put(E < 0 ? '-' : '+');
  const uint64_t ae = (uint64_t)(E < 0 ? -E : E);
  put_u64(o, ae, ae < 10 ? 2 : dec_len_u64(ae));
}
// exact "%.{p}lf" / "%.{p}e" for what the fast paths above do not cover: bg_decfmt.h
// a score-precision value (PrintScorePrecision: "%.{p}lf", or "%.{p}e" under --sci)
template <typename Out>
__device__ __forceinline__ bool put_real(Out& o, double v, int prec, bool sci) {
  uint64_t N;
  bool neg;
  if (v != v) {  // NaN: every NaN here comes from an invalid operation (sqrt of a negative
    // rounded variance, inf - inf), which on the reference's x86-64 build yields the
    // negative default NaN; glibc prints it as "-nan" under %lf and %e
    o.put('-'); o.put('n'); o.put('a'); o.put('n');
    return true;
  }
  if (v == __longlong_as_double(0x7ff0000000000000LL) || v == __longlong_as_double((long long)0xfff0000000000000ULL)) {
    if (v < 0) o.put('-');
    o.put('i'); o.put('n'); o.put('f');
    return true;
  }
  if (sci) {
    int E;
    if (prec <= 17 && sci_digits(v, prec, N, E, neg)) put_sci(o, N, E, neg, prec);
    else put_real_exact(o, v, prec, true);
    return true;
  }
  if (prec <= 17 && fixed_digits(v, prec, N, neg)) put_fixed(o, N, neg, prec);
  else put_real_exact(o, v, prec, false);
  return true;
}

// put_real's "%.{p}lf" for finite values whose digits fit 64 bits; false otherwise (NaN,
// infinities and huge values are left to the general formatter, RES_MAP)
template <typename Out>
__device__ __forceinline__ bool put_real_fixed(Out& o, double v, int prec) {
  uint64_t N;
  bool neg;
  if (prec > 17 || !fixed_digits(v, prec, N, neg)) return false;
  put_fixed(o, N, neg, prec);
  return true;
}
// RES_MAP formatted without the window / text / element / order-statistic operations and
// without --sci: a small kernel (the general one holds ~200 VGPRs and spills SGPRs for the
// operations a run does not use); bg_result_format falls back to RES_MAP on any value this
// path refuses
#define RES_MAPS 100
struct CountOut {  // measures only
  uint64_t n = 0;
  __device__ __forceinline__ void put_at(int, char) {}
  __device__ __forceinline__ void adv(int k) { n += k; }
  __device__ __forceinline__ void put(char) { ++n; }
};
struct LdsOut {
  char* p;
  __device__ __forceinline__ void put_at(int k, char c) { p[k] = c; }
  __device__ __forceinline__ void adv(int k) { p += k; }
  __device__ __forceinline__ void put(char c) { *p++ = c; }
};
// coordinates (< 10^12, at most 12 digits): SWAR digit groups where the sink is memory
__device__ __forceinline__ void put_coord(LdsOut& o, uint64_t v, int len) {
  if (len <= 12) {
    put_u64_lds(o.p, v, len);
    o.adv(len);
  } else {
    put_u64(o, v, len);
  }
}
__device__ __forceinline__ void put_coord(CountOut& o, uint64_t, int len) { o.adv(len); }
// a row rendered straight to HBM (oversized tiles): writes stop at the row's counted end, so
// a row that renders longer than the count pass measured (its inputs changed in between)
// cannot write past its slot or the text buffer; the mismatch is reported (BG_FMT_MISMATCH)
struct BoundOut {
  char* p;
  char* lim;
  __device__ __forceinline__ void put_at(int k, char c) {
    if (p + k < lim) p[k] = c;
  }
  __device__ __forceinline__ void adv(int k) { p += k; }
  __device__ __forceinline__ void put(char c) {
    if (p < lim) *p = c;
    ++p;
  }
};
__device__ __forceinline__ void put_coord(BoundOut& o, uint64_t v, int len) { put_u64(o, v, len); }

template <typename Out>
__device__ __forceinline__ void put_i64(Out& o, int64_t v) {
  if (v < 0) {
    o.put('-');
    const uint64_t u = (uint64_t)0 - (uint64_t)v;
    put_u64(o, u, dec_len_u64(u));
  } else {
    put_u64(o, (uint64_t)v, dec_len_u64((uint64_t)v));
  }
}

// "%s\t%lu\t%lu%s": chrom, start, end, verbatim rest (B3Rest print, Bed.hpp:321-325)
template <typename Out>
__device__ __forceinline__ void put_row(const FmtArgs& A, Out& o, int64_t s, int64_t e,
                                        const char* rest, uint32_t rl) {
  const uint32_t g = (uint32_t)(s >> BG_KEY_SHIFT);
  const uint32_t nl = A.name_len[g];
  const char* nm = A.names + A.name_off[g];
  for (uint32_t q = 0; q < nl; ++q) o.put(nm[q]);
  o.put('\t');
  const uint64_t cs = (uint64_t)(s & BG_COORD_MASK), ce = (uint64_t)(e & BG_COORD_MASK);
  put_coord(o, cs, dec_len_u64(cs));
  o.put('\t');
  put_coord(o, ce, dec_len_u64(ce));
  for (uint32_t q = 0; q < rl; ++q) o.put(rest[q]);
}

template <typename Out>
__device__ __forceinline__ void put_delim(const FmtArgs& A, Out& o) {
  for (int d = 0; d < A.dlen; ++d) o.put(A.delim[d]);
}

// getDistance(x, ref) of closest-features (ClosestFeature.cpp:244-255), same chromosome
__device__ __forceinline__ int64_t cf_dist(int64_t xs, int64_t xe, int64_t bs, int64_t be) {
  if (xe <= bs) return -((bs - xe) + 1);
  if (be <= xs) return (xs - be) + 1;
  return 0;
}

// one closest-features line: PrintAll (Printers.hpp:54-93) or PrintShortest (:112-200)
template <typename Out>
__device__ __forceinline__ void render_closest(const FmtArgs& A, uint64_t k, Out& o) {
  const int64_t bs = A.s[k], be = A.e[k];
  if (!A.no_ref) {
    put_row(A, o, bs, be, A.text + A.rest_off[k], A.rest_len[k]);
    put_delim(A, o);
  }
  const int64_t L = A.left[k], R = A.right[k];
  auto cand = [&](int64_t x, int zero_dist) {
    put_row(A, o, A.s2[x], A.e2[x], A.text2 + A.rest_off2[x], A.rest_len2[x]);
    if (A.print_dist) {
      put_delim(A, o);
      if (zero_dist) o.put('0');
      else put_i64(o, cf_dist(A.s2[x], A.e2[x], bs, be));
    }
  };
  auto na = [&]() {
    o.put('N');
    o.put('A');
    if (A.print_dist) {
      put_delim(A, o);
      o.put('N');
      o.put('A');
    }
  };
  if (!A.shortest) {
    if (L >= 0) cand(L, 0);
    else na();
    put_delim(A, o);
    if (R >= 0) cand(R, 0);
    else na();
    o.put('\n');
    return;
  }
  if (L < 0 && R < 0) {
    na();
    o.put('\n');
    return;
  }
  int64_t d1 = LLONG_MAX, d2 = LLONG_MAX;
  if (L >= 0) {
    if (A.e2[L] <= bs) {  // <= as getDistance
      d1 = (bs - A.e2[L]) + 1;
      if (R < 0) { cand(L, 0); o.put('\n'); return; }
    } else {  // overlapping or adjacent left: printed with distance 0
      cand(L, 1);
      o.put('\n');
      return;
    }
  }
  if (R >= 0) {
    if (L < 0) { cand(R, 0); o.put('\n'); return; }
    if (be <= A.s2[R]) d2 = (A.s2[R] - be) + 1;
    else { cand(R, 1); o.put('\n'); return; }
  }
  if (d1 <= d2) cand(L, 0);
  else cand(R, 0);
  o.put('\n');
}

__device__ __forceinline__ bool fmt_isws(char ch) { return ch == ' ' || (ch >= '\t' && ch <= '\r'); }

// map row m as the reference's map type prints it (Bed.hpp): B3Rest "%s\t%lu\t%lu%s",
// B4Rest "%s\t%lu\t%lu\t%s%s" (id, then what follows it), B5Rest "...\t%s\t%lf%s"
// (the score re-printed with "%lf", Formats.hpp:34)
template <typename Out>
__device__ __forceinline__ bool put_map_row(const FmtArgs& A, Out& o, uint64_t m, int sprec = -1) {
  const char* rp = A.text2 + A.rest_off2[m];
  const uint32_t rl = A.rest_len2[m];
  if (A.mapfields == 3) {
    put_row(A, o, A.s2[m], A.e2[m], rp, rl);
    return true;
  }
  put_row(A, o, A.s2[m], A.e2[m], rp, 0);
  uint32_t i = 0;
  while (i < rl && fmt_isws(rp[i])) ++i;
  o.put('\t');
  for (; i < rl && !fmt_isws(rp[i]); ++i) o.put(rp[i]);  // id
  if (A.mapfields == 5) {
    while (i < rl && fmt_isws(rp[i])) ++i;
    while (i < rl && !fmt_isws(rp[i])) ++i;  // the score's text, re-printed
    o.put('\t');
    if (sprec >= 0) {  // PrintAllScorePrecision: "%.{p}lf" / "%.{p}e"
      if (!put_real(o, A.score2[m], sprec, A.sci)) return false;
    } else {
      uint64_t N;
      bool neg;
      const double sv = A.score2[m];
      if (sv != sv || sv == __longlong_as_double(0x7ff0000000000000LL) ||
          sv == __longlong_as_double((long long)0xfff0000000000000ULL)) {
        if (!put_real(o, sv, 6, false)) return false;
      } else if (!fixed_digits(sv, 6, N, neg)) {
        put_real_exact(o, sv, 6, false);
      } else {
        put_fixed(o, N, neg, 6);
      }
    }
  }
  for (; i < rl; ++i) o.put(rp[i]);
  return true;
}

// the sweep's padding of the criterion (RangedDist under --range)
__device__ __forceinline__ int64_t fmt_pad(const FmtArgs& A) {
  return A.crit == BG_OVR_RANGE ? A.range : 0;
}

// the window's rows of reference row k in GenomicAddressCompare order (BedCompare.hpp:51-63):
// row order, except that a run of rows equal in (start, end) comes in heap-address order
// (A.maddr, bg_heap.hip); f returns false to stop
template <typename F>
__device__ __forceinline__ void map_window_genomic(const FmtArgs& A, uint64_t k, F f) {
  const int64_t s = A.s[k], e = A.e[k];
  auto member = [&](uint64_t m) {
    return bg_map_live(A.zin, A.zout, k, m) && bg_map_in(A.crit, A.ovr, A.range, A.perc, s, e, A.s2[m], A.e2[m]);
  };
  uint64_t skip = 0;  // rows below this went out with their tie run
  // --faster: the window is exactly [wlo, whi) (the sweep's deque), so a tie run is cut to it
  const uint64_t tend = A.crit == BG_OVR_FAST ? A.whi[k] : A.n2;
  bg_map_cands(A.s2, A.e2, A.wlo[k], A.whi[k], A.lrows, s, e, fmt_pad(A), [&](uint64_t m) {
    if (m < skip) return true;
    if (A.maddr && m + 1 < tend && A.s2[m + 1] == A.s2[m] && A.e2[m + 1] == A.e2[m]) {
      uint64_t t = m + 1;
      while (t < tend && A.s2[t] == A.s2[m] && A.e2[t] == A.e2[m]) ++t;
      skip = t;
      if (A.maord) {  // the whole run in address order (bg_heap_addr), its rows [m, t) taken
        uint64_t r0 = m, r1 = t;
        while (r0 > 0 && A.s2[r0 - 1] == A.s2[m] && A.e2[r0 - 1] == A.e2[m]) --r0;
        while (r1 < A.n2 && A.s2[r1] == A.s2[m] && A.e2[r1] == A.e2[m]) ++r1;
        for (uint64_t q = r0; q < r1; ++q) {
          const uint64_t u = A.maord[q];
          if (u < m || u >= t || !member(u)) continue;
          if (!f(u)) return false;
        }
        return true;
      }
      bool has = false;
      int64_t last = 0;
      for (;;) {  // the run's members by increasing address
        uint64_t best = ~0ULL;
        for (uint64_t u = m; u < t; ++u) {
          if (!member(u) || (has && A.maddr[u] <= last)) continue;
          if (best == ~0ULL || A.maddr[u] < A.maddr[best]) best = u;
        }
        if (best == ~0ULL) return true;
        if (!f(best)) return false;
        has = true;
        last = A.maddr[best];
      }
    }
    if (!member(m)) return true;
    return f(m);
  });
}

// --echo-map* of reference row k: the window's rows in genomic order (EchoMapBed's set,
// EchoMapBedVisitor.hpp:58-63) joined by --multidelim (PrintRangeDelim)
template <typename Out>
__device__ __forceinline__ bool put_echo_map(const FmtArgs& A, Out& o, uint64_t k, int op) {
  const int64_t s = A.s[k], e = A.e[k];
  bool first = true, ok = true;
  int64_t rs = 0, re = 0;
  map_window_genomic(A, k, [&](uint64_t m) {
    const int64_t ms = A.s2[m], me = A.e2[m];
    if (op == BG_MAP_ECHO_MAP_RANGE) {  // PrintGenomicRange (ProcessBedVisitorRow.hpp:433-456)
      if (first) { rs = ms; re = me; }
      else { rs = min(rs, ms); re = max(re, me); }
      first = false;
      return true;
    }
    if (!first) for (int d = 0; d < A.mdlen; ++d) o.put(A.mdelim[d]);
    first = false;
    if (op == BG_MAP_ECHO_MAP) {
      if (!put_map_row(A, o, m)) { ok = false; return false; }
    } else if (op == BG_MAP_ECHO_MAP_ID) {
      const char* rp = A.text2 + A.rest_off2[m];
      const uint32_t rl = A.rest_len2[m];
      uint32_t i = 0;
      while (i < rl && fmt_isws(rp[i])) ++i;
      for (; i < rl && !fmt_isws(rp[i]); ++i) o.put(rp[i]);
    } else if (op == BG_MAP_ECHO_MAP_SCORE) {
      if (!put_real(o, A.score2[m], A.prec, A.sci)) { ok = false; return false; }
    } else if (op == BG_MAP_ECHO_MAP_SIZE) {
      const uint64_t len = (uint64_t)(me - ms);
      put_u64(o, len, dec_len_u64(len));
    } else {  // BG_MAP_ECHO_OVERLAP_SIZE: |ref ∩ map row|, "%ld"
      const int64_t ov = min(e, me) - max(s, ms);
      const uint64_t len = ov > 0 ? (uint64_t)ov : 0;
      put_u64(o, len, dec_len_u64(len));
    }
    return true;
  });
  if (!ok) return false;
  if (op == BG_MAP_ECHO_MAP_RANGE && !first) put_row(A, o, rs, re, nullptr, 0);
  return true;
}

// the id (4th column) of map row m: the first token of its remainder
__device__ __forceinline__ const char* map_id(const FmtArgs& A, uint64_t m, uint32_t& len) {
  const char* rp = A.text2 + A.rest_off2[m];
  const uint32_t rl = A.rest_len2[m];
  uint32_t i = 0;
  while (i < rl && fmt_isws(rp[i])) ++i;
  uint32_t j = i;
  while (j < rl && !fmt_isws(rp[j])) ++j;
  len = j - i;
  return rp + i;
}
// std::string ordering (char_traits<char>::compare: bytes as unsigned char, then length)
__device__ __forceinline__ int id_cmp(const char* a, uint32_t la, const char* b, uint32_t lb) {
  const uint32_t n = la < lb ? la : lb;
  for (uint32_t i = 0; i < n; ++i)
    if (a[i] != b[i]) return (uint8_t)a[i] < (uint8_t)b[i] ? -1 : 1;
  return la < lb ? -1 : (la > lb ? 1 : 0);
}
// --echo-map-id-uniq: the window's ids as a sorted set (PrintUniqueRangeIDs,
// ProcessBedVisitorRow.hpp:361-385), by repeated selection of the next larger id
template <typename Out>
__device__ __forceinline__ void put_unique_ids(const FmtArgs& A, Out& o, uint64_t k) {
  const int64_t s = A.s[k], e = A.e[k];
  const char* prev = nullptr;
  uint32_t plen = 0;
  for (;;) {
    const char* best = nullptr;
    uint32_t blen = 0;
    bg_map_cands(A.s2, A.e2, A.wlo[k], A.whi[k], A.lrows, s, e, fmt_pad(A), [&](uint64_t m) {
      if (!bg_map_live(A.zin, A.zout, k, m) ||
          !bg_map_in(A.crit, A.ovr, A.range, A.perc, s, e, A.s2[m], A.e2[m]))
        return true;
      uint32_t l;
      const char* id = map_id(A, m, l);
      if (prev && id_cmp(id, l, prev, plen) <= 0) return true;
      if (!best || id_cmp(id, l, best, blen) < 0) { best = id; blen = l; }
      return true;
    });
    if (!best) return;
    if (prev) for (int d = 0; d < A.mdlen; ++d) o.put(A.mdelim[d]);
    for (uint32_t i = 0; i < blen; ++i) o.put(best[i]);
    prev = best;
    plen = blen;
  }
}

// value at sorted position p of the window's scores (a multiset: x is at positions
// [#{< x}, #{<= x}) ), by counting; windows are small, and this keeps no per-row buffer
// (dev: of the absolute deviations |x - med| instead, MedianAbsoluteDeviationVisitor.hpp:43-49)
__device__ __forceinline__ double mad_dev(double x, double med) {
  const double d = x - med;
  return d < 0 ? -d : d;
}
__device__ __forceinline__ double window_rank(const FmtArgs& A, uint64_t k, uint32_t p,
                                              bool dev = false, double med = 0.0) {
  const int64_t s = A.s[k], e = A.e[k];
  double out = 0.0;  // (every p < window size is found)
  bg_map_cands(A.s2, A.e2, A.wlo[k], A.whi[k], A.lrows, s, e, fmt_pad(A), [&](uint64_t i) {
    if (!bg_map_live(A.zin, A.zout, k, i) ||
        !bg_map_in(A.crit, A.ovr, A.range, A.perc, s, e, A.s2[i], A.e2[i]))
      return true;
    const double x = dev ? mad_dev(A.score2[i], med) : A.score2[i];
    uint32_t lt = 0, le = 0;
    bg_map_cands(A.s2, A.e2, A.wlo[k], A.whi[k], A.lrows, s, e, fmt_pad(A), [&](uint64_t j) {
      if (!bg_map_live(A.zin, A.zout, k, j) ||
          !bg_map_in(A.crit, A.ovr, A.range, A.perc, s, e, A.s2[j], A.e2[j]))
        return true;
      const double y = dev ? mad_dev(A.score2[j], med) : A.score2[j];
      lt += y < x;
      le += y <= x;
      return true;
    });
    if (lt <= p && p < le) { out = x; return false; }
    return true;
  });
  return out;
}

// RollingKthAverage::DoneReference (numerical/RollingKthAverageVisitor.hpp:61-92): with
// up = ceil(kth*n), down = floor(kth*n), each made zero-based when > 0, the average of the
// elements at up and up+1 when up == down, else the element at up
__device__ __forceinline__ double window_kth(const FmtArgs& A, uint64_t k, uint32_t n, double kth) {
  if (n == 1) return window_rank(A, k, 0);
  uint64_t up = (uint64_t)ceil(kth * (double)n), down = (uint64_t)floor(kth * (double)n);
  if (up > 0) --up;
  if (down > 0) --down;
  if (up == down) {
    const double one = window_rank(A, k, (uint32_t)up), two = window_rank(A, k, (uint32_t)up + 1);
    return (one + two) / 2.0;
  }
  return window_rank(A, k, (uint32_t)up);
}

// --min-element / --max-element[-rand]: the window row Extreme<PrintAllScorePrecision>
// prints (ExtremeVisitor.hpp:103-133). Stable: the set is ordered by
// ScoreThenGenomicCompareLesser/Greater (score, then chrom/start/end; BedCompare.hpp:263-288)
// and keeps the first of equivalent rows, which fixWindow adds in CoordRestAddressCompare
// order (full_rest, then address). -rand: CompValueThenAddress order, then RandTie's
// random pick among equal scores (the first of the set here: min lowest row, max highest).
__device__ __forceinline__ bool elem_better(const FmtArgs& A, int op, uint64_t m, uint64_t b) {
  const double x = A.score2[m], y = A.score2[b];
  const int64_t am = bg_maddr(A.maddr, m), ab = bg_maddr(A.maddr, b);
  if (op == BG_MAP_MIN_ELEMENT_RAND) return x != y ? x < y : am < ab;
  if (op == BG_MAP_MAX_ELEMENT_RAND) return x != y ? x > y : am > ab;
  const bool mx = op == BG_MAP_MAX_ELEMENT;
  if (x != y) return mx ? x > y : x < y;
  if (A.s2[m] != A.s2[b]) return mx ? A.s2[m] > A.s2[b] : A.s2[m] < A.s2[b];
  if (A.e2[m] != A.e2[b]) return mx ? A.e2[m] > A.e2[b] : A.e2[m] < A.e2[b];
  // --faster: rows join the set in file order (no fixWindow), and equal rows join and leave
  // the deque together: the set keeps the first in file order
  if (A.crit == BG_OVR_FAST) return m < b;
  const int c = bg_frest_cmp(A.text2, A.rest_off2, A.rest_len2, A.mapfields, m, b);
  return c != 0 ? c < 0 : am < ab;
}
template <typename Out>
__device__ __forceinline__ bool put_element(const FmtArgs& A, Out& o, uint64_t k, int op) {
  const int64_t s = A.s[k], e = A.e[k];
  uint64_t best = ~0ULL;
  bg_map_cands(A.s2, A.e2, A.wlo[k], A.whi[k], A.lrows, s, e, fmt_pad(A), [&](uint64_t m) {
    if (!bg_map_live(A.zin, A.zout, k, m) || !bg_map_in(A.crit, A.ovr, A.range, A.perc, s, e, A.s2[m], A.e2[m]))
      return true;
    if (best == ~0ULL || elem_better(A, op, m, best)) best = m;
    return true;
  });
  return put_map_row(A, o, best, A.prec);
}
// --wmean: WeightedAverage::DoneReference (bed/WeightedAverageVisitor.hpp:55-70) over its
// std::set<MapType*> (heap-address order, A.maddr; row order without a replay): sum of
// overlap/len(ref) * score, divided by the sum of the weights
__device__ __forceinline__ double window_wmean(const FmtArgs& A, uint64_t k) {
  const int64_t s = A.s[k], e = A.e[k];
  const double len = (double)(uint64_t)(e - s);
  double value = 0, wsum = 0;
  if (A.maddr) {  // by repeated selection of the next larger address
    bool has = false;
    int64_t last = 0;
    for (;;) {
      uint64_t best = ~0ULL;
      bg_map_cands(A.s2, A.e2, A.wlo[k], A.whi[k], A.lrows, s, e, fmt_pad(A), [&](uint64_t m) {
        if (!bg_map_live(A.zin, A.zout, k, m) || !bg_map_in(A.crit, A.ovr, A.range, A.perc, s, e, A.s2[m], A.e2[m]))
          return true;
        if (has && A.maddr[m] <= last) return true;
        if (best == ~0ULL || A.maddr[m] < A.maddr[best]) best = m;
        return true;
      });
      if (best == ~0ULL) break;
      const int64_t ov = min(e, A.e2[best]) - max(s, A.s2[best]);
      const double w = (double)(uint64_t)(ov > 0 ? ov : 0) / len;
      value += w * A.score2[best];
      wsum += w;
      has = true;
      last = A.maddr[best];
    }
    return value / wsum;
  }
  bg_map_cands(A.s2, A.e2, A.wlo[k], A.whi[k], A.lrows, s, e, fmt_pad(A), [&](uint64_t m) {
    const int64_t ms = A.s2[m], me = A.e2[m];
    if (!bg_map_live(A.zin, A.zout, k, m) || !bg_map_in(A.crit, A.ovr, A.range, A.perc, s, e, ms, me))
      return true;
    const int64_t ov = min(e, me) - max(s, ms);
    const double w = (double)(uint64_t)(ov > 0 ? ov : 0) / len;
    value += w * A.score2[m];
    wsum += w;
    return true;
  });
  return value / wsum;
}
__device__ __forceinline__ bool is_elem_op(int op) {
  return op >= BG_MAP_MIN_ELEMENT && op <= BG_MAP_MAX_ELEMENT_RAND;
}

// renders (or measures) line k; returns false on a value outside the GPU range
template <int KIND, typename Out>
__device__ __forceinline__ bool render(const FmtArgs& A, uint64_t k, Out& o) {
  if (KIND == RES_CLOSEST) {
    render_closest(A, k, o);
    return true;
  }
  if (KIND == RES_MAP || KIND == RES_MAPS) {
    constexpr bool FULL = KIND == RES_MAP;  // RES_MAPS: the plain numeric columns only
    // one value per operation (MultiVisitor.hpp:83-98); formats: Count/Indicator "%d",
    // OvrAggregate "%lu", OvrUnique "%u", Echo (ProcessBedVisitorRow.hpp:309-342), the rest
    // "%.{p}lf" or "NAN" (PrintScorePrecision, Formats.hpp:42-50)
    const int32_t c = A.cnt[k];
    if (A.skip_unmapped && c == 0) return true;
    for (int q = 0; q < A.nops; ++q) {
      if (q) put_delim(A, o);
      const int op = A.ops[q];
      if (op == BG_MAP_COUNT) {
        put_i64(o, (int64_t)c);
        continue;
      }
      if (op == BG_MAP_INDICATOR) {
        o.put(c > 0 ? '1' : '0');
        continue;
      }
      if (op == BG_MAP_BASES) {
        put_u64(o, A.bases[k], dec_len_u64(A.bases[k]));
        continue;
      }
      if (op == BG_MAP_BASES_UNIQ) {
        put_u64(o, (uint64_t)A.uniq[k], dec_len_u64((uint64_t)A.uniq[k]));
        continue;
      }
      if (FULL && op == BG_MAP_ECHO) {
        if (A.single) {  // the row as its own (map) type prints it
          if (!put_map_row(A, o, k)) return false;
        } else {
          put_row(A, o, A.s[k], A.e[k], A.text + A.rest_off[k], A.rest_len[k]);
        }
        continue;
      }
      if (FULL && is_elem_op(op)) {
        if (c <= 0) return true;  // the reference throws here: the line ends unfinished
        if (!put_element(A, o, k, op)) return false;
        continue;
      }
      if (FULL && op == BG_MAP_ECHO_MAP_ID_UNIQ) {
        put_unique_ids(A, o, k);
        continue;
      }
      if (FULL && op == BG_MAP_ECHO_REF_ROW_ID) {  // PrintRowID: "id-" ++rowID (a static shared by all)
        const uint64_t line = A.rrank ? A.rrank[k] : k;
        uint64_t j = 0;
        for (int q2 = 0; q2 < q; ++q2) j += A.ops[q2] == BG_MAP_ECHO_REF_ROW_ID;
        const uint64_t id = line * (uint64_t)A.nrid + j + 1;
        o.put('i'); o.put('d'); o.put('-');
        put_u64(o, id, dec_len_u64(id));
        continue;
      }
      if (FULL && op >= BG_MAP_ECHO_MAP && op <= BG_MAP_ECHO_MAP_RANGE) {
        if (!put_echo_map(A, o, k, op)) return false;
        continue;
      }
      if (op == BG_MAP_ECHO_SIZE) {
        const uint64_t len = (uint64_t)(A.e[k] - A.s[k]);
        put_u64(o, len, dec_len_u64(len));
        continue;
      }
      if (op == BG_MAP_ECHO_NAME) {  // "chrom:start-end"
        const uint32_t g = (uint32_t)(A.s[k] >> BG_KEY_SHIFT);
        const char* nm = A.names + A.name_off[g];
        for (uint32_t i = 0; i < A.name_len[g]; ++i) o.put(nm[i]);
        o.put(':');
        const uint64_t cs = (uint64_t)(A.s[k] & BG_COORD_MASK), ce = (uint64_t)(A.e[k] & BG_COORD_MASK);
        put_u64(o, cs, dec_len_u64(cs));
        o.put('-');
        put_u64(o, ce, dec_len_u64(ce));
        continue;
      }
      double v;
      if (op == BG_MAP_BASES_UNIQ_F) {
        v = (double)A.uniq[k] / (double)(A.e[k] - A.s[k]);
      } else if (c <= 0) {
        o.put('N'); o.put('A'); o.put('N');
        continue;
      } else if (op == BG_MAP_MEAN) {
        v = (A.dsum ? A.dsum[k] : (double)A.isum[k]) / (double)c;
      } else if (op == BG_MAP_SUM) {
        v = A.dsum ? A.dsum[k] : (double)A.isum[k];
      } else if (op == BG_MAP_VARIANCE || op == BG_MAP_STDEV || op == BG_MAP_CV) {
        // Variance / StdDev / CoeffVariation DoneReference (VarianceVisitor.hpp, StdevVisitor.hpp,
        // CoeffVariationVisitor.hpp:60-74) on the exact running sums, in their double order
        if (c <= 1) { o.put('N'); o.put('A'); o.put('N'); continue; }
        const double cnt = (double)c;
        const double sum = A.dsum ? A.dsum[k] : (double)A.isum[k];
        const double sq = A.dsq ? A.dsq[k] : (double)A.isq[k];
        const double numer = (cnt * sq) - (sum * sum);
        const double denom = (cnt * (cnt - 1));
        v = numer / denom;
        if (op != BG_MAP_VARIANCE) v = sqrt(v);
        if (op == BG_MAP_CV) {
          const double mean = sum / cnt;
          if (mean == 0) { o.put('N'); o.put('A'); o.put('N'); continue; }
          v = v / mean;
        }
      } else if (FULL && op == BG_MAP_MAD) {  // MedianAbsoluteDeviation::DoneReference (:70-110)
        if (c <= 1) { o.put('N'); o.put('A'); o.put('N'); continue; }
        const double med = window_kth(A, k, (uint32_t)c, 0.5);
        const uint32_t sz = (uint32_t)c;
        double mad;
        if (sz % 2 == 0) {
          mad = window_rank(A, k, sz / 2 - 1, true, med);
          mad += window_rank(A, k, sz / 2, true, med);
          mad /= 2.0;
        } else {
          mad = window_rank(A, k, sz / 2, true, med);
        }
        v = mad * (A.op_arg[q] > 0 ? A.op_arg[q] : 1.0);
      } else if (FULL && (op == BG_MAP_MEDIAN || op == BG_MAP_KTH)) {
        v = window_kth(A, k, (uint32_t)c, op == BG_MAP_MEDIAN ? 0.5 : A.op_arg[q]);
      } else if (FULL && op == BG_MAP_TMEAN) {
        v = A.tmv[q][k];
      } else if (FULL && op == BG_MAP_WMEAN) {
        v = window_wmean(A, k);
      } else {
        v = (op == BG_MAP_MIN) ? A.vmin[k] : A.vmax[k];
      }
      if (FULL) {
        if (!put_real(o, v, A.prec, A.sci)) return false;
      } else if (!put_real_fixed(o, v, A.prec)) {
        return false;  // (the general kind renders this run)
      }
    }
    o.put('\n');
    return true;
  }
  const uint64_t r = (KIND == RES_ROWS) ? A.rows[k] : k;
  const int64_t s = A.s[r], e = A.e[r];
  const uint32_t g = (uint32_t)(s >> BG_KEY_SHIFT);
  const uint32_t nl = A.name_len[g];
  const char* nm = A.names + A.name_off[g];
  for (uint32_t q = 0; q < nl; ++q) o.put(nm[q]);
  o.put('\t');
  const uint64_t cs = (uint64_t)(s & BG_COORD_MASK), ce = (uint64_t)(e & BG_COORD_MASK);
  put_coord(o, cs, dec_len_u64(cs));
  o.put('\t');
  put_coord(o, ce, dec_len_u64(ce));
  if (KIND == RES_ROWS) {
    const uint32_t rl = A.rest_len[r];
    const char* rp = A.text + A.rest_off[r];
    for (uint32_t q = 0; q < rl; ++q) o.put(rp[q]);
  } else if (KIND == RES_MULTI) {
    const uint32_t rl = A.rlen[k];
    const char* rp = (const char*)A.rows[k];
    if (A.rest_tab && rl) o.put('\t');
    for (uint32_t q = 0; q < rl; ++q) o.put(rp[q]);
  }
  o.put('\n');
  return true;
}

// bytes of every FT_TILE-row tile: one wave per tile (rows striped over the lanes, 64-lane
// shuffle reduction), FC_TILES tiles per workgroup, no workgroup barrier
#define FC_TILES 8
template <int KIND>
__global__ void __launch_bounds__(BG_NT) k_fmt_count(FmtArgs A, uint64_t* __restrict__ tb,
                                                     uint64_t ntiles, bg_dstatus* st) {
  const int lane = bg_lane();
  for (uint64_t t = (uint64_t)blockIdx.x * FC_TILES + bg_wave(); t < (uint64_t)(blockIdx.x + 1) * FC_TILES;
       t += BG_NT / 64) {
    if (t >= ntiles) return;
    CountOut co;
    const uint64_t base = t * FT_TILE + lane;
#pragma unroll 2
    for (int k = 0; k < FT_TILE / 64; ++k) {
      const uint64_t row = base + (uint64_t)k * 64;
      const uint64_t n0 = co.n;
      if (row < A.n && !render<KIND>(A, row, co)) bg_report(st, row, ERR_RANGE);
      if (A.rowlen && row < A.n) A.rowlen[row] = (uint32_t)(co.n - n0);
      if (KIND == RES_MAP && A.has_elem && row < A.n && A.cnt[row] <= 0)
        atomicMin(&st->stop_row, (unsigned long long)row);
    }
    uint64_t v = co.n;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if (lane == 0) tb[t] = v;
  }
}

// the row stripes unrolled: their byte offsets (my[]) stay in registers (not unrolled, the
// large render bodies left the loops rolled and my[] in scratch: 32 bytes per lane)
#ifndef BG_FMT_UNROLL
#define BG_FMT_UNROLL 1
#endif
#if BG_FMT_UNROLL
#define FMT_UNROLL _Pragma("unroll")
// (RES_MAP's render is too large to unroll; its loops stay rolled)
#pragma clang diagnostic ignored "-Wpass-failed"
#else
#define FMT_UNROLL
#endif
template <int KIND>
__global__ void __launch_bounds__(BG_NT) k_fmt_write(FmtArgs A, const uint64_t* __restrict__ toff,
                                                     char* __restrict__ out) {
  __shared__ uint64_t sh[BG_NT / 64 + 1];
  __shared__ __attribute__((aligned(16))) char buf[FT_LDS + 16];
  // rows are striped over the threads (coalesced column reads); a row's byte offset
  // in the tile = all bytes of the previous stripes + its prefix inside its stripe
  const uint64_t base = (uint64_t)blockIdx.x * FT_TILE + threadIdx.x;
  uint64_t my[FT_ROWS];
  uint64_t tot = 0;
FMT_UNROLL
  for (int k = 0; k < FT_ROWS; ++k) {
    const uint64_t row = base + (uint64_t)k * BG_NT;
    CountOut co;
    if (row < A.n) {
      if (A.rowlen) co.n = A.rowlen[row];
      else render<KIND>(A, row, co);
    }
    uint64_t st;
    my[k] = tot + block_excl_scan(co.n, OpSum(), (uint64_t)0, sh, &st);
    tot += st;
    if (KIND == RES_MAP && row == A.stop_row) *A.stop_out = toff[blockIdx.x] + my[k] + co.n;
  }
  const uint64_t dst0 = toff[blockIdx.x];
  bool mismatch = false;  // a row rendered to another length than it was placed with
  if (tot > FT_LDS) {  // oversized tile (long names / rests): render straight to HBM
  FMT_UNROLL
  for (int k = 0; k < FT_ROWS; ++k) {
      const uint64_t row = base + (uint64_t)k * BG_NT;
      if (row >= A.n) continue;
      const uint64_t len = A.rowlen ? A.rowlen[row] : 0;
      char* const p0 = out + dst0 + my[k];
      BoundOut o{p0, A.rowlen ? p0 + len : out + A.total};
      render<KIND>(A, row, o);
      mismatch |= A.rowlen && (uint64_t)(o.p - p0) != len;
    }
    if (mismatch && A.st) atomicOr(&A.st->flags, BG_FMT_MISMATCH);
    return;
  }
  // stage with the same alignment mod 16 as the destination, so every aligned 16-byte
  // chunk of the output is one aligned 16-byte LDS read
  const uint32_t skew = (uint32_t)(dst0 & 15);
FMT_UNROLL
  for (int k = 0; k < FT_ROWS; ++k) {
    const uint64_t row = base + (uint64_t)k * BG_NT;
    LdsOut o{buf + skew + my[k]};
    if (row < A.n) {
      render<KIND>(A, row, o);
      mismatch |= A.rowlen && (uint64_t)(o.p - (buf + skew + my[k])) != A.rowlen[row];
    }
  }
  if (mismatch && A.st) atomicOr(&A.st->flags, BG_FMT_MISMATCH);
  __syncthreads();
  // stream buf[skew, skew + tot) -> out[dst0, dst0 + tot)
  const uint64_t a0 = dst0, a1 = dst0 + tot;
  const uint64_t al0 = (a0 + 15) & ~15ULL, al1 = a1 & ~15ULL;
  const char* bb = buf + skew;
  if (al0 >= al1) {
    for (uint64_t p = a0 + threadIdx.x; p < a1; p += BG_NT) out[p] = bb[p - a0];
    return;
  }
  for (uint64_t p = a0 + threadIdx.x; p < al0; p += BG_NT) out[p] = bb[p - a0];
  for (uint64_t p = al1 + threadIdx.x; p < a1; p += BG_NT) out[p] = bb[p - a0];
  for (uint64_t p = al0 + 16ull * threadIdx.x; p < al1; p += 16ull * BG_NT)
    *reinterpret_cast<uint4*>(out + p) = *reinterpret_cast<const uint4*>(bb + (p - a0));
}

// RES_IVL rows ("%s\t%lu\t%lu\n"): thread t renders rows 2t and 2t+1 of the tile, both
// loaded up front as 16-byte pairs, so one block scan of the per-thread byte counts places
// them (k_fmt_write's general form scans once per row stripe and reloads each row to
// render it)
__device__ __forceinline__ uint32_t ivl_len(const FmtArgs& A, int64_t s, int64_t e) {
  return bg_ivl_len(A.name_len, s, e);
}
__device__ __forceinline__ void ivl_put(const FmtArgs& A, char* p, int64_t s, int64_t e) {
  const uint32_t g = (uint32_t)(s >> BG_KEY_SHIFT);
  const uint32_t nl = A.name_len[g];
  const char* nm = A.names + A.name_off[g];
  for (uint32_t q = 0; q < nl; ++q) p[q] = nm[q];
  p += nl;
  *p++ = '\t';
  const uint64_t cs = (uint64_t)(s & BG_COORD_MASK), ce = (uint64_t)(e & BG_COORD_MASK);
  const int l1 = dec_len_u64(cs), l2 = dec_len_u64(ce);
  put_u64_lds(p, cs, l1);
  p += l1;
  *p++ = '\t';
  put_u64_lds(p, ce, l2);
  p[l2] = '\n';
}

__global__ void __launch_bounds__(BG_NT) k_fmt_ivl_write(FmtArgs A, const uint64_t* __restrict__ toff,
                                                         char* __restrict__ out) {
  __shared__ uint32_t sh[BG_NT / 64 + 1];
  __shared__ __attribute__((aligned(16))) char buf[FT_LDS + 16];
  static_assert(FT_ROWS == 2, "two rows per thread");
  const uint64_t r0 = (uint64_t)blockIdx.x * FT_TILE + 2ull * threadIdx.x;
  int64_t s0 = 0, e0 = 0, s1 = 0, e1 = 0;
  const bool v0 = r0 < A.n, v1 = r0 + 1 < A.n;
  if (v1) {
    const longlong2 S = reinterpret_cast<const longlong2*>(A.s)[r0 >> 1];
    const longlong2 E = reinterpret_cast<const longlong2*>(A.e)[r0 >> 1];
    s0 = S.x; s1 = S.y; e0 = E.x; e1 = E.y;
  } else if (v0) {
    s0 = A.s[r0];
    e0 = A.e[r0];
  }
  const uint32_t l0 = v0 ? ivl_len(A, s0, e0) : 0u, l1 = v1 ? ivl_len(A, s1, e1) : 0u;
  uint32_t tot;
  const uint32_t my = block_excl_scan(l0 + l1, OpSum(), 0u, sh, &tot);
  const uint64_t dst0 = toff[blockIdx.x];
  if (tot > FT_LDS) {  // oversized tile (long names): render straight to HBM
    if (v0) ivl_put(A, out + dst0 + my, s0, e0);
    if (v1) ivl_put(A, out + dst0 + my + l0, s1, e1);
    return;
  }
  const uint32_t skew = (uint32_t)(dst0 & 15);
  if (v0) ivl_put(A, buf + skew + my, s0, e0);
  if (v1) ivl_put(A, buf + skew + my + l0, s1, e1);
  __syncthreads();
  const uint64_t a0 = dst0, a1 = dst0 + tot;
  const uint64_t al0 = (a0 + 15) & ~15ULL, al1 = a1 & ~15ULL;
  const char* bb = buf + skew;
  if (al0 >= al1) {
    for (uint64_t p = a0 + threadIdx.x; p < a1; p += BG_NT) out[p] = bb[p - a0];
    return;
  }
  for (uint64_t p = a0 + threadIdx.x; p < al0; p += BG_NT) out[p] = bb[p - a0];
  for (uint64_t p = al1 + threadIdx.x; p < a1; p += BG_NT) out[p] = bb[p - a0];
  for (uint64_t p = al0 + 16ull * threadIdx.x; p < al1; p += 16ull * BG_NT)
    *reinterpret_cast<uint4*>(out + p) = *reinterpret_cast<const uint4*>(bb + (p - a0));
}

// RES_ROWS rows (the input line re-rendered: "%s\t%lu\t%lu" + its rest + "\n", bedops
// --element-of / --not-element-of): k_fmt_ivl_write's layout — thread t renders rows 2t and
// 2t+1 of the tile (their row indices, keys and rest spans loaded up front), one block scan of
// the per-thread byte counts places them, LDS staging, 16-byte stores — instead of
// k_fmt_write<RES_ROWS>'s two renders per row (a counting one for the stripe scan, then the
// real one)
__device__ __forceinline__ void rows_put(const FmtArgs& A, char* p, uint64_t r, int64_t s, int64_t e,
                                         uint32_t g0 = ~0u, const char* nm0 = nullptr, uint32_t nl0 = 0) {
  const uint32_t g = (uint32_t)(s >> BG_KEY_SHIFT);
  if (g == g0) {  // the tile's first chromosome, staged in LDS
    for (uint32_t q = 0; q < nl0; ++q) p[q] = nm0[q];
    p += nl0;
  } else {
    const uint32_t nl = A.name_len[g];
    const char* nm = A.names + A.name_off[g];
    for (uint32_t q = 0; q < nl; ++q) p[q] = nm[q];
    p += nl;
  }
  *p++ = '\t';
  const uint64_t cs = (uint64_t)(s & BG_COORD_MASK), ce = (uint64_t)(e & BG_COORD_MASK);
  const int l1 = dec_len_u64(cs), l2 = dec_len_u64(ce);
  put_u64_lds(p, cs, l1);
  p += l1;
  *p++ = '\t';
  put_u64_lds(p, ce, l2);
  p += l2;
  const uint32_t rl = A.rest_len[r];
  const char* rp = A.text + A.rest_off[r];
  for (uint32_t q = 0; q < rl; ++q) p[q] = rp[q];
  p[rl] = '\n';
}
__global__ void __launch_bounds__(BG_NT) k_fmt_rows_write(FmtArgs A, const uint64_t* __restrict__ toff,
                                                          char* __restrict__ out) {
  __shared__ uint32_t sh[BG_NT / 64 + 1];
  __shared__ __attribute__((aligned(16))) char buf[FT_LDS + 16];
  __shared__ char nm0[BG_CHR_MAX + 1];
  static_assert(FT_ROWS == 2, "two rows per thread");
  const uint64_t k0 = (uint64_t)blockIdx.x * FT_TILE + 2ull * threadIdx.x;
  const bool v0 = k0 < A.n, v1 = k0 + 1 < A.n;
  {  // the tile's first row's chromosome name -> LDS (published by the scan's barrier)
    const uint64_t f = (uint64_t)blockIdx.x * FT_TILE;
    const uint32_t g = (uint32_t)(A.s[A.rows[f]] >> BG_KEY_SHIFT);
    if (threadIdx.x < A.name_len[g]) nm0[threadIdx.x] = A.names[A.name_off[g] + threadIdx.x];
  }
  const uint32_t g0 = (uint32_t)(A.s[A.rows[(uint64_t)blockIdx.x * FT_TILE]] >> BG_KEY_SHIFT);
  const uint32_t nl0 = A.name_len[g0];
  uint64_t r0 = 0, r1 = 0;
  if (v1) {
    const ulonglong2 R = reinterpret_cast<const ulonglong2*>(A.rows)[k0 >> 1];
    r0 = R.x;
    r1 = R.y;
  } else if (v0) {
    r0 = A.rows[k0];
  }
  const int64_t s0 = v0 ? A.s[r0] : 0, e0 = v0 ? A.e[r0] : 0;
  const int64_t s1 = v1 ? A.s[r1] : 0, e1 = v1 ? A.e[r1] : 0;
  const uint32_t l0 = v0 ? bg_ivl_len(A.name_len, s0, e0) + A.rest_len[r0] : 0u;
  const uint32_t l1 = v1 ? bg_ivl_len(A.name_len, s1, e1) + A.rest_len[r1] : 0u;
  uint32_t tot;
  const uint32_t my = block_excl_scan(l0 + l1, OpSum(), 0u, sh, &tot);
  const uint64_t dst0 = toff[blockIdx.x];
  if (tot > FT_LDS) {  // oversized tile (long names / rests): render straight to HBM
    if (v0) rows_put(A, out + dst0 + my, r0, s0, e0);
    if (v1) rows_put(A, out + dst0 + my + l0, r1, s1, e1);
    return;
  }
  const uint32_t skew = (uint32_t)(dst0 & 15);
  if (v0) rows_put(A, buf + skew + my, r0, s0, e0, g0, nm0, nl0);
  if (v1) rows_put(A, buf + skew + my + l0, r1, s1, e1, g0, nm0, nl0);
  __syncthreads();
  const uint64_t a0 = dst0, a1 = dst0 + tot;
  const uint64_t al0 = (a0 + 15) & ~15ULL, al1 = a1 & ~15ULL;
  const char* bb = buf + skew;
  if (al0 >= al1) {
    for (uint64_t p = a0 + threadIdx.x; p < a1; p += BG_NT) out[p] = bb[p - a0];
    return;
  }
  for (uint64_t p = a0 + threadIdx.x; p < al0; p += BG_NT) out[p] = bb[p - a0];
  for (uint64_t p = al1 + threadIdx.x; p < a1; p += BG_NT) out[p] = bb[p - a0];
  for (uint64_t p = al0 + 16ull * threadIdx.x; p < al1; p += 16ull * BG_NT)
    *reinterpret_cast<uint4*>(out + p) = *reinterpret_cast<const uint4*>(bb + (p - a0));
}

// a segmented RES_IVL (bg_result::nseg, straight from k_mp_tile): one workgroup per segment,
// its byte offset and printed size already scanned (seg_boff), so there is no count pass.
// The segment's pieces (up to BG_SEG_CAP, ~660 for 100M x 100M --intersect) go in rounds of
// BG_NT, one per thread (coalesced column loads, every lane busy): each round is placed by
// one block scan, rendered into LDS and streamed out as in k_fmt_ivl_write. toff[k] (the
// byte offset of row k * FT_TILE, kept for bg_result_chrom_spans) is written by whichever
// segment holds that row. (Measured on 100M x 100M --intersect, with k_mp_tile's segmented
// write 0.35 ms: 0.49 ms, against 0.117 + 0.381 ms for the count and write passes over a
// contiguous result, plus the 0.2 ms count pass of k_mp_tile this layout removes. Dense
// 512-row tiles located through per-piece byte prefixes: 0.50-0.55 ms with the prefixes
// making k_mp_tile 0.38-0.39 ms; four pieces per thread in one 32 KiB round: 0.69 ms; two
// per thread in rounds of 512: 0.56 ms.)
// (round 5) every round's keys are loaded up front (a segment holds at most BG_SEG_CAP =
// 4 rounds), so only the first round waits on HBM; and the chromosome name of the segment's
// first piece is staged in LDS — pieces of that chromosome (nearly all) copy it from there
// instead of byte loads from the global name table
#define SEG_R (BG_SEG_CAP / BG_NT)
__device__ __forceinline__ void ivl_put_nm(const FmtArgs& A, char* p, int64_t s, int64_t e, uint32_t g0,
                                           const char* nm0, uint32_t nl0) {
  const uint32_t g = (uint32_t)(s >> BG_KEY_SHIFT);
  if (g == g0) {
    for (uint32_t q = 0; q < nl0; ++q) p[q] = nm0[q];
    p += nl0;
  } else {
    const uint32_t nl = A.name_len[g];
    const char* nm = A.names + A.name_off[g];
    for (uint32_t q = 0; q < nl; ++q) p[q] = nm[q];
    p += nl;
  }
  *p++ = '\t';
  const uint64_t cs = (uint64_t)(s & BG_COORD_MASK), ce = (uint64_t)(e & BG_COORD_MASK);
  const int l1 = dec_len_u64(cs), l2 = dec_len_u64(ce);
  put_u64_lds(p, cs, l1);
  p += l1;
  *p++ = '\t';
  put_u64_lds(p, ce, l2);
  p[l2] = '\n';
}
__global__ void __launch_bounds__(BG_NT) k_fmt_ivl_seg(FmtArgs A, const uint64_t* __restrict__ seg_off,
                                                       const uint64_t* __restrict__ seg_boff,
                                                       char* __restrict__ out, uint64_t* __restrict__ toff) {
  static_assert(SEG_R * BG_NT == BG_SEG_CAP, "segment rounds");
  __shared__ uint32_t sh[BG_NT / 64 + 1];
  __shared__ __attribute__((aligned(16))) char buf[FT_LDS + 16];
  __shared__ char nm0[BG_CHR_MAX + 1];
  const uint64_t t = blockIdx.x;
  const uint64_t c0 = seg_off[t];
  const uint32_t n = (uint32_t)(seg_off[t + 1] - c0);
  const int64_t* S = A.s + t * BG_SEG_CAP;
  const int64_t* E = A.e + t * BG_SEG_CAP;
  int64_t ks[SEG_R], ke[SEG_R];
#pragma unroll
  for (int q = 0; q < SEG_R; ++q) {
    const uint32_t j = q * BG_NT + threadIdx.x;
    ks[q] = j < n ? S[j] : 0;
    ke[q] = j < n ? E[j] : 0;
  }
  const uint32_t g0 = n ? (uint32_t)(S[0] >> BG_KEY_SHIFT) : ~0u;
  const uint32_t nl0 = n ? A.name_len[g0] : 0u;
  if (threadIdx.x < nl0) nm0[threadIdx.x] = A.names[A.name_off[g0] + threadIdx.x];
  uint64_t dst0 = seg_boff[t];
#pragma unroll
  for (int q = 0; q < SEG_R; ++q) {
    const uint32_t r0 = q * BG_NT;
    if (r0 >= n) break;  // (block-uniform)
    const uint32_t j = r0 + threadIdx.x;
    const bool v = j < n;
    const int64_t s = ks[q], e = ke[q];
    const uint32_t l = v ? ivl_len(A, s, e) : 0u;
    uint32_t tot;
    const uint32_t my = block_excl_scan(l, OpSum(), 0u, sh, &tot);  // (its barrier also publishes nm0)
    if (v && (c0 + j) % FT_TILE == 0) toff[(c0 + j) / FT_TILE] = dst0 + my;
    if (tot > FT_LDS) {  // oversized round (long names): render straight to HBM
      if (v) ivl_put(A, out + dst0 + my, s, e);
    } else {
      const uint32_t skew = (uint32_t)(dst0 & 15);
      if (v) ivl_put_nm(A, buf + skew + my, s, e, g0, nm0, nl0);
      __syncthreads();
      const uint64_t a0 = dst0, a1 = dst0 + tot;
      const uint64_t al0 = (a0 + 15) & ~15ULL, al1 = a1 & ~15ULL;
      const char* bb = buf + skew;
      if (al0 >= al1) {
        for (uint64_t p = a0 + threadIdx.x; p < a1; p += BG_NT) out[p] = bb[p - a0];
      } else {
        for (uint64_t p = a0 + threadIdx.x; p < al0; p += BG_NT) out[p] = bb[p - a0];
        for (uint64_t p = al1 + threadIdx.x; p < a1; p += BG_NT) out[p] = bb[p - a0];
        for (uint64_t p = al0 + 16ull * threadIdx.x; p < al1; p += 16ull * BG_NT)
          *reinterpret_cast<uint4*>(out + p) = *reinterpret_cast<const uint4*>(bb + (p - a0));
      }
    }
    dst0 += tot;
    __syncthreads();  // buf and sh are reused by the next round
  }
}

// bytes of every FT_TILE-row tile of a RES_IVL result: the same two-rows-per-thread
// layout as k_fmt_ivl_write, one block reduction per tile
__global__ void __launch_bounds__(BG_NT) k_fmt_ivl_count(FmtArgs A, uint64_t* __restrict__ tb) {
  __shared__ uint32_t sh[BG_NT / 64];
  const uint64_t r0 = (uint64_t)blockIdx.x * FT_TILE + 2ull * threadIdx.x;
  uint32_t l = 0;
  if (r0 + 1 < A.n) {
    const longlong2 S = reinterpret_cast<const longlong2*>(A.s)[r0 >> 1];
    const longlong2 E = reinterpret_cast<const longlong2*>(A.e)[r0 >> 1];
    l = ivl_len(A, S.x, E.x) + ivl_len(A, S.y, E.y);
  } else if (r0 < A.n) {
    l = ivl_len(A, A.s[r0], A.e[r0]);
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) l += __shfl_xor(l, d, 64);
  if (bg_lane() == 0) sh[bg_wave()] = l;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int q = 0; q < BG_NT / 64; ++q) t += sh[q];
    tb[blockIdx.x] = t;
  }
}

static void fill_args(bg_result* r, FmtArgs& A) {
  memset(&A, 0, sizeof(A));
  bg_set* s = r->set;
  A.kind = r->kind;
  A.n = r->n;
  A.names = s->d_names;
  A.name_off = s->d_name_off;
  A.name_len = s->d_name_len;
  if (r->kind == RES_IVL) {
    A.s = r->s;
    A.e = r->e;
  } else if (r->kind == RES_MULTI) {
    A.s = r->s;
    A.e = r->e;
    A.rows = r->rows;
    A.rlen = r->rlen;
    A.rest_tab = r->rest_tab ? 1 : 0;
  } else if (r->kind == RES_ROWS) {
    bg_table* T = s->t[r->tab];
    A.s = T->ks;
    A.e = T->ke;
    A.rows = r->rows;
    A.text = T->text;
    A.rest_off = T->rest_off;
    A.rest_len = T->rest_len;
  } else if (r->kind == RES_CLOSEST) {
    bg_table* T = s->t[r->tab];
    bg_table* U = s->t[r->tab2];
    A.s = T->ks;
    A.e = T->ke;
    A.text = T->text;
    A.rest_off = T->rest_off;
    A.rest_len = T->rest_len;
    A.s2 = U->ks;
    A.e2 = U->ke;
    A.text2 = U->text;
    A.rest_off2 = U->rest_off;
    A.rest_len2 = U->rest_len;
    A.left = r->left;
    A.right = r->right;
    A.shortest = r->copts.shortest;
    A.print_dist = r->copts.print_dist;
    A.no_ref = r->copts.no_ref;
    A.dlen = (int)strnlen(r->copts.delim, 15);
    memcpy(A.delim, r->copts.delim, A.dlen);
  } else {
    A.s = s->t[r->tab]->ks;  // reference rows (chromosome spans)
    A.e = s->t[r->tab]->ke;
    A.cnt = r->cnt;
    A.isum = r->isum;
    A.isq = r->isq;
    A.dsum = r->dsum;
    A.dsq = r->dsq;
    A.rrank = r->rrank;
    A.nrid = 0;
    for (int q = 0; q < r->mopts.n_ops; ++q) A.nrid += r->mopts.ops[q] == BG_MAP_ECHO_REF_ROW_ID;
    for (int q = 0; q < 16; ++q) A.op_arg[q] = r->mopts.op_arg[q];
    A.vmin = r->vmin;
    A.vmax = r->vmax;
    A.bases = r->bases;
    A.uniq = r->uniq;
    A.text = s->t[r->tab]->text;  // --echo: the reference rows' remainders
    A.rest_off = s->t[r->tab]->rest_off;
    A.rest_len = s->t[r->tab]->rest_len;
    if (r->wlo) {  // --echo-map*
      const bg_table* M = s->t[r->map_tab];
      A.s2 = M->ks;
      A.e2 = M->ke;
      A.text2 = M->text;
      A.rest_off2 = M->rest_off;
      A.rest_len2 = M->rest_len;
      A.score2 = M->score;
      A.wlo = r->wlo;
      A.whi = r->whi;
      A.zin = r->zin;
      A.zout = r->zout;
      A.maddr = r->maddr;
      A.n2 = M->n;
      A.maord = r->maddr ? reinterpret_cast<const uint32_t*>(r->maddr + M->n) : nullptr;
      A.lrows = r->lrows;
      A.crit = r->mopts.faster ? BG_OVR_FAST : r->mopts.criterion;  // --faster: the deque is the window
      A.ovr = (int64_t)r->mopts.overlap_bp;
      A.range = (int64_t)r->mopts.range_bp;
      A.perc = r->perc;
      A.mapfields = r->mapfields;
      A.mdlen = (int)strnlen(r->mopts.multidelim, 15);
      memcpy(A.mdelim, r->mopts.multidelim, A.mdlen);
    }
    A.nops = r->mopts.n_ops;
    for (int k = 0; k < A.nops; ++k) A.ops[k] = r->mopts.ops[k];
    for (int k = 0; k < 16; ++k) A.tmv[k] = r->tmv[k];
    A.single = r->single ? 1 : 0;
    A.mapfields = r->mapfields;
    if (r->single && !r->wlo) {  // --echo prints rows with the map table's printer
      const bg_table* M = s->t[r->map_tab];
      A.s2 = M->ks;
      A.e2 = M->ke;
      A.text2 = M->text;
      A.rest_off2 = M->rest_off;
      A.rest_len2 = M->rest_len;
      A.score2 = M->score;
    }
    for (int k = 0; k < A.nops; ++k)
      if (A.ops[k] >= BG_MAP_MIN_ELEMENT && A.ops[k] <= BG_MAP_MAX_ELEMENT_RAND && !r->mopts.skip_unmapped)
        A.has_elem = 1;
    A.prec = r->mopts.precision;
    A.sci = r->mopts.scientific;
    A.skip_unmapped = r->mopts.skip_unmapped;
    A.dlen = (int)strnlen(r->mopts.delim, 15);
    memcpy(A.delim, r->mopts.delim, A.dlen);
  }
}

static bool map_simple_op_host(int op) {
  switch (op) {
    case BG_MAP_COUNT: case BG_MAP_INDICATOR: case BG_MAP_BASES: case BG_MAP_BASES_UNIQ: case BG_MAP_BASES_UNIQ_F:
    case BG_MAP_MEAN: case BG_MAP_SUM: case BG_MAP_VARIANCE: case BG_MAP_STDEV: case BG_MAP_CV: case BG_MAP_MIN:
    case BG_MAP_MAX: case BG_MAP_ECHO_SIZE: case BG_MAP_ECHO_NAME:
      return true;
  }
  return false;
}

extern "C" int bg_result_format(bg_ctx* c, bg_result* r, uint64_t* nbytes) {
  if (!c || !r) return BG_E_ARG;
  if (r->kind == RES_ROWS && !r->set->t[r->tab]->rest_off)
    return bg_fail(c, BG_E_ARG, "row result needs its table loaded as BG_BED3_REST");
  if (r->formatted) {
    if (nbytes) *nbytes = r->nbytes;
    return r->stopped ? bg_fail(c, BG_E_VISITOR, "Unable to process a 'NAN' with PrintAllScorePrecision.") : 0;
  }
  FmtArgs A;
  fill_args(r, A);
  A.stop_row = ~0ULL;
  if (r->kind == RES_IVL && r->nseg) {  // segmented: sizes known, one pass
    // every piece prints at most name + 3 + two 13-digit coordinates (< 2^40): with that
    // bound allocated up front, the counts come back with the kernel's completion (one host
    // round trip per format instead of one before and one after)
    const uint64_t line_max = (uint64_t)r->set->max_name_len + 3 + 2 * 13;
    const uint64_t bound = r->seg_nz * line_max;
    const bool ahead = bound <= (8ull << 30);
    uint64_t tots[2] = {0, 0};  // pieces, bytes
    int rc = 0;
    if (!ahead) {
      BG_HIP(c, hipMemcpyAsync(&tots[0], r->seg_off + r->nseg, 8, hipMemcpyDeviceToHost, c->stream));
      BG_HIP(c, hipMemcpyAsync(&tots[1], r->seg_boff + r->nseg, 8, hipMemcpyDeviceToHost, c->stream));
      BG_HIP(c, hipStreamSynchronize(c->stream));
      r->n = tots[0];
      r->n_pending = false;
    }
    const unsigned nt = bg_blocks(ahead ? r->seg_nz : r->n, FT_TILE);
    uint64_t* tb = (uint64_t*)bg_alloc(c, 8ull * (nt ? nt : 1));
    r->text = (char*)bg_alloc(c, (ahead ? bound : tots[1]) + 16);
    if (!tb || !r->text) return BG_E_NOMEM;
    BG_LAUNCH(c, "k_fmt_write", k_fmt_ivl_seg, dim3((unsigned)r->nseg), dim3(BG_NT), A, r->seg_off, r->seg_boff,
              r->text, tb);
    BG_HIP(c, hipGetLastError());
    if (ahead) {
      BG_HIP(c, hipMemcpyAsync(&tots[0], r->seg_off + r->nseg, 8, hipMemcpyDeviceToHost, c->stream));
      BG_HIP(c, hipMemcpyAsync(&tots[1], r->seg_boff + r->nseg, 8, hipMemcpyDeviceToHost, c->stream));
      BG_HIP(c, hipStreamSynchronize(c->stream));
      r->n = tots[0];
      r->n_pending = false;
    }
    (void)rc;
    const uint64_t total = tots[1];
    r->toff = tb;
    r->nbytes = total;
    r->formatted = true;
    if (nbytes) *nbytes = total;
    bg_mark(c, "format");
    return 0;
  }
  const unsigned nb = bg_blocks(r->n, FT_TILE);
  const unsigned nbc = bg_blocks(nb, FC_TILES);
  uint64_t* tb = (uint64_t*)bg_alloc(c, 8ull * (nb ? nb : 1));
  uint64_t* d_tot = (uint64_t*)bg_alloc(c, 8);
  if (!tb || !d_tot) return BG_E_NOMEM;
  BG_HIP(c, hipMemsetAsync(&c->dstat->first_bad, 0xff, 8, c->stream));
  BG_HIP(c, hipMemsetAsync(&c->dstat->stop_row, 0xff, 8, c->stream));
  static_assert(FT_TILE == BG_FMT_TILE, "format tile");
  if ((A.kind == RES_MAP || A.kind == RES_CLOSEST) && r->n) {
    A.rowlen = (uint32_t*)bg_alloc(c, 4 * r->n);  // (null: the write pass measures again)
  }
  bool simple = A.kind == RES_MAP && !A.sci && !A.has_elem;
  for (int k = 0; simple && k < A.nops; ++k) simple = map_simple_op_host(A.ops[k]);
count_again:
  if (nb && A.kind == RES_ROWS && r->tbytes) {  // summed by bg_element_of's compaction
    BG_HIP(c, hipMemcpyAsync(tb, r->tbytes, 8ull * nb, hipMemcpyDeviceToDevice, c->stream));
  } else if (nb) {
    switch (A.kind) {
      case RES_IVL: BG_LAUNCH(c, "k_fmt_count", k_fmt_ivl_count, dim3(nb), dim3(BG_NT), A, tb); break;
      case RES_ROWS: BG_LAUNCH(c, "k_fmt_count", k_fmt_count<RES_ROWS>, dim3(nbc), dim3(BG_NT), A, tb, (uint64_t)nb, c->dstat); break;
      case RES_MAP:
        if (simple) BG_LAUNCH(c, "k_fmt_count", k_fmt_count<RES_MAPS>, dim3(nbc), dim3(BG_NT), A, tb, (uint64_t)nb, c->dstat);
        else BG_LAUNCH(c, "k_fmt_count", k_fmt_count<RES_MAP>, dim3(nbc), dim3(BG_NT), A, tb, (uint64_t)nb, c->dstat);
        break;
      case RES_MULTI: BG_LAUNCH(c, "k_fmt_count", k_fmt_count<RES_MULTI>, dim3(nbc), dim3(BG_NT), A, tb, (uint64_t)nb, c->dstat); break;
      default: BG_LAUNCH(c, "k_fmt_count", k_fmt_count<RES_CLOSEST>, dim3(nbc), dim3(BG_NT), A, tb, (uint64_t)nb, c->dstat);
    }
    BG_HIP(c, hipGetLastError());
  }
  int rc = bg_scan_sum_u64(c, tb, tb, nb, d_tot);
  if (rc) return rc;
  uint64_t total = 0;
  BG_HIP(c, hipMemcpyAsync(c->hstat, c->dstat, sizeof(bg_dstatus), hipMemcpyDeviceToHost, c->stream));
  if ((rc = bg_fetch_u64(c, d_tot, &total))) return rc;
  if (c->hstat->first_bad != ~0ULL && simple) {  // a value the small kernel refuses: the general one
    simple = false;
    BG_HIP(c, hipMemsetAsync(&c->dstat->first_bad, 0xff, 8, c->stream));
    BG_HIP(c, hipMemsetAsync(&c->dstat->stop_row, 0xff, 8, c->stream));
    goto count_again;
  }
  if (c->hstat->first_bad != ~0ULL)
    return bg_fail(c, BG_E_UNSUPPORTED, "a value is outside the GPU formatter's range");
  r->text = (char*)bg_alloc(c, total + 16);
  if (!r->text) return BG_E_NOMEM;
  A.st = c->dstat;
  A.total = total;
  if (A.rowlen) BG_HIP(c, hipMemsetAsync(&c->dstat->flags, 0, 8, c->stream));
  uint64_t* d_stop = nullptr;
  if (c->hstat->stop_row != ~0ULL) {  // the text ends inside this row (k_fmt_write finds where)
    A.stop_row = c->hstat->stop_row;
    d_stop = (uint64_t*)bg_alloc(c, 8);
    if (!d_stop) return BG_E_NOMEM;
    A.stop_out = d_stop;
  }
  static const bool rows_fast = [] {  // BEDGPU_FMT_ROWS=0: k_fmt_write<RES_ROWS> (A/B)
    const char* e = getenv("BEDGPU_FMT_ROWS");
    return !(e && atoi(e) == 0);
  }();
  if (nb) {
    switch (A.kind) {
      case RES_IVL: BG_LAUNCH(c, "k_fmt_write", k_fmt_ivl_write, dim3(nb), dim3(BG_NT), A, tb, r->text); break;
      case RES_ROWS:
        if (rows_fast) BG_LAUNCH(c, "k_fmt_write", k_fmt_rows_write, dim3(nb), dim3(BG_NT), A, tb, r->text);
        else BG_LAUNCH(c, "k_fmt_write", k_fmt_write<RES_ROWS>, dim3(nb), dim3(BG_NT), A, tb, r->text);
        break;
      case RES_MAP:
        if (simple) BG_LAUNCH(c, "k_fmt_write", k_fmt_write<RES_MAPS>, dim3(nb), dim3(BG_NT), A, tb, r->text);
        else BG_LAUNCH(c, "k_fmt_write", k_fmt_write<RES_MAP>, dim3(nb), dim3(BG_NT), A, tb, r->text);
        break;
      case RES_MULTI: BG_LAUNCH(c, "k_fmt_write", k_fmt_write<RES_MULTI>, dim3(nb), dim3(BG_NT), A, tb, r->text); break;
      default: BG_LAUNCH(c, "k_fmt_write", k_fmt_write<RES_CLOSEST>, dim3(nb), dim3(BG_NT), A, tb, r->text);
    }
    BG_HIP(c, hipGetLastError());
    if (A.rowlen) {  // rows placed by the count pass's lengths must render to exactly those
      uint64_t fl = 0;
      if ((rc = bg_fetch_u64(c, (const uint64_t*)&c->dstat->flags, &fl))) return rc;
      if (fl & BG_FMT_MISMATCH)
        return bg_fail(c, BG_E_INTERNAL, "formatter: a row rendered to another length than counted (its inputs changed between the passes)");
    }
  }
  r->toff = tb;
  bg_release(c, d_tot);
  bg_release(c, A.rowlen);  // (stream-ordered: reused only by later work on c's stream)
  if (d_stop) {
    rc = bg_fetch_u64(c, d_stop, &total);
    bg_release(c, d_stop);
    if (rc) return rc;
    r->stopped = true;
  }
  r->nbytes = total;
  r->formatted = true;
  if (nbytes) *nbytes = total;
  bg_mark(c, "format");
  return r->stopped ? bg_fail(c, BG_E_VISITOR, "Unable to process a 'NAN' with PrintAllScorePrecision.") : 0;
}

// Byte offset of the first output line of every chromosome g of the set's dictionary;
// out[nchroms] = total bytes, so chromosome g's lines are text[out[g], out[g+1]).
// Used to reassemble per-GPU shards in strcmp chromosome order (multi-GPU path).
template <int KIND>
__global__ void k_chrom_spans(FmtArgs A, const uint64_t* __restrict__ toff, uint32_t nchroms,
                              uint64_t nbytes, uint64_t* __restrict__ out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g > nchroms) return;
  if (g == nchroms) { out[g] = nbytes; return; }
  const int64_t key = (int64_t)g << BG_KEY_SHIFT;
  uint64_t lo = 0, hi = A.n;  // first output row whose chromosome is >= g
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    const uint64_t r = (KIND == RES_ROWS) ? A.rows[mid] : mid;
    if (A.s[r] < key) lo = mid + 1;
    else hi = mid;
  }
  if (lo >= A.n) { out[g] = nbytes; return; }
  const uint64_t t = lo / FT_TILE;
  CountOut co;
  for (uint64_t j = t * FT_TILE; j < lo; ++j) render<KIND>(A, j, co);
  out[g] = toff[t] + co.n;
}

extern "C" int bg_result_chrom_spans(bg_ctx* c, bg_result* r, uint64_t* offsets, uint32_t cap) {
  if (!c || !r || !offsets) return BG_E_ARG;
  const uint32_t nc = (uint32_t)r->set->names.size();
  if (cap < nc + 1) return bg_fail(c, BG_E_ARG, "offsets buffer needs nchroms+1 entries");
  int rc = bg_result_format(c, r, nullptr);
  if (rc) return rc;
  if ((rc = bg_result_compact(c, r))) return rc;  // the row search reads contiguous pieces
  FmtArgs A;
  fill_args(r, A);
  uint64_t* d = (uint64_t*)bg_alloc(c, 8ull * (nc + 1));
  if (!d) return BG_E_NOMEM;
#define BG_SPANS(K) BG_LAUNCH(c, "k_chrom_spans", k_chrom_spans<K>, dim3(bg_blocks(nc + 1, 64)), dim3(64), A, r->toff, nc, r->nbytes, d)
  switch (A.kind) {
    case RES_IVL: BG_SPANS(RES_IVL); break;
    case RES_ROWS: BG_SPANS(RES_ROWS); break;
    case RES_MAP: BG_SPANS(RES_MAP); break;
    case RES_MULTI: BG_SPANS(RES_MULTI); break;
    default: BG_SPANS(RES_CLOSEST);
  }
#undef BG_SPANS
  BG_HIP(c, hipGetLastError());
  BG_HIP(c, hipMemcpyAsync(offsets, d, 8ull * (nc + 1), hipMemcpyDeviceToHost, c->stream));
  BG_HIP(c, hipStreamSynchronize(c->stream));
  bg_release(c, d);
  return 0;
}

extern "C" int bg_set_chroms(const bg_set* s, uint32_t* n) {
  if (!s || !n) return BG_E_ARG;
  *n = (uint32_t)s->names.size();
  return 0;
}

extern "C" const char* bg_set_chrom_name(const bg_set* s, uint32_t g) {
  if (!s || g >= s->names.size()) return nullptr;
  return s->names[g].c_str();
}

extern "C" int bg_result_copy_text_device(bg_ctx* c, bg_result* r, void* dst, uint64_t cap) {
  uint64_t n = 0;
  int rc = bg_result_format(c, r, &n);
  if (rc && rc != BG_E_VISITOR) return rc;
  if (cap < n) return bg_fail(c, BG_E_ARG, "device buffer too small");
  if (n) BG_HIP(c, hipMemcpyAsync(dst, r->text, n, hipMemcpyDeviceToDevice, c->stream));
  BG_HIP(c, hipStreamSynchronize(c->stream));
  return rc;
}
