// bg_decfmt.h — exact "%.{p}lf" / "%.{p}e" of any finite double at any precision, shared by
// the GPU formatter (bg_format.hip) and its CPU test (tests/cpu/test_decfmt.cpp, which
// compares it with glibc printf).
//
// bedmap prints scores with Formats::Format(double, prec, sci) (Formats.hpp:42-50): glibc
// printf of the exact binary value, rounded half-to-even at the last printed digit. The
// formatter's fast paths cover |v| * 10^p < 2^64 (and 1e-16 <= |v| < 2^128 under --sci) for
// p <= 17; this covers every other finite value and precision with O(1) state per thread:
// |v| = I + F, the integer part I held as base-10^9 groups and the fraction F = f / 2^k
// producing its digits nine at a time (f *= 10^9; the group is the bits of f at and above k).
// Two walks over the same digit stream: the first finds the rounding (the digit after the
// cut, and whether anything nonzero follows it) and the last printed digit that is not a 9;
// the second prints, with the carry applied at that digit.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define BG_DF __host__ __device__ __noinline__
#define BG_DF_INL __host__ __device__ __forceinline__
#else
#define BG_DF static
#define BG_DF_INL inline
#endif

struct DecStream {
  uint32_t ig[36];  // I in base 10^9, least significant group first (< 2^1024: 35 groups)
  int nig;          // groups of I (0: I == 0)
  int lead;         // digits of I's top group
  uint32_t f[36];   // F = f / 2^k (f < 2^k), 32-bit limbs, least significant first
  int nf, k;
  bool fz;          // f == 0: every later fraction digit is 0
  // the walk: I's digits (most significant first), then F's
  int gi;           // current group of I (counting down); -1 once in F
  uint32_t grp;     // current 9-digit group
  int gd;           // digits of grp still to give (from the top)

  BG_DF_INL void init(double v) {
    uint64_t bits;
    memcpy(&bits, &v, 8);
    const int bexp = (int)((bits >> 52) & 0x7ff);
    uint64_t m = bits & ((1ULL << 52) - 1);
    int ex;
    if (bexp == 0) ex = -1074;
    else {
      m |= 1ULL << 52;
      ex = bexp - 1075;
    }
    uint32_t L[36];  // I in 32-bit limbs
    int nl;
    nf = 0;
    k = 0;
    if (ex >= 0) {  // an integer: I = m << ex (< 2^1024), F = 0
      const int w = ex >> 5, b = ex & 31;
      for (int i = 0; i < w; ++i) L[i] = 0;
      const uint64_t lo = m << b, hi = b ? (m >> (64 - b)) : 0;
      L[w] = (uint32_t)lo;
      L[w + 1] = (uint32_t)(lo >> 32);
      L[w + 2] = (uint32_t)hi;
      nl = w + 3;
    } else {
      k = -ex;  // 1 .. 1074
      uint64_t ip = 0, fr = m;
      if (k < 64) {
        ip = m >> k;
        fr = m & ((1ULL << k) - 1);
      }
      L[0] = (uint32_t)ip;
      L[1] = (uint32_t)(ip >> 32);
      nl = 2;
      nf = (k >> 5) + 2;  // f < 2^(k + 30) after a multiply by 10^9
      for (int i = 0; i < nf; ++i) f[i] = 0;
      f[0] = (uint32_t)fr;
      f[1] = (uint32_t)(fr >> 32);
    }
    fz = true;
    for (int i = 0; i < nf; ++i)
      if (f[i]) fz = false;
    while (nl > 0 && L[nl - 1] == 0) --nl;
    nig = 0;
    while (nl > 0) {  // base 2^32 -> base 10^9 by long division
      uint64_t rem = 0;
      for (int i = nl - 1; i >= 0; --i) {
        const uint64_t cur = (rem << 32) | L[i];
        L[i] = (uint32_t)(cur / 1000000000u);
        rem = cur % 1000000000u;
      }
      ig[nig++] = (uint32_t)rem;
      while (nl > 0 && L[nl - 1] == 0) --nl;
    }
    lead = 0;
    if (nig)
      for (uint32_t t = ig[nig - 1]; t; t /= 10) ++lead;
  }
  // back to the stream's first digit (F restarts from the state init() left: callers copy)
  BG_DF_INL int int_digits() const { return nig ? 9 * (nig - 1) + lead : 0; }
  BG_DF_INL void start() {
    gi = nig - 1;
    if (gi >= 0) {
      grp = ig[gi];
      gd = lead;
    } else {
      grp = 0;
      gd = 0;
    }
  }
  // F's next 9 digits
  BG_DF_INL uint32_t frac9() {
    if (fz) return 0;
    uint64_t carry = 0;
    for (int i = 0; i < nf; ++i) {
      const uint64_t t = (uint64_t)f[i] * 1000000000u + carry;
      f[i] = (uint32_t)t;
      carry = t >> 32;
    }
    const int w = k >> 5, b = k & 31;
    const uint64_t two = ((uint64_t)(w + 1 < nf ? f[w + 1] : 0) << 32) | f[w];
    const uint32_t g = (uint32_t)(two >> b);  // < 10^9
    f[w] &= b ? ((1u << b) - 1) : 0u;
    for (int i = w + 1; i < nf; ++i) f[i] = 0;
    fz = true;
    for (int i = 0; i <= w && i < nf; ++i)
      if (f[i]) fz = false;
    return g;
  }
  static BG_DF_INL uint32_t pow10u(int e) {
    uint32_t p = 1;
    for (int i = 0; i < e; ++i) p *= 10;
    return p;
  }
  // the next digit
  BG_DF_INL int next() {
    if (gd == 0) {
      if (gi > 0) {
        grp = ig[--gi];
      } else {
        gi = -1;
        grp = frac9();
      }
      gd = 9;
    }
    --gd;
    return (int)((grp / pow10u(gd)) % 10u);
  }
  // every digit after the current one is 0
  BG_DF_INL bool rest_zero() const {
    if (grp % pow10u(gd)) return false;
    for (int i = gi - 1; i >= 0; --i)
      if (ig[i]) return false;
    return fz;
  }
  // in F with nothing but zeros to come
  BG_DF_INL bool exhausted() const { return gi < 0 && fz && grp % pow10u(gd) == 0; }
};

// prints finite v with prec digits after the point: "%.{prec}f" or (sci) "%.{prec}e"
template <typename Out>
BG_DF void put_real_exact(Out& o, double v, int prec, bool sci) {
  uint64_t bits;
  memcpy(&bits, &v, 8);
  const bool neg = (bits >> 63) != 0;
  // one stream at a time, re-initialised for each walk (private memory: ~300 bytes a thread)
  DecStream D;
  D.init(v);
  const bool zero = D.nig == 0 && D.fz;
  if (neg) o.put('-');
  if (sci && zero) {
    o.put('0');
    if (prec > 0) o.put('.');
    for (int i = 0; i < prec; ++i) o.put('0');
    o.put('e');
    o.put('+');
    o.put('0');
    o.put('0');
    return;
  }
  int E = 0;
  int64_t skip = 0;  // stream digits before the first kept one (sci of |v| < 1)
  int virt = 0;      // fixed, I == 0: a kept "0" the stream does not hold
  int64_t nkeep, nint;
  if (sci) {
    if (D.nig) {
      E = D.int_digits() - 1;
    } else {
      D.start();
      while (D.next() == 0) ++skip;
      E = -(int)(skip + 1);
    }
    nkeep = (int64_t)prec + 1;
    nint = 1;
  } else {
    virt = D.nig ? 0 : 1;
    nint = virt + D.int_digits();
    nkeep = nint + prec;
  }
  // walk 1: the rounding, and the last kept digit that is not a 9
  int64_t last_non9 = -1;
  bool up = false;
  {
    D.init(v);
    D.start();
    for (int64_t i = 0; i < skip; ++i) D.next();
    int lastd = 0;
    bool done = false;
    for (int64_t i = 0; i < nkeep; ++i) {
      if (i >= virt && D.exhausted()) {  // zeros to the end: no rounding
        last_non9 = nkeep - 1;
        done = true;
        break;
      }
      const int d = i < virt ? 0 : D.next();
      lastd = d;
      if (d != 9) last_non9 = i;
    }
    if (!done && !D.exhausted()) {
      const int r = D.next();
      up = r > 5 || (r == 5 && (!D.rest_zero() || (lastd & 1)));
    }
  }
  // walk 2: print
  D.init(v);
  D.start();
  for (int64_t i = 0; i < skip; ++i) D.next();
  const bool all9 = up && last_non9 < 0;  // 9.99 -> 10.00 (fixed) / 1.00e(E+1) (sci)
  if (sci && all9) {
    o.put('1');
    if (prec > 0) o.put('.');
    for (int i = 0; i < prec; ++i) o.put('0');
    ++E;
  } else {
    if (all9) o.put('1');  // fixed: one more integer digit
    for (int64_t i = 0; i < nkeep; ++i) {
      if (i == nint) o.put('.');
      int d = 0;
      if (i >= virt && !D.exhausted()) d = D.next();
      if (up) {
        if (all9 || i > last_non9) d = 0;
        else if (i == last_non9) d += 1;
      }
      o.put((char)('0' + d));
    }
  }
  if (sci) {
    o.put('e');
    o.put(E < 0 ? '-' : '+');
    const int ae = E < 0 ? -E : E;
    if (ae >= 100) o.put((char)('0' + ae / 100));
    o.put((char)('0' + (ae / 10) % 10));
    o.put((char)('0' + ae % 10));
  }
}
