// bg_strtod.h — correctly rounded decimal -> double for the score column, any exponent,
// shared by the GPU loader (bg_load.hip's parse_score) and its CPU test
// (tests/cpu/strtod_main.cpp, against glibc strtod).
//
// B5Rest reads the score with fscanf "%lf" (Bed.hpp:829-860), i.e. glibc strtod: the exact
// decimal value rounded half-to-even to a double, subnormals included, overflow to infinity.
// The loader's fast paths (Clinger, 128-bit) cover <= 19 significant digits with exponents
// in -26..37; this covers the rest — up to BG_SD_DIGITS significant digits (more: the caller
// refuses the row) at any exponent — with big integers in 32-bit limbs: value = D * 10^e,
// e >= 0: D * 10^e exactly, e < 0: q = floor(D * 2^s / 5^-e) by shift-subtract, the
// remainder as the sticky bit; then one rounding to 53 bits (fewer below 2^-1022).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define BG_SD __host__ __device__ __noinline__
#define BG_SD_INL __host__ __device__ __forceinline__
#else
#define BG_SD static
#define BG_SD_INL static inline
#endif

#define BG_SD_DIGITS 200  // significant digits held exactly
#define BG_SD_LIMBS 44    // 1.4K bits: D < 10^200 (665 bits), 5^524, D << s

struct BigU {
  uint32_t w[BG_SD_LIMBS];
  int n;  // limbs in use (w[n-1] != 0 unless n == 0)
};

BG_SD_INL void big_set(BigU& a, uint64_t v) {
  a.w[0] = (uint32_t)v;
  a.w[1] = (uint32_t)(v >> 32);
  a.n = a.w[1] ? 2 : (a.w[0] ? 1 : 0);
}
BG_SD_INL bool big_muladd(BigU& a, uint32_t m, uint32_t add) {  // a = a * m + add
  uint64_t c = add;
  for (int i = 0; i < a.n; ++i) {
    const uint64_t t = (uint64_t)a.w[i] * m + c;
    a.w[i] = (uint32_t)t;
    c = t >> 32;
  }
  if (c) {
    if (a.n >= BG_SD_LIMBS) return false;
    a.w[a.n++] = (uint32_t)c;
  }
  return true;
}
BG_SD_INL int big_bits(const BigU& a) {
  if (a.n == 0) return 0;
  uint32_t t = a.w[a.n - 1];
  int b = 0;
  while (t) {
    ++b;
    t >>= 1;
  }
  return 32 * (a.n - 1) + b;
}
BG_SD_INL bool big_shl(BigU& a, int s) {  // a <<= s
  if (a.n == 0 || s == 0) return true;
  const int w = s >> 5, b = s & 31;
  const int nn = a.n + w + 1;
  if (nn > BG_SD_LIMBS) return false;
  for (int i = nn - 1; i >= 0; --i) {
    const int src = i - w;
    uint32_t hi = (src >= 0 && src < a.n) ? a.w[src] : 0;
    uint32_t lo = (src - 1 >= 0 && src - 1 < a.n) ? a.w[src - 1] : 0;
    a.w[i] = b ? ((hi << b) | (lo >> (32 - b))) : hi;
  }
  a.n = nn;
  while (a.n > 0 && a.w[a.n - 1] == 0) --a.n;
  return true;
}
// bit i of (b << s)
BG_SD_INL uint32_t big_limb_shifted(const BigU& b, int s, int i) {  // limb i of b << s
  const int w = s >> 5, bb = s & 31;
  const int src = i - w;
  const uint32_t hi = (src >= 0 && src < b.n) ? b.w[src] : 0;
  const uint32_t lo = (src - 1 >= 0 && src - 1 < b.n) ? b.w[src - 1] : 0;
  return bb ? ((hi << bb) | (lo >> (32 - bb))) : hi;
}
// a >= (b << s)
BG_SD_INL bool big_ge_shifted(const BigU& a, const BigU& b, int s) {
  const int nb = b.n + (s >> 5) + 1;
  const int n = a.n > nb ? a.n : nb;
  for (int i = n - 1; i >= 0; --i) {
    const uint32_t x = i < a.n ? a.w[i] : 0, y = big_limb_shifted(b, s, i);
    if (x != y) return x > y;
  }
  return true;
}
// a -= (b << s), given a >= b << s
BG_SD_INL void big_sub_shifted(BigU& a, const BigU& b, int s) {
  int64_t br = 0;
  for (int i = 0; i < a.n; ++i) {
    const int64_t t = (int64_t)a.w[i] - (int64_t)big_limb_shifted(b, s, i) - br;
    a.w[i] = (uint32_t)t;
    br = t < 0 ? 1 : 0;
  }
  while (a.n > 0 && a.w[a.n - 1] == 0) --a.n;
}

// q * 2^e2 (+ sticky below q's last bit) rounded half-to-even to a double
BG_SD_INL double sd_round(uint64_t q, int e2, bool sticky) {
  int L = 0;
  for (uint64_t t = q; t; t >>= 1) ++L;
  const int lb = e2 + L - 1;                         // exponent of the leading bit
  int keep = lb >= -1022 ? 53 : 53 - (-1022 - lb);   // mantissa bits kept
  int d = L - keep;                                  // low bits dropped
  uint64_t mant;
  if (d <= 0) {
    mant = q << (-d);
    e2 += d;
  } else if (d > 64) {
    mant = 0;
    e2 += d;
  } else {
    const uint64_t rest = d == 64 ? q : (q & ((1ULL << d) - 1));
    const uint64_t half = 1ULL << (d - 1);
    mant = d == 64 ? 0 : (q >> d);
    const bool up = rest > half || (rest == half && (sticky || (mant & 1)));
    if (up) ++mant;
    e2 += d;
  }
  // (mant may now be 2^53: ldexp renormalises exactly)
  double r = (double)mant;
  // ldexp in two steps keeps subnormal results exact (no double rounding: mant fits)
  if (e2 < -1000) {
    r *= 0x1p-600;
    e2 += 600;
  }
  if (e2 > 1000) {
    r *= 0x1p+600;
    e2 -= 600;
  }
  int e = e2;
  while (e > 0) {
    const int st = e > 60 ? 60 : e;
    r *= (double)(1ULL << st);
    e -= st;
  }
  while (e < 0) {
    const int st = -e > 60 ? 60 : -e;
    r /= (double)(1ULL << st);
    e += st;
  }
  return r;
}

// |value| of the significant digits dg[0..nd) (no leading zeros, nd <= BG_SD_DIGITS) times
// 10^e, plus `more`: nonzero digits were dropped after them. false: out of this path's range
// (never for nd <= BG_SD_DIGITS)
BG_SD bool strtod_big(const uint8_t* dg, int nd, int e, bool more, double& out) {
  if (nd == 0) {
    out = 0;
    return true;
  }
  const int e10 = nd + e;  // value in [10^(e10-1), 10^e10)
  if (e10 > 310) {
    out = __builtin_inf();
    return true;
  }
  if (e10 < -324) {  // < 10^-325: below half the smallest subnormal
    out = 0;
    return true;
  }
  BigU D;
  D.n = 0;
  for (int i = 0; i < nd; ++i)
    if (!big_muladd(D, 10, dg[i])) return false;
  if (e >= 0) {  // an integer (more: a fraction below its last digit)
    for (int i = 0; i < e; ++i)
      if (!big_muladd(D, 10, 0)) return false;
    const int L = big_bits(D);
    const int s = L > 64 ? L - 64 : 0;  // top 64 bits, the rest sticky
    uint64_t q = 0;
    bool st = more;
    for (int i = 0; i < D.n; ++i) {
      const int lo = 32 * i;
      for (int b = 0; b < 32; ++b) {
        const int bit = lo + b;
        if (!((D.w[i] >> b) & 1)) continue;
        if (bit < s) st = true;
        else q |= 1ULL << (bit - s);
      }
    }
    out = sd_round(q, s, st);
    return true;
  }
  // e < 0: value = D / (5^k 2^k), k = -e
  const int k = -e;
  BigU S;
  big_set(S, 1);
  for (int i = 0; i < k; ++i)
    if (!big_muladd(S, 5, 0)) return false;
  // q = floor(D * 2^s / S) with 62..63 bits: s = 62 + bits(S) - bits(D)
  int s = 62 + big_bits(S) - big_bits(D);
  BigU X = D;
  int sS = 0;  // S shifted instead when s < 0
  if (s >= 0) {
    if (!big_shl(X, s)) return false;
  } else {
    sS = -s;
  }
  uint64_t q = 0;
  for (int b = 63; b >= 0; --b) {
    if (big_ge_shifted(X, S, sS + b)) {
      big_sub_shifted(X, S, sS + b);
      q |= 1ULL << b;
    }
  }
  const bool st = more || X.n != 0;
  out = sd_round(q, -s - k, st);
  return true;
}
