// bg_parse.h — branch-free BED field extraction shared by the GPU loader and its CPU
// unit test (tests/cpu/test_parse_helpers.cpp compiles this header with g++).
//
// A line's first 32 bytes are held as 8 little-endian dwords W[0..7]. Per dword, SWAR
// byte classification yields 4-bit groups for "whitespace" ({' ', \t..\r}) and "digit";
// the fields (chrom token, start digits, end digits) then fall out of count-trailing-
// zeros on the two 32-bit masks, and each number is converted 8 digits at a time with
// the 3-multiply SWAR decimal conversion. Anything the masks cannot decide (fields past
// 32 bytes, '+' signs, > 16 digits, malformed text) returns 0 and the caller takes the
// byte-by-byte path, which applies the full grammar and reports errors.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define BG_HD __host__ __device__ __forceinline__
#else
#define BG_HD static inline
#endif

BG_HD uint32_t bgp_ctz(uint32_t x) { return (uint32_t)__builtin_ctz(x); }

// bit 7 of each byte of m80 -> 4-bit group (byte 0 -> bit 0)
BG_HD uint32_t bgp_group4(uint32_t m80) {
  return ((((m80 >> 7) & 0x01010101u) * 0x00204081u) >> 21) & 0xFu;
}

// per-byte classes of one dword: ws4 = {' ', 0x09..0x0D}, dg4 = {'0'..'9'} (bit i = byte i).
// Both 4-bit groups come out of ONE multiply: byte i carries its ws flag in bit 0 and its
// digit flag in bit 4, and x * 0x00204081 gathers bit 0 of byte i at bit 21+i and bit 4 of
// byte i at bit 25+i (the 32 partial products land on distinct bits: no carries).
BG_HD void bgp_classify(uint32_t x, uint32_t& ws4, uint32_t& dg4) {
  const uint32_t hi = x & 0x80808080u;  // bytes >= 0x80 are neither
  const uint32_t lo7 = x & 0x7F7F7F7Fu;
  const uint32_t nz20 = ((lo7 ^ 0x20202020u) + 0x7F7F7F7Fu);  // bit 7: byte != ' '
  const uint32_t ge9 = lo7 + 0x77777777u;
  const uint32_t ge14 = lo7 + 0x72727272u;
  const uint32_t ws = (~nz20 | (ge9 & ~ge14)) & ~hi & 0x80808080u;
  const uint32_t ge48 = lo7 + 0x50505050u;
  const uint32_t ge58 = lo7 + 0x46464646u;
  const uint32_t dg = ge48 & ~ge58 & ~hi & 0x80808080u;
  const uint32_t p = ((ws >> 7) | (dg >> 3)) * 0x00204081u;
  ws4 = (p >> 21) & 0xFu;
  dg4 = (p >> 25) & 0xFu;
}

// bytes [o, o+4) of the 8-byte little-endian sequence (lo, hi), o in 0..3
BG_HD uint32_t bgp_align(uint32_t lo, uint32_t hi, uint32_t o) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbyte(hi, lo, o);
#else
  return o ? (lo >> (8 * o)) | (hi << (32 - 8 * o)) : lo;
#endif
}

// value of the first L (1..8) ASCII digits of v (first digit in the low byte)
BG_HD uint64_t bgp_swar8(uint64_t v, int L) {
  v -= 0x3030303030303030ull;
  v <<= 8 * (8 - L);
  v = (v * 10) + (v >> 8);
  v = (((v & 0x000000FF000000FFull) * (100 + (1000000ull << 32))) +
       (((v >> 16) & 0x000000FF000000FFull) * (1 + (10000ull << 32)))) >> 32;
  return v;
}

// value of L (1..16) ASCII digits held in lo8 (digits 0..7) and hi8 (8..15)
BG_HD uint64_t bgp_digits(uint64_t lo8, uint64_t hi8, int L) {
  if (L <= 8) return bgp_swar8(lo8, L);
  const int h = L - 8;  // leading digits, then the last 8
  const uint64_t head = bgp_swar8(lo8, h);
  const uint64_t tail = (h == 8) ? hi8 : ((lo8 >> (8 * h)) | (hi8 << (64 - 8 * h)));
  return head * 100000000ull + bgp_swar8(tail, 8);
}

// sum of byte products a.b[i] * w.b[i] + c (v_dot4_u32_u8 on the GPU), mod 2^32
BG_HD uint32_t bgp_udot4(uint32_t a, uint32_t w, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_udot4(a, w, c, false);
#else
  for (int i = 0; i < 4; ++i) c += ((a >> (8 * i)) & 0xFFu) * ((w >> (8 * i)) & 0xFFu);
  return c;
#endif
}

// four ASCII digits (first digit in the low byte) -> value, via two byte dot products
BG_HD uint32_t bgp_dig4(uint32_t d) {
  const uint32_t hi2 = bgp_udot4(d, 0x0000010Au, 0u);           // 10*x0 + x1 (+ 528)
  const uint32_t lo2 = bgp_udot4(d, 0x010A0000u, 0u - 53328u);  // 10*x2 + x3 (+ 528 - 53328)
  return hi2 * 100u + lo2;                                      // 100*(.. - 528) + ..
}

// value of the last L (1..12) ASCII digits of the 12 bytes d1|d2|d3 (the number's last
// digit is the high byte of d3); bytes before the number are ignored. Only 32-bit VALU
// work plus one 32x32->64 multiply-add.
BG_HD uint64_t bgp_digits_r(uint32_t d1, uint32_t d2, uint32_t d3, int L) {
  const int k1 = L >= 12 ? 0 : (L <= 8 ? 4 : 12 - L);  // leading bytes of d1 to ignore
  const int k2 = L >= 8 ? 0 : (L <= 4 ? 4 : 8 - L);
  const int k3 = L >= 4 ? 0 : 4 - L;
  const uint32_t m1 = (uint32_t)(~0ull << (8 * k1));  // bytes that belong to the number
  const uint32_t m2 = (uint32_t)(~0ull << (8 * k2));
  const uint32_t m3 = (uint32_t)(~0ull << (8 * k3));
  d1 = (d1 & m1) | (0x30303030u & ~m1);  // others read as '0'
  d2 = (d2 & m2) | (0x30303030u & ~m2);
  d3 = (d3 & m3) | (0x30303030u & ~m3);
  const uint32_t g23 = bgp_dig4(d2) * 10000u + bgp_dig4(d3);
  return (uint64_t)bgp_dig4(d1) * 100000000ull + g23;
}

// bgp_digits_r plus a check that the L number bytes are all ASCII digits (*ok cleared if
// not): the whitespace-only field split (bgp_fields_ws) finds number ends at whitespace and
// leaves the digit test to this
BG_HD uint64_t bgp_digits_rc(uint32_t d1, uint32_t d2, uint32_t d3, int L, bool& ok) {
  const int k1 = L >= 12 ? 0 : (L <= 8 ? 4 : 12 - L);
  const int k2 = L >= 8 ? 0 : (L <= 4 ? 4 : 8 - L);
  const int k3 = L >= 4 ? 0 : 4 - L;
  const uint32_t m1 = (uint32_t)(~0ull << (8 * k1));
  const uint32_t m2 = (uint32_t)(~0ull << (8 * k2));
  const uint32_t m3 = (uint32_t)(~0ull << (8 * k3));
  d1 = (d1 & m1) | (0x30303030u & ~m1);
  d2 = (d2 & m2) | (0x30303030u & ~m2);
  d3 = (d3 & m3) | (0x30303030u & ~m3);
  // byte x = d ^ '0' is a digit iff x < 10: bit 7 of x or of (x & 0x7F) + 0x76 flags the rest
  const uint32_t x1 = d1 ^ 0x30303030u, x2 = d2 ^ 0x30303030u, x3 = d3 ^ 0x30303030u;
  const uint32_t bad = (x1 | ((x1 & 0x7F7F7F7Fu) + 0x76767676u)) | (x2 | ((x2 & 0x7F7F7F7Fu) + 0x76767676u)) |
                       (x3 | ((x3 & 0x7F7F7F7Fu) + 0x76767676u));
  ok = ok && (bad & 0x80808080u) == 0;
  const uint32_t g23 = bgp_dig4(d2) * 10000u + bgp_dig4(d3);
  return (uint64_t)bgp_dig4(d1) * 100000000ull + g23;
}

// bit 7 of each byte of x: the byte is whitespace ({' ', 0x09..0x0D})
BG_HD uint32_t bgp_ws80(uint32_t x) {
  const uint32_t hi = x & 0x80808080u;
  const uint32_t lo7 = x & 0x7F7F7F7Fu;
  const uint32_t nz20 = ((lo7 ^ 0x20202020u) + 0x7F7F7F7Fu);  // bit 7: byte != ' '
  const uint32_t ge9 = lo7 + 0x77777777u;
  const uint32_t ge14 = lo7 + 0x72727272u;
  return (~nz20 | (ge9 & ~ge14)) & ~hi & 0x80808080u;
}
// whitespace classes of two dwords with ONE multiply (the bgp_classify gather with b's flags
// in a's digit slots): bits 0..3 = bytes of a, 4..7 = bytes of b
BG_HD uint32_t bgp_ws8(uint32_t a, uint32_t b) {
  const uint32_t p = ((bgp_ws80(a) >> 7) | (bgp_ws80(b) >> 3)) * 0x00204081u;
  return (p >> 21) & 0xFFu;
}

struct BgpFields {
  uint32_t a0, a1;  // chrom token [a0, a1)
  uint32_t s0, s1;  // start digits
  uint32_t e0, e1;  // end digits; rest starts at e1
};

// class masks of 32 bytes held as 8 dwords: bit j = byte j
BG_HD void bgp_classify8(const uint32_t W[8], uint32_t& WS, uint32_t& DG) {
  WS = 0;
  DG = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t w4, d4;
    bgp_classify(W[i], w4, d4);
    WS |= w4 << (4 * i);
    DG |= d4 << (4 * i);
  }
}

// index of the lowest set bit; 0xFFFFFFFF for 0 (v_ffbl_b32 semantics)
BG_HD uint32_t bgp_ffbl(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)(__ffs(x) - 1);
#else
  return x ? (uint32_t)__builtin_ctz(x) : 0xFFFFFFFFu;
#endif
}

// WS/DG: class masks of the line's first 32 bytes (bit j = byte j); len: line length
// (bytes before '\n'). returns 1: fields found; 0: undecided here (use the byte
// path); -1: blank line. Branch-free apart from the blank-line exit: every step runs and
// one flag collects the checks (keeps the exec mask and the SGPRs out of the hot loop).
BG_HD int bgp_fields_masks(uint32_t WS, uint32_t DG, uint32_t len, BgpFields& F) {
  const uint32_t endm = len < 32 ? (~0u << (len & 31)) : 0u;  // bytes past the line end
  WS |= endm;                                                  // act as whitespace
  DG &= ~endm;
  const uint32_t NW = ~WS;
  if (NW == 0) return len <= 32 ? -1 : 0;
  const uint32_t a0 = bgp_ffbl(NW);
  const uint32_t m1 = WS & (~0u << a0);
  const uint32_t a1 = bgp_ffbl(m1);
  const uint32_t m2 = NW & (~0u << (a1 & 31));
  const uint32_t s0 = bgp_ffbl(m2);
  const uint32_t m3 = ~DG & (~0u << (s0 & 31));
  const uint32_t s1 = bgp_ffbl(m3);
  const uint32_t m4 = NW & (~0u << (s1 & 31));
  const uint32_t e0 = bgp_ffbl(m4);
  const uint32_t m5 = ~DG & (~0u << (e0 & 31));
  const uint32_t e1 = bgp_ffbl(m5);
  // m1..m5 != 0 makes every index < 32
  bool ok = (m1 != 0) & (a1 < 31) & (m2 != 0) & (m3 != 0) & (m4 != 0) & (m5 != 0);
  ok &= ((DG >> (s0 & 31)) & 1u) != 0;   // start begins with a digit
  ok &= ((WS >> (s1 & 31)) & 1u) != 0;   // and ends at whitespace
  ok &= s1 < 31;
  ok &= ((DG >> (e0 & 31)) & 1u) != 0;   // end begins with a digit (may run to the line end)
  ok &= (s1 - s0 <= 16) & (e1 - e0 <= 16) & (e1 <= len);
  F.a0 = a0;
  F.a1 = a1;
  F.s0 = s0;
  F.s1 = s1;
  F.e0 = e0;
  F.e1 = e1;
  return ok ? 1 : 0;
}

// the same fields from the whitespace mask alone: a number runs to the next whitespace (or
// the line end) and the caller checks its bytes are digits (bgp_digits_rc), so every line
// this accepts (with the digit check passed) is one bgp_fields_masks accepts with the same
// fields; a number followed by another non-digit goes to the byte path
BG_HD int bgp_fields_ws(uint32_t WS, uint32_t len, BgpFields& F) {
  const uint32_t endm = len < 32 ? (~0u << (len & 31)) : 0u;
  WS |= endm;
  const uint32_t NW = ~WS;
  if (NW == 0) return len <= 32 ? -1 : 0;
  const uint32_t a0 = bgp_ffbl(NW);
  const uint32_t m1 = WS & (~0u << a0);
  const uint32_t a1 = bgp_ffbl(m1);
  const uint32_t m2 = NW & (~0u << (a1 & 31));
  const uint32_t s0 = bgp_ffbl(m2);
  const uint32_t m3 = WS & (~0u << (s0 & 31));
  const uint32_t s1 = bgp_ffbl(m3);
  const uint32_t m4 = NW & (~0u << (s1 & 31));
  const uint32_t e0 = bgp_ffbl(m4);
  const uint32_t m5 = WS & (~0u << (e0 & 31));
  const uint32_t e1 = bgp_ffbl(m5);
  bool ok = (m1 != 0) & (a1 < 31) & (m2 != 0) & (m3 != 0) & (m4 != 0) & (m5 != 0);
  ok &= s1 < 31;
  ok &= (s1 - s0 <= 16) & (e1 - e0 <= 16) & (e1 <= len);
  F.a0 = a0;
  F.a1 = a1;
  F.s0 = s0;
  F.s1 = s1;
  F.e0 = e0;
  F.e1 = e1;
  return ok ? 1 : 0;
}

// W: bytes [0, 32) of the line
BG_HD int bgp_fields(const uint32_t W[8], uint32_t len, BgpFields& F) {
  uint32_t WS, DG;
  bgp_classify8(W, WS, DG);
  return bgp_fields_masks(WS, DG, len, F);
}

// Token hash over 32-bit little-endian words of the token (zero padded), then the
// length: identical whether computed byte by byte or from 16-byte register windows.
BG_HD uint64_t bgp_hash_words(const uint32_t* w, uint32_t nwords, uint32_t len) {
  uint64_t h = 1469598103934665603ull;
  for (uint32_t i = 0; i < nwords; ++i) h = (h ^ w[i]) * 1099511628211ull;
  return (h ^ len) * 1099511628211ull;
}
// up to 16 token bytes given as lo (bytes 0..7) and hi (8..15) of the token start
BG_HD uint64_t bgp_hash16(uint64_t lo, uint64_t hi, uint32_t len) {
  if (len < 16) {
    if (len <= 8) {
      hi = 0;
      lo = len == 8 ? lo : (lo & ((1ull << (8 * len)) - 1));
    } else {
      hi &= (1ull << (8 * (len - 8))) - 1;
    }
  }
  uint32_t w[4] = {(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
  return bgp_hash_words(w, (len + 3) / 4, len);
}

// FNV-1a 64 over a chromosome token (run identity; same function everywhere)
#define BGP_FNV_OFF 1469598103934665603ull
#define BGP_FNV_PRIME 1099511628211ull
BG_HD uint64_t bgp_hash_step(uint64_t h, uint8_t b) { return (h ^ b) * BGP_FNV_PRIME; }
BG_HD uint64_t bgp_hash_final(uint64_t h, uint32_t len) { return (h ^ len) * BGP_FNV_PRIME; }
