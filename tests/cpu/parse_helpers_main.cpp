// CPU driver for bedops_amd/csrc/bg_parse.h (the loader's SWAR field extraction).
// Reads lines on stdin; for each prints "fast a0 a1 start end rest", "slow" or "blank".
#include <initializer_list>
#include <stdio.h>
#include <string.h>

#include "../../bedops_amd/csrc/bg_parse.h"

static int naive_ws(unsigned b) { return b == ' ' || (b >= 9 && b <= 13); }
static int naive_dg(unsigned b) { return b >= '0' && b <= '9'; }

int main() {
  // bgp_classify against a per-byte restatement: every byte value in every position
  for (uint32_t pos = 0; pos < 4; ++pos)
    for (uint32_t v = 0; v < 256; ++v)
      for (uint32_t fill : {0x00000000u, 0x20202020u, 0x39393939u, 0xFFFFFFFFu, 0x0A09300Bu}) {
        const uint32_t x = (fill & ~(0xFFu << (8 * pos))) | (v << (8 * pos));
        uint32_t ws, dg, w2 = 0, d2 = 0;
        bgp_classify(x, ws, dg);
        for (int i = 0; i < 4; ++i) {
          w2 |= (uint32_t)naive_ws((x >> (8 * i)) & 0xFF) << i;
          d2 |= (uint32_t)naive_dg((x >> (8 * i)) & 0xFF) << i;
        }
        if (ws != w2 || dg != d2) { printf("CLASSIFY %08x\n", x); return 1; }
      }
  // bgp_ws8 against bgp_classify's whitespace groups
  for (uint32_t v = 0; v < 256; ++v)
    for (uint32_t fill : {0x00000000u, 0x20202020u, 0x0D0A0920u, 0xFFFFFFFFu})
      for (uint32_t pos = 0; pos < 4; ++pos) {
        const uint32_t a = (fill & ~(0xFFu << (8 * pos))) | (v << (8 * pos)), b = ~a ^ (v << 8);
        uint32_t wa, wb, d;
        bgp_classify(a, wa, d);
        bgp_classify(b, wb, d);
        if (bgp_ws8(a, b) != (wa | (wb << 4))) { printf("WS8 %08x %08x\n", a, b); return 1; }
      }
  static char line[1 << 16];
  while (fgets(line, sizeof(line), stdin)) {
    size_t len = strlen(line);
    if (len && line[len - 1] == '\n') line[--len] = 0;
    unsigned char buf[64] = {0};
    memcpy(buf, line, len < 52 ? len : 52);
    uint32_t W[8];
    for (int i = 0; i < 8; ++i)
      W[i] = buf[4 * i] | (buf[4 * i + 1] << 8) | (buf[4 * i + 2] << 16) | ((uint32_t)buf[4 * i + 3] << 24);
    // the whitespace-only split (k_parse_set's path) with its digit checks, printed first
    {
      uint32_t WSm = 0;
      for (int i = 0; i < 8; i += 2) WSm |= bgp_ws8(W[i], W[i + 1]) << (4 * i);
      BgpFields G;
      const int r2 = bgp_fields_ws(WSm, (uint32_t)len, G);
      if (r2 == -1) printf("ws blank ");
      else if (r2 == 0 || G.s1 - G.s0 > 12 || G.e1 - G.e0 > 12) printf("ws slow ");
      else {
        bool ok = true;
        uint64_t v2[2];
        for (int which = 0; which < 2; ++which) {
          const uint32_t b0 = which ? G.e0 : G.s0, b1 = which ? G.e1 : G.s1;
          unsigned char w[12];
          for (int i = 0; i < 12; ++i) {
            const int at = (int)b1 - 12 + i;
            w[i] = at >= 0 ? (unsigned char)line[at] : 0x55;
          }
          uint32_t d[3];
          memcpy(d, w, 12);
          v2[which] = bgp_digits_rc(d[0], d[1], d[2], (int)(b1 - b0), ok);
        }
        if (ok) printf("ws fast %u %u %llu %llu %u ", G.a0, G.a1, (unsigned long long)v2[0], (unsigned long long)v2[1], G.e1);
        else printf("ws slow ");
      }
    }
    BgpFields F;
    int r = bgp_fields(W, (uint32_t)len, F);
    if (r == -1) { puts("blank"); continue; }
    if (r == 0) { puts("slow"); continue; }
    uint64_t lo = 0, hi = 0;
    unsigned char d[16] = {0};
    memcpy(d, line + F.s0, len - F.s0 < 16 ? len - F.s0 : 16);
    memcpy(&lo, d, 8);
    memcpy(&hi, d + 8, 8);
    uint64_t s = bgp_digits(lo, hi, (int)(F.s1 - F.s0));
    memset(d, 0, 16);
    memcpy(d, line + F.e0, len - F.e0 < 16 ? len - F.e0 : 16);
    memcpy(&lo, d, 8);
    memcpy(&hi, d + 8, 8);
    uint64_t e = bgp_digits(lo, hi, (int)(F.e1 - F.e0));
    // right-aligned form (the one the kernel uses): the 12 bytes ending at the last digit
    for (int which = 0; which < 2; ++which) {
      const uint32_t b0 = which ? F.e0 : F.s0, b1 = which ? F.e1 : F.s1;
      if (b1 - b0 > 12) continue;
      unsigned char w[12];
      for (int i = 0; i < 12; ++i) {
        const int at = (int)b1 - 12 + i;
        w[i] = at >= 0 ? (unsigned char)line[at] : 0x55;
      }
      uint32_t d[3];
      memcpy(d, w, 12);
      const uint64_t v = bgp_digits_r(d[0], d[1], d[2], (int)(b1 - b0));
      if (v != (which ? e : s)) { printf("MISMATCH %llu\n", (unsigned long long)v); return 1; }
    }
    printf("fast %u %u %llu %llu %u\n", F.a0, F.a1, (unsigned long long)s, (unsigned long long)e, F.e1);
  }
  return 0;
}
