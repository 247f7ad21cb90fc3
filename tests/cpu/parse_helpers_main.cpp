// CPU driver for bedops_amd/csrc/bg_parse.h (the loader's SWAR field extraction).
// Reads lines on stdin; for each prints "fast a0 a1 start end rest", "slow" or "blank".
#include <stdio.h>
#include <string.h>

#include "../../bedops_amd/csrc/bg_parse.h"

int main() {
  static char line[1 << 16];
  while (fgets(line, sizeof(line), stdin)) {
    size_t len = strlen(line);
    if (len && line[len - 1] == '\n') line[--len] = 0;
    unsigned char buf[64] = {0};
    memcpy(buf, line, len < 52 ? len : 52);
    uint32_t W[8];
    for (int i = 0; i < 8; ++i)
      W[i] = buf[4 * i] | (buf[4 * i + 1] << 8) | (buf[4 * i + 2] << 16) | ((uint32_t)buf[4 * i + 3] << 24);
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
    printf("fast %u %u %llu %llu %u\n", F.a0, F.a1, (unsigned long long)s, (unsigned long long)e, F.e1);
  }
  return 0;
}
