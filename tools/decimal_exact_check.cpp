// Host check of bg_load.hip decimal_exact / round_u128 (copied here) against glibc strtod on
// random and near-halfway spellings: g++ -O2 tools/decimal_exact_check.cpp && ./a.out
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cmath>
#include <cstring>
#include <random>
static double round_u128(unsigned __int128 N, int e2) {
  const uint64_t hi = (uint64_t)(N >> 64), lo = (uint64_t)N;
  const int lz = hi ? __builtin_clzll(hi) : 64 + __builtin_clzll(lo);
  N <<= lz; e2 -= lz;
  uint64_t mant = (uint64_t)(N >> 75);
  const unsigned __int128 rest = N & (((unsigned __int128)1 << 75) - 1), half = (unsigned __int128)1 << 74;
  if (rest > half || (rest == half && (mant & 1))) { ++mant; if (mant >> 53) { mant >>= 1; ++e2; } }
  return ldexp((double)mant, e2 + 75);
}
static bool decimal_exact(uint64_t m, int pw, double& out) {
  if (pw > 27 || pw < -26) return false;
  uint64_t f5 = 1;
  for (int k = 0; k < (pw < 0 ? -pw : pw); ++k) f5 *= 5;
  if (pw >= 0) { out = round_u128((unsigned __int128)m * f5, pw); return true; }
  const int s = 117 - (64 - __builtin_clzll(m));
  const unsigned __int128 num = (unsigned __int128)m << s;
  const unsigned __int128 q = num / f5, r = num - q * f5;
  out = round_u128((q << 1) | (r != 0 ? 1 : 0), -s - 1 + pw);
  return true;
}
int main() {
  std::mt19937_64 g(7);
  long bad = 0, n = 0;
  for (int it = 0; it < 3000000; ++it) {
    int digits = 1 + g() % 19;
    uint64_t m = 0;
    for (int i = 0; i < digits; ++i) m = m * 10 + g() % 10;
    if (!m) continue;
    int pw = (int)(g() % 54) - 26;
    if (it % 7 == 0) { // near halfway cases: m odd near 2^53..2^64 boundaries
      m = (1ULL << 53) + (g() % 1000);
    }
    double got;
    if (!decimal_exact(m, pw, got)) continue;
    char buf[64];
    snprintf(buf, sizeof buf, "%llue%d", (unsigned long long)m, pw);
    const double want = strtod(buf, nullptr);
    ++n;
    if (memcmp(&got, &want, 8)) { if (bad < 5) printf("bad %s got %.17g want %.17g\n", buf, got, want); ++bad; }
  }
  printf("checked %ld, mismatches %ld\n", n, bad);
}
