// CPU test of bedops_amd/csrc/bg_decfmt.h (the GPU formatter's exact "%.{p}lf"/"%.{p}e"
// path) against glibc printf, which the reference prints with (Formats.hpp:42-50).
// usage: decfmt <seed> <n>   -> prints "ok <checked>" or the first mismatch, exit 1
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../bedops_amd/csrc/bg_decfmt.h"

struct StrOut {
  std::string s;
  void put(char c) { s.push_back(c); }
};

static uint64_t sm(uint64_t& x) {  // splitmix64
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static int check(double v, int prec, bool sci, long& n) {
  if (!std::isfinite(v)) return 0;
  StrOut o;
  put_real_exact(o, v, prec, sci);
  std::string want(4000, '\0');
  int len = snprintf(&want[0], want.size(), sci ? "%.*e" : "%.*lf", prec, v);
  if (len >= (int)want.size()) {
    want.assign(len + 1, '\0');
    snprintf(&want[0], want.size(), sci ? "%.*e" : "%.*lf", prec, v);
  }
  want.resize(len);
  ++n;
  if (o.s != want) {
    uint64_t b;
    memcpy(&b, &v, 8);
    printf("MISMATCH bits=%016llx prec=%d sci=%d\n got  %s\n want %s\n", (unsigned long long)b, prec, (int)sci,
           o.s.c_str(), want.c_str());
    return 1;
  }
  return 0;
}

int main(int argc, char** argv) {
  uint64_t x = argc > 1 ? strtoull(argv[1], 0, 10) : 1;
  const long N = argc > 2 ? atol(argv[2]) : 20000;
  long n = 0;
  const int precs[] = {0, 1, 2, 3, 5, 6, 9, 10, 15, 16, 17, 18, 19, 20, 21, 25, 30, 40, 60, 100, 200, 340, 767, 1074, 1100};
  const double fixed[] = {0.0, -0.0, 0.5, 1.5, 2.5, -2.5, 0.125, 0.375, 9.995, 99.5, 999999.5, 0.05, 0.15, 0.25,
                          1e14, 1.23456789e14, 1e20, 1e22, 1e23, 1e300, -1e300, DBL_MAX, -DBL_MAX, DBL_MIN,
                          4.9406564584124654e-324, 2.2250738585072009e-308, 1e-16, 1e-17, 1e-300, 0.1, 1.0 / 3,
                          123456789.123456789, 9.999999999999999e22, 0.9999999, 0.99999999999, 5e-7, 4.9999999e-7,
                          1152921504606846976.0, 18446744073709551616.0, 9007199254740993.0, 0.000123};
  for (double v : fixed)
    for (int p : precs)
      for (int sc = 0; sc < 2; ++sc)
        if (check(v, p, sc, n)) return 1;
  for (long i = 0; i < N; ++i) {
    uint64_t r = sm(x), bits;
    const int kind = (int)(r % 4);
    double v;
    if (kind == 0) {  // any bit pattern
      bits = sm(x);
      memcpy(&v, &bits, 8);
    } else if (kind == 1) {  // decimal-looking scores around a random magnitude
      const int e = (int)(sm(x) % 60) - 30;
      v = (double)(sm(x) % 1000000) / 1000.0 * pow(10.0, e);
    } else if (kind == 2) {  // exact halves at many scales (ties for half-even)
      const int e = (int)(sm(x) % 40);
      v = ((double)(sm(x) % 100000) + 0.5) / pow(2.0, e % 12) * (e > 20 ? 1e10 : 1.0);
    } else {  // integers and near-integers around 2^53..2^80
      v = ldexp((double)(sm(x) >> 11), (int)(sm(x) % 40));
    }
    if (sm(x) & 1) v = -v;
    const int p = (sm(x) % 5 == 0) ? precs[sm(x) % (sizeof(precs) / sizeof(int))] : (int)(sm(x) % 25);
    if (check(v, p, sm(x) & 1, n)) return 1;
  }
  printf("ok %ld\n", n);
  return 0;
}
