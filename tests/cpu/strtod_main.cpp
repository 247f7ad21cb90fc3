// CPU test of bedops_amd/csrc/bg_strtod.h (the loader's exact score conversion past the fast
// paths) against glibc strtod, which B5Rest's fscanf "%lf" uses (Bed.hpp:829-860).
// usage: strtod <seed> <n> -> "ok <checked>" or the first mismatch (exit 1)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../bedops_amd/csrc/bg_strtod.h"

static uint64_t sm(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// "<digits>[.<digits>][e<exp>]" -> significant digits + exponent of the last one
static bool split(const std::string& t, std::string& dg, int& e) {
  int frac = 0;
  bool dot = false;
  dg.clear();
  size_t i = 0;
  for (; i < t.size(); ++i) {
    const char c = t[i];
    if (c == '.') { dot = true; continue; }
    if (c < '0' || c > '9') break;
    if (dot) ++frac;
    if (dg.empty() && c == '0') continue;
    dg.push_back(c);
  }
  // digits after the first significant one that were zeros before it were skipped: count
  // the fraction digits only from the significant ones by recomputing
  int ex = 0;
  if (i < t.size() && (t[i] == 'e' || t[i] == 'E')) ex = atoi(t.c_str() + i + 1);
  e = ex - frac;
  // trailing zeros of dg move into e
  while (!dg.empty() && dg.back() == '0') { dg.pop_back(); ++e; }
  return true;
}

static int check(const std::string& t, long& n) {
  std::string dg;
  int e;
  split(t, dg, e);
  if (dg.size() > BG_SD_DIGITS) return 0;
  uint8_t d[BG_SD_DIGITS];
  for (size_t i = 0; i < dg.size(); ++i) d[i] = (uint8_t)(dg[i] - '0');
  double got;
  if (!strtod_big(d, (int)dg.size(), e, false, got)) {
    printf("REFUSED %s\n", t.c_str());
    return 1;
  }
  const double want = strtod(t.c_str(), nullptr);
  ++n;
  if (memcmp(&got, &want, 8) != 0) {
    printf("MISMATCH %s\n got  %.17g\n want %.17g\n", t.c_str(), got, want);
    return 1;
  }
  return 0;
}

int main(int argc, char** argv) {
  uint64_t x = argc > 1 ? strtoull(argv[1], 0, 10) : 1;
  const long N = argc > 2 ? atol(argv[2]) : 100000;
  long n = 0;
  const char* fixed[] = {"0", "1", "1e300", "1e308", "1.7976931348623157e308", "1.7976931348623159e308",
                         "1e309", "2.2250738585072014e-308", "2.2250738585072011e-308", "4.9406564584124654e-324",
                         "2.4703282292062327e-324", "2.4703282292062328e-324", "3e-320", "1e-325", "9007199254740993",
                         "9007199254740992.5", "18446744073709551616", "123456789012345678901234567890", "0.1",
                         "1e23", "8.98846567431158e307", "4.5e15", "1e-300", "2.5e299", "0.000000000000000000000001"};
  for (const char* t : fixed)
    if (check(t, n)) return 1;
  char buf[512];
  for (long i = 0; i < N; ++i) {
    const int kind = (int)(sm(x) % 4);
    std::string t;
    if (kind == 0) {  // a random double printed with 17..40 digits (near-halfway strings)
      uint64_t b = sm(x) & 0x7FFFFFFFFFFFFFFFull;
      double v;
      memcpy(&v, &b, 8);
      if (!std::isfinite(v)) continue;
      snprintf(buf, sizeof(buf), "%.*e", 16 + (int)(sm(x) % 25), v);
      t = buf;
    } else if (kind == 1) {  // exact halfway points between neighbours: m+1/2 ulp printed exactly
      uint64_t b = (sm(x) & 0x7FEFFFFFFFFFFFFFull);
      double v, w;
      memcpy(&v, &b, 8);
      w = nextafter(v, INFINITY);
      long double h = ((long double)v + (long double)w) / 2;
      snprintf(buf, sizeof(buf), "%.*Le", 20 + (int)(sm(x) % 60), h);
      t = buf;
    } else if (kind == 2) {  // random digit strings, random exponents
      const int nd = 1 + (int)(sm(x) % (sm(x) % 4 == 0 ? 190 : 25));
      for (int k = 0; k < nd; ++k) t.push_back((char)('0' + sm(x) % 10));
      if (sm(x) & 1) t.insert(t.begin() + (sm(x) % t.size()), '.');
      t += "e" + std::to_string((int)(sm(x) % 700) - 350);
    } else {  // subnormal range
      snprintf(buf, sizeof(buf), "%llue-%d", (unsigned long long)(sm(x) % 100000000000ull), 308 + (int)(sm(x) % 30));
      t = buf;
    }
    if (check(t, n)) return 1;
  }
  printf("ok %ld\n", n);
  return 0;
}
