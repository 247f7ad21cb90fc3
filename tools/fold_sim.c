// Simulation of a speculative parallel fold of the decimal bedmap running sum (DESIGN.md
// sect. 4.2, measured and dropped): how many segment starts still change per repair round.
// gcc -O2 -o fold_sim tools/fold_sim.c && ./fold_sim <events> <segment> <mean window>
// simulate the segmented fold's convergence on a synthetic decimal event stream
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
static uint64_t rs = 88172645463325252ull;
static uint64_t xr(void) { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; }
static int same(double a, double b) { uint64_t x, y; memcpy(&x, &a, 8); memcpy(&y, &b, 8); return x == y; }
int main(int argc, char** argv) {
  const uint64_t E = argc > 1 ? atoll(argv[1]) : 20000000;
  const int L = argc > 2 ? atoi(argv[2]) : 256;
  const int mean_w = argc > 3 ? atoi(argv[3]) : 10;
  double* X = malloc(8 * E);
  double win[4096]; int wn = 0, wh = 0;  // ring of window scores (FIFO)
  uint64_t k = 0;
  while (k < E) {
    // each ref row: delete a few oldest, add a few new; sometimes empty the window
    int nd = (int)(xr() % 4), na = (int)(xr() % 4);
    if (xr() % 8 == 0) nd = wn;  // gap: window empties
    if (wn + na - nd > 2 * mean_w) na = 0;
    for (int i = 0; i < nd && wn > 0 && k < E; ++i) { X[k++] = -win[wh]; wh = (wh + 1) % 4096; --wn; }
    for (int i = 0; i < na && k < E; ++i) {
      double x = (double)(xr() % 100000) / 1000.0;
      win[(wh + wn) % 4096] = x; ++wn; X[k++] = x;
    }
  }
  double* SA = malloc(8 * E);
  double s = 0; for (uint64_t i = 0; i < E; ++i) { s += X[i]; SA[i] = s; }
  const uint64_t P = (E + L - 1) / L;
  double *st = malloc(8 * P), *ea = malloc(8 * P), *eb = malloc(8 * P), *S2 = malloc(8 * E);
  // totals and guesses
  double acc = 0;
  for (uint64_t j = 0; j < P; ++j) {
    double t = 0; for (uint64_t i = j * L; i < (j + 1) * L && i < E; ++i) t += X[i];
    st[j] = j ? acc : 0.0; acc += t;
  }
  for (uint64_t j = 0; j < P; ++j) { double t = st[j]; for (uint64_t i = j * L; i < (j + 1) * L && i < E; ++i) { t += X[i]; S2[i] = t; } ea[j] = t; }
  for (int r = 0; r < 64; ++r) {
    memcpy(eb, ea, 8 * P);
    uint64_t ch = 0, work = 0, minj = ~0ull;
    for (uint64_t j = 1; j < P; ++j) {
      double n = eb[j - 1];
      if (same(n, st[j])) { ea[j] = eb[j]; continue; }
      ++ch; if (j < minj) minj = j;
      st[j] = n; double t = n; int met = 0;
      uint64_t i = j * L, b = (j + 1) * L < E ? (j + 1) * L : E;
      for (; i < b; ++i) { t += X[i]; ++work; int eq = same(t, S2[i]); S2[i] = t; if (eq) { met = 1; break; } }
      ea[j] = met ? eb[j] : t;
    }
    printf("round %d: changed %llu work %llu min %llu\n", r, (unsigned long long)ch, (unsigned long long)work, (unsigned long long)minj);
    if (!ch) break;
  }
  uint64_t bad = 0; for (uint64_t i = 0; i < E; ++i) bad += !same(S2[i], SA[i]);
  printf("mismatches after rounds: %llu (E %llu P %llu)\n", (unsigned long long)bad, (unsigned long long)E, (unsigned long long)P);
  return 0;
}
