// CPU build of the GPU --ec grammar (bedops_amd/csrc/bg_check.h) over a file, with the same
// first-failure rule as bg_check.hip: prints "in <file>\n<code>\nSee row: <n>" or nothing.
// The message wording comes from bg_check_message() in the library; tests/test_check.py
// maps codes to text with the same table through ctypes.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../bedops_amd/csrc/bg_check.h"

int main(int argc, char** argv) {
  if (argc != 4) return 2;
  const int nf = atoi(argv[1]), rest = atoi(argv[2]);
  FILE* f = fopen(argv[3], "rb");
  if (!f) return 2;
  std::string t;
  char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof(buf), f)) > 0) t.append(buf, n);
  std::vector<std::pair<size_t, size_t>> L;  // getline lines
  size_t p = 0;
  while (p < t.size()) {
    size_t e = t.find('\n', p);
    if (e == std::string::npos) e = t.size();
    L.push_back({p, e - p});
    p = e + 1;
  }
  size_t F = ~(size_t)0;
  for (size_t i = 0; i < L.size(); ++i) {
    BgcRow R;
    if (bgc_line(t.data() + L[i].first, (uint32_t)L[i].second, nf, rest, R) != BGC_HEADER) { F = i; break; }
  }
  for (size_t i = 0; i < L.size(); ++i) {
    BgcRow R;
    const char* l = t.data() + L[i].first;
    const int code = bgc_line(l, (uint32_t)L[i].second, nf, rest, R);
    int err = 0;
    if (code == BGC_HEADER) err = i > F ? BGC_HEADER_LATE : 0;
    else if (code) err = code;
    else if (i > F) {
      BgcRow P;
      const char* pl = t.data() + L[i - 1].first;
      if (bgc_line(pl, (uint32_t)L[i - 1].second, nf, rest, P) == BGC_OK)
        err = bgc_order(pl, (uint32_t)L[i - 1].second, P, l, (uint32_t)L[i].second, R, rest);
    } else if (R.end <= R.start) {
      err = BGC_END_LE_START;
    }
    if (err) {
      printf("%zu %d %zu %zu\n", i + 1, err, L[i].first, L[i].second);
      return 1;
    }
  }
  return 0;
}
