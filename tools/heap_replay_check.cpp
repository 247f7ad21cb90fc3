// tools/heap_replay_check.cpp — runs the product's host heap replay (bedops_amd/csrc/
// bg_heap_replay.h, the code bg_heap_addr drives on the keyed rows) on the CPU over BED files,
// and prints the simulated address of every map row, one per line: tests/test_heap_replay.py
// compares them with oracle/bedmap_oracle.c --dump-addr on the same arguments. The row
// preparation restates what the device does before the replay (keys with chromosome ids in
// strcmp order, k_heap_lens, k_heap_rest_rank).
//   usage: heap_replay_check [bedmap options and operations] ref.bed [map.bed]
#include "../bedops_amd/csrc/bg_heap_replay.h"

#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>

namespace {
struct Row {
  std::string chrom, rest;  // rest: everything after `end` (with its leading tab)
  int64_t s = 0, e = 0;
};
bool read_bed(const char* path, std::vector<Row>& out) {
  FILE* f = fopen(path, "r");
  if (!f) return false;
  char* line = nullptr;
  size_t cap = 0;
  ssize_t n;
  while ((n = getline(&line, &cap, f)) > 0) {
    if (line[n - 1] == '\n') line[--n] = 0;
    if (!n) continue;
    Row r;
    char* p = line;
    char* t1 = strchr(p, '\t');
    if (!t1) continue;
    r.chrom.assign(p, t1 - p);
    char* q;
    r.s = strtoll(t1 + 1, &q, 10);
    r.e = strtoll(q + 1, &q, 10);
    r.rest = q;
    out.push_back(r);
  }
  free(line);
  fclose(f);
  return true;
}
bool ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }
// k_heap_lens: id length and the remainder after id (B4) / score (B5)
void lens(const std::string& rp, int fields, uint32_t& li, uint32_t& lr) {
  const uint32_t rl = (uint32_t)rp.size();
  if (fields == 3) {
    li = 0;
    lr = rl;
    return;
  }
  uint32_t i = 0;
  while (i < rl && ws(rp[i])) ++i;
  uint32_t j = i;
  while (j < rl && !ws(rp[j])) ++j;
  li = j - i;
  if (fields == 4) {
    lr = rl - j;
    return;
  }
  uint32_t k = j;
  while (k < rl && ws(rp[k])) ++k;
  while (k < rl && !ws(rp[k])) ++k;
  lr = rl - k;
}
// bg_frest: full_rest() of a row
std::string frest(const std::string& rp, int fields) {
  const size_t rl = rp.size();
  if (fields == 3) return rp;
  size_t i = 0;
  while (i < rl && ws(rp[i])) ++i;
  if (fields == 4) return rp.substr(i);
  size_t j = i;
  while (j < rl && !ws(rp[j])) ++j;
  size_t k = j;
  while (k < rl && ws(rp[k])) ++k;
  while (k < rl && !ws(rp[k])) ++k;
  return rp.substr(i, j - i) + rp.substr(k);
}
}  // namespace

int main(int argc, char** argv) {
  static const struct { const char* name; int op; int f; } OPS[] = {
      {"--count", BG_MAP_COUNT, 3}, {"--mean", BG_MAP_MEAN, 5}, {"--sum", BG_MAP_SUM, 5}, {"--min", BG_MAP_MIN, 5},
      {"--max", BG_MAP_MAX, 5}, {"--indicator", BG_MAP_INDICATOR, 3}, {"--bases", BG_MAP_BASES, 3},
      {"--bases-uniq", BG_MAP_BASES_UNIQ, 3}, {"--bases-uniq-f", BG_MAP_BASES_UNIQ_F, 3}, {"--echo", BG_MAP_ECHO, 3},
      {"--echo-ref-size", BG_MAP_ECHO_SIZE, 3}, {"--echo-ref-name", BG_MAP_ECHO_NAME, 3},
      {"--echo-map", BG_MAP_ECHO_MAP, 3}, {"--echo-map-id", BG_MAP_ECHO_MAP_ID, 4},
      {"--echo-map-score", BG_MAP_ECHO_MAP_SCORE, 5}, {"--echo-map-size", BG_MAP_ECHO_MAP_SIZE, 3},
      {"--echo-overlap-size", BG_MAP_ECHO_OVERLAP_SIZE, 3}, {"--echo-map-range", BG_MAP_ECHO_MAP_RANGE, 3},
      {"--median", BG_MAP_MEDIAN, 5}, {"--variance", BG_MAP_VARIANCE, 5}, {"--stdev", BG_MAP_STDEV, 5},
      {"--cv", BG_MAP_CV, 5}, {"--echo-map-id-uniq", BG_MAP_ECHO_MAP_ID_UNIQ, 4},
      {"--echo-ref-row-id", BG_MAP_ECHO_REF_ROW_ID, 3}, {"--min-element", BG_MAP_MIN_ELEMENT, 5},
      {"--max-element", BG_MAP_MAX_ELEMENT, 5}, {"--min-element-rand", BG_MAP_MIN_ELEMENT_RAND, 5},
      {"--max-element-rand", BG_MAP_MAX_ELEMENT_RAND, 5}, {"--wmean", BG_MAP_WMEAN, 5}};
  std::vector<int> ops;
  int fields = 3;
  bg_heap_spec spec;
  spec.crit = BG_OVR_BP;
  spec.ovr = 1;
  auto frac = [](const char* v) {  // PercentOverlapMapping's constructor (BedDistances.hpp:126-136)
    double p = strtod(v, nullptr);
    while (p > 1) p /= 10.0;
    p -= DBL_EPSILON;
    if (p <= 0.0) p = DBL_EPSILON;
    return p;
  };
  int a = 1;
  while (a < argc && !strncmp(argv[a], "--", 2)) {
    const char* o = argv[a++];
    bool found = false;
    for (const auto& k : OPS)
      if (!strcmp(o, k.name)) {
        ops.push_back(k.op);
        fields = std::max(fields, k.f);
        found = true;
      }
    if (found) continue;
    if (!strcmp(o, "--tmean")) { ops.push_back(BG_MAP_TMEAN); fields = 5; a += 2; }
    else if (!strcmp(o, "--kth")) { ops.push_back(BG_MAP_KTH); fields = 5; ++a; }
    else if (!strcmp(o, "--mad")) {
      ops.push_back(BG_MAP_MAD);
      fields = 5;
      if (a < argc && argv[a][0] && strspn(argv[a], ".-0123456789") == strlen(argv[a])) ++a;
    }
    else if (!strcmp(o, "--bp-ovr")) { spec.crit = BG_OVR_BP; spec.ovr = atoll(argv[a++]); }
    else if (!strcmp(o, "--range")) {
      spec.range = atoll(argv[a++]);
      if (spec.range == 0) { spec.crit = BG_OVR_BP; spec.ovr = 1; }
      else spec.crit = BG_OVR_RANGE;
    }
    else if (!strcmp(o, "--fraction-ref")) { spec.crit = BG_OVR_FRAC_REF; spec.perc = frac(argv[a++]); }
    else if (!strcmp(o, "--fraction-map")) { spec.crit = BG_OVR_FRAC_MAP; spec.perc = frac(argv[a++]); }
    else if (!strcmp(o, "--fraction-either")) { spec.crit = BG_OVR_FRAC_EITHER; spec.perc = frac(argv[a++]); }
    else if (!strcmp(o, "--fraction-both")) { spec.crit = BG_OVR_FRAC_BOTH; spec.perc = frac(argv[a++]); }
    else if (!strcmp(o, "--exact")) spec.crit = BG_OVR_EXACT;
    else if (!strcmp(o, "--faster")) spec.faster = true;
    else if (!strcmp(o, "--skip-unmapped")) spec.skip_unmapped = true;
    else if (!strcmp(o, "--delim") || !strcmp(o, "--multidelim") || !strcmp(o, "--prec")) ++a;
    else if (!strcmp(o, "--sci") || !strcmp(o, "--sweep-all")) {}
    else { fprintf(stderr, "heap_replay_check: unsupported option %s\n", o); return 2; }
  }
  const int nf = argc - a;
  if (nf < 1 || nf > 2 || ops.empty()) { fprintf(stderr, "heap_replay_check: bad usage\n"); return 2; }
  std::vector<Row> ref, map;
  if (!read_bed(argv[a], nf == 2 ? ref : map) || (nf == 2 && !read_bed(argv[a + 1], map))) return 2;
  const bool single = nf == 1;
  std::map<std::string, int> ids;  // chromosome ids in strcmp order
  for (const auto& r : ref) ids[r.chrom] = 0;
  for (const auto& r : map) ids[r.chrom] = 0;
  std::vector<std::string> names;
  for (auto& kv : ids) {
    kv.second = (int)names.size();
    names.push_back(kv.first);
  }
  auto key = [&](const Row& r, int64_t v) { return ((int64_t)ids[r.chrom] << BG_KEY_SHIFT) | v; };
  const uint64_t nm = map.size(), nr = ref.size();
  std::vector<int64_t> MS(nm), ME(nm), RS(nr), RE(nr);
  std::vector<uint32_t> li(nm), lr(nm), rrank(nm, 0), rlr(nr);
  std::vector<std::string> fr(nm);
  for (uint64_t m = 0; m < nm; ++m) {
    MS[m] = key(map[m], map[m].s);
    ME[m] = key(map[m], map[m].e);
    lens(map[m].rest, fields, li[m], lr[m]);
    fr[m] = frest(map[m].rest, fields);
  }
  for (uint64_t m = 0; m < nm; ++m) {  // k_heap_rest_rank
    uint64_t lo = m, hi = m + 1;
    while (lo > 0 && MS[lo - 1] == MS[m] && ME[lo - 1] == ME[m]) --lo;
    while (hi < nm && MS[hi] == MS[m] && ME[hi] == ME[m]) ++hi;
    for (uint64_t j = lo; j < hi; ++j)
      if (j != m && strcmp(fr[j].c_str(), fr[m].c_str()) < 0) ++rrank[m];
  }
  for (uint64_t r = 0; r < nr; ++r) {
    RS[r] = key(ref[r], ref[r].s);
    RE[r] = key(ref[r], ref[r].e);
    rlr[r] = (uint32_t)ref[r].rest.size();
  }
  spec.nops = (int)ops.size();
  spec.ops = ops.data();
  std::vector<int64_t> addr(nm + 1);
  Replay P;
  P.RS = RS.data();
  P.RE = RE.data();
  P.MS = MS.data();
  P.ME = ME.data();
  P.nr = single ? nm : nr;
  P.nm = nm;
  P.single = single;
  P.fields = fields;
  P.mli = li.data();
  P.mlr = lr.data();
  P.rlr = rlr.data();
  P.rrank = rrank.data();
  P.mlc.resize(nm);
  for (uint64_t m = 0; m < nm; ++m) P.mlc[m] = (uint32_t)map[m].chrom.size();
  P.rlc.resize(nr);
  for (uint64_t r = 0; r < nr; ++r) P.rlc[r] = (uint32_t)ref[r].chrom.size();
  P.spec = &spec;
  P.addr = addr.data();
  P.keyed.resize(ops.size());
  if (single) P.run1();
  else P.run2();
  for (uint64_t m = 0; m < nm; ++m) printf("%lld\n", (long long)addr[m]);
  return 0;
}
