/*
 * oracle/bedmap_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C) of `bedmap [--bp-ovr N] [--delim D] [--prec P] [--sci]
 * [--skip-unmapped] <--count|--mean>... ref.bed map.bed` on the reference's exact
 * event order:
 *   two-file window sweep ........... interfaces/src/algorithm/sweep/WindowSweepImpl.cpp:168-256
 *   overlap "distance" .............. interfaces/general-headers/data/bed/BedDistances.hpp:80-118
 *   window repair (fixWindow) ....... algorithm/visitors/bed/BedBaseVisitor.hpp:131-215
 *   set order (start,end,rest,addr) . data/bed/BedCompare.hpp:143-194 (row index stands in
 *                                     for the heap address: allocation order)
 *   fan-out / row printing .......... algorithm/visitors/other/MultiVisitor.hpp:71-98
 *   Count ("%d") .................... algorithm/visitors/numerical/CountVisitor.hpp:34-64
 *   Average (running double) ........ algorithm/visitors/numerical/AverageVisitor.hpp:35-75,
 *                                     "%.{prec}lf"/"%.{prec}e" utility/Formats.hpp:42-50,
 *                                     "NAN" interfaces/src/data/measurement/NaN.cpp:26
 *   argv grammar (subset) ........... applications/bed/bedmap/src/Input.hpp:75-367
 * Map rows are read as BED5 (chrom start end id score) when --mean is requested
 * (bedmap/src/Input.hpp:395-410 MapFields), else as BED3.
 * Only used by tests/ and bench.py's cpu_baseline; never linked into the product.
 */
#include "bedio.h"

static chrom_pool_t POOL;
static const bedfile_t *REF, *MAP;

/* Overlapping(ovr)(a,b) for a map row vs a ref row (BedDistances.hpp:95-115);
 * sign convention: 0 = in range, <0 = a "before" b, >0 otherwise. */
static int overlap_cmp(int ac, uint64_t as, uint64_t ae, int64_t aid, int bc, uint64_t bs,
                       uint64_t be, int64_t bid, uint64_t ovr) {
  if (ac != bc) {
    int v = strcmp(POOL.names[ac], POOL.names[bc]);
    if (v != 0) return v > 0 ? 1 : -1;
  }
  uint64_t mn = as > bs ? as : bs, mx = ae < be ? ae : be;
  if (mx > mn) {
    if (mx - mn >= ovr) return 0;
    if (as != bs) return as < bs ? -1 : 1;
    if (ae != be) return ae < be ? -1 : 1;
    return aid < bid ? -1 : 1;
  }
  return as < bs ? -1 : 1;
}
/* Ref2Map(r, m) / Map2Ref(m, r) */
static int r2m(int64_t r, int64_t m, uint64_t ovr) {
  return overlap_cmp(REF->chrom[r], REF->start[r], REF->end[r], -1 - r, MAP->chrom[m],
                     MAP->start[m], MAP->end[m], m, ovr);
}
static int m2r(int64_t m, int64_t r, uint64_t ovr) {
  return overlap_cmp(MAP->chrom[m], MAP->start[m], MAP->end[m], m, REF->chrom[r],
                     REF->start[r], REF->end[r], -1 - r, ovr);
}

/* ordered set of map rows by (start, end, row) */
typedef struct { int64_t* v; int64_t n, cap; } oset_t;
static int mless(int64_t a, int64_t b) {
  if (MAP->start[a] != MAP->start[b]) return MAP->start[a] < MAP->start[b];
  if (MAP->end[a] != MAP->end[b]) return MAP->end[a] < MAP->end[b];
  return a < b;
}
static int64_t os_lb(const oset_t* s, int64_t x) {
  int64_t lo = 0, hi = s->n;
  while (lo < hi) {
    int64_t mid = (lo + hi) / 2;
    if (mless(s->v[mid], x)) lo = mid + 1; else hi = mid;
  }
  return lo;
}
static void os_insert(oset_t* s, int64_t x) {
  int64_t p = os_lb(s, x);
  if (p < s->n && s->v[p] == x) return;
  if (s->n == s->cap) { s->cap = s->cap ? 2 * s->cap : 64; s->v = (int64_t*)realloc(s->v, (size_t)s->cap * 8); }
  memmove(s->v + p + 1, s->v + p, (size_t)(s->n - p) * 8);
  s->v[p] = x;
  s->n++;
}
static int os_erase(oset_t* s, int64_t x) {
  int64_t p = os_lb(s, x);
  if (p < s->n && s->v[p] == x) {
    memmove(s->v + p, s->v + p + 1, (size_t)(s->n - p - 1) * 8);
    s->n--;
    return 1;
  }
  return 0;
}

/* visitors */
enum { V_COUNT = 1, V_MEAN = 2 };
static int VIS[64], NVIS;
static int count_;
static double sum_;
static int counter_;
static long cnt_; /* MultiVisitor's own add/delete balance */
static const char* DELIM = "|";
static int PREC = 6, SCI = 0, SKIP_UNMAPPED = 0;

static void v_add(int64_t m) {
  for (int i = 0; i < NVIS; ++i) {
    if (VIS[i] == V_COUNT) ++count_;
    else { sum_ += MAP->score[m]; ++counter_; }
  }
  ++cnt_;
}
static void v_del(int64_t m) {
  for (int i = 0; i < NVIS; ++i) {
    if (VIS[i] == V_COUNT) --count_;
    else { sum_ -= MAP->score[m]; --counter_; }
  }
  --cnt_;
}
static void v_done(void) {
  if (SKIP_UNMAPPED && cnt_ == 0) return;
  char fmt[32];
  snprintf(fmt, sizeof(fmt), SCI ? "%%.%de" : "%%.%dlf", PREC);
  for (int i = 0; i < NVIS; ++i) {
    if (i) fputs(DELIM, stdout);
    if (VIS[i] == V_COUNT) printf("%d", count_);
    else if (counter_ > 0) printf(fmt, sum_ / counter_);
    else fputs("NAN", stdout);
  }
  fputc('\n', stdout);
}

int main(int argc, char** argv) {
  uint64_t ovr = 1;
  int a = 1, need5 = 0;
  const char* only_chrom = NULL;
  while (a < argc - 2 || (a < argc && strncmp(argv[a], "--", 2) == 0)) {
    const char* o = argv[a++];
    if (!strcmp(o, "--count")) VIS[NVIS++] = V_COUNT;
    else if (!strcmp(o, "--mean")) { VIS[NVIS++] = V_MEAN; need5 = 1; }
    else if (!strcmp(o, "--bp-ovr") && a < argc) ovr = strtoull(argv[a++], 0, 10);
    else if (!strcmp(o, "--delim") && a < argc) DELIM = argv[a++];
    else if (!strcmp(o, "--prec") && a < argc) PREC = atoi(argv[a++]);
    else if (!strcmp(o, "--chrom") && a < argc) only_chrom = argv[a++];
    else if (!strcmp(o, "--sci")) SCI = 1;
    else if (!strcmp(o, "--skip-unmapped")) SKIP_UNMAPPED = 1;
    else if (!strcmp(o, "--ec") || !strcmp(o, "--header") || !strcmp(o, "--sweep-all")) {}
    else { fprintf(stderr, "bedmap_oracle: unsupported option %s\n", o); return 2; }
  }
  if (NVIS == 0 || argc - a != 2) { fprintf(stderr, "bedmap_oracle: bad usage\n"); return 2; }
  static bedfile_t ref, map;
  FILE* fr = open_input(argv[a]);
  FILE* fm = open_input(argv[a + 1]);
  if (!fr || !fm) { fprintf(stderr, "bedmap_oracle: cannot open input\n"); return 2; }
  read_bed3(fr, &POOL, &ref, 0);
  if (need5) read_bed5(fm, &POOL, &map);
  else read_bed3(fm, &POOL, &map, 0);
  if (only_chrom) {
    bedfile_t* fs[2] = {&ref, &map};
    for (int q = 0; q < 2; ++q) {
      bedfile_t* f = fs[q];
      int64_t k = 0;
      for (int64_t j = 0; j < f->n; ++j) {
        if (strcmp(POOL.names[f->chrom[j]], only_chrom) != 0) continue;
        f->chrom[k] = f->chrom[j]; f->start[k] = f->start[j]; f->end[k] = f->end[j];
        if (f->score) f->score[k] = f->score[j];
        ++k;
      }
      f->n = k;
    }
  }
  REF = &ref;
  MAP = &map;
  static char obuf[1 << 20];
  setvbuf(stdout, obuf, _IOFBF, sizeof(obuf));

  /* sweep() overload2 with Overlapping(0); visitor distance Overlapping(ovr) */
  int64_t* win = (int64_t*)malloc(sizeof(int64_t) * (size_t)(map.n + 1));
  int64_t wh = 0, wt = 0; /* deque [wh, wt) */
  int64_t mi = 0, cache = -1;
  oset_t vwin = {0}, vcache = {0}, lst = {0};
  for (int64_t r = 0; r < ref.n; ++r) {
    while (wt > wh && m2r(win[wh], r, 0) < 0) { /* OnDelete */
      int64_t m = win[wh++];
      if (os_erase(&vwin, m)) v_del(m);
      else os_erase(&vcache, m);
    }
    while (cache >= 0 || mi < map.n) {
      int64_t m;
      if (cache >= 0) { m = cache; cache = -1; }
      else m = mi++;
      int v = r2m(r, m, 0);
      if (v == 0) { win[wt++] = m; os_insert(&vcache, m); } /* OnAdd -> cache_ */
      else if (v < 0) { cache = m; break; }
    }
    /* OnDone: fixWindow (deletions first, then insertions), then DoneReference */
    lst.n = 0;
    for (int64_t i = 0; i < vwin.n;) {
      int64_t m = vwin.v[i];
      if (m2r(m, r, ovr) != 0) {
        v_del(m);
        os_insert(&lst, m);
        memmove(vwin.v + i, vwin.v + i + 1, (size_t)(vwin.n - i - 1) * 8);
        vwin.n--;
      } else ++i;
    }
    for (int64_t i = 0; i < vcache.n;) {
      int64_t m = vcache.v[i];
      if (m2r(m, r, ovr) == 0) {
        v_add(m);
        os_insert(&vwin, m);
        memmove(vcache.v + i, vcache.v + i + 1, (size_t)(vcache.n - i - 1) * 8);
        vcache.n--;
      } else ++i;
    }
    for (int64_t i = 0; i < lst.n; ++i) os_insert(&vcache, lst.v[i]);
    v_done();
  }
  fflush(stdout);
  return 0;
}
