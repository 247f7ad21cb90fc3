/*
 * oracle/bedmap_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C) of `bedmap [overlap-option] [--delim D] [--prec P] [--sci]
 * [--skip-unmapped] <operations>... ref.bed map.bed` on the reference's exact event order:
 *   two-file window sweep ........... interfaces/src/algorithm/sweep/WindowSweepImpl.cpp:168-256
 *   sweep / visitor distances ....... applications/bed/bedmap/src/Bedmap.cpp:95-155 (the sweep
 *                                     runs on Overlapping(0), or RangedDist(R) for --range;
 *                                     the visitors filter with the chosen criterion)
 *   criteria ........................ interfaces/general-headers/data/bed/BedDistances.hpp:
 *                                     RangedDist :41-67, Overlapping :80-118,
 *                                     PercentOverlapMapping/Reference/Either/Both :123-288,
 *                                     Exact :293-317
 *   window repair (fixWindow) ....... algorithm/visitors/bed/BedBaseVisitor.hpp:131-215
 *   set order (start,end,rest,addr) . data/bed/BedCompare.hpp:143-194; the address of a map
 *                                     row comes from oracle/heapsim.h (the reference's glibc
 *                                     allocator replayed over the sweep's new/delete calls;
 *                                     row index in single-file mode)
 *   fan-out / row printing .......... algorithm/visitors/other/MultiVisitor.hpp:71-98
 *   visitors ........................ numerical/CountVisitor.hpp ("%d"), AverageVisitor.hpp and
 *                                     SumVisitor.hpp (running double), ExtremeVisitor.hpp (min/max),
 *                                     IndicatorVisitor.hpp, bed/OvrAggregateVisitor.hpp ("%lu"),
 *                                     bed/OvrUniqueVisitor.hpp ("%u"), bed/OvrUniqueFractionVisitor.hpp,
 *                                     other/EchoVisitor.hpp with PrintAll / PrintLength /
 *                                     PrintSpanName (helpers/ProcessBedVisitorRow.hpp:309-342);
 *                                     VarianceVisitor.hpp / StdevVisitor.hpp / CoeffVariationVisitor.hpp
 *                                     (running double sums), Median / RollingKthAverageVisitor.hpp:61-92;
 *                                     Extreme<PrintAllScorePrecision> for --min/max-element[-rand]
 *                                     (ExtremeVisitor.hpp:84-135 with Bed::ScoreThenGenomicCompare*,
 *                                     BedCompare.hpp:263-288, or CompValueThenAddress*,
 *                                     OrderCompare.hpp:31-47; printer ProcessBedVisitorRow.hpp:181-207),
 *                                     TrimmedMeanVisitor.hpp:40-220, bed/WeightedAverageVisitor.hpp:40-80;
 *                                     option names: helpers/NamedVisitors.hpp:52-250
 *   single-file mode ................ Bedmap.cpp:196-246 -> sweep overload 1,
 *                                     WindowSweepImpl.cpp:66-162 (rows are their own map rows,
 *                                     read as the map type, Bedmap.cpp:660-700)
 *   number formats .................. "%.{prec}lf"/"%.{prec}e" utility/Formats.hpp:42-50,
 *                                     "NAN" interfaces/src/data/measurement/NaN.cpp:26
 *   argv grammar (subset) ........... applications/bed/bedmap/src/Input.hpp:75-367
 * Map rows are read as BED5 (chrom start end id score) when a score operation is requested
 * (bedmap/src/Input.hpp:395-410 MapFields), else as BED3; the reference file keeps its
 * remainder (B3Rest) for --echo.
 * Only used by tests/ and bench.py's cpu_baseline; never linked into the product.
 */
#include <float.h>
#include <math.h>

#include "bedio.h"
#include "heapsim.h"

static chrom_pool_t POOL;
static const bedfile_t *REF, *MAP;

enum { C_BP, C_RANGE, C_FREF, C_FMAP, C_FEITHER, C_FBOTH, C_EXACT };
static int CRIT = C_BP;
static uint64_t OVR = 1, RANGE = 0;
static double PERC = 1.0; /* PercentOverlapMapping::perc_ after its constructor */

typedef struct { int c; uint64_t s, e; int64_t id; } row_t;
static int64_t* ADDR; /* simulated heap address of each map row (NULL: row index) */
#define A_(m) (ADDR ? ADDR[m] : (m))
static int SINGLE; /* single-file mode: the reference rows are the map rows (same objects) */
/* Overlapping's last tie-break compares the two rows' addresses (BedDistances.hpp:108-110):
 * the simulated heap address of a map row, and of the live reference row (two are alive) */
static int64_t REFA[2];
static row_t R_(int64_t r) { row_t x = {REF->chrom[r], REF->start[r], REF->end[r], SINGLE ? A_(r) : REFA[r & 1]}; return x; }
static row_t M_(int64_t m) { row_t x = {MAP->chrom[m], MAP->start[m], MAP->end[m], A_(m)}; return x; }
static int chrom_cmp(int a, int b) {
  if (a == b) return 0;
  int v = strcmp(POOL.names[a], POOL.names[b]);
  return v > 0 ? 1 : (v < 0 ? -1 : 0);
}

/* Overlapping(ovr)(a, b), BedDistances.hpp:97-115 */
static int d_overlap(row_t a, row_t b, uint64_t ovr) {
  int v = chrom_cmp(a.c, b.c);
  if (v) return v;
  uint64_t mn = a.s > b.s ? a.s : b.s, mx = a.e < b.e ? a.e : b.e;
  if (mx > mn) {
    if (mx - mn >= ovr) return 0;
    if (a.s != b.s) return a.s < b.s ? -1 : 1;
    if (a.e != b.e) return a.e < b.e ? -1 : 1;
    return a.id < b.id ? -1 : 1;
  }
  return a.s < b.s ? -1 : 1;
}
/* RangedDist(R)(a, b), BedDistances.hpp:57-64 */
static int d_ranged(row_t a, row_t b) {
  int v = chrom_cmp(a.c, b.c);
  if (v) return v;
  if (a.s < b.e) return (a.e + RANGE > b.s) ? 0 : -1;
  return (b.e + RANGE > a.s) ? 0 : 1;
}
/* PercentOverlapMapping::Ref2Map(ref, map), BedDistances.hpp:142-179 (fraction of map's size) */
static int d_pmap(row_t ref, row_t map) {
  int v = chrom_cmp(ref.c, map.c);
  if (v) return v;
  if (ref.e < map.s) return -1;
  if (map.e < ref.s) return 1;
  if (PERC <= DBL_EPSILON) return 0;
  double sz, total = (double)(map.e - map.s);
  int direction;
  if (ref.s <= map.s) {
    sz = (ref.e >= map.e) ? (double)(map.e - map.s) : (double)(ref.e - map.s);
    direction = -1;
  } else {
    sz = (ref.e >= map.e) ? (double)(map.e - ref.s) : (double)(ref.e - ref.s);
    direction = 1;
  }
  if (sz / total >= PERC) return 0;
  return direction;
}
/* the visitor distance's Map2Ref(map, ref); fixWindow uses only its zero-ness */
static int crit_m2r(int64_t m, int64_t r) {
  row_t a = M_(m), b = R_(r);
  switch (CRIT) {
    case C_RANGE: return d_ranged(a, b);
    case C_FMAP: return -d_pmap(b, a);          /* Mapping::Map2Ref = -Ref2Map(ref, map) */
    case C_FREF: return d_pmap(a, b);           /* Reference::Map2Ref = -(-Base::Ref2Map(map, ref)) */
    case C_FEITHER: {                           /* Either::Ref2Map, :233-241, negated */
      int v1 = d_pmap(b, a);
      if (v1 == 0) return 0;
      int v2 = -d_pmap(a, b);
      if (v2 == 0) return 0;
      return -v1;
    }
    case C_FBOTH: {                             /* Both::Ref2Map, :268-276, negated */
      int v1 = d_pmap(b, a);
      if (v1 != 0) return -v1;
      int v2 = -d_pmap(a, b);
      if (v2 != 0) return -v2;
      return 0;
    }
    case C_EXACT: {                             /* Exact::Ref2Map(ref, map), negated */
      int v = chrom_cmp(b.c, a.c);
      if (v) return -v;
      if (b.s != a.s) return b.s < a.s ? 1 : -1;
      if (b.e != a.e) return b.e < a.e ? 1 : -1;
      return 0;
    }
    default: return d_overlap(a, b, OVR);
  }
}
/* the criterion's own Ref2Map(ref, map) (--faster sweeps with it, Bedmap.cpp:287-290):
 * Overlapping / RangedDist operator() (:97-115, :57-64); PercentOverlapBoth::Ref2Map
 * (:268-276); Exact::Ref2Map (:300-309) */
static int crit_r2m(int64_t r, int64_t m) {
  row_t a = R_(r), b = M_(m);
  switch (CRIT) {
    case C_RANGE: return d_ranged(a, b);
    case C_FBOTH: {
      int v1 = d_pmap(a, b);
      if (v1 != 0) return v1;
      return -d_pmap(b, a);
    }
    case C_EXACT: {
      int v = chrom_cmp(a.c, b.c);
      if (v) return v;
      if (a.s != b.s) return a.s < b.s ? -1 : 1;
      if (a.e != b.e) return a.e < b.e ? -1 : 1;
      return 0;
    }
    default: return d_overlap(a, b, OVR);
  }
}
/* the sweep distance: Overlapping(0), or RangedDist(R) for --range; with --faster the
 * criterion itself (Bedmap.cpp:728-745) */
static int FASTER; /* --faster: no BedBaseVisitor, the visitors see the sweep's calls */
static int sweep_r2m(int64_t r, int64_t m) {
  if (FASTER) return crit_r2m(r, m);
  return CRIT == C_RANGE ? d_ranged(R_(r), M_(m)) : d_overlap(R_(r), M_(m), 0);
}
static int sweep_m2r(int64_t m, int64_t r) {
  if (FASTER) return crit_m2r(m, r);
  return CRIT == C_RANGE ? d_ranged(M_(m), R_(r)) : d_overlap(M_(m), R_(r), 0);
}

/* ordered set of map rows by (start, end, row) */
typedef struct { int64_t* v; int64_t n, cap; } oset_t;
static int mless(int64_t a, int64_t b) {
  if (MAP->start[a] != MAP->start[b]) return MAP->start[a] < MAP->start[b];
  if (MAP->end[a] != MAP->end[b]) return MAP->end[a] < MAP->end[b];
  return A_(a) < A_(b);
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

/* BedBaseVisitor's set order (CoordRestAddressCompare, BedCompare.hpp:143-194): start, end,
 * then strcmp of full_rest() (B3Rest: the remainder after end; B4Rest/B5Rest: id + the
 * remainder after id / score, Bed.hpp:301,537,788), then the address (row index here).
 * Add/Delete calls of fixWindow come in this order; it decides the running doubles'
 * rounding for rows of equal coordinates. */
static int MAPFIELDS = 3; /* map row type: B3Rest / B4Rest / B5Rest (Bedmap.cpp:601-655) */
static const char* frest_part(int64_t m, int part) {
  if (MAPFIELDS >= 4) return part == 0 ? MAP->id[m] : (MAP->rest ? MAP->rest[m] : "");
  return part == 0 ? (MAP->rest ? MAP->rest[m] : "") : "";
}
static int frest_cmp(int64_t a, int64_t b) {
  const char *pa = frest_part(a, 0), *pb = frest_part(b, 0);
  int ia = 0, ib = 0;
  for (;;) {
    if (!*pa && ia == 0) { pa = frest_part(a, 1); ia = 1; continue; }
    if (!*pb && ib == 0) { pb = frest_part(b, 1); ib = 1; continue; }
    const unsigned char x = (unsigned char)*pa, y = (unsigned char)*pb;
    if (x != y) return x < y ? -1 : 1;
    if (!x) return 0;
    ++pa;
    ++pb;
  }
}
static int rless(int64_t a, int64_t b) {
  if (MAP->start[a] != MAP->start[b]) return MAP->start[a] < MAP->start[b];
  if (MAP->end[a] != MAP->end[b]) return MAP->end[a] < MAP->end[b];
  int v = frest_cmp(a, b);
  if (v) return v < 0;
  return A_(a) < A_(b);
}
static void ev_push(oset_t* s, int64_t x) {
  if (s->n == s->cap) { s->cap = s->cap ? 2 * s->cap : 64; s->v = (int64_t*)realloc(s->v, (size_t)s->cap * 8); }
  s->v[s->n++] = x;
}
static void sort_rless(int64_t* v, int64_t n) { /* insertion sort: runs are short */
  for (int64_t i = 1; i < n; ++i) {
    int64_t x = v[i], j = i;
    while (j > 0 && rless(x, v[j - 1])) { v[j] = v[j - 1]; --j; }
    v[j] = x;
  }
}

/* visitors */
enum { V_COUNT = 1, V_MEAN, V_SUM, V_MIN, V_MAX, V_INDICATOR, V_BASES, V_BASES_UNIQ,
       V_BASES_UNIQ_F, V_ECHO, V_ECHO_SIZE, V_ECHO_NAME, V_ECHO_MAP, V_ECHO_MAP_ID,
       V_ECHO_MAP_SCORE, V_ECHO_MAP_SIZE, V_ECHO_OVERLAP_SIZE, V_ECHO_MAP_RANGE, V_MEDIAN,
       V_KTH, V_VARIANCE, V_STDEV, V_CV, V_ECHO_MAP_ID_UNIQ, V_ECHO_REF_ROW_ID, V_MAD,
       V_MIN_EL, V_MAX_EL, V_MIN_EL_RAND, V_MAX_EL_RAND, V_TMEAN, V_WMEAN };
static double VARG[64];      /* --kth argument per visitor */
static double sq_;           /* Variance-family running sum of squares */
static int VIS[64], NVIS;
static int count_;     /* Count / Indicator */
static double sum_;    /* Average / Sum: one running double (they see the same events) */
static int counter_;
static long cnt_;      /* MultiVisitor's own add/delete balance */
static const char* DELIM = "|";
static const char* MULTIDELIM = ";";
static int PREC = 6, SCI = 0, SKIP_UNMAPPED = 0;
static oset_t VWIN;    /* the visitor window (BedBaseVisitor::win_) */

/* Extreme<.., Bed::ScoreThenGenomicCompare{Lesser,Greater}> (--min-element/--max-element):
 * a std::set keyed by (score, chrom, start, end) — an Add equivalent to a member is
 * dropped, a Delete erases the equivalent member (ExtremeVisitor.hpp:92-98). Both orders
 * share that equivalence, so one literal set serves both. */
static oset_t EXT;
static int ext_equiv(int64_t a, int64_t b) {
  return MAP->score[a] == MAP->score[b] && MAP->chrom[a] == MAP->chrom[b] &&
         MAP->start[a] == MAP->start[b] && MAP->end[a] == MAP->end[b];
}
static void ext_add(int64_t m) {
  for (int64_t i = 0; i < EXT.n; ++i) if (ext_equiv(EXT.v[i], m)) return;
  if (EXT.n == EXT.cap) { EXT.cap = EXT.cap ? 2 * EXT.cap : 64; EXT.v = (int64_t*)realloc(EXT.v, (size_t)EXT.cap * 8); }
  EXT.v[EXT.n++] = m;
}
static void ext_del(int64_t m) {
  for (int64_t i = 0; i < EXT.n; ++i)
    if (ext_equiv(EXT.v[i], m)) { EXT.v[i] = EXT.v[--EXT.n]; return; }
}
/* ScoreThenGenomicCompareLesser(a, b) (BedCompare.hpp:263-278) */
static int sg_less(int64_t a, int64_t b) {
  if (MAP->score[a] != MAP->score[b]) return MAP->score[a] < MAP->score[b];
  int v = chrom_cmp(MAP->chrom[a], MAP->chrom[b]);
  if (v) return v < 0;
  if (MAP->start[a] != MAP->start[b]) return MAP->start[a] < MAP->start[b];
  return MAP->end[a] < MAP->end[b];
}

/* TrimmedMean (TrimmedMeanVisitor.hpp:40-220): scoresBuf_ is a std::set ordered by
 * CompValueThenAddressLesser (score, then address = row index); each marker is an element
 * (-1 = end()) with its position and running double sum. */
typedef struct { int64_t el; size_t pos; double sum; } tm_mark_t;
typedef struct {
  double lo, hi;
  int doKth, symmetric;
  oset_t buf;
  tm_mark_t L, U;
} tmean_t;
static tmean_t TM[64];
static int vl_less(int64_t a, int64_t b) {
  if (MAP->score[a] != MAP->score[b]) return MAP->score[a] < MAP->score[b];
  return A_(a) < A_(b);
}
static int64_t tm_rank(const oset_t* s, int64_t x) {
  int64_t lo = 0, hi = s->n;
  while (lo < hi) { int64_t mid = (lo + hi) / 2; if (vl_less(s->v[mid], x)) lo = mid + 1; else hi = mid; }
  return lo;
}
static void tm_init(tmean_t* t, double lo, double hi) {
  memset(t, 0, sizeof(*t));
  t->lo = lo; t->hi = hi;
  t->L.el = t->U.el = -1;
  const double eps = DBL_EPSILON;
  if (fabs(1.0 - lo - hi) <= eps) t->doKth = 1;
  if (fabs(lo - hi) <= eps) t->symmetric = 1;
}
/* add(): after the insert */
static void tm_mark_add(tmean_t* t, tm_mark_t* k, int64_t m) {
  if (k->el < 0) { k->el = t->buf.v[0]; k->pos = 0; k->sum = MAP->score[m]; }
  else if (vl_less(m, k->el)) { ++k->pos; k->sum += MAP->score[m]; }
}
/* remove(): before the erase */
static void tm_mark_del(tmean_t* t, tm_mark_t* k, int64_t m) {
  if (vl_less(m, k->el)) { --k->pos; k->sum -= MAP->score[m]; }
  else if (m == k->el) {
    k->sum -= MAP->score[m];
    const int64_t r = tm_rank(&t->buf, k->el);
    if (r != 0) { k->el = t->buf.v[r - 1]; --k->pos; }
    else if (r + 1 < t->buf.n) { k->el = t->buf.v[r + 1]; k->sum += MAP->score[k->el]; }
    else k->el = -1;
  }
}
static void tm_add(tmean_t* t, int64_t m) {
  int64_t p = tm_rank(&t->buf, m);
  if (t->buf.n == t->buf.cap) { t->buf.cap = t->buf.cap ? 2 * t->buf.cap : 64; t->buf.v = (int64_t*)realloc(t->buf.v, (size_t)t->buf.cap * 8); }
  memmove(t->buf.v + p + 1, t->buf.v + p, (size_t)(t->buf.n - p) * 8);
  t->buf.v[p] = m;
  t->buf.n++;
  if (t->lo > 0 && !t->doKth) tm_mark_add(t, &t->L, m);
  tm_mark_add(t, &t->U, m);
}
static void tm_del(tmean_t* t, int64_t m) {
  if (t->lo > 0 && !t->doKth) tm_mark_del(t, &t->L, m);
  tm_mark_del(t, &t->U, m);
  int64_t p = tm_rank(&t->buf, m);
  memmove(t->buf.v + p, t->buf.v + p + 1, (size_t)(t->buf.n - p - 1) * 8);
  t->buf.n--;
}
static double tm_iround(double d) {
  double d1 = ceil(d);
  return (d >= 0) ? ((d1 - d > 0.5) ? floor(d) : d1) : ((d1 - d >= 0.5) ? floor(d) : d1);
}
/* doneRef(): walk the marker to newPos, summing what it passes */
static void tm_walk(tmean_t* t, tm_mark_t* k, size_t np) {
  int64_t r = tm_rank(&t->buf, k->el);
  while (np > k->pos) { ++r; k->sum += MAP->score[t->buf.v[r]]; ++k->pos; }
  while (np < k->pos) { k->sum -= MAP->score[t->buf.v[r]]; --r; --k->pos; }
  k->el = t->buf.v[r];
}
/* DoneReference(): 1 = value in *out, 0 = NAN */
static int tm_done(tmean_t* t, double* out) {
  if (t->buf.n == 0) return 0;
  const size_t size = (size_t)t->buf.n;
  size_t kl = (size_t)tm_iround(t->lo * (double)size);
  size_t kh = (size_t)tm_iround(t->hi * (double)size);
  kh = size - kh;
  if (t->symmetric) {
    kl = kl > size - kh ? kl : size - kh;
    kh = size - kl;
  }
  const int doLow = kl > 0;
  if (doLow) --kl;
  if (kh > 0) --kh;
  if (!t->doKth && doLow) tm_walk(t, &t->L, kl);
  tm_walk(t, &t->U, kh);
  if (t->doKth || t->U.pos == t->L.pos) *out = MAP->score[t->U.el];
  else if (doLow) *out = (t->U.sum - t->L.sum) / (double)(t->U.pos - t->L.pos);
  else *out = t->U.sum / (double)(t->U.pos + 1);
  return 1;
}

/* std::set node traffic. A B3Rest map row (32-byte object) shares the 48-byte chunk class with
 * the 40-byte _Rb_tree_node<MapType*> of every set the sweep's visitors keep, so for B3Rest maps
 * the address of a row depends on those nodes too (B4Rest / B5Rest rows use 64-byte chunks and
 * are not disturbed). Modelled containers:
 *   BedBaseVisitor's cache_ / win_ (BedBaseVisitor.hpp:139-153, fixWindow :185-211; the list
 *     nodes of fixWindow use 32-byte chunks and are left out);
 *   EchoMapBed / EchoMapIntersectLength / OvrAggregate: one node per Add (EchoMapBedVisitor.hpp:49-55,
 *     EchoMapIntersectLengthVisitor.hpp:56-62, OvrAggregateVisitor.hpp:57-67);
 *   OvrUnique(-Fract): a set keyed on coordinates (GenomicCompare), so rows with equal
 *     coordinates share one node, stored by the first of them (OvrUniqueVisitor.hpp:51-58). */
#define NODE_REQ 40
static heapsim_t HS;
static int NODES_ON;
static int64_t *NCACHE, *NWIN, *CREP; /* CREP: first row with the same coordinates */
static int64_t *NV[64], *HOLD[64];
static int vset(int v) {
  switch (v) {
    case V_ECHO_MAP: case V_ECHO_MAP_ID: case V_ECHO_MAP_SCORE: case V_ECHO_MAP_SIZE: case V_ECHO_MAP_RANGE:
    case V_ECHO_MAP_ID_UNIQ: case V_ECHO_OVERLAP_SIZE: case V_BASES: return 1;
    case V_BASES_UNIQ: case V_BASES_UNIQ_F: return 2;
  }
  return 0;
}
static void nodes_init(int64_t n) {
  NODES_ON = 1;
  NCACHE = (int64_t*)malloc((size_t)(n + 1) * 8);
  NWIN = (int64_t*)malloc((size_t)(n + 1) * 8);
  CREP = (int64_t*)malloc((size_t)(n + 1) * 8);
  for (int64_t m = 0; m <= n; ++m) NCACHE[m] = NWIN[m] = -1;
  for (int64_t m = 0; m < n; ++m)
    CREP[m] = (m && MAP->chrom[m] == MAP->chrom[m - 1] && MAP->start[m] == MAP->start[m - 1] &&
               MAP->end[m] == MAP->end[m - 1]) ? CREP[m - 1] : m;
  for (int q = 0; q < NVIS; ++q) {
    if (!vset(VIS[q])) continue;
    NV[q] = (int64_t*)malloc((size_t)(n + 1) * 8);
    HOLD[q] = (int64_t*)malloc((size_t)(n + 1) * 8);
    for (int64_t m = 0; m <= n; ++m) NV[q][m] = -1;
  }
}
static void n_new(int64_t* s, int64_t k) { s[k] = hs_malloc(&HS, NODE_REQ); }
static void n_free(int64_t* s, int64_t k) {
  if (s[k] >= 0) { hs_free(&HS, NODE_REQ, s[k]); s[k] = -1; }
}
/* MultiVisitor::Add / Delete: each visitor in command-line order (MultiVisitor.hpp:71-81) */
static void vis_add(int64_t m) {
  for (int q = 0; q < NVIS; ++q) {
    const int k = vset(VIS[q]);
    if (k == 1) n_new(NV[q], m);
    else if (k == 2 && NV[q][CREP[m]] < 0) { n_new(NV[q], CREP[m]); HOLD[q][CREP[m]] = m; }
  }
}
static void vis_del(int64_t m) {
  for (int q = 0; q < NVIS; ++q) {
    const int k = vset(VIS[q]);
    if (k == 1) n_free(NV[q], m);
    else if (k == 2) n_free(NV[q], CREP[m]);
  }
}
/* a temporary copy of a row (of `fields` columns + rest). Copy constructors allocate chrom_
 * (Bed.hpp:70-72), id_ (B4/B5, :404), then rest_ and fullrest_ (B3Rest :291-294, B4Rest
 * :509-512); B5Rest's copy constructor sizes rest_ / fullrest_ as strlen(p + 1), one byte
 * short of the string (Bed.hpp:757-759; for an empty string the length read past it is taken
 * as 0: such an allocation is in the smallest chunk class either way). The destructor frees
 * rest_, fullrest_, id_, then chrom_ (Bed.hpp:622-626 / 876-881, 477-480, 100-104). */
typedef struct { int64_t c, i, r, f; size_t lc, li, lr, lf; int fields; } tmprow_t;
static size_t slen(const char* p) { return p ? strlen(p) : 0; }
static void tmp_sizes(tmprow_t* t, const bedfile_t* f, int64_t i, int copy) {
  const size_t c = strlen(POOL.names[f->chrom[i]]), d = t->fields >= 4 ? slen(f->id[i]) : 0;
  const size_t r = f->rest ? slen(f->rest[i]) : 0;
  t->lc = c + 1;
  t->li = d + 1;
  if (copy && t->fields == 5) {
    t->lr = r ? r - 1 : 0;
    t->lf = d + r ? d + r - 1 : 0;
  } else {
    t->lr = r + 1;
    t->lf = d + r + 1;
  }
}
static void tmp_copy(tmprow_t* t, const bedfile_t* f, int64_t i, int fields) {
  t->fields = fields;
  tmp_sizes(t, f, i, 1);
  t->c = hs_malloc(&HS, t->lc);
  if (fields >= 4) t->i = hs_malloc(&HS, t->li);
  t->r = hs_malloc(&HS, t->lr);
  if (fields >= 4) t->f = hs_malloc(&HS, t->lf);
}
/* operator=: chrom_ (Bed.hpp:92-97), id_ (:468-474), then rest_ / fullrest_ freed and
 * re-allocated (:304-312, :609-619, :864-874) */
static void tmp_assign(tmprow_t* t, const bedfile_t* f, int64_t i) {
  tmprow_t n = *t;
  tmp_sizes(&n, f, i, 0);
  hs_free(&HS, t->lc, t->c);
  t->c = hs_malloc(&HS, n.lc);
  if (t->fields >= 4) { hs_free(&HS, t->li, t->i); t->i = hs_malloc(&HS, n.li); }
  hs_free(&HS, t->lr, t->r);
  if (t->fields >= 4) hs_free(&HS, t->lf, t->f);
  t->r = hs_malloc(&HS, n.lr);
  if (t->fields >= 4) t->f = hs_malloc(&HS, n.lf);
  t->lc = n.lc; t->li = n.li; t->lr = n.lr; t->lf = n.lf;
}
static void tmp_drop(const tmprow_t* t) {
  hs_free(&HS, t->lr, t->r);
  if (t->fields >= 4) { hs_free(&HS, t->lf, t->f); hs_free(&HS, t->li, t->i); }
  hs_free(&HS, t->lc, t->c);
}
/* EchoMapIntersectLength::DoneReference (EchoMapIntersectLengthVisitor.hpp:64-73): per map
 * row a copy of the reference row, and a std::vector<long> growing 1, 2, 4, 8, ... */
static void heap_intersect_lengths(int64_t r) {
  int64_t buf = -1;
  size_t cap = 0;
  for (int64_t k = 0; k < VWIN.n; ++k) {
    tmprow_t t;
    tmp_copy(&t, REF, r, SINGLE ? MAPFIELDS : 3);
    if ((size_t)k == cap) { /* _M_realloc_insert: allocate, move, free the old buffer */
      const size_t nc = cap ? 2 * cap : 1;
      const int64_t nb = hs_malloc(&HS, nc * 8);
      if (cap) hs_free(&HS, cap * 8, buf);
      buf = nb;
      cap = nc;
    }
    tmp_drop(&t);
  }
  if (cap) hs_free(&HS, cap * 8, buf);
}

static void v_add(int64_t m) {
  if (NODES_ON) vis_add(m);
  ++count_;
  if (MAP->score) {
    sum_ += MAP->score[m]; sq_ += MAP->score[m] * MAP->score[m]; ++counter_;
    ext_add(m);
    for (int i = 0; i < NVIS; ++i) if (VIS[i] == V_TMEAN) tm_add(&TM[i], m);
  }
  ++cnt_;
}
static void v_del(int64_t m) {
  if (NODES_ON) vis_del(m);
  --count_;
  if (MAP->score) {
    sum_ -= MAP->score[m]; sq_ -= MAP->score[m] * MAP->score[m]; --counter_;
    ext_del(m);
    for (int i = 0; i < NVIS; ++i) if (VIS[i] == V_TMEAN) tm_del(&TM[i], m);
  }
  --cnt_;
}
static void put_real(double v) {
  char fmt[32];
  snprintf(fmt, sizeof(fmt), SCI ? "%%.%de" : "%%.%dlf", PREC);
  printf(fmt, v);
}
/* OvrAggregate::coordCompare(ref, map), OvrAggregateVisitor.hpp:77-97 */
static unsigned long ovr_agg(int64_t r, int64_t m) {
  uint64_t ts = REF->start[r], te = REF->end[r], vs = MAP->start[m], ve = MAP->end[m];
  if (ts >= vs) {
    if (ve > ts) return ve > te ? te - ts : ve - ts;
    return 0;
  }
  if (te > vs) return ve < te ? ve - vs : te - vs;
  return 0;
}
/* BasicCoords::overlap length, Bed.hpp:172-190 */
static uint64_t ovr_len(uint64_t as, uint64_t ae, uint64_t bs, uint64_t be) {
  uint64_t mn = as > bs ? as : bs, mx = ae < be ? ae : be;
  return mx > mn ? mx - mn : 0;
}
/* OvrUnique::DoneReference, OvrUniqueVisitor.hpp:62-78 (its set is in genomic order) */
static unsigned int ovr_uniq(int q, int64_t r) {
  unsigned int ovr = 0;
  if (VWIN.n == 0) return 0;
  /* the set holds one row per distinct coordinates (GenomicCompare): equal rows are adjacent
   * in the window's order; the temporary is a copy of the row the set stored */
  tmprow_t t;
  if (NODES_ON) tmp_copy(&t, MAP, HOLD[q][CREP[VWIN.v[0]]], MAPFIELDS);
  uint64_t ts = MAP->start[VWIN.v[0]], te = MAP->end[VWIN.v[0]];
  const uint64_t rs = REF->start[r], re = REF->end[r];
  for (int64_t i = 1; i < VWIN.n; ++i) {
    const uint64_t s = MAP->start[VWIN.v[i]], e = MAP->end[VWIN.v[i]];
    if (s == MAP->start[VWIN.v[i - 1]] && e == MAP->end[VWIN.v[i - 1]]) continue;
    if (ovr_len(ts, te, s, e)) {
      ts = ts < s ? ts : s;
      te = te > e ? te : e;
    } else {
      ovr += (unsigned int)ovr_len(ts, te, rs, re);
      ts = s;
      te = e;
      if (NODES_ON) tmp_assign(&t, MAP, HOLD[q][CREP[VWIN.v[i]]]);
    }
  }
  ovr += (unsigned int)ovr_len(ts, te, rs, re);
  if (NODES_ON) tmp_drop(&t);
  return ovr;
}
/* one map row as its type prints it: B3Rest "%s\t%lu\t%lu%s", B4Rest "...\t%s%s",
 * B5Rest "...\t%s\t%lf%s" (Bed.hpp; Formats.hpp:34 "%lf") */
static void print_map_row_p(int64_t m, int prec_score) {
  printf("%s\t%" PRIu64 "\t%" PRIu64, POOL.names[MAP->chrom[m]], MAP->start[m], MAP->end[m]);
  if (MAPFIELDS >= 4) printf("\t%s", MAP->id[m]);
  if (MAPFIELDS >= 5) {
    fputc('\t', stdout);
    if (prec_score) put_real(MAP->score[m]);
    else printf("%lf", MAP->score[m]);
  }
  fputs(MAP->rest ? MAP->rest[m] : "", stdout);
}
static void print_map_row(int64_t m) { print_map_row_p(m, 0); }
static void echo_map(int how, int64_t r) {
  if (how == V_ECHO_MAP_RANGE) { /* PrintGenomicRange<PrintBED3>, ProcessBedVisitorRow.hpp:433-456 */
    if (VWIN.n == 0) return;
    uint64_t s = MAP->start[VWIN.v[0]], e = MAP->end[VWIN.v[0]];
    for (int64_t k = 1; k < VWIN.n; ++k) {
      if (s > MAP->start[VWIN.v[k]]) s = MAP->start[VWIN.v[k]];
      if (e < MAP->end[VWIN.v[k]]) e = MAP->end[VWIN.v[k]];
    }
    printf("%s\t%" PRIu64 "\t%" PRIu64, POOL.names[MAP->chrom[VWIN.v[0]]], s, e);
    return;
  }
  for (int64_t k = 0; k < VWIN.n; ++k) { /* PrintRangeDelim: genomic (set) order */
    const int64_t m = VWIN.v[k];
    if (k) fputs(MULTIDELIM, stdout);
    switch (how) {
      case V_ECHO_MAP: print_map_row(m); break;
      case V_ECHO_MAP_ID: fputs(MAP->id[m], stdout); break;
      case V_ECHO_MAP_SCORE: put_real(MAP->score[m]); break;
      case V_ECHO_MAP_SIZE: printf("%" PRIu64, MAP->end[m] - MAP->start[m]); break;
      case V_ECHO_OVERLAP_SIZE: /* EchoMapIntersectLengthVisitor.hpp:66-75, "%ld" */
        printf("%ld", (long)ovr_len(REF->start[r], REF->end[r], MAP->start[m], MAP->end[m]));
        break;
    }
  }
}
static int dcmp(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : (x > y ? 1 : 0);
}
/* RollingKthAverage::DoneReference on the window's sorted scores (RollingKthAverageVisitor.hpp:61-92) */
static double kth_value(double kth) {
  const size_t n = (size_t)VWIN.n;
  double* v = (double*)malloc(n * sizeof(double));
  for (size_t i = 0; i < n; ++i) v[i] = MAP->score[VWIN.v[i]];
  qsort(v, n, sizeof(double), dcmp);
  size_t up = (size_t)ceil(kth * (double)n), down = (size_t)floor(kth * (double)n);
  if (up > 0) --up;
  if (down > 0) --down;
  double r;
  if (n == 1) r = v[0];
  else if (up == down) r = (v[up] + v[up + 1]) / 2.0;
  else r = v[up];
  free(v);
  return r;
}
static void put_kth(double kth) {
  if (VWIN.n == 0) { fputs("NAN", stdout); return; }
  put_real(kth_value(kth));
}
/* MedianAbsoluteDeviation::DoneReference (MedianAbsoluteDeviationVisitor.hpp:70-110) */
static void put_mad(double mult) {
  const size_t n = (size_t)VWIN.n;
  if (n <= 1) { fputs("NAN", stdout); return; }
  const double med = kth_value(0.5);
  double* v = (double*)malloc(n * sizeof(double));
  for (size_t i = 0; i < n; ++i) {
    const double d = MAP->score[VWIN.v[i]] - med;
    v[i] = d < 0 ? -d : d;
  }
  qsort(v, n, sizeof(double), dcmp);
  double mad;
  if (n % 2 == 0) { mad = v[n / 2 - 1]; mad += v[n / 2]; mad /= 2.0; }
  else mad = v[n / 2];
  free(v);
  put_real(mad * mult);
}
static int scmp(const void* a, const void* b) { return strcmp(*(char* const*)a, *(char* const*)b); }
/* PrintUniqueRangeIDs (ProcessBedVisitorRow.hpp:361-385): std::set<std::string> of the ids */
static void put_unique_ids(void) {
  if (VWIN.n == 0) return;
  char** v = (char**)malloc((size_t)VWIN.n * sizeof(char*));
  for (int64_t i = 0; i < VWIN.n; ++i) v[i] = MAP->id[VWIN.v[i]];
  qsort(v, (size_t)VWIN.n, sizeof(char*), scmp);
  for (int64_t i = 0; i < VWIN.n; ++i) {
    if (i && !strcmp(v[i], v[i - 1])) continue;
    if (i) fputs(MULTIDELIM, stdout);
    fputs(v[i], stdout);
  }
  free(v);
}
static unsigned long ROWID; /* PrintRowID's static counter (ProcessBedVisitorRow.hpp:347-355) */
static void v_done(int64_t r) {
  if (SKIP_UNMAPPED && cnt_ == 0) return;
  for (int i = 0; i < NVIS; ++i) {
    if (i) fputs(DELIM, stdout);
    switch (VIS[i]) {
      case V_COUNT: printf("%d", count_); break;
      case V_INDICATOR: printf("%d", count_ > 0 ? 1 : 0); break;
      case V_MEAN:
        if (counter_ > 0) put_real(sum_ / counter_); else fputs("NAN", stdout);
        break;
      case V_SUM:
        if (counter_ > 0) put_real(sum_); else fputs("NAN", stdout);
        break;
      case V_MIN:
      case V_MAX: {
        if (VWIN.n == 0) { fputs("NAN", stdout); break; }
        double b = MAP->score[VWIN.v[0]];
        for (int64_t k = 1; k < VWIN.n; ++k) {
          const double x = MAP->score[VWIN.v[k]];
          if (VIS[i] == V_MIN ? x < b : x > b) b = x;
        }
        put_real(b);
        break;
      }
      case V_BASES: {
        unsigned long o = 0;
        for (int64_t k = 0; k < VWIN.n; ++k) o += ovr_agg(r, VWIN.v[k]);
        printf("%lu", o);
        break;
      }
      case V_BASES_UNIQ: printf("%u", ovr_uniq(i, r)); break;
      case V_BASES_UNIQ_F:
        put_real((double)ovr_uniq(i, r) / (double)(REF->end[r] - REF->start[r]));
        break;
      case V_ECHO:
        if (SINGLE) { print_map_row(r); break; } /* the row as its (map) type prints it */
        printf("%s\t%" PRIu64 "\t%" PRIu64 "%s", POOL.names[REF->chrom[r]], REF->start[r], REF->end[r],
               REF->rest ? REF->rest[r] : "");
        break;
      case V_MIN_EL: case V_MAX_EL: case V_MIN_EL_RAND: case V_MAX_EL_RAND: {
        /* an empty set hands NaN to PrintAllScorePrecision, which throws
         * (ProcessBedVisitorRow.hpp:206-208): bedmap stops with what it printed so far */
        if (VWIN.n == 0) {
          fflush(stdout);
          fputs("May use bedmap --help for more help.\n\nError: Unable to process a 'NAN' with PrintAllScorePrecision.\n", stderr);
          exit(EXIT_FAILURE);
        }
        int64_t b = -1;
        if (VIS[i] == V_MIN_EL || VIS[i] == V_MAX_EL) { /* m_.begin() of the literal set */
          for (int64_t k = 0; k < EXT.n; ++k) {
            const int64_t x = EXT.v[k];
            if (b < 0 || (VIS[i] == V_MIN_EL ? sg_less(x, b) : sg_less(b, x))) b = x;
          }
        } else { /* RandTie picks at random among equal scores: this restatement takes the
                  * set's first (min: lowest address, max: highest) */
          for (int64_t k = 0; k < VWIN.n; ++k) {
            const int64_t x = VWIN.v[k];
            if (b < 0 || (VIS[i] == V_MIN_EL_RAND ? vl_less(x, b) : vl_less(b, x))) b = x;
          }
        }
        print_map_row_p(b, 1);
        break;
      }
      case V_TMEAN: {
        double v;
        if (tm_done(&TM[i], &v)) put_real(v); else fputs("NAN", stdout);
        break;
      }
      case V_WMEAN: { /* WeightedAverage::DoneReference over std::set<MapType*> (address order) */
        if (VWIN.n == 0) { fputs("NAN", stdout); break; }
        int64_t* v = (int64_t*)malloc((size_t)VWIN.n * 8);
        memcpy(v, VWIN.v, (size_t)VWIN.n * 8);
        for (int64_t p = 1; p < VWIN.n; ++p) { /* address order */
          int64_t x = v[p], q = p;
          while (q > 0 && A_(v[q - 1]) > A_(x)) { v[q] = v[q - 1]; --q; }
          v[q] = x;
        }
        double value = 0, weightSum = 0;
        const double len = (double)(REF->end[r] - REF->start[r]);
        for (int64_t p = 0; p < VWIN.n; ++p) {
          const int64_t m = v[p];
          const double w = (double)ovr_len(REF->start[r], REF->end[r], MAP->start[m], MAP->end[m]) / len;
          value += w * MAP->score[m];
          weightSum += w;
        }
        free(v);
        value /= weightSum;
        put_real(value);
        break;
      }
      case V_ECHO_SIZE: printf("%" PRIu64, REF->end[r] - REF->start[r]); break;
      case V_ECHO_MAP_ID_UNIQ: put_unique_ids(); break;
      case V_ECHO_REF_ROW_ID: printf("id-%lu", ++ROWID); break;
      case V_MEDIAN: put_kth(0.5); break;
      case V_KTH: put_kth(VARG[i]); break;
      case V_MAD: put_mad(VARG[i]); break;
      case V_VARIANCE: case V_STDEV: case V_CV: {
        const double count = (double)counter_;
        if (count <= 1) { fputs("NAN", stdout); break; }
        const double numer = (count * sq_) - (sum_ * sum_);
        const double denom = (count * (count - 1));
        double v = numer / denom;
        if (VIS[i] != V_VARIANCE) v = sqrt(v);
        if (VIS[i] == V_CV) {
          const double mean = sum_ / count;
          if (mean == 0) { fputs("NAN", stdout); break; }
          v = v / mean;
        }
        put_real(v);
        break;
      }
      case V_ECHO_MAP: case V_ECHO_MAP_ID: case V_ECHO_MAP_SCORE: case V_ECHO_MAP_SIZE:
      case V_ECHO_OVERLAP_SIZE: case V_ECHO_MAP_RANGE:
        if (NODES_ON && VIS[i] == V_ECHO_OVERLAP_SIZE) heap_intersect_lengths(r);
        if (NODES_ON && VIS[i] == V_ECHO_MAP_RANGE && VWIN.n) { /* PrintGenomicRange's copy, ProcessBedVisitorRow.hpp:446 */
          tmprow_t t;
          tmp_copy(&t, MAP, VWIN.v[0], MAPFIELDS);
          tmp_drop(&t);
        }
        echo_map(VIS[i], r);
        break;
      case V_ECHO_NAME:
        printf("%s:%" PRIu64 "-%" PRIu64, POOL.names[REF->chrom[r]], REF->start[r], REF->end[r]);
        break;
    }
  }
  fputc('\n', stdout);
}

/* PercentOverlapMapping's constructor, BedDistances.hpp:126-136 */
static double parse_frac(const char* v) {
  double p = strtod(v, NULL);
  while (p > 1) p /= 10.0;
  p -= DBL_EPSILON;
  if (p <= 0.0) p = DBL_EPSILON;
  return p;
}

/* the reference's heap traffic for one row object (Bed.hpp constructors / readline /
 * destructors): object; ChromInfo() new char[1]; Bed4() new char[1] (B4/B5); readline
 * re-allocates chrom_ and id_, then rest_ and fullrest_ (B4/B5: id + rest); the destructor
 * frees rest_, fullrest_, id_, chrom_, then the object */
typedef struct { int64_t o, c, i, r, f; size_t lc, li, lr; } rowmem_t;
static void row_new(rowmem_t* x, int fields, size_t lc, size_t li, size_t lr) {
  x->lc = lc; x->li = li; x->lr = lr;
  x->o = hs_malloc(&HS, fields == 3 ? 32 : (fields == 4 ? 48 : 56));
  const int64_t c1 = hs_malloc(&HS, 1);
  const int64_t i1 = fields >= 4 ? hs_malloc(&HS, 1) : 0;
  hs_free(&HS, 1, c1);
  x->c = hs_malloc(&HS, lc + 1);
  if (fields >= 4) { hs_free(&HS, 1, i1); x->i = hs_malloc(&HS, li + 1); }
  x->r = hs_malloc(&HS, lr + 1);
  if (fields >= 4) x->f = hs_malloc(&HS, lr + 1 + li + 1);
}
static void row_del(const rowmem_t* x, int fields) {
  hs_free(&HS, x->lr + 1, x->r);
  if (fields >= 4) { hs_free(&HS, x->lr + 1 + x->li + 1, x->f); hs_free(&HS, x->li + 1, x->i); }
  hs_free(&HS, x->lc + 1, x->c);
  hs_free(&HS, fields == 3 ? 32 : (fields == 4 ? 48 : 56), x->o);
}
static rowmem_t* MMEM;
static rowmem_t RMEM[2];
static void map_new(int64_t m) { /* m == MAP->n: the row read at end of file (never freed) */
  if (m < MAP->n)
    row_new(&MMEM[m], MAPFIELDS, strlen(POOL.names[MAP->chrom[m]]), MAPFIELDS >= 4 ? strlen(MAP->id[m]) : 0,
            MAP->rest ? strlen(MAP->rest[m]) : 0);
  else
    row_new(&MMEM[m], MAPFIELDS, 0, 0, 0);
  ADDR[m] = MMEM[m].o;
}
static void ref_new(int64_t r) {
  if (r < REF->n)
    row_new(&RMEM[r & 1], 3, strlen(POOL.names[REF->chrom[r]]), 0, REF->rest ? strlen(REF->rest[r]) : 0);
  else
    row_new(&RMEM[r & 1], 3, 0, 0, 0);
  REFA[r & 1] = RMEM[r & 1].o;
}

static oset_t vcache, lst, ev, dl;
/* one file under the Overlapping specialisation: rows shorter than the required overlap
 * reach no visitor (WindowSweepImpl.specialize.cpp:66-67, 110-111) */
static int f_visible(int64_t m) { return !SINGLE || CRIT != C_BP || MAP->end[m] - MAP->start[m] >= (FASTER ? OVR : 0); }
/* BedBaseVisitor::OnDelete (:145-154); --faster: MultiVisitor's Delete straight away */
static void on_delete(int64_t m) {
  if (FASTER) {
    if (f_visible(m)) { os_erase(&VWIN, m); v_del(m); }
    return;
  }
  if (os_erase(&VWIN, m)) {
    v_del(m);
    if (NODES_ON) n_free(NWIN, m);
  } else {
    os_erase(&vcache, m);
    if (NODES_ON) n_free(NCACHE, m);
  }
}
/* BedBaseVisitor::OnAdd (:139-143, into its cache); --faster: MultiVisitor's Add */
static void on_add(int64_t m) {
  if (FASTER) {
    if (f_visible(m)) { os_insert(&VWIN, m); v_add(m); }
    return;
  }
  os_insert(&vcache, m);
  if (NODES_ON) n_new(NCACHE, m);
}
/* BedBaseVisitor::OnDone: fixWindow (deletions first, then insertions), then DoneReference;
 * --faster: DoneReference on the window as the sweep left it */
static void on_done(int64_t r) {
  if (FASTER) { v_done(r); return; }
  lst.n = 0;
  ev.n = 0;
  for (int64_t i = 0; i < VWIN.n;) {
    int64_t m = VWIN.v[i];
    if (crit_m2r(m, r) != 0) {
      ev_push(&ev, m);
      os_insert(&lst, m);
      memmove(VWIN.v + i, VWIN.v + i + 1, (size_t)(VWIN.n - i - 1) * 8);
      VWIN.n--;
    } else ++i;
  }
  sort_rless(ev.v, ev.n);
  for (int64_t i = 0; i < ev.n; ++i) {
    v_del(ev.v[i]);
    if (NODES_ON) n_free(NWIN, ev.v[i]); /* Delete, lst.push_back, win_.erase */
  }
  dl.n = 0;
  for (int64_t i = 0; i < ev.n; ++i) ev_push(&dl, ev.v[i]);
  ev.n = 0;
  for (int64_t i = 0; i < vcache.n;) {
    int64_t m = vcache.v[i];
    if (crit_m2r(m, r) == 0) {
      ev_push(&ev, m);
      os_insert(&VWIN, m);
      memmove(vcache.v + i, vcache.v + i + 1, (size_t)(vcache.n - i - 1) * 8);
      vcache.n--;
    } else ++i;
  }
  sort_rless(ev.v, ev.n);
  for (int64_t i = 0; i < ev.n; ++i) {
    v_add(ev.v[i]);
    if (NODES_ON) { n_new(NWIN, ev.v[i]); n_free(NCACHE, ev.v[i]); } /* Add, win_.insert, cache_.erase */
  }
  for (int64_t i = 0; i < lst.n; ++i) os_insert(&vcache, lst.v[i]);
  if (NODES_ON)
    for (int64_t i = 0; i < dl.n; ++i) n_new(NCACHE, dl.v[i]); /* cache_.insert(lst), in list order */
  v_done(r);
}

int main(int argc, char** argv) {
  int a = 1, need5 = 0, need4 = 0, rest = 0;
  const char* only_chrom = NULL;
  const char* dump_addr = NULL;
  static const struct { const char* name; int v; int score; } OPS[] = {
      {"--count", V_COUNT, 0},         {"--mean", V_MEAN, 1},           {"--sum", V_SUM, 1},
      {"--min", V_MIN, 1},             {"--max", V_MAX, 1},             {"--indicator", V_INDICATOR, 0},
      {"--bases", V_BASES, 0},         {"--bases-uniq", V_BASES_UNIQ, 0},
      {"--bases-uniq-f", V_BASES_UNIQ_F, 0},                            {"--echo", V_ECHO, 0},
      {"--echo-ref-size", V_ECHO_SIZE, 0},                              {"--echo-ref-name", V_ECHO_NAME, 0},
      {"--echo-map", V_ECHO_MAP, 0},   {"--echo-map-id", V_ECHO_MAP_ID, 0}, {"--echo-map-score", V_ECHO_MAP_SCORE, 1},
      {"--echo-map-size", V_ECHO_MAP_SIZE, 0}, {"--echo-overlap-size", V_ECHO_OVERLAP_SIZE, 0},
      {"--echo-map-range", V_ECHO_MAP_RANGE, 0}, {"--median", V_MEDIAN, 1},
      {"--variance", V_VARIANCE, 1},   {"--stdev", V_STDEV, 1},         {"--cv", V_CV, 1},
      {"--echo-map-id-uniq", V_ECHO_MAP_ID_UNIQ, 0}, {"--echo-ref-row-id", V_ECHO_REF_ROW_ID, 0},
      {"--min-element", V_MIN_EL, 1}, {"--max-element", V_MAX_EL, 1},
      {"--min-element-rand", V_MIN_EL_RAND, 1}, {"--max-element-rand", V_MAX_EL_RAND, 1},
      {"--wmean", V_WMEAN, 1}};
  while (a < argc - 2 || (a < argc && strncmp(argv[a], "--", 2) == 0)) {
    const char* o = argv[a++];
    int found = 0;
    for (size_t k = 0; k < sizeof(OPS) / sizeof(OPS[0]); ++k)
      if (!strcmp(o, OPS[k].name)) {
        VIS[NVIS++] = OPS[k].v;
        need5 |= OPS[k].score;
        if (OPS[k].v == V_ECHO_MAP_ID || OPS[k].v == V_ECHO_MAP_ID_UNIQ) need4 = 1;
        rest |= OPS[k].v == V_ECHO;
        found = 1;
      }
    if (found) continue;
    if (!strcmp(o, "--mad")) { /* optional multiplier when the next argument is all reals (Input.hpp:275-288) */
      VARG[NVIS] = 1.0;
      if (a < argc && argv[a][0] && strspn(argv[a], ".-0123456789") == strlen(argv[a])) VARG[NVIS] = strtod(argv[a++], NULL);
      VIS[NVIS++] = V_MAD;
      need5 = 1;
      continue;
    }
    if (!strcmp(o, "--tmean") && a + 1 < argc) {
      const double lo = strtod(argv[a], NULL), hi = strtod(argv[a + 1], NULL);
      a += 2;
      tm_init(&TM[NVIS], lo, hi);
      VIS[NVIS++] = V_TMEAN;
      need5 = 1;
      continue;
    }
    if (!strcmp(o, "--kth") && a < argc) {
      VARG[NVIS] = strtod(argv[a++], NULL);
      VIS[NVIS++] = V_KTH;
      need5 = 1;
      continue;
    }
    if (!strcmp(o, "--bp-ovr") && a < argc) { CRIT = C_BP; OVR = strtoull(argv[a++], 0, 10); }
    else if (!strcmp(o, "--range") && a < argc) {
      RANGE = strtoull(argv[a++], 0, 10);
      if (RANGE == 0) { CRIT = C_BP; OVR = 1; } /* --range 0 == --bp-ovr 1, Input.hpp:165-171 */
      else CRIT = C_RANGE;
    }
    else if (!strcmp(o, "--fraction-ref") && a < argc) { CRIT = C_FREF; PERC = parse_frac(argv[a++]); }
    else if (!strcmp(o, "--fraction-map") && a < argc) { CRIT = C_FMAP; PERC = parse_frac(argv[a++]); }
    else if (!strcmp(o, "--fraction-either") && a < argc) { CRIT = C_FEITHER; PERC = parse_frac(argv[a++]); }
    else if (!strcmp(o, "--fraction-both") && a < argc) { CRIT = C_FBOTH; PERC = parse_frac(argv[a++]); }
    else if (!strcmp(o, "--exact")) CRIT = C_EXACT;
    else if (!strcmp(o, "--delim") && a < argc) DELIM = argv[a++];
    else if (!strcmp(o, "--multidelim") && a < argc) MULTIDELIM = argv[a++];
    else if (!strcmp(o, "--prec") && a < argc) PREC = atoi(argv[a++]);
    else if (!strcmp(o, "--chrom") && a < argc) only_chrom = argv[a++];
    else if (!strcmp(o, "--sci")) SCI = 1;
    else if (!strcmp(o, "--skip-unmapped")) SKIP_UNMAPPED = 1;
    else if (!strcmp(o, "--faster")) FASTER = 1;
    else if (!strcmp(o, "--dump-addr") && a < argc) dump_addr = argv[a++]; /* the replayed addresses */
    else if (!strcmp(o, "--ec") || !strcmp(o, "--header") || !strcmp(o, "--sweep-all")) {}
    else { fprintf(stderr, "bedmap_oracle: unsupported option %s\n", o); return 2; }
  }
  const int nfiles = argc - a;
  if (NVIS == 0 || nfiles < 1 || nfiles > 2) { fprintf(stderr, "bedmap_oracle: bad usage\n"); return 2; }
  SINGLE = nfiles == 1;
  static bedfile_t ref, map;
  FILE* fr = open_input(argv[a]);
  FILE* fm = SINGLE ? NULL : open_input(argv[a + 1]);
  if (!fr || (!SINGLE && !fm)) { fprintf(stderr, "bedmap_oracle: cannot open input\n"); return 2; }
  MAPFIELDS = need5 ? 5 : (need4 ? 4 : 3);
  if (!SINGLE) {
    read_bed3(fr, &POOL, &ref, 1); /* rest_ kept for --echo and for its heap size */
    (void)rest;
    fr = fm;
  }
  if (need5) read_bed5(fr, &POOL, &map);
  else if (need4) read_bed4(fr, &POOL, &map);
  else read_bed3(fr, &POOL, &map, 1);
  if (only_chrom) {
    bedfile_t* fs[2] = {&ref, &map};
    for (int q = SINGLE ? 1 : 0; q < 2; ++q) {
      bedfile_t* f = fs[q];
      int64_t k = 0;
      for (int64_t j = 0; j < f->n; ++j) {
        if (strcmp(POOL.names[f->chrom[j]], only_chrom) != 0) continue;
        f->chrom[k] = f->chrom[j]; f->start[k] = f->start[j]; f->end[k] = f->end[j];
        if (f->score) f->score[k] = f->score[j];
        if (f->rest) f->rest[k] = f->rest[j];
        if (f->id) f->id[k] = f->id[j];
        ++k;
      }
      f->n = k;
    }
  }
  REF = SINGLE ? &map : &ref;
  MAP = &map;
  nodes_init(map.n);
  static char obuf[1 << 20];
  setvbuf(stdout, obuf, _IOFBF, sizeof(obuf));

  int64_t* win = (int64_t*)malloc(sizeof(int64_t) * (size_t)(map.n + 1));
  if (SINGLE) { /* sweep() overload 1, WindowSweepImpl.cpp:66-162 */
    int64_t wh = 0, wt = 0, index = 0, next = 0, cache = -1, cur = -1;
    int reset = 1;
    /* heap addresses: the iterator reads one row ahead (its constructor reads row 0, each
     * ++start the next); the sweep deletes rows as they leave the deque */
    ADDR = (int64_t*)calloc((size_t)map.n + 1, sizeof(int64_t));
    MMEM = (rowmem_t*)calloc((size_t)map.n + 1, sizeof(rowmem_t));
    map_new(0);
    for (;;) {
      if (!(next < map.n || cache >= 0 || wt > wh)) break;
      if (!reset) {
        cur = win[wh + index]; /* OnStart */
        while (wt > wh && sweep_m2r(win[wh], cur) < 0) {
          on_delete(win[wh]);
          row_del(&MMEM[win[wh]], MAPFIELDS);
          ++wh;
          --index;
        }
      } else if (next >= map.n && cache < 0) {
        break; /* OnEnd; the rest of the window is deleted on behalf of no reference */
      }
      while (cache >= 0 || next < map.n) {
        int64_t b;
        if (cache >= 0) { b = cache; cache = -1; }
        else { b = next++; map_new(next); } /* ++start */
        if (wt == wh || reset || sweep_r2m(win[wh + index], b) == 0) {
          if (reset) {
            reset = 0;
            index = 0;
            cur = b; /* OnStart(bPtr) */
            while (wt > wh) { on_delete(win[wh]); row_del(&MMEM[win[wh]], MAPFIELDS); ++wh; }
          }
          win[wt++] = b;
          on_add(b); /* OnAdd */
        } else {
          cache = b;
          break;
        }
      }
      on_done(cur);
      reset = ++index >= wt - wh;
    }
  } else {
    /* sweep() overload 2 with the sweep distance; fixWindow with the visitor distance */
    int64_t wh = 0, wt = 0; /* deque [wh, wt) */
    int64_t mi = 0, cache = -1;
    /* heap addresses: the iterators read one row ahead (ref first, Bedmap.cpp:282-284) */
    ADDR = (int64_t*)calloc((size_t)map.n + 1, sizeof(int64_t));
    MMEM = (rowmem_t*)calloc((size_t)map.n + 1, sizeof(rowmem_t));
    ref_new(0);
    map_new(0);
    for (int64_t r = 0; r < ref.n; ++r) {
      ref_new(r + 1); /* ++refStart */
      while (wt > wh && sweep_m2r(win[wh], r) < 0) { on_delete(win[wh]); row_del(&MMEM[win[wh]], MAPFIELDS); ++wh; }
      while (cache >= 0 || mi < map.n) {
        int64_t m;
        if (cache >= 0) { m = cache; cache = -1; }
        else { m = mi++; map_new(mi); } /* ++mapFromStart */
        int v = sweep_r2m(r, m);
        if (v == 0) { win[wt++] = m; on_add(m); } /* OnAdd -> cache_ */
        else if (v < 0) { cache = m; break; }
        else row_del(&MMEM[m], MAPFIELDS);
      }
      on_done(r);
      row_del(&RMEM[r & 1], 3); /* delete rPtr */
    }
  }
  fflush(stdout);
  if (dump_addr) {
    FILE* fa = fopen(dump_addr, "w");
    if (!fa) return 2;
    for (int64_t m = 0; m < map.n; ++m) fprintf(fa, "%" PRId64 "\n", ADDR[m]);
    fclose(fa);
  }
  return 0;
}
