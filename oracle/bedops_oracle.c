/*
 * oracle/bedops_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C) of the reference `bedops` sweep: the hot-path modes
 * --merge, --intersect, --difference, --element-of, --not-element-of, and the
 * remaining operations --complement, --chop, --symmdiff, --partition, --everything
 * with --range padding.
 * Used only by tests/ (parity checker), __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg. It is never linked into libbedgpu or the bedops_amd CLIs.
 *
 * It restates the reference's streaming control flow (not just the set semantics),
 * so zero-length rows, duplicates, nesting and adjacency behave exactly as in the
 * reference:
 *   reader with LIFO push-back ............ applications/bed/bedops/src/BedPadReader.hpp:87-167
 *   getNextFileMergedCoords ............... applications/bed/bedops/src/Bedops.cpp:791-814
 *   mergeOverlap .......................... Bedops.cpp:864-886
 *   intersectOverlap ...................... Bedops.cpp:855-859
 *   nextMergeAllLines (k-way union) ....... Bedops.cpp:1186-1243
 *   nextIntersectLine ..................... Bedops.cpp:1105-1181
 *   nextDifferenceLine / doDifference ..... Bedops.cpp:950-1018 / :500-524
 *   nextElementOfLine / doElementOf ....... Bedops.cpp:1023-1100 / :538-566
 *   threshold parsing (-e/-n N | P%) ...... applications/bed/bedops/src/Input.hpp:344-382
 * Parity of this restatement is pinned by the reference's own KATs
 * (applications/bed/bedops/test/TestPlan.xml, via tests/golden/testplan.json) and by
 * the reference output hashes recorded in SURVEY.md Appendix D (tests/test_oracle.py).
 *
 * usage: bedops_oracle [--ec] [--chrom C] [--range L:R|S]
 *            <-m|-i|-d|-e [N|P%]|-n [N|P%]|-c [-L]|-w [bp] [--stagger nt] [-x]|-s|-p|-u>
 *            file1 [file2 ...]
 */
#include "bedio.h"

static chrom_pool_t POOL;

typedef struct {
  int chrom;
  uint64_t start, end;
  int64_t row; /* source row (for the element-of "rest" column) */
  uint64_t id; /* object identity: the address tie-break of GenomicAddressCompare */
} rec_t;

static uint64_t NEXT_ID = 1;

typedef struct {
  const bedfile_t* f;
  int64_t pos;
  rec_t* stk;
  int sp, cap;
} reader_t;

static int rd_has(const reader_t* r) { return r->sp > 0 || r->pos < r->f->n; }
static int rd_read(reader_t* r, rec_t* out) {
  if (r->sp > 0) { *out = r->stk[--r->sp]; return 1; }
  if (r->pos >= r->f->n) return 0;
  out->chrom = r->f->chrom[r->pos];
  out->start = r->f->start[r->pos];
  out->end = r->f->end[r->pos];
  out->row = r->pos;
  out->id = NEXT_ID++;
  r->pos++;
  return 1;
}
static void rd_push(reader_t* r, const rec_t* x) {
  if (r->sp == r->cap) {
    r->cap = r->cap ? 2 * r->cap : 16;
    r->stk = (rec_t*)realloc(r->stk, (size_t)r->cap * sizeof(rec_t));
  }
  r->stk[r->sp++] = *x;
}

static int chrcmp(int a, int b) { return a == b ? 0 : strcmp(POOL.names[a], POOL.names[b]); }

static void emit3(const rec_t* x) {
  printf("%s\t%" PRIu64 "\t%" PRIu64 "\n", POOL.names[x->chrom], x->start, x->end);
}

/* mergeOverlap(p1, p2): union of two rows if they overlap or touch (Bedops.cpp:864-886) */
static int merge_pair(const rec_t* p1, const rec_t* p2, rec_t* out) {
  if (chrcmp(p1->chrom, p2->chrom) != 0) return 0;
  if (p1->start < p2->start) {
    if (p1->end < p2->start) return 0;
    *out = *p1;
  } else if (p1->start > p2->start) {
    if (p2->end < p1->start) return 0;
    *out = *p2;
  } else {
    *out = *p1;
  }
  out->end = p1->end > p2->end ? p1->end : p2->end;
  return 1;
}

/* getNextFileMergedCoords: next within-file merged piece (Bedops.cpp:791-814) */
static int next_file_merged(reader_t* r, rec_t* out) {
  rec_t cur, nx, m;
  if (!rd_read(r, &cur)) return 0;
  while (rd_has(r)) {
    rd_read(r, &nx);
    if (merge_pair(&nx, &cur, &m)) {
      cur = m;
    } else {
      rd_push(r, &nx);
      break;
    }
  }
  *out = cur;
  return 1;
}

/* nextMergeAllLines(lo, hi): next component of the union of files [lo,hi)
 * (Bedops.cpp:1186-1243). */
static int next_merge_all(reader_t* rd, int lo, int hi, rec_t* out) {
  int best = -1;
  rec_t bt, cur;
  for (int i = lo; i < hi; ++i) {
    if (!rd_has(&rd[i])) continue;
    rd_read(&rd[i], &bt);
    rd_push(&rd[i], &bt);
    if (best < 0) { best = i; cur = bt; continue; }
    int v = chrcmp(bt.chrom, cur.chrom);
    if (v < 0 || (v == 0 && bt.start < cur.start)) { best = i; cur = bt; }
  }
  if (best < 0) return 0;
  rd_read(&rd[best], &cur);
  for (int i = lo; i < hi; ++i) {
    if (!rd_has(&rd[i])) continue;
    int have = rd_read(&rd[i], &bt), v = 0;
    /* absorb rows ending inside the current piece */
    while ((v = chrcmp(bt.chrom, cur.chrom)) == 0 && bt.end <= cur.end) {
      have = rd_read(&rd[i], &bt);
      if (!have) break;
    }
    if (have && v == 0 && bt.start <= cur.end && bt.end > cur.end) {
      cur.end = bt.end; /* grew: rescan every file */
      i = lo - 1;
    } else if (have) {
      rd_push(&rd[i], &bt);
    }
  }
  *out = cur;
  return 1;
}

/* nextIntersectLine (Bedops.cpp:1105-1181) */
static int next_intersect(reader_t* rd, int nf, rec_t* out) {
  rec_t best, nx;
  int have_best = 0;
  for (int i = 0; i < nf; ++i) { /* the greatest of the per-file next merged pieces */
    if (!rd_has(&rd[i])) return 0;
    next_file_merged(&rd[i], &nx);
    rd_push(&rd[i], &nx);
    if (!have_best) { best = nx; have_best = 1; continue; }
    int v = chrcmp(nx.chrom, best.chrom);
    if ((v == 0 && nx.start > best.start) || v > 0) best = nx;
  }
  rec_t cur = best;
  int marker = -1;
  uint64_t minEnd = UINT64_MAX;
  for (int i = 0; i < nf; ++i) {
    if (!rd_has(&rd[i])) return 0;
    next_file_merged(&rd[i], &nx);
    int v = chrcmp(nx.chrom, cur.chrom);
    while (v < 0 || (v == 0 && nx.end <= cur.start)) { /* skip pieces left of cur */
      if (!next_file_merged(&rd[i], &nx)) return 0;
      v = chrcmp(nx.chrom, cur.chrom);
    }
    rd_push(&rd[i], &nx);
    if (v > 0 || nx.start >= cur.end) { /* no overlap: restart from this piece */
      cur = nx;
      i = -1;
      marker = -1;
      minEnd = UINT64_MAX;
      continue;
    }
    /* intersectOverlap (Bedops.cpp:855-859); overlap is guaranteed here */
    uint64_t lo = cur.start > nx.start ? cur.start : nx.start;
    uint64_t hi = cur.end < nx.end ? cur.end : nx.end;
    cur.start = lo;
    cur.end = hi;
    if (nx.end < minEnd) { minEnd = nx.end; marker = i; }
  }
  next_file_merged(&rd[marker], &nx); /* consume the piece that ends first */
  *out = cur;
  return 1;
}

/* nextDifferenceLine state machine (Bedops.cpp:950-1018), driven like doDifference
 * (Bedops.cpp:500-524). Returns: 0 stop, 1 emit *out, 2 call again. */
typedef struct {
  int has_ref, has_non;
  rec_t ref, non;
} diff_state_t;

static int next_difference(reader_t* rd, int nf, diff_state_t* st, rec_t* out) {
  if (!st->has_ref && !rd_has(&rd[0])) return 0;
  if (!st->has_non) {
    if (!st->has_ref) st->has_ref = next_file_merged(&rd[0], &st->ref);
    if (!st->has_ref) return 0;
    *out = st->ref;
    st->has_ref = 0;
    return 1;
  }
  if (!st->has_ref) st->has_ref = next_file_merged(&rd[0], &st->ref);
  if (!st->has_ref) return 0;
  int v = chrcmp(st->non.chrom, st->ref.chrom);
  while (v < 0 || (v == 0 && st->non.end <= st->ref.start)) {
    st->has_non = next_merge_all(rd, 1, nf, &st->non);
    if (!st->has_non) { *out = st->ref; st->has_ref = 0; return 1; }
    v = chrcmp(st->non.chrom, st->ref.chrom);
  }
  if (v > 0 || st->non.start >= st->ref.end) { /* no overlap with the reference piece */
    *out = st->ref;
    st->has_ref = 0;
    return 1;
  }
  if (st->non.start <= st->ref.start && st->non.end >= st->ref.end) { /* fully covered */
    st->has_ref = next_file_merged(&rd[0], &st->ref);
    return 2;
  }
  if (st->non.start > st->ref.start) { /* piece up to the covering start */
    *out = st->ref;
    out->end = st->non.start;
    st->ref.start = st->non.end;
    v = 0;
    while (v == 0 && st->non.end >= st->ref.end) {
      st->has_ref = next_file_merged(&rd[0], &st->ref);
      if (!st->has_ref) break;
      v = chrcmp(st->non.chrom, st->ref.chrom);
    }
    return 1;
  }
  st->ref.start = st->non.end; /* clip the reference piece from the left */
  return 2;
}

static void do_difference(reader_t* rd, int nf) {
  diff_state_t st;
  memset(&st, 0, sizeof(st));
  st.has_non = next_merge_all(rd, 1, nf, &st.non);
  rec_t o;
  for (;;) {
    int r = next_difference(rd, nf, &st, &o);
    if (r == 0) break;
    if (r == 1) emit3(&o);
  }
}

/* merged non-reference pieces with LIFO re-use, as the std::deque mergeList of
 * doElementOf (Bedops.cpp:538-566, getNextMerge :832-842) */
typedef struct {
  rec_t* q;
  int64_t head, tail, cap; /* ring buffer */
} deque_t;
static int64_t dq_size(const deque_t* d) { return d->tail - d->head; }
static void dq_grow(deque_t* d) {
  int64_t n = dq_size(d), nc = d->cap ? 2 * d->cap : 64;
  rec_t* q = (rec_t*)malloc((size_t)nc * sizeof(rec_t));
  for (int64_t i = 0; i < n; ++i) q[i] = d->q[(d->head + i) % d->cap];
  free(d->q);
  d->q = q; d->head = 0; d->tail = n; d->cap = nc;
}
static void dq_push_back(deque_t* d, const rec_t* x) {
  if (dq_size(d) == d->cap) dq_grow(d);
  d->q[d->tail % d->cap] = *x;
  d->tail++;
}
static void dq_push_front(deque_t* d, const rec_t* x) {
  if (dq_size(d) == d->cap) dq_grow(d);
  if (d->head == 0) { d->head += d->cap; d->tail += d->cap; }
  d->head--;
  d->q[d->head % d->cap] = *x;
}
static int dq_pop_front(deque_t* d, rec_t* x) {
  if (!dq_size(d)) return 0;
  *x = d->q[d->head % d->cap];
  d->head++;
  return 1;
}

static int get_next_merge(deque_t* d, reader_t* rd, int nf, rec_t* out) {
  if (dq_pop_front(d, out)) return 1;
  return next_merge_all(rd, 1, nf, out);
}

/* doElementOf / nextElementOfLine (Bedops.cpp:538-566, 1023-1100) */
static void do_element_of(reader_t* rd, int nf, const bedfile_t* ref, double thres, int use_pct,
                          int invert) {
  deque_t dq;
  memset(&dq, 0, sizeof(dq));
  rec_t first;
  if (next_merge_all(rd, 1, nf, &first)) dq_push_back(&dq, &first);
  rec_t* topush = NULL;
  int64_t tpcap = 0;
  for (int64_t ri = 0; ri < ref->n; ++ri) {
    rec_t r = {ref->chrom[ri], ref->start[ri], ref->end[ri], ri};
    int keep; /* decision for this reference row */
    rec_t m;
    if (!get_next_merge(&dq, rd, nf, &m)) {
      keep = invert; /* nothing left to be an element of */
    } else {
      int v = chrcmp(m.chrom, r.chrom), exhausted = 0;
      while (v < 0 || (v == 0 && m.end <= r.start)) {
        if (!get_next_merge(&dq, rd, nf, &m)) { exhausted = 1; break; }
        v = chrcmp(m.chrom, r.chrom);
      }
      if (exhausted) {
        keep = invert;
      } else {
        double overlap = 0, range = (double)(r.end - r.start);
        int64_t np = 0;
        if (np == tpcap) { tpcap = tpcap ? 2 * tpcap : 64; topush = (rec_t*)realloc(topush, (size_t)tpcap * sizeof(rec_t)); }
        topush[np++] = m;
        for (;;) {
          if (v > 0 || m.start >= r.end) break;
          uint64_t lo = m.start > r.start ? m.start : r.start;
          uint64_t hi = m.end < r.end ? m.end : r.end;
          /* intersectOverlap; NADA_NOTHING=(1,0) adds (uint64)(0-1) (unreachable here) */
          overlap += (hi >= lo) ? (double)(hi - lo) : (double)(uint64_t)(0ULL - 1ULL);
          if (!get_next_merge(&dq, rd, nf, &m)) break;
          if (np == tpcap) { tpcap = 2 * tpcap; topush = (rec_t*)realloc(topush, (size_t)tpcap * sizeof(rec_t)); }
          topush[np++] = m;
          v = chrcmp(m.chrom, r.chrom);
        }
        if (dq_size(&dq) == 0) {
          for (int64_t k = 0; k < np; ++k) dq_push_back(&dq, &topush[k]);
        } else {
          for (int64_t k = np - 1; k >= 0; --k) dq_push_front(&dq, &topush[k]);
        }
        int is_el = use_pct ? (overlap / range >= thres) : (overlap >= thres);
        keep = invert ? !is_el : is_el;
      }
    }
    if (keep)
      printf("%s\t%" PRIu64 "\t%" PRIu64 "%s\n", POOL.names[r.chrom], r.start, r.end, ref->rest[ri]);
  }
  free(topush);
  free(dq.q);
}

/* ------------------------------------------------------------------------------------
 * The remaining bedops operations, restated from the same
 * streaming control flow so that zero-length rows, ties and padding behave as in
 * the reference:
 *   --range L:R / S padding ............... BedPadReader.hpp:71-284 (ReadLine :109-167,
 *                                           getFirst :194-277), Input.hpp:86-127
 *   --complement [-L] ..................... Bedops.cpp:475-489 (doComplement),
 *                                           :891-945 (nextComplementLine)
 *   --chop [bp] [--stagger nt] [-x] ....... Bedops.cpp:437-467 (doChop), Input.hpp:224-258
 *   --symmdiff ............................ Bedops.cpp:697-747, :1343-1467
 *   --partition ........................... Bedops.cpp:614-686, :1249-1337
 *   --everything .......................... Bedops.cpp:752-786, :1472-1518
 * ------------------------------------------------------------------------------------ */

/* --range padding as a pure transform of one file's row stream (BedPadReader.hpp).
 * The reader consumes rows strictly in order, so applying it up front is the same
 * stream the sweep sees. Arithmetic mirrors the reference's types: uint64 coordinates,
 * int pads, the vaporise tests in double (:134) or uint64 (:212). */
typedef struct {
  int chrom;
  uint64_t start, end;
  int64_t row, ord;
} prow_t;

static int prow_cmp(const void* a, const void* b) { /* GenomicCompare, stable by ord */
  const prow_t* x = (const prow_t*)a;
  const prow_t* y = (const prow_t*)b;
  int v = chrcmp(x->chrom, y->chrom);
  if (v) return v;
  if (x->start != y->start) return x->start < y->start ? -1 : 1;
  if (x->end != y->end) return x->end < y->end ? -1 : 1;
  return x->ord < y->ord ? -1 : (x->ord > y->ord);
}

typedef struct {
  prow_t* v;
  int64_t n, cap;
} prows_t;

static void prows_add(prows_t* p, int c, uint64_t s, uint64_t e, int64_t row) {
  if (p->n == p->cap) {
    p->cap = p->cap ? 2 * p->cap : 1024;
    p->v = (prow_t*)realloc(p->v, (size_t)p->cap * sizeof(prow_t));
  }
  prow_t r = {c, s, e, row, p->n};
  p->v[p->n++] = r;
}

/* getFirst (BedPadReader.hpp:194-277): rows with start <= |lpad| are clamped to 0 (or
 * vaporised), until the first row with a larger start that survives; the group is
 * re-sorted (ties keep input order) and handed out first. */
static int64_t pad_get_first(const bedfile_t* f, int64_t i, int lpad, int rpad, prows_t* out,
                             int* last_chr) {
  const uint64_t lpd = (uint64_t)(lpad < 0 ? -(int64_t)lpad : lpad);
  prows_t g = {0};
  while (i < f->n) {
    int c = f->chrom[i];
    uint64_t s = f->start[i], e = f->end[i];
    int64_t row = i++;
    if (s > lpd) {
      s -= lpd;
      if (e + (uint64_t)(int64_t)rpad > s) { /* uint64 arithmetic, as the reference */
        prows_add(&g, c, s, e + (uint64_t)(int64_t)rpad, row);
        break;
      }
      continue; /* vaporised (lpad < 0 and rpad < lpad) */
    }
    if ((double)e + rpad <= 0) continue;
    prows_add(&g, c, 0, e + (uint64_t)(int64_t)rpad, row);
  }
  qsort(g.v, (size_t)g.n, sizeof(prow_t), prow_cmp);
  for (int64_t k = 0; k < g.n; ++k) {
    prows_add(out, g.v[k].chrom, g.v[k].start, g.v[k].end, g.v[k].row);
    *last_chr = g.v[k].chrom;
  }
  free(g.v);
  return i;
}

static void pad_file(bedfile_t* f, int lpad, int rpad) {
  if (lpad == 0 && rpad == 0) return;
  prows_t o = {0};
  int last_chr = -1;
  int64_t i = 0;
  if (lpad < 0) i = pad_get_first(f, i, lpad, rpad, &o, &last_chr); /* constructor :79-81 */
  while (i < f->n) {
    int c = f->chrom[i];
    uint64_t s = f->start[i], e = f->end[i];
    if (rpad < 0 || lpad > 0) { /* :127-136 (start may wrap: then it vaporises) */
      uint64_t s2 = s + (uint64_t)(int64_t)lpad;
      if ((double)e + rpad > (double)s2) prows_add(&o, c, s2, e + (uint64_t)(int64_t)rpad, i);
      ++i;
    } else if (lpad < 0) { /* :137-149 */
      if (c != last_chr) {
        i = pad_get_first(f, i, lpad, rpad, &o, &last_chr);
      } else {
        prows_add(&o, c, s - (uint64_t)(-(int64_t)lpad), e + (uint64_t)(int64_t)rpad, i);
        ++i;
      }
    } else { /* rpad > 0, lpad == 0 (:150-155) */
      prows_add(&o, c, s, e + (uint64_t)(int64_t)rpad, i);
      ++i;
    }
  }
  bedfile_t g;
  memset(&g, 0, sizeof(g));
  for (int64_t k = 0; k < o.n; ++k)
    bf_push(&g, o.v[k].chrom, o.v[k].start, o.v[k].end, f->rest ? f->rest[o.v[k].row] : NULL,
            f->rest != NULL, f->score ? f->score[o.v[k].row] : 0.0, f->score != NULL);
  free(o.v);
  *f = g; /* the original arrays are leaked: the oracle is a one-shot process */
}

/* doComplement / nextComplementLine (Bedops.cpp:475-489, :891-945) */
static void do_complement(reader_t* rd, int nf, int full_left) {
  rec_t last, nx;
  int have_last = 0;
  for (;;) {
    if (!have_last) {
      if (!next_merge_all(rd, 0, nf, &last)) return;
      have_last = 1;
      if (full_left && last.start != 0) { /* new chromosome: gap from base 0 */
        rec_t t = last;
        t.start = 0;
        t.end = last.start;
        emit3(&t);
        continue;
      }
    }
    if (!next_merge_all(rd, 0, nf, &nx)) return;
    if (chrcmp(nx.chrom, last.chrom) != 0) {
      last = nx;
      if (full_left && last.start != 0) {
        rec_t t = last;
        t.start = 0;
        t.end = last.start;
        emit3(&t);
      }
      continue;
    }
    rec_t g = last;
    g.start = last.end;
    g.end = nx.start;
    emit3(&g);
    last = nx;
  }
}

/* doChop (Bedops.cpp:437-467) over the merged components */
static void do_chop(reader_t* rd, int nf, uint64_t chunk, uint64_t stagger, int exclude_short) {
  rec_t r;
  while (next_merge_all(rd, 0, nf, &r)) {
    for (uint64_t i = r.start; i < r.end;) {
      rec_t c = r;
      c.start = i;
      c.end = i + chunk;
      if (c.end > r.end) {
        if (exclude_short) break;
        c.end = r.end;
      }
      emit3(&c);
      i += stagger ? stagger : chunk;
    }
  }
}

/* nextSymmetricDiffLine (Bedops.cpp:1343-1467). Returns 0 (nothing left),
 * 1 (*out is the next piece) or 2 (call again). */
static int next_symmdiff(reader_t* rd, int nf, int* all_mins, int* all_next, rec_t* out) {
  rec_t mn, next, look, b;
  int have_min = 0, have_next = 0, nm = 0, nn = 0;
  for (int i = 0; i < nf; ++i) {
    if (!rd_has(&rd[i])) continue;
    if (!have_min) {
      next_file_merged(&rd[i], &mn);
      rd_push(&rd[i], &mn);
      have_min = 1;
      have_next = 0;
      nn = 0;
      nm = 0;
      all_mins[nm++] = i;
      continue;
    }
    next_file_merged(&rd[i], &look);
    rd_push(&rd[i], &look);
    int v = chrcmp(look.chrom, mn.chrom);
    if (v > 0) continue;
    if (v < 0) {
      mn = look;
      have_next = 0;
      nn = 0;
      nm = 0;
      all_mins[nm++] = i;
      continue;
    }
    if (look.start < mn.start) {
      next = mn;
      have_next = 1;
      memcpy(all_next, all_mins, (size_t)nm * sizeof(int));
      nn = nm;
      nm = 0;
      mn = look;
      all_mins[nm++] = i;
    } else if (look.start == mn.start) {
      all_mins[nm++] = i;
    } else if (!have_next || look.start < next.start) {
      nn = 0;
      all_next[nn++] = i;
      next = look;
      have_next = 1;
    } else if (look.start == next.start) {
      all_next[nn++] = i;
    }
  }
  if (nm == 0) return 0;
  uint64_t min_second = UINT64_MAX, next_first = UINT64_MAX;
  for (int x = 0; x < nm; ++x) {
    rd_read(&rd[all_mins[x]], &b);
    rd_push(&rd[all_mins[x]], &b);
    if (b.end < min_second) min_second = b.end;
  }
  if (nn) {
    rd_read(&rd[all_next[0]], &b);
    rd_push(&rd[all_next[0]], &b);
    if (b.start < next_first) next_first = b.start;
  }
  if (nm == 1 && nn == 0) { /* case 1 */
    rd_read(&rd[all_mins[0]], out);
    return 1;
  }
  if (nn == 0) { /* case 2: the shared prefix is covered by several files */
    for (int x = 0; x < nm; ++x) {
      rd_read(&rd[all_mins[x]], &b);
      if (min_second != b.end) {
        b.start = min_second;
        rd_push(&rd[all_mins[x]], &b);
      }
    }
    return 2;
  }
  if (nm == 1) { /* case 3 */
    rd_read(&rd[all_mins[0]], &b);
    if (min_second > next_first) {
      rec_t c = b;
      c.id = NEXT_ID++;
      c.end = next_first;
      b.start = next_first;
      rd_push(&rd[all_mins[0]], &b);
      *out = c;
    } else {
      *out = b;
    }
    return 1;
  }
  if (min_second > next_first) { /* case 4 */
    for (int x = 0; x < nm; ++x) {
      rd_read(&rd[all_mins[x]], &b);
      b.start = next_first;
      rd_push(&rd[all_mins[x]], &b);
    }
  } else {
    for (int x = 0; x < nm; ++x) {
      rd_read(&rd[all_mins[x]], &b);
      if (b.end != min_second) {
        b.start = min_second;
        rd_push(&rd[all_mins[x]], &b);
      }
    }
  }
  return 2;
}

/* doSymmetricDifference (Bedops.cpp:697-747): pieces are joined with mergeOverlap */
static void do_symmdiff(reader_t* rd, int nf) {
  int* all_mins = (int*)malloc((size_t)nf * sizeof(int));
  int* all_next = (int*)malloc((size_t)nf * sizeof(int));
  int first = 1, have_rec = 0;
  rec_t to_record, o, ov;
  for (;;) {
    int r = next_symmdiff(rd, nf, all_mins, all_next, &o);
    if (r == 0) {
      if (!first) emit3(&to_record);
      break;
    }
    if (r == 2) continue;
    if (!have_rec || chrcmp(to_record.chrom, o.chrom) != 0) {
      if (!first && have_rec) emit3(&to_record);
      to_record = o;
      have_rec = 1;
    } else if (!merge_pair(&o, &to_record, &ov)) {
      if (!first) emit3(&to_record);
      to_record = o;
    } else {
      to_record = ov;
    }
    first = 0;
  }
  free(all_mins);
  free(all_next);
}

/* std::priority_queue with GenomicAddressCompare (max first) or its inverse (min
 * first); the address tie-break is the record identity (Bedops.cpp:158-176,
 * BedCompare.hpp:50-74). */
typedef struct {
  rec_t* a;
  int64_t n, cap;
  int min_first;
} heap_t;

static int ga_less(const rec_t* x, const rec_t* y) {
  int v = chrcmp(x->chrom, y->chrom);
  if (v) return v < 0;
  if (x->start != y->start) return x->start < y->start;
  if (x->end != y->end) return x->end < y->end;
  return x->id < y->id;
}
/* "x belongs above y" */
static int hp_above(const heap_t* h, const rec_t* x, const rec_t* y) {
  return h->min_first ? ga_less(x, y) : ga_less(y, x);
}
static void hp_push(heap_t* h, const rec_t* x) {
  if (h->n == h->cap) {
    h->cap = h->cap ? 2 * h->cap : 64;
    h->a = (rec_t*)realloc(h->a, (size_t)h->cap * sizeof(rec_t));
  }
  int64_t k = h->n++;
  while (k > 0) {
    int64_t p = (k - 1) / 2;
    if (!hp_above(h, x, &h->a[p])) break;
    h->a[k] = h->a[p];
    k = p;
  }
  h->a[k] = *x;
}
static rec_t* hp_top(heap_t* h) { return &h->a[0]; }
static void hp_pop(heap_t* h, rec_t* out) {
  if (out) *out = h->a[0];
  rec_t x = h->a[--h->n];
  int64_t k = 0;
  for (;;) {
    int64_t c = 2 * k + 1;
    if (c >= h->n) break;
    if (c + 1 < h->n && hp_above(h, &h->a[c + 1], &h->a[c])) ++c;
    if (!hp_above(h, &h->a[c], &x)) break;
    h->a[k] = h->a[c];
    k = c;
  }
  if (h->n) h->a[k] = x;
}

/* nextPartitionGroup (Bedops.cpp:1249-1337) */
static void next_partition_group(reader_t* rd, int nf, heap_t* pq) {
  rec_t minelem, bt;
  int mn = -1, have = 0, val = 1;
  for (int i = 0; i < nf; ++i) {
    if (!rd_has(&rd[i])) continue;
    rd_read(&rd[i], &bt);
    rd_push(&rd[i], &bt);
    if (!have || (val = chrcmp(bt.chrom, minelem.chrom)) < 0) {
      if (mn >= 0) rd_push(&rd[mn], &minelem);
      mn = i;
      rd_read(&rd[mn], &minelem);
      have = 1;
    } else if (val == 0 && (bt.start < minelem.start ||
                            (bt.start == minelem.start && bt.end < minelem.end))) {
      rd_push(&rd[mn], &minelem);
      mn = i;
      rd_read(&rd[mn], &minelem);
    }
  }
  if (!have) return;
  hp_push(pq, &minelem);
  heap_t lcl = {0};
  for (int i = 0; i < nf; ++i) {
    lcl.n = 0;
    lcl.min_first = 0;
    while (rd_has(&rd[i])) {
      rd_read(&rd[i], &bt);
      if (chrcmp(bt.chrom, minelem.chrom) != 0 || bt.start > minelem.end) {
        rd_push(&rd[i], &bt);
        break;
      } else if (bt.start == minelem.end) {
        hp_push(&lcl, &bt);
        continue;
      }
      if (bt.start == minelem.start) {
        if (bt.end == minelem.end) continue; /* duplicate */
        bt.start = minelem.end;
        hp_push(&lcl, &bt);
        while (rd_has(&rd[i])) {
          rd_read(&rd[i], &bt);
          if (bt.start == minelem.end) {
            hp_push(&lcl, &bt);
          } else {
            rd_push(&rd[i], &bt);
            break;
          }
        }
      } else if (bt.end <= minelem.end) { /* nested or shared end */
        hp_push(pq, &bt);
      } else {
        rec_t cpy = bt;
        cpy.id = NEXT_ID++;
        cpy.start = minelem.end;
        hp_push(&lcl, &cpy);
        bt.end = minelem.end;
        hp_push(pq, &bt);
      }
    }
    while (lcl.n) {
      rd_push(&rd[i], hp_top(&lcl));
      hp_pop(&lcl, NULL);
    }
  }
  free(lcl.a);
}

/* doPartitions (Bedops.cpp:614-686) */
static void do_partition(reader_t* rd, int nf) {
  heap_t pq = {0};
  pq.min_first = 1;
  rec_t mn, curr, ct, lcl, z;
  for (;;) {
    next_partition_group(rd, nf, &pq);
    if (!pq.n) break;
    hp_pop(&pq, &mn);
    if (!pq.n) {
      emit3(&mn);
      continue;
    }
    lcl = mn;
    curr = mn;
    while (pq.n) {
      hp_pop(&pq, &ct);
      if (curr.end <= ct.start) {
        emit3(&curr);
        curr = ct;
      } else if (ct.start == curr.start) {
        if (ct.end == curr.end) continue; /* duplicate */
        ct.start = curr.end;
        hp_push(&pq, &ct);
        while ((z = *hp_top(&pq)).start == curr.start) {
          hp_pop(&pq, NULL);
          z.start = curr.end;
          hp_push(&pq, &z);
        }
        ct = *hp_top(&pq); /* not popped */
        lcl.start = curr.start;
        lcl.end = ct.start;
        emit3(&lcl);
        if (curr.end != ct.start) {
          curr.start = ct.start;
          hp_push(&pq, &curr);
        }
        hp_pop(&pq, &curr);
      } else {
        lcl.start = curr.start;
        lcl.end = ct.start;
        emit3(&lcl);
        curr.start = ct.start;
        hp_push(&pq, &curr);
        hp_push(&pq, &ct);
        hp_pop(&pq, &curr);
      }
    }
    emit3(&curr);
  }
  free(pq.a);
}

/* doUnionAll / nextUnionAllLine (Bedops.cpp:752-786, :1472-1518); rows keep their rest */
static void do_everything(reader_t* rd, int nf, const bedfile_t* files) {
  rec_t first, nx;
  for (;;) {
    int marker = -1;
    for (int i = 0; i < nf; ++i) {
      if (!rd_has(&rd[i])) continue;
      if (marker < 0) {
        rd_read(&rd[i], &first);
        rd_push(&rd[i], &first);
        marker = i;
        continue;
      }
      rd_read(&rd[i], &nx);
      rd_push(&rd[i], &nx);
      int v = chrcmp(nx.chrom, first.chrom);
      int take = v < 0;
      if (v == 0) {
        if (nx.start != first.start) take = nx.start < first.start;
        else if (nx.end != first.end) take = nx.end < first.end;
        else take = strcmp(files[i].rest[nx.row], files[marker].rest[first.row]) < 0;
      }
      if (take) {
        first = nx;
        marker = i;
      }
    }
    if (marker < 0) return;
    rd_read(&rd[marker], &first);
    printf("%s\t%" PRIu64 "\t%" PRIu64 "%s\n", POOL.names[first.chrom], first.start, first.end,
           files[marker].rest[first.row]);
  }
}

/* -e/-n overlap spec (Input.hpp:344-382). Returns 1 if argument was consumed. */
static int parse_subset(const char* s, double* thres, int* use_pct) {
  size_t L = strlen(s);
  const char* pct = strchr(s, '%');
  if (pct) {
    if (pct[1] != '\0') return -1;
    const char* v = s;
    if (*v == '-') ++v;
    if (v == pct) return -1;
    for (const char* p = v; p < pct; ++p)
      if (!strchr(".0123456789", *p)) return -1;
    char buf[64];
    size_t n = (size_t)(pct - v) < sizeof(buf) - 1 ? (size_t)(pct - v) : sizeof(buf) - 1;
    memcpy(buf, v, n);
    buf[n] = 0;
    double d = 0;
    sscanf(buf, "%lf", &d); /* stringstream >> double */
    d /= 100.0;
    if (d > 1) return -1;
    *thres = d;
    *use_pct = 1;
    if (d == 0) { *thres = 1; *use_pct = 0; }
    return 1;
  }
  const char* q = s;
  if (*q == '-') ++q;
  if (*q == 0) return 0;
  for (size_t i = (size_t)(q - s); i < L; ++i)
    if (s[i] < '0' || s[i] > '9') return 0;
  *thres = (double)atoi(q);
  *use_pct = 0;
  return 1;
}

/* --range L:R | S (Input.hpp:86-127) */
static int parse_range(const char* v, int* lpad, int* rpad) {
  const char* colon = strchr(v, ':');
  if (colon) {
    if (colon == v || !colon[1]) return -1;
    *lpad = atoi(v);
    *rpad = atoi(colon + 1);
  } else {
    int r = atoi(v);
    *lpad = -r;
    *rpad = r;
  }
  return 0;
}

static int all_digits(const char* s) {
  if (!*s) return 1; /* find_first_not_of on "" is npos */
  for (; *s; ++s)
    if (*s < '0' || *s > '9') return 0;
  return 1;
}

int main(int argc, char** argv) {
  int a = 1, mode = 0;
  const char* only_chrom = NULL; /* --chrom: restrict every input to one chromosome */
  double thres = 1.0;
  int use_pct = 1, lpad = 0, rpad = 0, full_left = 0, chop_x = 0;
  uint64_t chop_bp = 1, chop_stagger = 0;
  while (a < argc && argv[a][0] == '-' && argv[a][1] != '\0') {
    const char* o = argv[a];
    if (!strcmp(o, "--ec") || !strcmp(o, "--header")) { ++a; continue; }
    if (!strcmp(o, "--chrom") && a + 1 < argc) { only_chrom = argv[a + 1]; a += 2; continue; }
    if (!strcmp(o, "--range") && a + 1 < argc) {
      if (parse_range(argv[a + 1], &lpad, &rpad)) { fprintf(stderr, "bedops_oracle: bad --range\n"); return 2; }
      a += 2;
      continue;
    }
    if (!strcmp(o, "-m") || !strcmp(o, "--merge")) mode = 'm';
    else if (!strcmp(o, "-i") || !strcmp(o, "--intersect")) mode = 'i';
    else if (!strcmp(o, "-d") || !strcmp(o, "--difference")) mode = 'd';
    else if (!strcmp(o, "-e") || !strcmp(o, "--element-of")) mode = 'e';
    else if (!strcmp(o, "-n") || !strcmp(o, "--not-element-of")) mode = 'n';
    else if (!strcmp(o, "-c") || !strcmp(o, "--complement")) mode = 'c';
    else if (!strcmp(o, "-s") || !strcmp(o, "--symmdiff")) mode = 's';
    else if (!strcmp(o, "-p") || !strcmp(o, "--partition")) mode = 'p';
    else if (!strcmp(o, "-u") || !strcmp(o, "--everything")) mode = 'u';
    else if (!strcmp(o, "-w") || !strcmp(o, "--chop")) mode = 'w';
    else { fprintf(stderr, "bedops_oracle: unsupported option %s\n", o); return 2; }
    ++a;
    if ((mode == 'e' || mode == 'n') && a < argc) {
      FILE* t = fopen(argv[a], "r");
      if (t) fclose(t);
      else {
        int r = parse_subset(argv[a], &thres, &use_pct);
        if (r < 0) { fprintf(stderr, "bedops_oracle: bad overlap spec\n"); return 2; }
        if (r > 0) ++a;
      }
    } else if (mode == 'c') { /* Input.hpp:207-220 */
      if (a < argc && !strcmp(argv[a], "-L")) { full_left = 1; ++a; }
    } else if (mode == 'w') { /* Input.hpp:221-258 */
      while (a < argc) {
        if (!strcmp(argv[a], "--stagger") && a + 1 < argc) {
          chop_stagger = strtoull(argv[a + 1], NULL, 10);
          a += 2;
        } else if (!strcmp(argv[a], "-x")) {
          chop_x = 1;
          ++a;
        } else if (all_digits(argv[a])) {
          chop_bp = strtoull(argv[a], NULL, 10);
          ++a;
        } else {
          break;
        }
      }
    }
    /* process flags may also follow the operation (Input.hpp:74-263 loops over all) */
    while (a < argc && (!strcmp(argv[a], "--ec") || !strcmp(argv[a], "--header") ||
                        !strcmp(argv[a], "--chrom") || !strcmp(argv[a], "--range"))) {
      if (!strcmp(argv[a], "--ec") || !strcmp(argv[a], "--header")) { ++a; continue; }
      if (a + 1 >= argc) break;
      if (!strcmp(argv[a], "--chrom")) only_chrom = argv[a + 1];
      else if (parse_range(argv[a + 1], &lpad, &rpad)) { fprintf(stderr, "bedops_oracle: bad --range\n"); return 2; }
      a += 2;
    }
    break;
  }
  int nf = argc - a;
  int minf = (mode == 'i' || mode == 'd' || mode == 'e' || mode == 'n' || mode == 's') ? 2 : 1;
  if (!mode || nf < minf) { fprintf(stderr, "bedops_oracle: bad usage\n"); return 2; }
  bedfile_t* files = (bedfile_t*)calloc((size_t)nf, sizeof(bedfile_t));
  for (int i = 0; i < nf; ++i) {
    FILE* fp = open_input(argv[a + i]);
    if (!fp) { fprintf(stderr, "bedops_oracle: cannot open %s\n", argv[a + i]); return 2; }
    /* B3Rest for every file of --everything and the reference of element-of
     * (Bedops.cpp:402-421), B3NoRest otherwise */
    read_bed3(fp, &POOL, &files[i], mode == 'u' || ((mode == 'e' || mode == 'n') && i == 0));
    if (fp != stdin) fclose(fp);
    if (only_chrom) { /* AllocateIterator_BED_starch.hpp:113-160 seeks to that chromosome */
      bedfile_t* f = &files[i];
      int64_t k = 0;
      for (int64_t j = 0; j < f->n; ++j) {
        if (strcmp(POOL.names[f->chrom[j]], only_chrom) != 0) continue;
        f->chrom[k] = f->chrom[j]; f->start[k] = f->start[j]; f->end[k] = f->end[j];
        if (f->rest) f->rest[k] = f->rest[j];
        ++k;
      }
      f->n = k;
    }
    /* every file is padded except the element-of reference (Bedops.cpp:230-236) */
    if (!((mode == 'e' || mode == 'n') && i == 0)) pad_file(&files[i], lpad, rpad);
  }
  reader_t* rd = (reader_t*)calloc((size_t)nf, sizeof(reader_t));
  for (int i = 0; i < nf; ++i) rd[i].f = &files[i];
  static char obuf[1 << 20];
  setvbuf(stdout, obuf, _IOFBF, sizeof(obuf));
  rec_t o;
  switch (mode) {
    case 'm':
      while (next_merge_all(rd, 0, nf, &o)) emit3(&o);
      break;
    case 'i':
      while (next_intersect(rd, nf, &o)) emit3(&o);
      break;
    case 'd':
      do_difference(rd, nf);
      break;
    case 'e':
    case 'n':
      do_element_of(rd, nf, &files[0], thres, use_pct, mode == 'n');
      break;
    case 'c':
      do_complement(rd, nf, full_left);
      break;
    case 'w':
      do_chop(rd, nf, chop_bp, chop_stagger, chop_x);
      break;
    case 's':
      do_symmdiff(rd, nf);
      break;
    case 'p':
      do_partition(rd, nf);
      break;
    case 'u':
      do_everything(rd, nf, files);
      break;
  }
  fflush(stdout);
  return 0;
}
