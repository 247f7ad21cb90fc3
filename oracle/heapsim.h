/*
 * oracle/heapsim.h — TEST INFRASTRUCTURE ONLY.
 *
 * The reference breaks ties between equal map rows by their heap ADDRESS:
 *   - BedBaseVisitor's window, CoordRestAddressCompare ............ BedCompare.hpp:143-156
 *   - EchoMapBed's set, GenomicAddressCompare ...................... BedCompare.hpp:51-63
 *   - TrimmedMean / RollingKth, CompValueThenAddressLesser ........ utility/OrderCompare.hpp
 *   - WeightedAverage's std::set<MapType*> (address order only) .... WeightedAverageVisitor.hpp:86
 * Rows are `new`-ed one at a time by allocate_iterator (AllocateIterator_BED_starch.hpp:205-215;
 * the iterator reads one row ahead, and the read at end of file allocates one last row that is
 * never freed) and `delete`-d by the sweep (WindowSweepImpl.cpp:207-233,240-253), so an
 * address is a function of the sequence of allocations and frees. This models the glibc
 * allocator the reference links (glibc 2.35 malloc.c) for those calls: per chunk size a
 * thread cache of 7 entries (LIFO, tcache_put/tcache_get) and, for chunks <= 128 bytes, a
 * LIFO fast bin; a malloc that misses the cache pops the fast bin and stashes the rest of
 * that bin into the cache (_int_malloc's fastbin path); a miss on both takes fresh memory
 * from the top of the heap (increasing addresses). Chunk size = request + 8 rounded up to
 * 16, at least 32. Modelled (oracle/bedmap_oracle.c): the row objects and their strings,
 * the std::set nodes of BedBaseVisitor and of the visitors keeping one per row or per
 * coordinates (40 bytes: the 48-byte chunks of B3Rest row objects), and DoneReference's
 * temporaries (row copies, EchoMapIntersectLength's vector). Not modelled: the sweep's deque
 * blocks and fixWindow's list nodes (other chunk sizes than any row object's).
 * Not modelled: malloc_consolidate (only when the heap grows while fast bins are occupied, or
 * on large requests), which a multi-megabyte sweep window can trigger.
 */
#ifndef ORACLE_HEAPSIM_H
#define ORACLE_HEAPSIM_H
#include <stdint.h>
#include <stdlib.h>

#define HS_CLASSES 66 /* chunk sizes 32 .. 1056 in steps of 16 */
typedef struct {
  int64_t* v;
  int64_t n, cap;
} hs_list_t;
typedef struct {
  hs_list_t tc[HS_CLASSES], fb[HS_CLASSES];
  int64_t top;
} heapsim_t;

static size_t hs_chunk(size_t req) {
  size_t c = (req + 8 + 15) & ~(size_t)15;
  return c < 32 ? 32 : c;
}
static void hs_push(hs_list_t* l, int64_t a) {
  if (l->n == l->cap) {
    l->cap = l->cap ? 2 * l->cap : 64;
    l->v = (int64_t*)realloc(l->v, (size_t)l->cap * sizeof(int64_t));
  }
  l->v[l->n++] = a;
}
static int64_t hs_malloc(heapsim_t* h, size_t req) {
  const size_t c = hs_chunk(req);
  const int k = (int)(c / 16 - 2);
  if (k >= HS_CLASSES) { /* large: fresh memory (not reused by the small classes) */
    const int64_t a = h->top;
    h->top += (int64_t)c;
    return a;
  }
  if (h->tc[k].n) return h->tc[k].v[--h->tc[k].n];
  if (h->fb[k].n) {
    const int64_t a = h->fb[k].v[--h->fb[k].n];
    while (h->tc[k].n < 7 && h->fb[k].n) hs_push(&h->tc[k], h->fb[k].v[--h->fb[k].n]);
    return a;
  }
  const int64_t a = h->top;
  h->top += (int64_t)c;
  return a;
}
static void hs_free(heapsim_t* h, size_t req, int64_t a) {
  const size_t c = hs_chunk(req);
  const int k = (int)(c / 16 - 2);
  if (k >= HS_CLASSES) return;
  if (h->tc[k].n < 7) hs_push(&h->tc[k], a);
  else hs_push(&h->fb[k], a); /* chunks > 128 B would go to the unsorted bin: LIFO here */
}
#endif
