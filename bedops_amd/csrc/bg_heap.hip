// bg_heap.hip — the heap addresses the reference breaks ties with, for bedmap.
//
// The reference orders equal map rows by their heap ADDRESS: BedBaseVisitor's window
// (CoordRestAddressCompare, BedCompare.hpp:143-156) and so the decimal running sums' event
// order; EchoMapBed's set (GenomicAddressCompare, BedCompare.hpp:51-63) and so the order of
// --echo-map* lists; TrimmedMean's set (CompValueThenAddressLesser, OrderCompare.hpp);
// WeightedAverage's std::set<MapType*> (address order only, WeightedAverageVisitor.hpp:86);
// the element operations' tie between equal rows. Rows are `new`-ed one at a time by
// allocate_iterator (AllocateIterator_BED_starch.hpp:205-215: one row read ahead; the read at
// end of file allocates a last row that is never freed) and `delete`-d by the sweep
// (WindowSweepImpl.cpp:207-253), so an address is a function of the program's allocation
// sequence under glibc's allocator: per chunk size a 7-entry LIFO thread cache, then a LIFO
// fast bin (a cache miss pops the bin and stashes the rest of it into the cache), then fresh
// memory from the top of the heap. The calls replayed (the same model is restated, as test
// infrastructure, in oracle/heapsim.h + oracle/bedmap_oracle.c and checked there against the
// reference's own output, tests/test_ref_fixtures.py):
//   - every row object and its strings (Bed.hpp constructors / readline / destructors), map
//     rows and the two live reference rows;
//   - the std::set nodes (40 bytes: the 48-byte chunks of B3Rest row objects) of
//     BedBaseVisitor's cache_ / win_ (BedBaseVisitor.hpp:139-153, fixWindow :185-211) and of
//     the visitors that keep one per row (EchoMapBed, EchoMapIntersectLength, OvrAggregate)
//     or one per distinct coordinates (OvrUnique, OvrUniqueFract);
//   - the temporaries of DoneReference: EchoMapIntersectLength's copy of the reference row
//     per map row and its growing std::vector<long> (EchoMapIntersectLengthVisitor.hpp:64-73),
//     PrintGenomicRange's copy of the first map row (ProcessBedVisitorRow.hpp:446), OvrUnique's
//     running copy (OvrUniqueVisitor.hpp:63-78); B5Rest's copy constructor allocates its
//     remainder strings one byte short (strlen(p + 1), Bed.hpp:757-759).
// Overlapping's last tie-break compares two rows' addresses (BedDistances.hpp:108-110): for
// bedmap --faster --bp-ovr N the sweep's decision on an equal reference / map row pair
// shorter than N (delete the map row now or hold it) is replayed with the simulated
// addresses; the device windows do not depend on it (bg_internal.h, bg_fs_ovl).
//
// The replay is one pass over the sweep's calls: sequential by nature, so it runs on the
// host over the keyed coordinates, and only when an operation can see an address tie (bg_map
// decides). Not modelled: malloc_consolidate (heap growth while fast bins hold chunks), which
// very large windows can trigger.
#include <string.h>
#include <algorithm>
#include "bg_heap_replay.h"

// per map row: id length and the remainder length the row's readline stores (restBuf):
// B3Rest everything after `end`; B4Rest after the id token; B5Rest after the score token
__global__ void k_heap_lens(const char* __restrict__ text, const uint64_t* __restrict__ rest_off,
                            const uint32_t* __restrict__ rest_len, uint64_t n, int fields,
                            uint32_t* __restrict__ li, uint32_t* __restrict__ lr) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  const char* rp = text + rest_off[m];
  const uint32_t rl = rest_len[m];
  if (fields == 3) {
    li[m] = 0;
    lr[m] = rl;
    return;
  }
  uint32_t i = 0;
  while (i < rl && bg_frest_ws(rp[i])) ++i;
  uint32_t j = i;
  while (j < rl && !bg_frest_ws(rp[j])) ++j;
  li[m] = j - i;
  if (fields == 4) {
    lr[m] = rl - j;
    return;
  }
  uint32_t k = j;
  while (k < rl && bg_frest_ws(rp[k])) ++k;
  while (k < rl && !bg_frest_ws(rp[k])) ++k;
  lr[m] = rl - k;
}

// rank of map row m's full_rest() among the rows of equal (start, end) around it (rows equal
// in all three have equal ranks): the third key of CoordRestAddressCompare, in which
// fixWindow's Add / Delete calls come. The runs come from their start flags (one compaction,
// no per-row walk); a run of up to HEAP_RUN_DEV rows is ranked here, one thread per row and
// one comparison per other row of its run; a longer run (PCR duplicates, placeholder rows: a
// run of L rows would cost L^2) is listed for the host, which sorts it in O(L log L) as the
// reference's std::set does (heap_long_ranks).
#define HEAP_RUN_DEV 64
__global__ void k_heap_run_flags(const int64_t* __restrict__ S, const int64_t* __restrict__ E, uint64_t n,
                                 uint8_t* __restrict__ f) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m < n) f[m] = m == 0 || S[m] != S[m - 1] || E[m] != E[m - 1];
}
__global__ void k_heap_rest_rank(const uint64_t* __restrict__ run0, uint64_t nrun, uint64_t n,
                                 const char* __restrict__ text, const uint64_t* __restrict__ rest_off,
                                 const uint32_t* __restrict__ rest_len, int fields, uint32_t* __restrict__ rank,
                                 uint64_t* __restrict__ longs, unsigned long long* __restrict__ nlong) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  uint64_t a = 0, b = nrun;  // the last run starting at or before m
  while (b - a > 1) {
    const uint64_t mid = (a + b) >> 1;
    if (run0[mid] <= m) a = mid;
    else b = mid;
  }
  const uint64_t lo = run0[a], hi = a + 1 < nrun ? run0[a + 1] : n;
  uint32_t r = 0;
  if (hi - lo > HEAP_RUN_DEV) {
    if (m == lo) longs[atomicAdd(nlong, 1ULL)] = a;
    r = 0;  // (the host's sort)
  } else if (hi - lo > 1 && rest_off) {
    for (uint64_t j = lo; j < hi; ++j)
      if (j != m && bg_frest_cmp(text, rest_off, rest_len, fields, j, m) < 0) ++r;
  }
  rank[m] = r;
}
// full_rest() lengths, then bytes, of the rows of listed runs (rows [row0[k], row0[k] + len[k]))
__global__ void k_heap_rest_len(const uint64_t* __restrict__ rows, uint64_t nrows, const char* __restrict__ text,
                                const uint64_t* __restrict__ rest_off, const uint32_t* __restrict__ rest_len,
                                int fields, uint64_t* __restrict__ len) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrows) return;
  const char *p1, *p2;
  uint32_t l1, l2;
  bg_frest(text, rest_off, rest_len, fields, rows[i], p1, l1, p2, l2);
  len[i] = l1 + l2;
}
__global__ void k_heap_rest_copy(const uint64_t* __restrict__ rows, uint64_t nrows, const char* __restrict__ text,
                                 const uint64_t* __restrict__ rest_off, const uint32_t* __restrict__ rest_len,
                                 int fields, const uint64_t* __restrict__ off, char* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrows) return;
  const char *p1, *p2;
  uint32_t l1, l2;
  bg_frest(text, rest_off, rest_len, fields, rows[i], p1, l1, p2, l2);
  char* o = out + off[i];
  for (uint32_t k = 0; k < l1; ++k) o[k] = p1[k];
  for (uint32_t k = 0; k < l2; ++k) o[l1 + k] = p2[k];
}

// full_rest() of each listed map row to the host: row i's bytes are txt[off[i], off[i + 1])
int bg_frest_gather(bg_ctx* c, const bg_table* M, int fields, const std::vector<uint64_t>& rows,
                    std::vector<char>& txt, std::vector<uint64_t>& off) {
  const uint64_t nr = rows.size();
  off.assign(nr + 1, 0);
  txt.clear();
  if (!nr) return 0;
  BgHold hold(c);
  uint64_t* drows = hold((uint64_t*)bg_alloc(c, 8 * nr));
  uint64_t* dlen = hold((uint64_t*)bg_alloc(c, 8 * (nr + 1)));
  if (!drows || !dlen) return BG_E_NOMEM;
  BG_HIP(c, hipMemcpyAsync(drows, rows.data(), 8 * nr, hipMemcpyHostToDevice, c->stream));
  BG_LAUNCH(c, "k_heap_rest_len", k_heap_rest_len, dim3(bg_blocks(nr, BG_NT)), dim3(BG_NT), drows, nr, M->text,
            M->rest_off, M->rest_len, fields, dlen);
  std::vector<uint64_t> len(nr);
  BG_HIP(c, hipMemcpyAsync(len.data(), dlen, 8 * nr, hipMemcpyDeviceToHost, c->stream));
  BG_HIP(c, hipStreamSynchronize(c->stream));
  for (uint64_t i = 0; i < nr; ++i) off[i + 1] = off[i] + len[i];
  char* dtxt = hold((char*)bg_alloc(c, off[nr] + 1));
  if (!dtxt) return BG_E_NOMEM;
  BG_HIP(c, hipMemcpyAsync(dlen, off.data(), 8 * nr, hipMemcpyHostToDevice, c->stream));
  BG_LAUNCH(c, "k_heap_rest_copy", k_heap_rest_copy, dim3(bg_blocks(nr, BG_NT)), dim3(BG_NT), drows, nr, M->text,
            M->rest_off, M->rest_len, fields, dlen, dtxt);
  txt.resize(off[nr] + 1);
  BG_HIP(c, hipMemcpyAsync(txt.data(), dtxt, off[nr], hipMemcpyDeviceToHost, c->stream));
  BG_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

// the ranks of the runs longer than HEAP_RUN_DEV: their rows' full_rest() strings to the
// host, each run sorted (strcmp order: bytes as unsigned, a prefix first), equal strings equal
// ranks, written into hrank
static int heap_long_ranks(bg_ctx* c, const bg_table* M, int fields, const uint64_t* d_run0, uint64_t nrun,
                           const std::vector<uint64_t>& longs, std::vector<uint32_t>& hrank) {
  const uint64_t nm = M->n;
  std::vector<uint64_t> h0(nrun);
  BG_HIP(c, hipMemcpyAsync(h0.data(), d_run0, 8 * nrun, hipMemcpyDeviceToHost, c->stream));
  BG_HIP(c, hipStreamSynchronize(c->stream));
  std::vector<uint64_t> rows;
  for (uint64_t a : longs) {
    const uint64_t lo = h0[a], hi = a + 1 < nrun ? h0[a + 1] : nm;
    for (uint64_t m = lo; m < hi; ++m) rows.push_back(m);
  }
  std::vector<char> txt;
  std::vector<uint64_t> off;
  int rc = bg_frest_gather(c, M, fields, rows, txt, off);
  if (rc) return rc;
  auto less = [&](uint64_t i, uint64_t j) {  // rows[i] vs rows[j] by full_rest()
    return bg_bytes_less(txt.data() + off[i], off[i + 1] - off[i], txt.data() + off[j], off[j + 1] - off[j]);
  };
  uint64_t i0 = 0;
  std::vector<uint64_t> ix;
  for (uint64_t a : longs) {
    const uint64_t n = (a + 1 < nrun ? h0[a + 1] : nm) - h0[a];
    ix.resize(n);
    for (uint64_t k = 0; k < n; ++k) ix[k] = i0 + k;
    std::sort(ix.begin(), ix.end(), less);
    uint32_t rk = 0;
    for (uint64_t k = 0; k < n; ++k) {
      if (k > 0 && less(ix[k - 1], ix[k])) rk = (uint32_t)k;  // equal strings share a rank
      hrank[rows[ix[k]]] = rk;
    }
    i0 += n;
  }
  return 0;
}

// does any map row equal its predecessor in (start, end) [and full_rest() when `rest`]?
__global__ void k_heap_ties(const int64_t* __restrict__ S, const int64_t* __restrict__ E, uint64_t n,
                            const char* __restrict__ text, const uint64_t* __restrict__ rest_off,
                            const uint32_t* __restrict__ rest_len, int fields, int rest,
                            unsigned int* __restrict__ any) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (m >= n) return;
  if (S[m] != S[m - 1] || E[m] != E[m - 1]) return;
  if (rest && rest_off && bg_frest_cmp(text, rest_off, rest_len, fields, m - 1, m) != 0) return;
  atomicOr(any, 1u);
}


// the simulated address of every map row, on the device (*out, bg_alloc'ed), for bg_map
// (R == M: one file)
int bg_heap_addr(bg_ctx* c, bg_set* set, const bg_table* R, const bg_table* M, int fields,
                 const bg_heap_spec* spec, int64_t** out) {
  *out = nullptr;
  if (spec->nops > kMaxVis) return bg_fail(c, BG_E_UNSUPPORTED, "too many operations for the heap replay");
  const bool single = R == M;
  const uint64_t nr = R->n, nm = M->n;
  std::vector<int64_t> hRS(single ? 0 : nr), hRE(single ? 0 : nr), hMS(nm), hME(nm);
  std::vector<uint32_t> hli(nm, 0), hlr(nm, 0), hrl(single ? 0 : nr, 0), hrank(nm, 0);
  uint32_t* dli = nullptr;
  uint32_t* dlr = nullptr;
  uint32_t* drk = nullptr;
  if (nm && M->rest_off) {
    dli = (uint32_t*)bg_alloc(c, 4 * nm);
    dlr = (uint32_t*)bg_alloc(c, 4 * nm);
    if (!dli || !dlr) return BG_E_NOMEM;
    BG_LAUNCH(c, "k_heap_lens", k_heap_lens, dim3(bg_blocks(nm, BG_NT)), dim3(BG_NT), M->text, M->rest_off,
              M->rest_len, nm, fields, dli, dlr);
    BG_HIP(c, hipGetLastError());
    BG_HIP(c, hipMemcpyAsync(hli.data(), dli, 4 * nm, hipMemcpyDeviceToHost, c->stream));
    BG_HIP(c, hipMemcpyAsync(hlr.data(), dlr, 4 * nm, hipMemcpyDeviceToHost, c->stream));
  }
  uint64_t* run0 = nullptr;
  uint64_t nrun = 0;
  std::vector<uint64_t> longs;
  if (nm && M->rest_off && !spec->faster) {
    drk = (uint32_t*)bg_alloc(c, 4 * nm);
    uint8_t* f = (uint8_t*)bg_alloc(c, nm);
    uint64_t* dl = (uint64_t*)bg_alloc(c, 8 * (nm + 1));  // long runs (count in the last slot)
    if (!drk || !f || !dl) return BG_E_NOMEM;
    BG_LAUNCH(c, "k_heap_run_flags", k_heap_run_flags, dim3(bg_blocks(nm, BG_NT)), dim3(BG_NT), M->ks, M->ke, nm, f);
    int rc = bg_compact_flags(c, f, nm, &run0, &nrun);
    if (rc) return rc;
    BG_HIP(c, hipMemsetAsync(dl + nm, 0, 8, c->stream));
    BG_LAUNCH(c, "k_heap_rest_rank", k_heap_rest_rank, dim3(bg_blocks(nm, BG_NT)), dim3(BG_NT), run0, nrun, nm,
              M->text, M->rest_off, M->rest_len, fields, drk, dl, (unsigned long long*)(dl + nm));
    BG_HIP(c, hipGetLastError());
    BG_HIP(c, hipMemcpyAsync(hrank.data(), drk, 4 * nm, hipMemcpyDeviceToHost, c->stream));
    uint64_t nl = 0;
    if ((rc = bg_fetch_u64(c, dl + nm, &nl))) return rc;
    if (nl) {
      longs.resize(nl);
      BG_HIP(c, hipMemcpyAsync(longs.data(), dl, 8 * nl, hipMemcpyDeviceToHost, c->stream));
      BG_HIP(c, hipStreamSynchronize(c->stream));
      std::sort(longs.begin(), longs.end());
      if ((rc = heap_long_ranks(c, M, fields, run0, nrun, longs, hrank))) return rc;
    }
    bg_release(c, f);
    bg_release(c, dl);
    bg_release(c, run0);
  }
  if (nr && !single) {
    BG_HIP(c, hipMemcpyAsync(hRS.data(), R->ks, 8 * nr, hipMemcpyDeviceToHost, c->stream));
    BG_HIP(c, hipMemcpyAsync(hRE.data(), R->ke, 8 * nr, hipMemcpyDeviceToHost, c->stream));
    if (R->rest_len) BG_HIP(c, hipMemcpyAsync(hrl.data(), R->rest_len, 4 * nr, hipMemcpyDeviceToHost, c->stream));
  }
  if (nm) {
    BG_HIP(c, hipMemcpyAsync(hMS.data(), M->ks, 8 * nm, hipMemcpyDeviceToHost, c->stream));
    BG_HIP(c, hipMemcpyAsync(hME.data(), M->ke, 8 * nm, hipMemcpyDeviceToHost, c->stream));
  }
  BG_HIP(c, hipStreamSynchronize(c->stream));
  bg_release(c, dli);
  bg_release(c, dlr);
  bg_release(c, drk);
  auto name_len = [&](int64_t key) -> uint32_t {
    const uint64_t g = (uint64_t)(key >> BG_KEY_SHIFT);
    return g < set->names.size() ? (uint32_t)set->names[g].size() : 0;
  };
  std::vector<int64_t> addr(nm + 1);
  Replay P;
  P.RS = hRS.data();
  P.RE = hRE.data();
  P.MS = hMS.data();
  P.ME = hME.data();
  P.nr = single ? nm : nr;
  P.nm = nm;
  P.single = single;
  P.fields = fields;
  P.mli = hli.data();
  P.mlr = hlr.data();
  P.rlr = hrl.data();
  P.rrank = hrank.data();
  P.mlc.resize(nm);
  for (uint64_t m = 0; m < nm; ++m) P.mlc[m] = name_len(hMS[m]);
  if (!single) {  // the reference file is read as B3Rest (Bedmap.cpp:624-654)
    P.rlc.resize(nr);
    for (uint64_t r = 0; r < nr; ++r) P.rlc[r] = name_len(hRS[r]);
  }
  P.spec = spec;
  P.addr = addr.data();
  P.keyed.resize((size_t)spec->nops);
  if (single) P.run1();
  else P.run2();
  // after the nm addresses: each run of rows equal in (start, end) listed by increasing address
  // (uint32 row indices, identity outside runs), so the formatter walks a tie run in
  // GenomicAddressCompare order in O(run) instead of selecting the next address each time
  std::vector<uint32_t> ord(nm);
  for (uint64_t m = 0; m < nm;) {
    uint64_t t = m + 1;
    while (t < nm && hMS[t] == hMS[m] && hME[t] == hME[m]) ++t;
    for (uint64_t u = m; u < t; ++u) ord[u] = (uint32_t)u;
    if (t - m > 1)
      std::sort(ord.begin() + (ptrdiff_t)m, ord.begin() + (ptrdiff_t)t,
                [&](uint32_t a, uint32_t b) { return addr[a] < addr[b]; });
    m = t;
  }
  int64_t* d = (int64_t*)bg_alloc(c, 8 * (nm ? nm : 1) + 4 * nm);
  if (!d) return BG_E_NOMEM;
  if (nm) {
    BG_HIP(c, hipMemcpyAsync(d, addr.data(), 8 * nm, hipMemcpyHostToDevice, c->stream));
    BG_HIP(c, hipMemcpyAsync(d + nm, ord.data(), 4 * nm, hipMemcpyHostToDevice, c->stream));
  }
  BG_HIP(c, hipStreamSynchronize(c->stream));
  *out = d;
  return 0;
}

// any adjacent map rows equal in (start, end) [and full_rest()]?
int bg_heap_ties(bg_ctx* c, const bg_table* M, int fields, bool rest, bool* any) {
  *any = false;
  if (M->n < 2) return 0;
  unsigned int* d = (unsigned int*)bg_alloc(c, 4);
  if (!d) return BG_E_NOMEM;
  BG_HIP(c, hipMemsetAsync(d, 0, 4, c->stream));
  BG_LAUNCH(c, "k_heap_ties", k_heap_ties, dim3(bg_blocks(M->n - 1, BG_NT)), dim3(BG_NT), M->ks, M->ke, M->n,
            M->text, M->rest_off, M->rest_len, fields, rest ? 1 : 0, d);
  BG_HIP(c, hipGetLastError());
  unsigned int h = 0;
  BG_HIP(c, hipMemcpyAsync(&h, d, 4, hipMemcpyDeviceToHost, c->stream));
  BG_HIP(c, hipStreamSynchronize(c->stream));
  bg_release(c, d);
  *any = h != 0;
  return 0;
}
