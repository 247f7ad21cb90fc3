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
// fixWindow's Add / Delete calls come. Runs of equal coordinates are short; a run of L rows
// costs L^2 comparisons.
__global__ void k_heap_rest_rank(const int64_t* __restrict__ S, const int64_t* __restrict__ E, uint64_t n,
                                 const char* __restrict__ text, const uint64_t* __restrict__ rest_off,
                                 const uint32_t* __restrict__ rest_len, int fields, uint32_t* __restrict__ rank) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  const int64_t s = S[m], e = E[m];
  uint64_t lo = m, hi = m + 1;
  while (lo > 0 && S[lo - 1] == s && E[lo - 1] == e) --lo;
  while (hi < n && S[hi] == s && E[hi] == e) ++hi;
  uint32_t r = 0;
  if (hi - lo > 1 && rest_off)
    for (uint64_t j = lo; j < hi; ++j)
      if (j != m && bg_frest_cmp(text, rest_off, rest_len, fields, j, m) < 0) ++r;
  rank[m] = r;
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
  if (nm && M->rest_off && !spec->faster) {
    drk = (uint32_t*)bg_alloc(c, 4 * nm);
    if (!drk) return BG_E_NOMEM;
    BG_LAUNCH(c, "k_heap_rest_rank", k_heap_rest_rank, dim3(bg_blocks(nm, BG_NT)), dim3(BG_NT), M->ks, M->ke, nm,
              M->text, M->rest_off, M->rest_len, fields, drk);
    BG_HIP(c, hipGetLastError());
    BG_HIP(c, hipMemcpyAsync(hrank.data(), drk, 4 * nm, hipMemcpyDeviceToHost, c->stream));
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
  int64_t* d = (int64_t*)bg_alloc(c, 8 * (nm ? nm : 1));
  if (!d) return BG_E_NOMEM;
  if (nm) BG_HIP(c, hipMemcpyAsync(d, addr.data(), 8 * nm, hipMemcpyHostToDevice, c->stream));
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
