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
// (WindowSweepImpl.cpp:207-253), so an address is a function of that call sequence under
// glibc's allocator: per chunk size a 7-entry LIFO thread cache, then a LIFO fast bin (a
// cache miss pops the bin and stashes the rest of it into the cache), then fresh memory from
// the top of the heap. Only the chunk size of the map row OBJECT matters (B3Rest 32 B ->
// 48-byte chunks, B4Rest 48 B / B5Rest 56 B -> 64), and in it: the row objects, and any row
// string (chrom, id, remainder, id + remainder) whose length puts it in the same chunk size.
// The same model is restated, as test infrastructure, in oracle/heapsim.h and checked there
// against the reference's own output (tests/test_ref_fixtures.py).
//
// The replay is one pass over the sweep's allocation/free sequence: sequential by nature, so
// it runs on the host over the keyed coordinates, and only when an operation can see an
// address tie (bg_map decides). Not modelled: malloc_consolidate (heap growth while fast bins
// hold chunks), which very large windows can trigger.
#include "bg_internal.h"

#include <unordered_map>
#include <vector>

// chunk size of a `new char[len + 1]` / `new T` of `req` bytes (request + 8, 16-aligned, >= 32)
static inline uint64_t hs_chunk(uint64_t req) {
  const uint64_t c = (req + 8 + 15) & ~15ULL;
  return c < 32 ? 32 : c;
}

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

namespace {
struct HeapClass {  // one chunk size of glibc's allocator: tcache + fast bin + top
  std::vector<int64_t> tc, fb;
  int64_t top = 0;
  int64_t get() {
    if (!tc.empty()) {
      const int64_t a = tc.back();
      tc.pop_back();
      return a;
    }
    if (!fb.empty()) {
      const int64_t a = fb.back();
      fb.pop_back();
      while (tc.size() < 7 && !fb.empty()) {
        tc.push_back(fb.back());
        fb.pop_back();
      }
      return a;
    }
    return top++;
  }
  void put(int64_t a) {
    if (tc.size() < 7) tc.push_back(a);
    else fb.push_back(a);
  }
};
struct RowStr {  // in-class string chunks of a live row: chrom, id, rest, id + rest (-1: none)
  int64_t a[4] = {-1, -1, -1, -1};
};
}  // namespace

// host replay of sweep overload 2 (WindowSweepImpl.cpp:168-256) over the keyed rows; addr[m]
// = the simulated address of map row m's object
// (fast_crit >= 0: bedmap --faster, the sweep runs with that criterion's Ref2Map / Map2Ref,
// bg_fs_r2m / bg_fs_m2r)
static void heap_replay(const int64_t* RS, const int64_t* RE, uint64_t nr, const uint8_t* rflag,
                        bool ref_obj_in_class, const int64_t* MS, const int64_t* ME, uint64_t nm,
                        const uint8_t* mflag, bool ranged, int64_t range, int64_t* addr, int fast_crit,
                        int64_t ovr, double perc) {
  HeapClass H;
  std::unordered_map<uint64_t, RowStr> mstr;
  RowStr rstr[2];
  int64_t robj[2] = {-1, -1};
  // construction: object, then (after the 1-byte placeholders, other sizes) chrom, id, rest,
  // id + rest; destruction: rest, id + rest, id, chrom, object (Bed.hpp)
  auto make = [&](uint8_t f, RowStr& s) {
    for (int q : {0, 1, 2, 3})
      s.a[q] = (f >> q) & 1 ? H.get() : -1;
  };
  auto drop = [&](const RowStr& s) {
    for (int q : {2, 3, 1, 0})
      if (s.a[q] >= 0) H.put(s.a[q]);
  };
  auto map_new = [&](uint64_t m) {  // m == nm: the row read at end of file (never freed)
    addr[m] = H.get();
    const uint8_t f = m < nm ? mflag[m] : 0;
    if (f) make(f, mstr[m]);
  };
  auto map_del = [&](uint64_t m) {
    const uint8_t f = mflag[m];
    if (f) {
      auto it = mstr.find(m);
      drop(it->second);
      mstr.erase(it);
    }
    H.put(addr[m]);
  };
  auto ref_new = [&](uint64_t r) {
    const int k = (int)(r & 1);
    if (ref_obj_in_class) robj[k] = H.get();
    rstr[k] = RowStr();
    if (r < nr && rflag[r]) make(rflag[r], rstr[k]);
  };
  auto ref_del = [&](uint64_t r) {
    const int k = (int)(r & 1);
    drop(rstr[k]);
    if (ref_obj_in_class) H.put(robj[k]);
  };
  auto chr = [](int64_t k) { return k >> BG_KEY_SHIFT; };
  // the sweep distance: Overlapping(0) (BedDistances.hpp:97-115) or RangedDist(R) (:57-64)
  auto dist = [&](int64_t as, int64_t ae, int64_t bs, int64_t be) -> int {
    const int64_t ca = chr(as), cb = chr(bs);
    if (ca != cb) return ca < cb ? -1 : 1;
    if (ranged) {
      if (as < be) return (ae + range > bs) ? 0 : -1;
      return (be + range > as) ? 0 : 1;
    }
    const int64_t mn = as > bs ? as : bs, mx = ae < be ? ae : be;
    if (mx > mn) return 0;
    return as < bs ? -1 : 1;
  };
  std::vector<uint64_t> win;
  size_t wh = 0;
  uint64_t mi = 0;
  int64_t cache = -1;
  ref_new(0);  // the iterators (ref first, Bedmap.cpp:282-284)
  map_new(0);
  for (uint64_t r = 0; r < nr; ++r) {
    ref_new(r + 1);  // ++refStart
    auto pop = [&](uint64_t w) {
      return fast_crit >= 0 ? bg_fs_m2r(fast_crit, ovr, range, perc, MS[w], ME[w], RS[r], RE[r]) < 0
                            : dist(MS[w], ME[w], RS[r], RE[r]) < 0;
    };
    while (wh < win.size() && pop(win[wh])) map_del(win[wh++]);
    if (wh > 4096 && wh * 2 > win.size()) {
      win.erase(win.begin(), win.begin() + (ptrdiff_t)wh);
      wh = 0;
    }
    while (cache >= 0 || mi < nm) {
      uint64_t m;
      if (cache >= 0) {
        m = (uint64_t)cache;
        cache = -1;
      } else {
        m = mi++;
        map_new(mi);  // ++mapFromStart
      }
      const int v = fast_crit >= 0 ? bg_fs_r2m(fast_crit, ovr, range, perc, RS[r], RE[r], MS[m], ME[m])
                                   : dist(RS[r], RE[r], MS[m], ME[m]);
      if (v == 0) win.push_back(m);
      else if (v < 0) {
        cache = (int64_t)m;
        break;
      } else {
        map_del(m);
      }
    }
    ref_del(r);
  }
}

// one file (R == M): sweep overload 1 (WindowSweepImpl.cpp:66-162; Overlapping
// specialisation WindowSweepImpl.specialize.cpp:40-138, same calls): the iterator's
// constructor reads row 0 and each ++start the next row; rows are deleted as they leave the
// deque (pops, and the whole deque when a reference row runs past its end)
static void heap_replay_single(const int64_t* S, const int64_t* E, uint64_t n, const uint8_t* mflag, bool ranged,
                               int64_t range, int64_t* addr, int fast_crit, int64_t ovr, double perc) {
  HeapClass H;
  std::unordered_map<uint64_t, RowStr> mstr;
  auto make = [&](uint8_t f, RowStr& s) {
    for (int q : {0, 1, 2, 3})
      s.a[q] = (f >> q) & 1 ? H.get() : -1;
  };
  auto drop = [&](const RowStr& s) {
    for (int q : {2, 3, 1, 0})
      if (s.a[q] >= 0) H.put(s.a[q]);
  };
  auto row_new = [&](uint64_t m) {  // m == n: the read past the last row (never freed)
    addr[m] = H.get();
    const uint8_t f = m < n ? mflag[m] : 0;
    if (f) make(f, mstr[m]);
  };
  auto row_del = [&](uint64_t m) {
    if (mflag[m]) {
      auto it = mstr.find(m);
      drop(it->second);
      mstr.erase(it);
    }
    H.put(addr[m]);
  };
  auto dist = [&](uint64_t a, uint64_t b) -> int {  // the sweep distance (a, b)
    const int64_t as = S[a], ae = E[a], bs = S[b], be = E[b];
    const int64_t ca = as >> BG_KEY_SHIFT, cb = bs >> BG_KEY_SHIFT;
    if (ca != cb) return ca < cb ? -1 : 1;
    if (ranged) {
      if (as < be) return (ae + range > bs) ? 0 : -1;
      return (be + range > as) ? 0 : 1;
    }
    const int64_t mn = as > bs ? as : bs, mx = ae < be ? ae : be;
    if (mx > mn) return 0;
    return as < bs ? -1 : 1;
  };
  auto r2m = [&](uint64_t r, uint64_t b) {
    return fast_crit >= 0 ? bg_fs_r2m(fast_crit, ovr, range, perc, S[r], E[r], S[b], E[b]) : dist(r, b);
  };
  auto m2r = [&](uint64_t w, uint64_t r) {
    return fast_crit >= 0 ? bg_fs_m2r(fast_crit, ovr, range, perc, S[w], E[w], S[r], E[r]) : dist(w, r);
  };
  std::vector<uint64_t> win;
  size_t wh = 0, index = 0;
  uint64_t next = 0;
  int64_t cache = -1;
  bool reset = true;
  row_new(0);
  for (;;) {
    if (!(next < n || cache >= 0 || win.size() > wh)) break;
    if (!reset) {
      const uint64_t cur = win[wh + index];
      while (win.size() > wh && m2r(win[wh], cur) < 0) {
        row_del(win[wh++]);
        --index;
      }
      if (wh > 4096 && wh * 2 > win.size()) {
        win.erase(win.begin(), win.begin() + (ptrdiff_t)wh);
        wh = 0;
      }
    } else if (next >= n && cache < 0) {
      break;
    }
    while (cache >= 0 || next < n) {
      uint64_t b;
      if (cache >= 0) {
        b = (uint64_t)cache;
        cache = -1;
      } else {
        b = next++;
        row_new(next);  // ++start
      }
      if (win.size() == wh || reset || r2m(win[wh + index], b) == 0) {
        if (reset) {
          reset = false;
          index = 0;
          while (win.size() > wh) row_del(win[wh++]);
          win.clear();
          wh = 0;
        }
        win.push_back(b);
      } else {
        cache = (int64_t)b;
        break;
      }
    }
    reset = ++index >= win.size() - wh;
  }
}

// the simulated address of every map row, on the device (*out, bg_alloc'ed), for bg_map
// (R == M: one file)
int bg_heap_addr(bg_ctx* c, bg_set* set, const bg_table* R, const bg_table* M, int fields, bool ranged,
                 int64_t range, int64_t** out, int fast_crit, int64_t ovr, double perc) {
  *out = nullptr;
  const uint64_t nr = R->n, nm = M->n;
  std::vector<int64_t> hRS(nr), hRE(nr), hMS(nm), hME(nm);
  std::vector<uint32_t> hli(nm, 0), hlr(nm, 0), hrl(nr, 0);
  uint32_t* dli = nullptr;
  uint32_t* dlr = nullptr;
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
  if (nr) {
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
  // the map object's chunk size, and which strings of each row share it
  const uint64_t K = hs_chunk(fields == 3 ? 32 : (fields == 4 ? 48 : 56));
  auto in = [&](uint64_t len) { return hs_chunk(len + 1) == K; };
  auto name_len = [&](int64_t key) -> uint64_t {
    const uint64_t g = (uint64_t)(key >> BG_KEY_SHIFT);
    return g < set->names.size() ? set->names[g].size() : 0;
  };
  std::vector<uint8_t> mflag(nm), rflag(nr);
  for (uint64_t m = 0; m < nm; ++m) {
    const uint64_t li = hli[m], lr = hlr[m];
    uint8_t f = in(name_len(hMS[m])) ? 1 : 0;
    if (fields >= 4) {
      f |= in(li) ? 2 : 0;
      f |= in(lr) ? 4 : 0;
      f |= hs_chunk(lr + 1 + li + 1) == K ? 8 : 0;
    } else {
      f |= in(lr) ? 4 : 0;
    }
    mflag[m] = f;
  }
  for (uint64_t r = 0; r < nr; ++r)  // the reference file is read as B3Rest (Bedmap.cpp:624-654)
    rflag[r] = (uint8_t)((in(name_len(hRS[r])) ? 1 : 0) | (in(hrl[r]) ? 4 : 0));
  std::vector<int64_t> addr(nm + 1);
  if (R == M)
    heap_replay_single(hMS.data(), hME.data(), nm, mflag.data(), ranged, range, addr.data(), fast_crit, ovr, perc);
  else
    heap_replay(hRS.data(), hRE.data(), nr, rflag.data(), hs_chunk(32) == K, hMS.data(), hME.data(), nm,
              mflag.data(), ranged, range, addr.data(), fast_crit, ovr, perc);
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
