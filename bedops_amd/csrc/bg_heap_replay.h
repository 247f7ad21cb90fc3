// bg_heap_replay.h — the host replay of the reference's allocation sequence for bedmap
// (bg_heap.hip drives it over the keyed rows; tools/heap_replay_check.cpp runs it on the CPU
// against oracle/bedmap_oracle.c's addresses). Host code only.
#pragma once
#include "bg_internal.h"

#include <algorithm>
#include <unordered_map>
#include <vector>

// chunk size of a `new char[len + 1]` / `new T` of `req` bytes (request + 8, 16-aligned, >= 32)
static inline uint64_t hs_chunk(uint64_t req) {
  const uint64_t c = (req + 8 + 15) & ~15ULL;
  return c < 32 ? 32 : c;
}

namespace {
// glibc's allocator for the replayed calls: per chunk size (32 .. 1056 bytes) a 7-entry LIFO
// thread cache and a LIFO fast bin; larger chunks come from the top and are not reused here
struct Heap {
  static constexpr int NC = 66;
  std::vector<int64_t> tc[NC], fb[NC];
  int64_t top = 0;
  int64_t get(uint64_t req) {
    const uint64_t c = hs_chunk(req);
    const uint64_t k = c / 16 - 2;
    int64_t a;
    if (k < NC) {
      auto& T = tc[k];
      auto& F = fb[k];
      if (!T.empty()) {
        a = T.back();
        T.pop_back();
        return a;
      }
      if (!F.empty()) {  // _int_malloc's fast-bin path stashes the rest of the bin
        a = F.back();
        F.pop_back();
        while (T.size() < 7 && !F.empty()) {
          T.push_back(F.back());
          F.pop_back();
        }
        return a;
      }
    }
    a = top;
    top += (int64_t)c;
    return a;
  }
  void put(uint64_t req, int64_t a) {
    const uint64_t k = hs_chunk(req) / 16 - 2;
    if (k >= NC) return;
    if (tc[k].size() < 7) tc[k].push_back(a);
    else fb[k].push_back(a);
  }
};

// one row object and its strings: object; ChromInfo() new char[1]; Bed4() new char[1] (B4/B5);
// readline re-allocates chrom_ and id_, then rest_ and fullrest_; the destructor frees rest_,
// fullrest_, id_, chrom_, then the object
struct RowMem {
  int64_t o = -1, c = -1, i = -1, r = -1, f = -1;
  uint32_t lc = 0, li = 0, lr = 0;
};
// a temporary copy of a row (see Tmp in the replay)
struct Tmp {
  int64_t c = -1, i = -1, r = -1, f = -1;
  uint64_t lc = 0, li = 0, lr = 0, lf = 0;
};

constexpr int kMaxVis = 16;
// the replay's state of a live map row
struct Live {
  RowMem mem;
  int64_t nbase = -1;  // its node in BedBaseVisitor's cache_ or win_
  int64_t nv[kMaxVis];
  uint64_t crep = 0;   // first row of its run of equal (start, end)
  bool inwin = false;  // in win_ (visitors have seen it), else in cache_
};

// rows addressed by index in a ring that holds every live row (all live rows are >= lo)
struct Ring {
  std::vector<Live> buf;
  uint64_t mask = 0;
  Live& at(uint64_t m) { return buf[m & mask]; }
  void need(uint64_t lo, uint64_t m) {  // make row m addressable, keeping rows [lo, m)
    if (buf.empty()) {
      buf.resize(1024);
      mask = 1023;
    }
    if (m - lo < buf.size()) return;
    size_t n = buf.size();
    while (m - lo >= n) n *= 2;
    std::vector<Live> nb(n);
    for (uint64_t k = lo; k < m; ++k) nb[k & (n - 1)] = buf[k & mask];
    buf.swap(nb);
    mask = n - 1;
  }
};

// visitor containers: 1 one node per row (EchoMapBed family, EchoMapIntersectLength,
// OvrAggregate); 2 one node per distinct coordinates (OvrUnique, OvrUniqueFract)
static int vis_set(int op) {
  switch (op) {
    case BG_MAP_ECHO_MAP: case BG_MAP_ECHO_MAP_ID: case BG_MAP_ECHO_MAP_SCORE: case BG_MAP_ECHO_MAP_SIZE:
    case BG_MAP_ECHO_MAP_RANGE: case BG_MAP_ECHO_MAP_ID_UNIQ: case BG_MAP_ECHO_OVERLAP_SIZE: case BG_MAP_BASES:
      return 1;
    case BG_MAP_BASES_UNIQ: case BG_MAP_BASES_UNIQ_F:
      return 2;
  }
  return 0;
}

struct Replay {
  // inputs (host copies)
  const int64_t *RS, *RE, *MS, *ME;
  uint64_t nr, nm;
  bool single;
  int fields;
  const uint32_t *mli, *mlr, *rlr, *rrank;
  std::vector<uint32_t> mlc, rlc;  // chromosome name lengths
  const bg_heap_spec* spec;
  int64_t* addr;  // out: object address of each map row
  // state
  Heap H;
  Ring L;
  RowMem rmem[2];
  int64_t refa[2] = {0, 0};
  std::vector<uint64_t> win;  // the sweep's deque [wh, win.size())
  size_t wh = 0;
  int64_t cache = -1;
  uint64_t lo_live = 0;
  long cnt = 0;  // MultiVisitor's add/delete balance
  uint64_t prev_crep = 0;
  std::vector<std::unordered_map<uint64_t, std::pair<int64_t, uint64_t>>> keyed;  // crep -> (node, holder)
  std::vector<uint64_t> ev, dl;

  uint64_t objsize() const { return fields == 3 ? 32 : (fields == 4 ? 48 : 56); }
  void row_new(RowMem& x, int fl, uint32_t lc, uint32_t li, uint32_t lr) {
    x.lc = lc;
    x.li = li;
    x.lr = lr;
    x.o = H.get(fl == 3 ? 32 : (fl == 4 ? 48 : 56));
    const int64_t c1 = H.get(1);
    const int64_t i1 = fl >= 4 ? H.get(1) : 0;
    H.put(1, c1);
    x.c = H.get(lc + 1);
    if (fl >= 4) {
      H.put(1, i1);
      x.i = H.get(li + 1);
    }
    x.r = H.get(lr + 1);
    if (fl >= 4) x.f = H.get((uint64_t)lr + 1 + li + 1);
  }
  void row_del(const RowMem& x, int fl) {
    H.put(x.lr + 1, x.r);
    if (fl >= 4) {
      H.put((uint64_t)x.lr + 1 + x.li + 1, x.f);
      H.put(x.li + 1, x.i);
    }
    H.put(x.lc + 1, x.c);
    H.put(fl == 3 ? 32 : (fl == 4 ? 48 : 56), x.o);
  }
  uint64_t lowest_live(uint64_t next) const {
    uint64_t lo = next;
    if (wh < win.size()) lo = std::min<uint64_t>(lo, win[wh]);
    if (cache >= 0) lo = std::min<uint64_t>(lo, (uint64_t)cache);
    return lo;
  }
  void map_new(uint64_t m) {  // m == nm: the row read at end of file (never freed)
    // live: the deque, the held row, and row m - 1 (read, not yet placed)
    L.need(std::min<uint64_t>(lowest_live(m), m ? m - 1 : 0), m);
    Live& x = L.at(m);
    x = Live();
    for (int q = 0; q < kMaxVis; ++q) x.nv[q] = -1;
    if (m < nm) {
      row_new(x.mem, fields, mlc[m], mli[m], mlr[m]);
      x.crep = prev_crep = (m && MS[m] == MS[m - 1] && ME[m] == ME[m - 1]) ? prev_crep : m;
    } else {
      row_new(x.mem, fields, 0, 0, 0);
    }
    addr[m] = x.mem.o;
  }
  void map_del(uint64_t m) { row_del(L.at(m).mem, fields); }
  void ref_new(uint64_t r) {
    const int k = (int)(r & 1);
    if (r < nr) row_new(rmem[k], 3, rlc[r], 0, rlr[r]);
    else row_new(rmem[k], 3, 0, 0, 0);
    refa[k] = rmem[k].o;
  }
  void ref_del(uint64_t r) { row_del(rmem[r & 1], 3); }

  // -- distances ---------------------------------------------------------------------
  int64_t ida(uint64_t r) const { return single ? addr[r] : refa[r & 1]; }
  // Overlapping(ovr)(a, b) with its address tie (BedDistances.hpp:97-115)
  static int ovl(int64_t as, int64_t ae, int64_t bs, int64_t be, int64_t ovr, int64_t pa, int64_t pb) {
    const int64_t ca = as >> BG_KEY_SHIFT, cb = bs >> BG_KEY_SHIFT;
    if (ca != cb) return ca > cb ? 1 : -1;
    const int64_t mn = as > bs ? as : bs, mx = ae < be ? ae : be;
    if (mx > mn) {
      if (mx - mn >= ovr) return 0;
      if (as != bs) return as < bs ? -1 : 1;
      if (ae != be) return ae < be ? -1 : 1;
      return pa < pb ? -1 : 1;
    }
    return as < bs ? -1 : 1;
  }
  const int64_t* rs() const { return single ? MS : RS; }
  const int64_t* re() const { return single ? ME : RE; }
  // the sweep's Ref2Map(r, m) / Map2Ref(m, r): Overlapping(0) or RangedDist(R); --faster the
  // criterion itself (Bedmap.cpp:287-290)
  int sweep_r2m(uint64_t r, uint64_t m) const {
    const int64_t s = rs()[r], e = re()[r];
    if (spec->faster) {
      if (spec->crit == BG_OVR_BP) return ovl(s, e, MS[m], ME[m], spec->ovr, ida(r), addr[m]);
      return bg_fs_r2m(spec->crit, spec->ovr, spec->range, spec->perc, s, e, MS[m], ME[m]);
    }
    if (spec->crit == BG_OVR_RANGE) return bg_fs_ranged(s, e, MS[m], ME[m], spec->range);
    return ovl(s, e, MS[m], ME[m], 0, 0, 0);
  }
  int sweep_m2r(uint64_t m, uint64_t r) const {
    const int64_t s = rs()[r], e = re()[r];
    if (spec->faster) {
      if (spec->crit == BG_OVR_BP) return ovl(MS[m], ME[m], s, e, spec->ovr, addr[m], ida(r));
      return bg_fs_m2r(spec->crit, spec->ovr, spec->range, spec->perc, MS[m], ME[m], s, e);
    }
    if (spec->crit == BG_OVR_RANGE) return bg_fs_ranged(MS[m], ME[m], s, e, spec->range);
    return ovl(MS[m], ME[m], s, e, 0, 0, 0);
  }
  // the visitors' criterion (fixWindow keeps a row iff Map2Ref is 0)
  bool crit_in(uint64_t m, uint64_t r) const {
    return bg_map_in(spec->crit, spec->ovr, spec->range, spec->perc, rs()[r], re()[r], MS[m], ME[m]);
  }
  // CoordRestAddressCompare
  bool rless(uint64_t a, uint64_t b) const {
    if (MS[a] != MS[b]) return MS[a] < MS[b];
    if (ME[a] != ME[b]) return ME[a] < ME[b];
    if (rrank[a] != rrank[b]) return rrank[a] < rrank[b];
    return addr[a] < addr[b];
  }
  // one file under the Overlapping specialisation: rows shorter than the required overlap
  // reach no visitor (WindowSweepImpl.specialize.cpp:66-67, 110-111)
  bool visible(uint64_t m) const {
    return !single || spec->crit != BG_OVR_BP || ME[m] - MS[m] >= (spec->faster ? spec->ovr : 0);
  }

  // -- visitors (MultiVisitor: each in command-line order, MultiVisitor.hpp:71-81) ------
  void vis_add(uint64_t m) {
    Live& x = L.at(m);
    for (int q = 0; q < spec->nops; ++q) {
      const int k = vis_set(spec->ops[q]);
      if (k == 1) x.nv[q] = H.get(40);
      else if (k == 2) {
        auto& K = keyed[q];
        if (K.find(x.crep) == K.end()) K[x.crep] = {H.get(40), m};
      }
    }
    ++cnt;
  }
  void vis_del(uint64_t m) {
    Live& x = L.at(m);
    for (int q = 0; q < spec->nops; ++q) {
      const int k = vis_set(spec->ops[q]);
      if (k == 1 && x.nv[q] >= 0) {
        H.put(40, x.nv[q]);
        x.nv[q] = -1;
      } else if (k == 2) {
        auto& K = keyed[q];
        auto it = K.find(x.crep);
        if (it != K.end()) {
          H.put(40, it->second.first);
          K.erase(it);
        }
      }
    }
    --cnt;
  }
  void on_add(uint64_t m) {
    if (spec->faster) {
      if (visible(m)) {
        L.at(m).inwin = true;
        vis_add(m);
      }
      return;
    }
    L.at(m).nbase = H.get(40);  // cache_.insert
  }
  void on_delete(uint64_t m) {
    Live& x = L.at(m);
    if (spec->faster) {
      if (visible(m)) {
        x.inwin = false;
        vis_del(m);
      }
      return;
    }
    if (x.inwin) vis_del(m);  // Delete, win_.erase; else cache_.erase
    x.inwin = false;
    H.put(40, x.nbase);
    x.nbase = -1;
  }

  // -- DoneReference temporaries ----------------------------------------------------
  // a copy of a row of `fl` columns: chrom_, id_, rest_, fullrest_ (B5Rest: one byte short)
  void tmp_sizes(Tmp& t, int fl, uint64_t lc, uint64_t li, uint64_t lr, bool copy) const {
    t.lc = lc + 1;
    t.li = li + 1;
    if (copy && fl == 5) {
      t.lr = lr ? lr - 1 : 0;
      t.lf = li + lr ? li + lr - 1 : 0;
    } else {
      t.lr = lr + 1;
      t.lf = li + lr + 1;
    }
  }
  void tmp_copy(Tmp& t, int fl, uint64_t lc, uint64_t li, uint64_t lr) {
    tmp_sizes(t, fl, lc, li, lr, true);
    t.c = H.get(t.lc);
    if (fl >= 4) t.i = H.get(t.li);
    t.r = H.get(t.lr);
    if (fl >= 4) t.f = H.get(t.lf);
  }
  void tmp_assign(Tmp& t, int fl, uint64_t lc, uint64_t li, uint64_t lr) {
    Tmp n;
    tmp_sizes(n, fl, lc, li, lr, false);
    H.put(t.lc, t.c);
    t.c = H.get(n.lc);
    if (fl >= 4) {
      H.put(t.li, t.i);
      t.i = H.get(n.li);
    }
    H.put(t.lr, t.r);
    if (fl >= 4) H.put(t.lf, t.f);
    t.r = H.get(n.lr);
    if (fl >= 4) t.f = H.get(n.lf);
    t.lc = n.lc;
    t.li = n.li;
    t.lr = n.lr;
    t.lf = n.lf;
  }
  void tmp_drop(const Tmp& t, int fl) {
    H.put(t.lr, t.r);
    if (fl >= 4) {
      H.put(t.lf, t.f);
      H.put(t.li, t.i);
    }
    H.put(t.lc, t.c);
  }
  void tmp_copy_map(Tmp& t, uint64_t m) { tmp_copy(t, fields, mlc[m], mli[m], mlr[m]); }
  void done(uint64_t r) {
    if (spec->skip_unmapped && cnt == 0) return;  // MultiVisitor::DoneReference, :84-98
    for (int q = 0; q < spec->nops; ++q) {
      const int op = spec->ops[q];
      if (op == BG_MAP_ECHO_OVERLAP_SIZE) {  // EchoMapIntersectLengthVisitor.hpp:64-73
        int64_t buf = -1;
        uint64_t cap = 0;
        for (long k = 0; k < cnt; ++k) {
          Tmp t;
          if (single) tmp_copy_map(t, r);
          else tmp_copy(t, 3, rlc[r], 0, rlr[r]);
          if ((uint64_t)k == cap) {  // _M_realloc_insert: allocate, move, free the old buffer
            const uint64_t nc = cap ? 2 * cap : 1;
            const int64_t nb = H.get(nc * 8);
            if (cap) H.put(cap * 8, buf);
            buf = nb;
            cap = nc;
          }
          tmp_drop(t, single ? fields : 3);
        }
        if (cap) H.put(cap * 8, buf);
      } else if (op == BG_MAP_ECHO_MAP_RANGE) {  // PrintGenomicRange's copy of the first row
        uint64_t first = ~0ULL;
        for (size_t k = wh; k < win.size(); ++k) {
          const uint64_t m = win[k];
          if (!L.at(m).inwin) continue;
          if (first == ~0ULL) first = m;
          else if (MS[m] == MS[first] && ME[m] == ME[first]) {
            if (addr[m] < addr[first]) first = m;
          } else {
            break;
          }
        }
        if (first != ~0ULL) {
          Tmp t;
          tmp_copy_map(t, first);
          tmp_drop(t, fields);
        }
      } else if (op == BG_MAP_BASES_UNIQ || op == BG_MAP_BASES_UNIQ_F) {  // OvrUniqueVisitor.hpp:63-78
        auto& K = keyed[q];
        bool have = false;
        Tmp t;
        int64_t ts = 0, te = 0, ps = 0, pe = 0;
        for (size_t k = wh; k < win.size(); ++k) {
          const uint64_t m = win[k];
          const Live& x = L.at(m);
          if (!x.inwin) continue;
          const int64_t s = MS[m], e = ME[m];
          if (!have) {
            tmp_copy_map(t, K[x.crep].second);
            ts = s;
            te = e;
            have = true;
          } else {
            if (s == ps && e == pe) continue;  // one node per distinct coordinates
            const int64_t mn = ts > s ? ts : s, mx = te < e ? te : e;
            if (mx > mn) {  // overlap: eunion
              ts = ts < s ? ts : s;
              te = te > e ? te : e;
            } else {  // tmpOvrRange = **i
              const uint64_t h = K[x.crep].second;
              tmp_assign(t, fields, mlc[h], mli[h], mlr[h]);
              ts = s;
              te = e;
            }
          }
          ps = s;
          pe = e;
        }
        if (have) tmp_drop(t, fields);
      }
    }
  }
  // BedBaseVisitor::OnDone: fixWindow (deletions, insertions, cache_.insert(lst)), then
  // DoneReference; --faster: DoneReference only
  void on_done(uint64_t r) {
    if (!spec->faster) {
      ev.clear();
      for (size_t k = wh; k < win.size(); ++k)
        if (L.at(win[k]).inwin && !crit_in(win[k], r)) ev.push_back(win[k]);
      std::sort(ev.begin(), ev.end(), [&](uint64_t a, uint64_t b) { return rless(a, b); });
      for (uint64_t m : ev) {  // Delete, lst.push_back, win_.erase
        Live& x = L.at(m);
        vis_del(m);
        H.put(40, x.nbase);
        x.nbase = -1;
        x.inwin = false;
      }
      dl.swap(ev);
      ev.clear();
      for (size_t k = wh; k < win.size(); ++k) {
        const uint64_t m = win[k];
        const Live& x = L.at(m);
        if (!x.inwin && x.nbase >= 0 && crit_in(m, r)) ev.push_back(m);
      }
      std::sort(ev.begin(), ev.end(), [&](uint64_t a, uint64_t b) { return rless(a, b); });
      for (uint64_t m : ev) {  // Add, win_.insert, cache_.erase
        Live& x = L.at(m);
        vis_add(m);
        const int64_t n = H.get(40);
        H.put(40, x.nbase);
        x.nbase = n;
        x.inwin = true;
      }
      for (uint64_t m : dl) L.at(m).nbase = H.get(40);  // cache_.insert(lst), list order
    }
    done(r);
  }

  // -- the sweeps -------------------------------------------------------------------
  // overload 2 (WindowSweepImpl.cpp:168-256), the iterators reading one row ahead (ref first,
  // Bedmap.cpp:282-284)
  void run2() {
    uint64_t mi = 0;
    ref_new(0);
    map_new(0);
    for (uint64_t r = 0; r < nr; ++r) {
      ref_new(r + 1);  // ++refStart
      while (wh < win.size() && sweep_m2r(win[wh], r) < 0) {
        on_delete(win[wh]);
        map_del(win[wh++]);
      }
      compact();
      while (cache >= 0 || mi < nm) {
        uint64_t m;
        if (cache >= 0) {
          m = (uint64_t)cache;
          cache = -1;
        } else {
          m = mi++;
          map_new(mi);  // ++mapFromStart
        }
        const int v = sweep_r2m(r, m);
        if (v == 0) {
          win.push_back(m);
          on_add(m);
        } else if (v < 0) {
          cache = (int64_t)m;
          break;
        } else {
          map_del(m);
        }
      }
      on_done(r);
      ref_del(r);
    }
  }
  // overload 1 (WindowSweepImpl.cpp:66-162; Overlapping specialisation
  // WindowSweepImpl.specialize.cpp:40-138, same calls): the iterator's constructor reads row 0
  // and each ++start the next; rows are deleted as they leave the deque
  void run1() {
    uint64_t next = 0;
    size_t index = 0;
    uint64_t cur = 0;
    bool reset = true;
    map_new(0);
    for (;;) {
      if (!(next < nm || cache >= 0 || win.size() > wh)) break;
      if (!reset) {
        cur = win[wh + index];  // OnStart
        while (win.size() > wh && sweep_m2r(win[wh], cur) < 0) {
          on_delete(win[wh]);
          map_del(win[wh++]);
          --index;
        }
        compact();
      } else if (next >= nm && cache < 0) {
        break;
      }
      while (cache >= 0 || next < nm) {
        uint64_t b;
        if (cache >= 0) {
          b = (uint64_t)cache;
          cache = -1;
        } else {
          b = next++;
          map_new(next);  // ++start
        }
        if (win.size() == wh || reset || sweep_r2m(win[wh + index], b) == 0) {
          if (reset) {
            reset = false;
            index = 0;
            cur = b;  // OnStart(bPtr)
            while (win.size() > wh) {
              on_delete(win[wh]);
              map_del(win[wh++]);
            }
            win.clear();
            wh = 0;
          }
          win.push_back(b);
          on_add(b);
        } else {
          cache = (int64_t)b;
          break;
        }
      }
      on_done(cur);
      reset = ++index >= win.size() - wh;
    }
  }
  void compact() {
    if (wh > 4096 && wh * 2 > win.size()) {
      win.erase(win.begin(), win.begin() + (ptrdiff_t)wh);
      wh = 0;
    }
  }
};
}  // namespace
