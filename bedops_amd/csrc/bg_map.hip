// bg_map.hip — K5: bedmap <operations> ref map, under every overlap criterion.
//
// Reference: WindowSweep::sweep overload 2 (interfaces/src/algorithm/sweep/
// WindowSweepImpl.cpp:168-256) keeps a deque window of map rows under the SWEEP distance
// (Overlapping(0), or RangedDist(R) for --range: applications/bed/bedmap/src/Bedmap.cpp:
// 95-155); BedBaseVisitor::fixWindow (algorithm/visitors/bed/BedBaseVisitor.hpp:184-215)
// keeps the members whose VISITOR distance Map2Ref(map, ref) is 0, and the visitors
// aggregate over that final window. For every reference row r that yields the multiset
//   S(r) = { m : same chrom, m in the sweep window of r, criterion(r, m) }
// with the criteria of data/bed/BedDistances.hpp (Overlapping :80-118, RangedDist :41-67,
// PercentOverlapMapping/Reference/Either/Both :123-288 in the reference's double
// arithmetic, Exact :293-317). Verified against the oracle's restatement of the sweep
// (oracle/bedmap_oracle.c) by randomized differential tests (tests/test_gpu_parity.py).
// GPU form: map rows are start-sorted, so with L = the longest map row every candidate
// starts in [r.s - R - L + 1, r.e + R) (R = 0 except --range), clamped to r's chromosome.
// Each workgroup bounds the candidate range of its 256 rows with two searches over the
// whole map table; each row's own searches then run over that cache-resident slice, and
// one thread per reference row walks its candidates in start order, accumulating
//   count, exact integer score sum, min / max score, Σ overlap bp (OvrAggregate
//   OvrAggregateVisitor.hpp:77-97) and the bp of r covered by the union of S(r)
//   (OvrUnique, OvrUniqueVisitor.hpp:62-78: pieces merged in genomic order).
// Exactness: Average/Sum keep ONE running double across the file (AverageVisitor.hpp:46-54,
// SumVisitor.hpp:47-51); it equals the exact per-row integer sum whenever scores are
// integers and partial sums stay below 2^53. Other inputs are refused (BG_E_UNSUPPORTED)
// rather than approximated. Min/max involve no arithmetic and take any score.
// Zero-length rows (k_mz_*): under Overlapping(0) a zero-length row overlaps nothing, and
// the sweep then (a) deletes every unread map row starting at or before a zero-length
// reference row, (b) pops every window row starting before it, and (c) stops reading at a
// zero-length map row starting after the current reference start (it is cached, and hides
// the rows behind it). The window is then no longer "every overlapping map row": each map
// row m is a window member of the reference rows [zin[m], zout[m]) only, computed from the
// map-stream position after each reference row (k_mz_walk) — see k_mz_member.
#include <cfloat>
#include <climits>
#include <cstring>

#include "bg_internal.h"

#define NEED_SUM 1u
#define NEED_EXT 2u
#define NEED_BASES 4u
#define NEED_UNIQ 8u
#define NEED_SQ 32u   // sum of squares (Variance, StdDev, CV)
#define NEED_WIN 16u  // --echo-map*: keep each row's candidate range for the formatter

struct MapArgs {
  const int64_t* RS;
  const int64_t* RE;
  uint64_t nr;
  const int64_t* MS;
  const int64_t* ME;
  const double* SC;
  uint64_t nm;
  int64_t L;       // longest map row
  int64_t ovr;     // --bp-ovr
  int64_t range;   // --range R
  double perc;     // PercentOverlapMapping::perc_ (set up on the host as its constructor does)
  uint32_t need;   // NEED_* columns to compute
  int32_t* cnt;
  int64_t* isum;
  double* vmin;
  double* vmax;
  uint64_t* bases;
  uint32_t* uniq;
  int64_t* isq;
  uint64_t* wlo;
  uint64_t* whi;
  LongRows lrows;      // rows longer than L by length class (bg_map_cands); L = its threshold
  const int64_t* zin;  // zero-length rows: window membership (bg_map_live), else null
  const int64_t* zout;
  int64_t touch;       // 1: rows that only touch the reference row can be in S(r) (tiny fractions)
  bg_dstatus* st;
};

__device__ __forceinline__ int64_t wmax64(int64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = max(v, (int64_t)__shfl_xor(v, d, 64));
  return v;
}

// m in S(r)? (bg_map_in with the criterion folded at compile time)
template <int CRIT>
__device__ __forceinline__ bool map_in(int64_t s, int64_t e, int64_t ms, int64_t me,
                                       const MapArgs& A) {
  return bg_map_in(CRIT, A.ovr, A.range, A.perc, s, e, ms, me);
}

// first index k in [lo, hi) with X[k] >= v, X in LDS
__device__ __forceinline__ uint32_t lds_lower_bound(const int64_t* X, uint32_t lo, uint32_t hi,
                                                    int64_t v) {
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (X[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

#define MAP_SLICE 3072  // map starts staged per workgroup (24 KiB of LDS)

// CRIT == BG_OVR_FAST (bedmap --faster, bg_faster.hip): the window [wlo, whi) of every row
// is an input, its members are the rows that joined the sweep's deque (zin), and no criterion
// is re-tested
// (staging the candidates' ends and scores beside their starts, 72 KiB of LDS, measured 6.5 ->
// 12.0 ms on 50M x 500M, round 5: 2 workgroups per CU; the workgroups' candidate ranges from
// separate pre-kernels measured 6.62 -> 6.93 ms)
template <int CRIT, bool ZM, bool LONG>
__global__ void __launch_bounds__(BG_NT) k_map_ops(MapArgs A) {
  __shared__ int64_t wmax[BG_NT / 64];
  __shared__ uint64_t bnd[2];
  __shared__ int64_t xs[MAP_SLICE];  // the workgroup's candidate starts, when they fit
  constexpr bool FAST = CRIT == BG_OVR_FAST;
  const uint64_t r0 = (uint64_t)blockIdx.x * BG_NT;
  const uint64_t r = r0 + threadIdx.x;
  const bool live = r < A.nr;
  const int64_t s = live ? A.RS[r] : 0, e = live ? A.RE[r] : 0;
  const int64_t g = s & ~BG_COORD_MASK;  // the row's chromosome in key space
  const int64_t pad = (CRIT == BG_OVR_RANGE) ? A.range : 0;
  const int64_t klo = max(g, s - pad - A.L + 1 - A.touch);          // non-decreasing in r
  // (--exact: a zero-length row matches rows starting at its end, itself in one-file mode;
  // tiny fractions: rows touching either end)
  const int64_t khi = min(g + (1LL << BG_KEY_SHIFT), e + pad + (CRIT == BG_OVR_EXACT ? 1 : A.touch));
  uint64_t blo = 0, bhi = 0;
  if (!FAST) {
    const int64_t hm = wmax64(live ? khi : LLONG_MIN);
    if (bg_lane() == 0) wmax[bg_wave()] = hm;
    __syncthreads();
    if (threadIdx.x == 0) bnd[0] = lower_bound_i64(A.MS, A.nm, klo);  // row r0 is live
    if (threadIdx.x == 64) {
      int64_t m = wmax[0];
      for (int w = 1; w < BG_NT / 64; ++w) m = max(m, wmax[w]);
      bnd[1] = lower_bound_i64(A.MS, A.nm, m);
    }
    __syncthreads();
    blo = bnd[0];
    bhi = max(bnd[0], bnd[1]);
  }
  // the slice every row of this workgroup searches: staged in LDS when it fits (a search
  // level then costs an LDS read instead of an L2 round trip)
  const bool staged = !FAST && bhi - blo <= MAP_SLICE;
  if (staged) {
    for (uint32_t i = threadIdx.x; i < bhi - blo; i += BG_NT) {
      xs[i] = A.MS[blo + i];
    }
    __syncthreads();
  }
  if (!live) return;
  uint64_t lo, hi;
  if (FAST) {
    lo = A.wlo[r];
    hi = A.whi[r];
  } else if (staged) {
    const uint32_t n = (uint32_t)(bhi - blo);
    const uint32_t l = lds_lower_bound(xs, 0, n, klo);
    lo = blo + l;
    hi = blo + lds_lower_bound(xs, l, n, khi);
  } else {
    lo = lower_bound_in(A.MS, blo, bhi, klo);
    hi = lower_bound_in(A.MS, lo, bhi, khi);
  }
  if (A.wlo && !FAST) {
    A.wlo[r] = lo;
    A.whi[r] = hi;
  }
  int32_t c = 0;
  int64_t sum = 0, sq = 0;
  double vmin = 0, vmax = 0;
  uint64_t bases = 0;
  uint32_t uniq = 0;                // unsigned int arithmetic, as OvrUnique's
  int64_t us = 0, ue = LLONG_MIN;  // current union piece
  auto visit = [&](int64_t ms, int64_t me, double x) {  // one member of S(r), in start order
    if (A.need & (NEED_SUM | NEED_EXT)) {
      sum += (int64_t)x;
      if (A.need & NEED_SQ) sq += (int64_t)x * (int64_t)x;
      if (c == 0) vmin = vmax = x;
      else {
        if (x < vmin) vmin = x;
        if (x > vmax) vmax = x;
      }
    }
    ++c;
    if (A.need & NEED_BASES) bases += (uint64_t)max(min(e, me) - max(s, ms), (int64_t)0);
    if (A.need & NEED_UNIQ) {
      // OvrUnique merges a row into the current piece only when they overlap by > 0 bp
      // (BasicCoords::overlap, Bed.hpp:172-190): a zero-length row closes the piece
      if (min(ue, me) > max(us, ms)) {
        us = min(us, ms);
        ue = max(ue, me);
      } else {
        if (ue > us) uniq += (uint32_t)max(min(e, ue) - max(s, us), (int64_t)0);
        us = ms;
        ue = me;
      }
    }
  };
  if (LONG) {  // short range + the long rows' class ranges, merged in index order
    bg_map_cands(A.MS, A.ME, lo, hi, A.lrows, s, e, pad, [&](uint64_t m) {
      const int64_t ms = A.MS[m], me = A.ME[m];
      if ((!ZM || bg_map_live(A.zin, A.zout, r, m)) && map_in<CRIT>(s, e, ms, me, A))
        visit(ms, me, (A.need & (NEED_SUM | NEED_EXT)) ? A.SC[m] : 0.0);
      return true;
    });
  } else {
  // candidates in groups of MU: the group's loads are issued together (they are
  // independent; one at a time, every candidate paid a cache round trip)
  constexpr int MU = 4;
  for (uint64_t m0 = lo; m0 < hi; m0 += MU) {
    int64_t ms[MU], me[MU];
    double sc[MU];
    bool live_m[MU];
#pragma unroll
    for (int j = 0; j < MU; ++j) {
      const uint64_t m = min(m0 + j, hi - 1);
      ms[j] = staged ? xs[m - blo] : A.MS[m];
      me[j] = A.ME[m];
      sc[j] = (A.need & (NEED_SUM | NEED_EXT)) ? A.SC[m] : 0.0;
      live_m[j] = !ZM || bg_map_live(A.zin, A.zout, r, m);
    }
#pragma unroll
    for (int j = 0; j < MU; ++j) {
      if (m0 + j >= hi || !live_m[j] || !map_in<CRIT>(s, e, ms[j], me[j], A)) continue;
      visit(ms[j], me[j], sc[j]);
    }
  }
  }
  if ((A.need & NEED_UNIQ) && ue > us) uniq += (uint32_t)max(min(e, ue) - max(s, us), (int64_t)0);
  A.cnt[r] = c;
  if (A.isum) {
    A.isum[r] = sum;
    if (sum >= (1LL << 53) || sum <= -(1LL << 53)) atomicOr(&A.st->flags, 4ULL);
  }
  if (A.isq) {
    A.isq[r] = sq;
    if (sq >= (1LL << 53) || sq < 0) atomicOr(&A.st->flags, 4ULL);
  }
  if (A.vmin) { A.vmin[r] = vmin; A.vmax[r] = vmax; }
  if (A.bases) A.bases[r] = bases;
  if (A.uniq) A.uniq[r] = uniq;
}

// ------------------------------- zero-length rows ---------------------------------
// The map-stream position p_i after reference row i (the index of the row it leaves
// cached, WindowSweepImpl.cpp:214-234): starting from p_{i-1}, rows are consumed until one
// starts after r.start without overlapping r, i.e. (map rows start-sorted)
//   p_i = min(max(p_{i-1}, A_i), Z(max(p_{i-1}, C_i)))
// with C_i = first map row starting after r.start, A_i = first starting at or after r.end
// (= C_i for a zero-length r) and Z(x) = first zero-length map row at index >= x. When no
// earlier reference row ends past r.start + 1, p_{i-1} <= C_i and p_i = min(A_i, Z(C_i))
// does not depend on the past: those rows start the segments k_mz_walk replays, one thread
// per segment.
__global__ void k_mz_flags(const int64_t* __restrict__ S, const int64_t* __restrict__ E,
                           const int64_t* __restrict__ PM, uint64_t n, uint8_t* __restrict__ f) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  f[i] = PM ? (S[i] + 1 >= PM[i]) : (S[i] == E[i]);  // segment start | zero-length row
}

__device__ __forceinline__ uint64_t mz_next_zero(const uint64_t* zm, uint64_t nz, uint64_t nm,
                                                 uint64_t x) {
  uint64_t lo = 0, hi = nz;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (zm[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo < nz ? zm[lo] : nm;
}

__global__ void k_mz_walk(const int64_t* __restrict__ RS, const int64_t* __restrict__ RE,
                          uint64_t nr, const int64_t* __restrict__ MS, uint64_t nm,
                          const uint64_t* __restrict__ zm, uint64_t nz,
                          const uint64_t* __restrict__ seg, uint64_t nseg, int64_t* __restrict__ P) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nseg) return;
  const uint64_t i0 = seg[k], i1 = k + 1 < nseg ? seg[k + 1] : nr;
  uint64_t p = 0;
  for (uint64_t i = i0; i < i1; ++i) {
    const int64_t s = RS[i], e = RE[i];
    const uint64_t pp = (i == i0) ? 0 : p;
    const uint64_t C = upper_bound_in(MS, min(pp, nm), nm, s);
    const uint64_t A = (e > s) ? lower_bound_in(MS, C, nm, e) : C;
    p = min(max(pp, A), mz_next_zero(zm, nz, nm, max(pp, C)));
    P[i] = (int64_t)p;
  }
}

// Map row m is consumed by reference row i* = first i with p_i > m, and enters the window
// iff it overlaps r_{i*} (else it is deleted, :232-233). It leaves at the first
// zero-length reference row after i* that starts after m.start (which pops every window
// row starting before it, :207-211); a non-empty reference row only pops rows that end at
// or before its start, which no later row overlaps. zin = i* (INT64_MAX: never a member),
// zout = that zero-length row (nr: none).
__global__ void k_mz_member(const int64_t* __restrict__ RS, const int64_t* __restrict__ RE,
                            uint64_t nr, const int64_t* __restrict__ MS,
                            const int64_t* __restrict__ ME, uint64_t nm,
                            const int64_t* __restrict__ P, const uint64_t* __restrict__ zr,
                            uint64_t nzr, int64_t* __restrict__ zin, int64_t* __restrict__ zout) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nm) return;
  const int64_t ms = MS[m], me = ME[m];
  const uint64_t is = upper_bound_i64(P, nr, (int64_t)m);
  const bool added = is < nr && min(RE[is], me) > max(RS[is], ms);
  zin[m] = added ? (int64_t)is : LLONG_MAX;
  uint64_t lo = 0, hi = nzr;  // first zero-length row index > is
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (zr[mid] <= is) lo = mid + 1;
    else hi = mid;
  }
  uint64_t lo2 = 0, hi2 = nzr;  // first zero-length row starting after ms
  while (lo2 < hi2) {
    const uint64_t mid = (lo2 + hi2) >> 1;
    if (RS[zr[mid]] <= ms) lo2 = mid + 1;
    else hi2 = mid;
  }
  const uint64_t k = max(lo, lo2);
  zout[m] = k < nzr ? (int64_t)zr[k] : (int64_t)nr;
}

// One file (sweep overload 1, WindowSweepImpl.specialize.cpp:40-138, run with Overlapping(0)
// under every criterion but --range, Bedmap.cpp:108-152): the deque after row i's pops and
// reads is [f_i, p_i) (every row joins it), the --faster replay's own chains with the sweep
// distance Overlapping(0) (bg_faster_windows); f and p never decrease, so row m is a member
// for the rows i with f_i <= m < p_i: mz_in = the first i with p_i > m, mz_out = the first
// i with f_i > m. BedBaseVisitor then re-tests each member with the criterion (fixWindow,
// BedBaseVisitor.hpp:184-215), as k_map_ops does for bg_map_live members.
__global__ void k_mz_single(const uint64_t* __restrict__ f, const uint64_t* __restrict__ p, uint64_t n,
                            int64_t* __restrict__ zin, int64_t* __restrict__ zout) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  zin[m] = (int64_t)upper_bound_i64((const int64_t*)p, n, (int64_t)m);
  zout[m] = (int64_t)upper_bound_i64((const int64_t*)f, n, (int64_t)m);
}
static int map_zero_prep_single(bg_ctx* c, const bg_table* R, bg_result* res) {
  const uint64_t n = R->n;
  if (!n) return 0;
  res->zin = (int64_t*)bg_alloc(c, 8 * n);
  res->zout = (int64_t*)bg_alloc(c, 8 * n);
  uint64_t* f = (uint64_t*)bg_alloc(c, 8 * n);
  uint64_t* p = (uint64_t*)bg_alloc(c, 8 * n);
  int64_t* j0 = (int64_t*)bg_alloc(c, 8 * n);
  int64_t* j1 = (int64_t*)bg_alloc(c, 8 * n);
  int rc = (!res->zin || !res->zout || !f || !p || !j0 || !j1) ? BG_E_NOMEM : 0;
  if (!rc) rc = bg_faster_windows(c, R, R, BG_OVR_BP, 0, 0, 1.0, true, f, p, j0, j1);
  if (!rc) {
    BG_LAUNCH(c, "k_mz_single", k_mz_single, dim3(bg_blocks(n, BG_NT)), dim3(BG_NT), f, p, n, res->zin, res->zout);
    rc = bg_hip_ok(c, hipGetLastError());
  }
  bg_release(c, f);
  bg_release(c, p);
  bg_release(c, j0);
  bg_release(c, j1);
  return rc;
}

// Two files under a tiny fraction (perc_ <= DBL_EPSILON): S(r) takes every deque member
// not strictly apart from r, so the windows are the sweep's deque (overload 2 under
// Overlapping(0), Bedmap.cpp:108-138): [f_i, p_i) over the rows that joined it, from the
// --faster replay's chains; a joined row m is a member for i in [first p_i > m, first f_i > m)
__global__ void k_mz_deque(const uint64_t* __restrict__ f, const uint64_t* __restrict__ p, uint64_t nr,
                           const int64_t* __restrict__ joined, uint64_t nm, int64_t* __restrict__ zin,
                           int64_t* __restrict__ zout) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nm) return;
  zin[m] = joined[m] == INT64_MAX ? INT64_MAX : (int64_t)upper_bound_i64((const int64_t*)p, nr, (int64_t)m);
  zout[m] = (int64_t)upper_bound_i64((const int64_t*)f, nr, (int64_t)m);
}
static int map_deque_prep(bg_ctx* c, const bg_table* R, const bg_table* M, bg_result* res) {
  const uint64_t nr = R->n, nm = M->n;
  if (!nr || !nm) return 0;
  res->zin = (int64_t*)bg_alloc(c, 8 * nm);
  res->zout = (int64_t*)bg_alloc(c, 8 * nm);
  uint64_t* f = (uint64_t*)bg_alloc(c, 8 * nr);
  uint64_t* p = (uint64_t*)bg_alloc(c, 8 * nr);
  int64_t* j0 = (int64_t*)bg_alloc(c, 8 * nm);
  int64_t* j1 = (int64_t*)bg_alloc(c, 8 * nm);
  int rc = (!res->zin || !res->zout || !f || !p || !j0 || !j1) ? BG_E_NOMEM : 0;
  if (!rc) rc = bg_faster_windows(c, R, M, BG_OVR_BP, 0, 0, 1.0, false, f, p, j0, j1);
  if (!rc) {
    BG_LAUNCH(c, "k_mz_deque", k_mz_deque, dim3(bg_blocks(nm, BG_NT)), dim3(BG_NT), f, p, nr, j0, nm, res->zin,
              res->zout);
    rc = bg_hip_ok(c, hipGetLastError());
  }
  bg_release(c, f);
  bg_release(c, p);
  bg_release(c, j0);
  bg_release(c, j1);
  return rc;
}

static int map_zero_prep(bg_ctx* c, const bg_table* R, const bg_table* M, bg_result* res) {
  const uint64_t nr = R->n, nm = M->n;
  if (!nr || !nm) return 0;
  res->zin = (int64_t*)bg_alloc(c, 8 * nm);
  res->zout = (int64_t*)bg_alloc(c, 8 * nm);
  int64_t* PM = (int64_t*)bg_alloc(c, 8 * nr);
  int64_t* P = (int64_t*)bg_alloc(c, 8 * nr);
  uint8_t* f = (uint8_t*)bg_alloc(c, max(nr, nm));
  if (!res->zin || !res->zout || !PM || !P || !f) return BG_E_NOMEM;
  int rc = bg_scan_max_i64(c, R->ke, PM, nr, LLONG_MIN);
  if (rc) return rc;
  uint64_t *seg = nullptr, *zm = nullptr, *zr = nullptr, nseg = 0, nz = 0, nzr = 0;
  BG_LAUNCH(c, "k_mz_flags", k_mz_flags, dim3(bg_blocks(nr, BG_NT)), dim3(BG_NT), R->ks, R->ke, PM, nr, f);
  if ((rc = bg_compact_flags(c, f, nr, &seg, &nseg))) return rc;
  BG_LAUNCH(c, "k_mz_flags", k_mz_flags, dim3(bg_blocks(nm, BG_NT)), dim3(BG_NT), M->ks, M->ke,
            (const int64_t*)nullptr, nm, f);
  if ((rc = bg_compact_flags(c, f, nm, &zm, &nz))) return rc;
  BG_LAUNCH(c, "k_mz_flags", k_mz_flags, dim3(bg_blocks(nr, BG_NT)), dim3(BG_NT), R->ks, R->ke,
            (const int64_t*)nullptr, nr, f);
  if ((rc = bg_compact_flags(c, f, nr, &zr, &nzr))) return rc;
  if (nseg)
    BG_LAUNCH(c, "k_mz_walk", k_mz_walk, dim3(bg_blocks(nseg, BG_NT)), dim3(BG_NT), R->ks, R->ke, nr,
              M->ks, nm, zm, nz, seg, nseg, P);
  BG_LAUNCH(c, "k_mz_member", k_mz_member, dim3(bg_blocks(nm, BG_NT)), dim3(BG_NT), R->ks, R->ke, nr,
            M->ks, M->ke, nm, P, zr, nzr, res->zin, res->zout);
  BG_HIP(c, hipGetLastError());
  bg_release(c, PM);
  bg_release(c, P);
  bg_release(c, f);
  bg_release(c, seg);
  bg_release(c, zm);
  bg_release(c, zr);
  return 0;
}

// ------------------------------- running doubles (decimal scores) ------------------
// Average / Sum / Variance keep ONE running double (sum_, squareSum_) for the whole file
// (AverageVisitor.hpp:46-54, SumVisitor.hpp:47-51, VarianceVisitor.hpp:45-55): with
// non-integer scores every printed value depends on the exact order of all earlier Add and
// Delete calls, and two runs that start from different sums never re-converge (measured:
// DESIGN.md §5.2), so the sums are replayed exactly, in the reference's event order:
//   at reference row i (after row i-1 left S(r_{i-1}) as BedBaseVisitor::win_):
//   (a) the sweep pops the deque front while Map2Ref(front, r_i) < 0 (WindowSweepImpl.cpp:
//       207-211): members of S(r_{i-1}) popped there are Deleted in file order; a member m
//       is popped iff it is poppable (ends R or more before r_i.start, or lies on an
//       earlier chromosome) and no earlier row still in the deque is not, i.e. m < f_i, the
//       first candidate of r_i that is not poppable (a row before it that is not poppable
//       would overlap r_i, and every row overlapping r_i was added to the deque);
//   (b) fixWindow Deletes the other members of S(r_{i-1}) that fail the criterion for r_i,
//   (c) then Adds the rows of S(r_i) \ S(r_{i-1}) — both in set order
//       (CoordRestAddressCompare: start, end, id + remainder, address ~ row index).
// k_mev counts and writes that event stream (+score / -score, and +-fl(score^2) for the
// Variance family); k_mev_chain folds it with one wavefront in order (the only sequential
// step: one FP64 add per event on the critical path), and k_mev_pick reads each row's sums
// after its last event.
struct EvArgs {
  const int64_t* RS;
  const int64_t* RE;
  uint64_t nr;
  const int64_t* MS;
  const int64_t* ME;
  const double* SC;
  uint64_t nm;
  const uint64_t* wlo;
  const uint64_t* whi;
  int64_t ovr, range;
  double perc;
  const char* text;  // map text + remainder spans: full_rest() for the set order
  const uint64_t* rest_off;
  const uint32_t* rest_len;
  int mapfields;
  const int64_t* addr;  // simulated heap addresses (bg_heap.hip), null: row order
  const uint32_t* ro;   // each run of equal starts in set order (k_ev_rank), null: select
  const ulonglong2* P;  // first 16 bytes of each row's full_rest(), big-endian, 0-padded (k_ev_keys)
  const uint32_t* PL;   // full_rest() length
  const int64_t* zin;   // --faster: rows that joined the deque (zin != INT64_MAX), else null
  // zero-length rows (not --faster): map row m is a sweep-window member of the reference rows
  // [mz_in[m], mz_out[m]) only (k_mz_member, k_mz_single), else null
  const int64_t* mz_in;
  const int64_t* mz_out;
  bool mz_exact;  // the membership is the deque itself (one file; tiny fractions): pops = leaving it
};
__device__ __forceinline__ bool ev_live(const EvArgs& A, uint64_t r, uint64_t m) {
  return bg_map_live(A.mz_in, A.mz_out, r, m);
}

__device__ __forceinline__ int ev_rest_cmp(const EvArgs& A, uint64_t a, uint64_t b) {
  return bg_frest_cmp(A.text, A.rest_off, A.rest_len, A.mapfields, a, b);
}
// strcmp order of full_rest(a) and full_rest(b) from the 16-byte prefixes; the byte
// comparison only when both strings run past the prefix and it ties
__device__ __forceinline__ int ev_rest_cmp_k(const EvArgs& A, uint64_t a, uint64_t b) {
  const ulonglong2 x = A.P[a], y = A.P[b];
  if (x.x != y.x) return x.x < y.x ? -1 : 1;
  if (x.y != y.y) return x.y < y.y ? -1 : 1;
  const uint32_t la = A.PL[a], lb = A.PL[b];
  if (min(la, lb) < 16) return la == lb ? 0 : (la < lb ? -1 : 1);
  return ev_rest_cmp(A, a, b);
}
// CoordRestAddressCompare for two rows of equal start
__device__ __forceinline__ bool ev_less(const EvArgs& A, uint64_t a, uint64_t b) {
  if (A.ME[a] != A.ME[b]) return A.ME[a] < A.ME[b];
  const int c = A.P ? ev_rest_cmp_k(A, a, b) : ev_rest_cmp(A, a, b);
  if (c != 0) return c < 0;
  return bg_maddr(A.addr, a) < bg_maddr(A.addr, b);
}
// first index in (m, b] whose start differs from MS[m] (starts are sorted): a gallop, so a
// lone row costs one load and a run of g equal starts O(log g)
__device__ __forceinline__ uint64_t ev_run_hi(const int64_t* MS, uint64_t m, uint64_t b) {
  const int64_t v = MS[m];
  uint64_t lo = m + 1;
  if (lo >= b || MS[lo] != v) return lo;
  uint64_t step = 1;  // MS[lo] == v
  while (lo + step < b && MS[lo + step] == v) {
    lo += step;
    step <<= 1;
  }
  uint64_t hi = min(lo + step, b);  // MS[hi] != v, or hi == b
  while (hi - lo > 1) {
    const uint64_t mid = lo + (hi - lo) / 2;
    if (MS[mid] == v) lo = mid;
    else hi = mid;
  }
  return hi;
}
// first index f <= m with MS[f..m] all equal to MS[m]
__device__ __forceinline__ uint64_t ev_run_lo(const int64_t* MS, uint64_t m) {
  const int64_t v = MS[m];
  if (m == 0 || MS[m - 1] != v) return m;
  uint64_t hi = m - 1, step = 1;  // MS[hi] == v
  while (hi >= step && MS[hi - step] == v) {
    hi -= step;
    step <<= 1;
  }
  // the run starts in (hi - step, hi]; hi - step may be "before 0"
  uint64_t lo = hi >= step ? hi - step : 0;  // MS[lo] != v unless lo == 0 and it is equal
  if (lo == 0 && MS[0] == v) return 0;
  while (hi - lo > 1) {
    const uint64_t mid = lo + (hi - lo) / 2;
    if (MS[mid] == v) hi = mid;
    else lo = mid;
  }
  return hi;
}
// the rows of [a, b) that satisfy `pred`, in set order (rows are start-sorted: only runs of
// equal starts need ordering). With A.ro each whole run is visited in its precomputed set
// order (O(run) per walk); without it, by selection (O(run^2): 10k equal rows made every
// window that holds them take 10^8 comparisons)
template <typename Pred, typename Emit>
__device__ __forceinline__ void ev_walk(const EvArgs& A, uint64_t a, uint64_t b, Pred pred, Emit emit) {
  uint64_t m = a;
  while (m < b) {
    const uint64_t g1 = ev_run_hi(A.MS, m, b);
    if (g1 - m == 1) {
      if (pred(m)) emit(m);
    } else if (A.ro) {
      // the whole run (the window may cut it)
      const uint64_t f0 = m == a ? ev_run_lo(A.MS, m) : m;
      const uint64_t f1 = g1 == b ? ev_run_hi(A.MS, m, A.nm) : g1;
      for (uint64_t q = f0; q < f1; ++q) {
        const uint64_t t = A.ro[q];
        if (t >= m && t < g1 && pred(t)) emit(t);
      }
    } else {
      uint64_t last = ~0ULL;
      for (;;) {
        uint64_t best = ~0ULL;
        for (uint64_t t = m; t < g1; ++t) {
          if (!pred(t)) continue;
          if (last != ~0ULL && !ev_less(A, last, t)) continue;
          if (best == ~0ULL || ev_less(A, t, best)) best = t;
        }
        if (best == ~0ULL) break;
        emit(best);
        last = best;
      }
    }
    m = g1;
  }
}

// A.ro: the rank of row t in its run of equal starts under CoordRestAddressCompare (a
// strict total order: addresses are distinct), counted against the whole run — O(run) per
// row, so O(run^2) once per map instead of per window, for runs of up to EV_RUN_DEV rows;
// longer runs (a pile of reads at one position) are listed in `longs` (count in *nlong) and
// sorted on the host in O(run log run) (ev_long_order)
#define EV_RUN_DEV 2048
__global__ void __launch_bounds__(BG_NT) k_ev_rank(EvArgs A, uint32_t* __restrict__ ro, uint64_t* __restrict__ longs,
                                                   unsigned long long* __restrict__ nlong) {
  const uint64_t t = (uint64_t)blockIdx.x * BG_NT + threadIdx.x;
  if (t >= A.nm) return;
  const int64_t s = A.MS[t];
  const bool alone = (t == 0 || A.MS[t - 1] != s) && (t + 1 >= A.nm || A.MS[t + 1] != s);
  if (alone) {
    ro[t] = (uint32_t)t;
    return;
  }
  const uint64_t f0 = ev_run_lo(A.MS, t), f1 = ev_run_hi(A.MS, t, A.nm);
  if (f1 - f0 > EV_RUN_DEV) {
    if (t == f0) longs[atomicAdd(nlong, 1ULL)] = f0;
    return;
  }
  uint64_t r = 0;
  // (ME, prefix) decide almost every pair: independent loads, no byte walks
  const int64_t te = A.ME[t];
  const ulonglong2 tp = A.P[t];
#pragma unroll 4
  for (uint64_t u = f0; u < f1; ++u) {
    const int64_t ue = A.ME[u];
    const ulonglong2 up = A.P[u];
    bool less;
    if (ue != te) less = ue < te;
    else if (up.x != tp.x) less = up.x < tp.x;
    else if (up.y != tp.y) less = up.y < tp.y;
    else less = u != t && ev_less(A, u, t);
    r += less ? 1 : 0;
  }
  ro[f0 + r] = (uint32_t)t;
}

// A.P / A.PL: the first 16 bytes of every map row's full_rest() (big-endian: integer order =
// strcmp order of the prefixes; 0-padded) and its length
__global__ void __launch_bounds__(BG_NT) k_ev_keys(EvArgs A, ulonglong2* __restrict__ P, uint32_t* __restrict__ PL) {
  const uint64_t t = (uint64_t)blockIdx.x * BG_NT + threadIdx.x;
  if (t >= A.nm) return;
  uint64_t hi = 0, lo = 0;
  uint32_t len = 0;
  if (A.rest_off) {
    const char *p1, *p2;
    uint32_t l1, l2;
    bg_frest(A.text, A.rest_off, A.rest_len, A.mapfields, t, p1, l1, p2, l2);
    len = l1 + l2;
    for (uint32_t q = 0; q < 16 && q < len; ++q) {
      const uint64_t b = (uint8_t)(q < l1 ? p1[q] : p2[q - l1]);
      if (q < 8) hi |= b << (56 - 8 * q);
      else lo |= b << (56 - 8 * (q - 8));
    }
  }
  P[t] = make_ulonglong2(hi, lo);
  PL[t] = len;
}

// the visitor events between reference rows i-1 and i, in the reference's order:
// (a) sweep pops and (b) fixWindow Deletes of S(r_{i-1}) members (skipped when !dels),
// then (c) the Adds of S(r_i) \ S(r_{i-1})
template <int CRIT, typename Del, typename Add>
__device__ __forceinline__ void ev_events(const EvArgs& A, uint64_t i, bool dels, Del emit_del, Add emit_add) {
  if constexpr (CRIT == BG_OVR_FAST) {
    // --faster: the visitors see the sweep's own calls (no BedBaseVisitor in between): the
    // front pops [f_{i-1}, f_i) (WindowSweepImpl.cpp:207-211; one file :92-96 and the whole
    // deque on a restart :132-136), then each row read into the deque (:219-221; :139-140),
    // both in file order
    if (i > 0 && dels)
      for (uint64_t m = A.wlo[i - 1]; m < A.wlo[i]; ++m)
        if (A.zin[m] != INT64_MAX) emit_del(m);
    for (uint64_t m = i ? A.whi[i - 1] : 0; m < A.whi[i]; ++m)
      if (A.zin[m] != INT64_MAX) emit_add(m);
    return;
  }
  const int64_t s = A.RS[i], e = A.RE[i];
  const int64_t g = s & ~BG_COORD_MASK;
  const int64_t R = (CRIT == BG_OVR_RANGE) ? A.range : 0;
  const uint64_t lo = A.wlo[i], hi = A.whi[i];
  const bool hp = i > 0;
  const int64_t ps = hp ? A.RS[i - 1] : 0, pe = hp ? A.RE[i - 1] : 0;
  const uint64_t plo = hp ? A.wlo[i - 1] : 0, phi = hp ? A.whi[i - 1] : 0;
  uint64_t f = lo;  // first candidate of r_i that the sweep cannot pop
  while (f < hi && A.ME[f] + R <= s) ++f;
  // S(r) = the sweep-window members (every candidate, or the zero-length replay's [mz_in,
  // mz_out)) that meet the criterion; the sweep itself deletes the rows it pops at r_i and,
  // with zero-length rows, every member whose window membership ends at r_i (a zero-length
  // reference row's pops, WindowSweepImpl.cpp:207-211; one file, a restart :132-136)
  auto in_prev = [&](uint64_t m) {
    return hp && m >= plo && m < phi && ev_live(A, i - 1, m) &&
           bg_map_in(CRIT, A.ovr, A.range, A.perc, ps, pe, A.MS[m], A.ME[m]);
  };
  auto in_cur = [&](uint64_t m) {
    return (A.MS[m] & ~BG_COORD_MASK) == g && ev_live(A, i, m) &&
           bg_map_in(CRIT, A.ovr, A.range, A.perc, s, e, A.MS[m], A.ME[m]);
  };
  auto popped = [&](uint64_t m) {
    if (A.mz_exact) return !ev_live(A, i, m);
    return (m < f && ((A.ME[m] & ~BG_COORD_MASK) != g || A.ME[m] + R <= s)) || (A.mz_in && !ev_live(A, i, m));
  };
  if (hp && dels) {
    for (uint64_t m = plo; m < phi; ++m)  // (a) in deque (file) order
      if (in_prev(m) && popped(m)) emit_del(m);
    ev_walk(A, plo, phi, [&](uint64_t m) { return in_prev(m) && !popped(m) && !in_cur(m); }, emit_del);
  }
  ev_walk(A, lo, hi, [&](uint64_t m) { return in_cur(m) && !in_prev(m); }, emit_add);  // (c)
}

template <int CRIT, bool WRITE>
__global__ void __launch_bounds__(BG_NT) k_mev(EvArgs A, uint64_t* __restrict__ cnt,
                                               const uint64_t* __restrict__ off,
                                               double* __restrict__ X, double* __restrict__ X2) {
  const uint64_t i = (uint64_t)blockIdx.x * BG_NT + threadIdx.x;
  if (i >= A.nr) return;
  uint64_t k = 0;
  const uint64_t base = WRITE ? off[i] : 0;
  auto emit_del = [&](uint64_t m) {
    if (WRITE) {
      const double x = A.SC[m];
      X[base + k] = -x;
      if (X2) X2[base + k] = -(x * x);
    }
    ++k;
  };
  auto emit_add = [&](uint64_t m) {
    if (WRITE) {
      const double x = A.SC[m];
      X[base + k] = x;
      if (X2) X2[base + k] = x * x;
    }
    ++k;
  };
  ev_events<CRIT>(A, i, true, emit_del, emit_add);
  if (!WRITE) cnt[i] = k;
}

__device__ __forceinline__ double readlane_f64(double v, int j) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, j);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), j);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// one wavefront folds the whole event stream in order: SA[k] = sum_ after event k
// (QA: squareSum_); `s += x` with x = -score for a Delete is exactly `sum_ -= score`.
// The fold is a chain of dependent FP64 adds, so nothing else may sit on it: blocks of
// MC_BLK events are staged in LDS by all 64 lanes (coalesced loads issued one block AHEAD,
// in flight while the chain runs), lane 0 alone walks the block (an LDS read that does not
// depend on the sum, the add, an LDS write of the partial sum), and the partial sums go
// back to HBM coalesced. (Round 2 broadcast each event with two v_readlane and captured
// the sum with a lane select: five VALU ops per event around the add, 4 ns per event.)
#define MC_BLK 1024
#define MC_G 32  // values lane 0 holds in registers per half-step of the chain
// lane 0's fold of one staged block: the values of the next MC_G events are read from LDS
// into registers before the adds of the current MC_G (two register sets, no copies)
template <bool SQ>
__device__ __forceinline__ void mev_fold(const double* xs, const double* ys, double* ss, double* qs,
                                         double& s, double& q) {
  double a[MC_G], b[MC_G], ay[MC_G], by[MC_G];
#pragma unroll
  for (int j = 0; j < MC_G; ++j) {
    a[j] = xs[j];
    if (SQ) ay[j] = ys[j];
  }
  for (int g = 0; g < MC_BLK; g += 2 * MC_G) {
#pragma unroll
    for (int j = 0; j < MC_G; ++j) {
      b[j] = xs[g + MC_G + j];
      if (SQ) by[j] = ys[g + MC_G + j];
    }
#pragma unroll
    for (int j = 0; j < MC_G; ++j) {
      s += a[j];
      ss[g + j] = s;
      if (SQ) {
        q += ay[j];
        qs[g + j] = q;
      }
    }
    if (g + 2 * MC_G < MC_BLK) {
#pragma unroll
      for (int j = 0; j < MC_G; ++j) {
        a[j] = xs[g + 2 * MC_G + j];
        if (SQ) ay[j] = ys[g + 2 * MC_G + j];
      }
    }
#pragma unroll
    for (int j = 0; j < MC_G; ++j) {
      s += b[j];
      ss[g + MC_G + j] = s;
      if (SQ) {
        q += by[j];
        qs[g + MC_G + j] = q;
      }
    }
  }
}

__global__ void __launch_bounds__(64) k_mev_chain(const double* __restrict__ X,
                                                  const double* __restrict__ X2, uint64_t E,
                                                  double* __restrict__ SA, double* __restrict__ QA) {
  __shared__ double xs[MC_BLK], ys[MC_BLK], ss[MC_BLK], qs[MC_BLK];
  constexpr int PER = MC_BLK / 64;
  const int lane = threadIdx.x;
  const bool sq = X2 != nullptr;
  double s = 0.0, q = 0.0;  // lane 0's running sums
  double px[PER], py[PER];
  auto fetch = [&](uint64_t b) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const uint64_t k = b + (uint64_t)i * 64 + lane;
      px[i] = k < E ? X[k] : 0.0;
      py[i] = (sq && k < E) ? X2[k] : 0.0;
    }
  };
  fetch(0);
  for (uint64_t b = 0; b < E; b += MC_BLK) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      xs[i * 64 + lane] = px[i];
      ys[i * 64 + lane] = py[i];
    }
    __syncthreads();
    if (b + MC_BLK < E) fetch(b + MC_BLK);  // the next block in flight during the fold
    // the last block is padded with +0.0 events: they only follow every real event, and
    // the sums after them are never stored
    if (lane == 0) {
      if (sq) mev_fold<true>(xs, ys, ss, qs, s, q);
      else mev_fold<false>(xs, ys, ss, qs, s, q);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const uint64_t k = b + (uint64_t)i * 64 + lane;
      if (k < E) {
        SA[k] = ss[i * 64 + lane];
        if (QA) QA[k] = qs[i * 64 + lane];
      }
    }
    __syncthreads();  // the next block's staging overwrites xs/ss
  }
}

// each row's running sums after its last event (0 before any event: the visitors start at 0)
__global__ void k_mev_pick(const uint64_t* __restrict__ off, uint64_t nr, const double* __restrict__ SA,
                           const double* __restrict__ QA, double* __restrict__ dsum,
                           double* __restrict__ dsq) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nr) return;
  const uint64_t end = off[i + 1];
  dsum[i] = end ? SA[end - 1] : 0.0;
  if (dsq) dsq[i] = end ? QA[end - 1] : 0.0;
}

// A.ro for every run of equal map starts: k_ev_rank, then the long runs it listed sorted here
// by (end, full_rest(), address) — CoordRestAddressCompare's order for rows of one start
static int ev_order(bg_ctx* c, const EvArgs& E, const bg_table* M, int fields, uint32_t* ro) {
  const uint64_t nm = E.nm;
  BgHold hold(c);
  uint64_t* dl = hold((uint64_t*)bg_alloc(c, 8 * (nm + 1)));
  if (!dl) return BG_E_NOMEM;
  BG_HIP(c, hipMemsetAsync(dl + nm, 0, 8, c->stream));
  BG_LAUNCH(c, "k_ev_rank", k_ev_rank, dim3(bg_blocks(nm, BG_NT)), dim3(BG_NT), E, ro, dl,
            (unsigned long long*)(dl + nm));
  int rc = bg_hip_ok(c, hipGetLastError());
  uint64_t nl = 0;
  if (rc || (rc = bg_fetch_u64(c, dl + nm, &nl))) return rc;
  if (nl) {
    std::vector<uint64_t> f0(nl);
    BG_HIP(c, hipMemcpyAsync(f0.data(), dl, 8 * nl, hipMemcpyDeviceToHost, c->stream));
    std::vector<int64_t> ms(nm), me(nm), ad;
    BG_HIP(c, hipMemcpyAsync(ms.data(), E.MS, 8 * nm, hipMemcpyDeviceToHost, c->stream));
    BG_HIP(c, hipMemcpyAsync(me.data(), E.ME, 8 * nm, hipMemcpyDeviceToHost, c->stream));
    if (E.addr) {
      ad.resize(nm);
      BG_HIP(c, hipMemcpyAsync(ad.data(), E.addr, 8 * nm, hipMemcpyDeviceToHost, c->stream));
    }
    BG_HIP(c, hipStreamSynchronize(c->stream));
    std::vector<uint64_t> rows, run;  // run k: rows[run[k], run[k + 1])
    for (uint64_t a : f0) {
      run.push_back(rows.size());
      for (uint64_t m = a; m < nm && ms[m] == ms[a]; ++m) rows.push_back(m);
    }
    run.push_back(rows.size());
    std::vector<char> txt;
    std::vector<uint64_t> off;
    if (M->rest_off && (rc = bg_frest_gather(c, M, fields, rows, txt, off))) return rc;
    auto less = [&](uint64_t i, uint64_t j) {  // rows[i] vs rows[j]
      const uint64_t a = rows[i], b = rows[j];
      if (me[a] != me[b]) return me[a] < me[b];
      if (M->rest_off) {
        const char *x = txt.data() + off[i], *y = txt.data() + off[j];
        const uint64_t lx = off[i + 1] - off[i], ly = off[j + 1] - off[j];
        if (bg_bytes_less(x, lx, y, ly)) return true;
        if (bg_bytes_less(y, ly, x, lx)) return false;
      }
      return (E.addr ? ad[a] : (int64_t)a) < (E.addr ? ad[b] : (int64_t)b);
    };
    std::vector<uint64_t> ix;
    std::vector<uint32_t> out;
    for (uint64_t k = 0; k + 1 < run.size(); ++k) {
      ix.resize(run[k + 1] - run[k]);
      for (uint64_t i = 0; i < ix.size(); ++i) ix[i] = run[k] + i;
      std::sort(ix.begin(), ix.end(), less);
      out.resize(ix.size());
      for (uint64_t i = 0; i < ix.size(); ++i) out[i] = (uint32_t)rows[ix[i]];
      BG_HIP(c, hipMemcpyAsync(ro + rows[run[k]], out.data(), 4 * out.size(), hipMemcpyHostToDevice, c->stream));
      BG_HIP(c, hipStreamSynchronize(c->stream));
    }
  }
  return 0;
}

template <int CRIT>
static int map_running_sums_t(bg_ctx* c, const EvArgs& A, bool need_sq, bg_result* res) {
  const uint64_t nr = A.nr;
  const unsigned nb = bg_blocks(nr, BG_NT);
  uint64_t* off = (uint64_t*)bg_alloc(c, 8 * (nr + 1));
  if (!off) return BG_E_NOMEM;
  BG_LAUNCH(c, "k_mev_count", (k_mev<CRIT, false>), dim3(nb), dim3(BG_NT), A, off,
            (const uint64_t*)nullptr, (double*)nullptr, (double*)nullptr);
  BG_HIP(c, hipGetLastError());
  int rc = bg_scan_sum_u64(c, off, off, nr, off + nr);
  uint64_t E = 0;
  if (rc || (rc = bg_fetch_u64(c, off + nr, &E))) return rc;
  const uint64_t E1 = E ? E : 1;
  double* X = (double*)bg_alloc(c, 8 * E1);
  double* X2 = need_sq ? (double*)bg_alloc(c, 8 * E1) : nullptr;
  double* SA = (double*)bg_alloc(c, 8 * E1);
  double* QA = need_sq ? (double*)bg_alloc(c, 8 * E1) : nullptr;
  if (!X || !SA || (need_sq && (!X2 || !QA))) return BG_E_NOMEM;
  BG_LAUNCH(c, "k_mev_write", (k_mev<CRIT, true>), dim3(nb), dim3(BG_NT), A, (uint64_t*)nullptr,
            (const uint64_t*)off, X, X2);
  if (E) BG_LAUNCH(c, "k_mev_chain", k_mev_chain, dim3(1), dim3(64), X, X2, E, SA, QA);
  BG_LAUNCH(c, "k_mev_pick", k_mev_pick, dim3(nb), dim3(BG_NT), off, nr, SA, QA, res->dsum, res->dsq);
  BG_HIP(c, hipGetLastError());
  bg_release(c, off);
  bg_release(c, X);
  bg_release(c, X2);
  bg_release(c, SA);
  bg_release(c, QA);
  return 0;
}

static int map_running_sums(bg_ctx* c, int crit, const EvArgs& A, bool need_sq, bg_result* res) {
  switch (crit) {
    case BG_OVR_BP: return map_running_sums_t<BG_OVR_BP>(c, A, need_sq, res);
    case BG_OVR_RANGE: return map_running_sums_t<BG_OVR_RANGE>(c, A, need_sq, res);
    case BG_OVR_FRAC_REF: return map_running_sums_t<BG_OVR_FRAC_REF>(c, A, need_sq, res);
    case BG_OVR_FRAC_MAP: return map_running_sums_t<BG_OVR_FRAC_MAP>(c, A, need_sq, res);
    case BG_OVR_FRAC_EITHER: return map_running_sums_t<BG_OVR_FRAC_EITHER>(c, A, need_sq, res);
    case BG_OVR_FRAC_BOTH: return map_running_sums_t<BG_OVR_FRAC_BOTH>(c, A, need_sq, res);
    case BG_OVR_FAST: return map_running_sums_t<BG_OVR_FAST>(c, A, need_sq, res);
    default: return map_running_sums_t<BG_OVR_EXACT>(c, A, need_sq, res);
  }
}

// ------------------------------- --tmean: TrimmedMean replayed --------------------------
// TrimmedMean (numerical/TrimmedMeanVisitor.hpp:40-220) keeps its window in a std::set
// ordered by (score, address) (CompValueThenAddressLesser, OrderCompare.hpp:31-38) and two
// markers, each an element with its position and a running double (lowerSum_/upperSum_)
// moved by every Add/Delete (add :153-163, remove :165-184) and walked to the trim points
// in DoneReference (doneRef :186-200). Positions equal the marker's rank, so the state is
// the sorted window + two ranks + two doubles; the doubles carry rounding from row to row.
// When S(r_{i-1}) and S(r_i) share no row, the Deletes empty the set, the last removal
// sends both markers to end(), and the next Add restarts them (sum = score): nothing is
// carried across such a row. The rows are cut there into independent segments (k_tm_seg),
// and one thread per segment replays the visitor exactly, in the event order of ev_events,
// on a sorted copy of the window in HBM scratch sized by the segment's largest window.
// Addresses: the replayed heap addresses (bg_heap.hip) when a tie is possible, as in ev_less.
struct TmArgs {
  double lo, hi;  // lowerKth_, upperKth_
  int doKth, symmetric, lower;  // lower: the lower marker is maintained (lowerKth_ > 0 && !doKth_)
};
struct TmMark {
  bool valid;  // not end()
  uint64_t pos;
  double sum;
};
__device__ __forceinline__ bool tm_less(double va, uint64_t ia, double vb, uint64_t ib) {
  if (va != vb) return va < vb;
  return ia < ib;
}
template <int CRIT>
__global__ void k_tm_seg(EvArgs A, uint64_t* __restrict__ flag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.nr) return;
  uint64_t st = 1;
  if (i > 0) {
    const int64_t s = A.RS[i], e = A.RE[i], ps = A.RS[i - 1], pe = A.RE[i - 1];
    const int64_t g = s & ~BG_COORD_MASK;
    const uint64_t lo = max(A.wlo[i], A.wlo[i - 1]), hi = min(A.whi[i], A.whi[i - 1]);
    if ((ps & ~BG_COORD_MASK) == g)
      for (uint64_t m = lo; m < hi; ++m)
        if ((A.MS[m] & ~BG_COORD_MASK) == g && (CRIT != BG_OVR_FAST || A.zin[m] != INT64_MAX) &&
            (CRIT == BG_OVR_FAST || (ev_live(A, i, m) && ev_live(A, i - 1, m))) &&
            bg_map_in(CRIT, A.ovr, A.range, A.perc, s, e, A.MS[m], A.ME[m]) &&
            bg_map_in(CRIT, A.ovr, A.range, A.perc, ps, pe, A.MS[m], A.ME[m])) {
        st = 0;
        break;
      }
  }
  flag[i] = st;
}
// segment starts (flag scanned to pos), then each segment's largest window (cnt)
__global__ void k_tm_list(const uint64_t* __restrict__ flag, const uint64_t* __restrict__ pos, uint64_t n,
                          uint64_t* __restrict__ seg) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && flag[i]) seg[pos[i]] = i;
}
__global__ void k_tm_cap(const uint64_t* __restrict__ seg, uint64_t nseg, uint64_t nr,
                         const int32_t* __restrict__ cnt, uint64_t* __restrict__ cap) {
  const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nseg) return;
  const uint64_t a = seg[q], b = q + 1 < nseg ? seg[q + 1] : nr;
  int32_t mx = 0;
  for (uint64_t i = a; i < b; ++i) mx = max(mx, cnt[i]);
  cap[q] = (uint64_t)mx;
}
__device__ __forceinline__ double tm_iround(double d) {
  const double d1 = ceil(d);
  return (d >= 0) ? ((d1 - d > 0.5) ? floor(d) : d1) : ((d1 - d >= 0.5) ? floor(d) : d1);
}
// the sorted window's element moves, TM_B at a time (all loads of a batch issued before its
// stores: one HBM round trip per TM_B elements instead of per element; a window of 10^4
// equal-coordinate rows took 3-4 s one element at a time)
#define TM_B 16
// [p, n) -> [p + 1, n + 1), from the top
__device__ __forceinline__ void tm_shift_up(double* V, uint64_t* X, uint64_t p, uint64_t n) {
  uint64_t t = n;  // next destination + 1
  while (t >= p + 1 + TM_B) {
    double v[TM_B];
    uint64_t x[TM_B];
#pragma unroll
    for (int i = 0; i < TM_B; ++i) {
      v[i] = V[t - 1 - i];
      x[i] = X[t - 1 - i];
    }
#pragma unroll
    for (int i = 0; i < TM_B; ++i) {
      V[t - i] = v[i];
      X[t - i] = x[i];
    }
    t -= TM_B;
  }
  for (; t > p; --t) {
    V[t] = V[t - 1];
    X[t] = X[t - 1];
  }
}
// [p + 1, n) -> [p, n - 1), from the bottom
__device__ __forceinline__ void tm_shift_down(double* V, uint64_t* X, uint64_t p, uint64_t n) {
  uint64_t t = p;  // next destination
  while (t + 1 + TM_B <= n) {
    double v[TM_B];
    uint64_t x[TM_B];
#pragma unroll
    for (int i = 0; i < TM_B; ++i) {
      v[i] = V[t + 1 + i];
      x[i] = X[t + 1 + i];
    }
#pragma unroll
    for (int i = 0; i < TM_B; ++i) {
      V[t + i] = v[i];
      X[t + i] = x[i];
    }
    t += TM_B;
  }
  for (; t + 1 < n; ++t) {
    V[t] = V[t + 1];
    X[t] = X[t + 1];
  }
}
template <int CRIT>
__global__ void k_tm_replay(EvArgs A, TmArgs T, const uint64_t* __restrict__ seg, uint64_t nseg,
                            const uint64_t* __restrict__ soff, double* __restrict__ SV,
                            uint64_t* __restrict__ SI, double* __restrict__ out) {
  const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nseg) return;
  const uint64_t a = seg[q], b = q + 1 < nseg ? seg[q + 1] : A.nr;
  double* V = SV + soff[q];  // the set, ascending (score, row)
  uint64_t* X = SI + soff[q];
  uint64_t n = 0;
  TmMark L = {false, 0, 0.0}, U = {false, 0, 0.0};
  auto rank = [&](double v, uint64_t m) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (tm_less(V[mid], X[mid], v, m)) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  };
  auto mark_add = [&](TmMark& k, uint64_t p, double v) {  // after the insert at p
    if (!k.valid) { k.valid = true; k.pos = 0; k.sum = v; }
    else if (p <= k.pos) { ++k.pos; k.sum += v; }  // ptr < *marker
  };
  auto mark_del = [&](TmMark& k, uint64_t p, double v) {  // before the erase of rank p
    if (p < k.pos) { --k.pos; k.sum -= v; }
    else if (p == k.pos) {
      k.sum -= v;
      if (k.pos != 0) --k.pos;
      else if (n > 1) k.sum += V[1];  // ++marker: its successor (rank 0 after the erase)
      else k.valid = false;
    }
  };
  auto del = [&](uint64_t m) {
    const double v = A.SC[m];
    const uint64_t p = rank(v, (uint64_t)bg_maddr(A.addr, m));
    if (T.lower) mark_del(L, p, v);
    mark_del(U, p, v);
    tm_shift_down(V, X, p, n);
    --n;
  };
  auto add = [&](uint64_t m) {
    const double v = A.SC[m];
    const uint64_t am = (uint64_t)bg_maddr(A.addr, m);
    const uint64_t p = rank(v, am);
    tm_shift_up(V, X, p, n);
    V[p] = v;
    X[p] = am;
    ++n;
    if (T.lower) mark_add(L, p, v);
    mark_add(U, p, v);
  };
  auto walk = [&](TmMark& k, uint64_t np) {
    while (np > k.pos) { ++k.pos; k.sum += V[k.pos]; }
    while (np < k.pos) { k.sum -= V[k.pos]; --k.pos; }
  };
  for (uint64_t i = a; i < b; ++i) {
    // the first row of a segment starts from the emptied set (its Deletes reset everything)
    ev_events<CRIT>(A, i, i > a, del, add);
    if (n == 0) { out[i] = 0.0; continue; }  // NAN (the formatter prints it from cnt)
    const uint64_t size = n;
    uint64_t kl = (uint64_t)tm_iround(T.lo * (double)size);
    uint64_t kh = (uint64_t)tm_iround(T.hi * (double)size);
    kh = size - kh;
    if (T.symmetric) {
      kl = max(kl, size - kh);
      kh = size - kl;
    }
    const bool doLow = kl > 0;
    if (doLow) --kl;
    if (kh > 0) --kh;
    if (!T.doKth && doLow) walk(L, kl);
    walk(U, kh);
    double r;
    if (T.doKth || U.pos == L.pos) r = V[U.pos];
    else if (doLow) r = (U.sum - L.sum) / (double)(U.pos - L.pos);
    else r = U.sum / (double)(U.pos + 1);
    out[i] = r;
  }
}

template <int CRIT>
static int map_tmean_t(bg_ctx* c, const EvArgs& A, const int32_t* cnt, const bg_map_opts* o, bg_result* res) {
  const uint64_t nr = A.nr;
  const unsigned nb = bg_blocks(nr, BG_NT);
  uint64_t* flag = (uint64_t*)bg_alloc(c, 8 * nr);
  uint64_t* pos = (uint64_t*)bg_alloc(c, 8 * (nr + 1));
  if (!flag || !pos) return BG_E_NOMEM;
  BG_LAUNCH(c, "k_tm_seg", k_tm_seg<CRIT>, dim3(nb), dim3(BG_NT), A, flag);
  BG_HIP(c, hipGetLastError());
  int rc = bg_scan_sum_u64(c, flag, pos, nr, pos + nr);
  uint64_t nseg = 0;
  if (rc || (rc = bg_fetch_u64(c, pos + nr, &nseg))) return rc;
  uint64_t* seg = (uint64_t*)bg_alloc(c, 8 * (nseg ? nseg : 1));
  uint64_t* soff = (uint64_t*)bg_alloc(c, 8 * (nseg + 1));
  if (!seg || !soff) return BG_E_NOMEM;
  BG_LAUNCH(c, "k_tm_list", k_tm_list, dim3(nb), dim3(BG_NT), flag, pos, nr, seg);
  const unsigned ns = bg_blocks(nseg ? nseg : 1, BG_NT);
  BG_LAUNCH(c, "k_tm_cap", k_tm_cap, dim3(ns), dim3(BG_NT), seg, nseg, nr, cnt, soff);
  BG_HIP(c, hipGetLastError());
  uint64_t slots = 0;
  if ((rc = bg_scan_sum_u64(c, soff, soff, nseg, soff + nseg)) || (rc = bg_fetch_u64(c, soff + nseg, &slots)))
    return rc;
  double* SV = (double*)bg_alloc(c, 8 * (slots ? slots : 1));
  uint64_t* SI = (uint64_t*)bg_alloc(c, 8 * (slots ? slots : 1));
  if (!SV || !SI) return BG_E_NOMEM;
  for (int q = 0; q < o->n_ops && !rc; ++q) {
    if (o->ops[q] != BG_MAP_TMEAN) continue;
    TmArgs T;
    T.lo = o->op_arg[q];
    T.hi = o->op_arg2[q];
    // the constructor's tests, in the same double arithmetic (TrimmedMeanVisitor.hpp:62-73)
    T.doKth = fabs(1.0 - T.lo - T.hi) <= DBL_EPSILON;
    T.symmetric = fabs(T.lo - T.hi) <= DBL_EPSILON;
    T.lower = T.lo > 0 && !T.doKth;
    res->tmv[q] = (double*)bg_alloc(c, 8 * nr);
    if (!res->tmv[q]) return BG_E_NOMEM;
    if (nseg) BG_LAUNCH(c, "k_tm_replay", k_tm_replay<CRIT>, dim3(ns), dim3(BG_NT), A, T, seg, nseg, soff, SV, SI,
                        res->tmv[q]);
    rc = bg_hip_ok(c, hipGetLastError());
  }
  BG_HIP(c, hipStreamSynchronize(c->stream));
  bg_release(c, flag);
  bg_release(c, pos);
  bg_release(c, seg);
  bg_release(c, soff);
  bg_release(c, SV);
  bg_release(c, SI);
  return rc;
}

static int map_tmean(bg_ctx* c, int crit, const EvArgs& A, const int32_t* cnt, const bg_map_opts* o,
                     bg_result* res) {
  switch (crit) {
    case BG_OVR_BP: return map_tmean_t<BG_OVR_BP>(c, A, cnt, o, res);
    case BG_OVR_RANGE: return map_tmean_t<BG_OVR_RANGE>(c, A, cnt, o, res);
    case BG_OVR_FRAC_REF: return map_tmean_t<BG_OVR_FRAC_REF>(c, A, cnt, o, res);
    case BG_OVR_FRAC_MAP: return map_tmean_t<BG_OVR_FRAC_MAP>(c, A, cnt, o, res);
    case BG_OVR_FRAC_EITHER: return map_tmean_t<BG_OVR_FRAC_EITHER>(c, A, cnt, o, res);
    case BG_OVR_FRAC_BOTH: return map_tmean_t<BG_OVR_FRAC_BOTH>(c, A, cnt, o, res);
    case BG_OVR_FAST: return map_tmean_t<BG_OVR_FAST>(c, A, cnt, o, res);
    default: return map_tmean_t<BG_OVR_EXACT>(c, A, cnt, o, res);
  }
}

// ------------------------------- long rows by length class --------------------------
#define BG_LONG_THR 4096
__global__ void k_len_class(const int64_t* __restrict__ S, const int64_t* __restrict__ E, uint64_t n,
                            int64_t thr, uint8_t* __restrict__ cls) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t len = E[i] - S[i];
  uint8_t c = 0;
  if (len > thr) {  // class k + 1: (thr << k, thr << (k + 1)]
    int k = 0;
    while ((thr << (k + 1)) < len) ++k;
    c = (uint8_t)(k + 1);
  }
  cls[i] = c;
}
__global__ void k_is_class(const uint8_t* __restrict__ cls, uint64_t n, uint8_t want, uint8_t* __restrict__ f) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) f[i] = cls[i] == want;
}
__global__ void k_gather_i64(const int64_t* __restrict__ src, const uint64_t* __restrict__ idx, uint64_t n,
                             int64_t* __restrict__ dst) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}

// the map table's rows longer than BG_LONG_THR, grouped by length class (index order in
// each class), with their starts: res->lrows
static int map_long_rows(bg_ctx* c, const bg_table* M, bg_result* res) {
  const uint64_t n = M->n;
  uint8_t* cls = (uint8_t*)bg_alloc(c, n);
  uint8_t* f = (uint8_t*)bg_alloc(c, n);
  if (!cls || !f) return BG_E_NOMEM;
  BG_LAUNCH(c, "k_len_class", k_len_class, dim3(bg_blocks(n, BG_NT)), dim3(BG_NT), M->ks, M->ke, n,
            (int64_t)BG_LONG_THR, cls);
  std::vector<uint64_t*> lists;
  std::vector<uint64_t> counts;
  int maxc = 0;
  while (((int64_t)BG_LONG_THR << (maxc + 1)) < M->maxlen && maxc + 1 < BG_LONG_MAXC) ++maxc;
  for (int k = 0; k <= maxc; ++k) {
    BG_LAUNCH(c, "k_is_class", k_is_class, dim3(bg_blocks(n, BG_NT)), dim3(BG_NT), cls, n, (uint8_t)(k + 1), f);
    uint64_t* idx = nullptr;
    uint64_t cnt = 0;
    int rc = bg_compact_flags(c, f, n, &idx, &cnt);
    if (rc) return rc;
    lists.push_back(idx);
    counts.push_back(cnt);
  }
  uint64_t tot = 0;
  std::vector<uint64_t> coff(lists.size() + 1, 0);
  for (size_t k = 0; k < lists.size(); ++k) coff[k + 1] = coff[k] + counts[k];
  tot = coff.back();
  uint64_t* idx = (uint64_t*)bg_alloc(c, 8 * (tot ? tot : 1));
  int64_t* ls = (int64_t*)bg_alloc(c, 8 * (tot ? tot : 1));
  uint64_t* dco = (uint64_t*)bg_alloc(c, 8 * coff.size());
  if (!idx || !ls || !dco) return BG_E_NOMEM;
  for (size_t k = 0; k < lists.size(); ++k) {
    if (counts[k]) BG_HIP(c, hipMemcpyAsync(idx + coff[k], lists[k], 8 * counts[k], hipMemcpyDeviceToDevice, c->stream));
    bg_release(c, lists[k]);
  }
  if (tot) BG_LAUNCH(c, "k_gather_i64", k_gather_i64, dim3(bg_blocks(tot, BG_NT)), dim3(BG_NT), M->ks, idx, tot, ls);
  BG_HIP(c, hipMemcpyAsync(dco, coff.data(), 8 * coff.size(), hipMemcpyHostToDevice, c->stream));
  BG_HIP(c, hipStreamSynchronize(c->stream));  // coff is a host vector
  bg_release(c, cls);
  bg_release(c, f);
  res->lrows = LongRows{idx, ls, dco, (int)lists.size(), (int64_t)BG_LONG_THR};
  return 0;
}

// 1 per reference row that prints a line (MultiVisitor.hpp:83-84 skips rows without maps)
__global__ void k_map_printed(const int32_t* __restrict__ cnt, uint64_t n, uint64_t* __restrict__ f) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) f[i] = cnt[i] > 0 ? 1 : 0;
}

// force_running: integer scores whose window sums (or sums of squares) reach 2^53, where
// the reference's running doubles (AverageVisitor.hpp:46-54) round: the same replay of its
// doubles in event order as decimal scores (map_running_sums), instead of exact int64 sums
static int map_impl(bg_ctx* c, bg_set* set, int ref, int map, const bg_map_opts* opts, bg_result** out,
                    bool force_running);

extern "C" int bg_map(bg_ctx* c, bg_set* set, int ref, int map, const bg_map_opts* opts,
                      bg_result** out) {
  return map_impl(c, set, ref, map, opts, out, false);
}

static int map_impl(bg_ctx* c, bg_set* set, int ref, int map, const bg_map_opts* opts, bg_result** out,
                    bool force_running) {
  if (!c || !set || !opts || !out || ref < 0 || map < 0 || ref >= (int)set->t.size() ||
      map >= (int)set->t.size() || opts->n_ops <= 0 || opts->n_ops > 16)
    return BG_E_ARG;
  {
    const int f[2] = {ref, map};
    int rc0 = bg_need_rows(c, set, f, 2, "bedmap");
    if (rc0) return rc0;
  }
  bg_table* R = set->t[ref];
  bg_table* M = set->t[map];
  uint32_t need = 0;
  bool need_sum = false, need_ext = false;
  int mapfields = 3;  // map row type (bedmap/src/Input.hpp:401-418 MapFields)
  bool need_rrank = false, tmean = false;
  for (int k = 0; k < opts->n_ops; ++k) {
    switch (opts->ops[k]) {
      case BG_MAP_COUNT: case BG_MAP_INDICATOR: case BG_MAP_ECHO_SIZE: case BG_MAP_ECHO_NAME: break;
      case BG_MAP_MEAN: case BG_MAP_SUM: need_sum = true; break;
      case BG_MAP_MIN: case BG_MAP_MAX: need_ext = true; break;
      case BG_MAP_BASES: need |= NEED_BASES; break;
      case BG_MAP_BASES_UNIQ: case BG_MAP_BASES_UNIQ_F: need |= NEED_UNIQ; break;
      case BG_MAP_ECHO:
        if (!R->rest_off) return bg_fail(c, BG_E_ARG, "--echo needs the reference file loaded as BG_BED3_REST");
        break;
      case BG_MAP_ECHO_REF_ROW_ID: need_rrank = opts->skip_unmapped != 0; break;
      case BG_MAP_ECHO_MAP: case BG_MAP_ECHO_MAP_ID: case BG_MAP_ECHO_MAP_ID_UNIQ:
        if (!M->rest_off) return bg_fail(c, BG_E_ARG, "--echo-map/--echo-map-id need the map file loaded with its remainder (BG_BED3_REST / BG_BED5_REST)");
        need |= NEED_WIN;
        if (opts->ops[k] != BG_MAP_ECHO_MAP && mapfields < 4) mapfields = 4;
        break;
      case BG_MAP_ECHO_MAP_SCORE:
        need_ext = true;  // the map scores (no arithmetic)
        need |= NEED_WIN;
        break;
      case BG_MAP_ECHO_MAP_SIZE: case BG_MAP_ECHO_OVERLAP_SIZE: case BG_MAP_ECHO_MAP_RANGE:
        need |= NEED_WIN;
        break;
      case BG_MAP_KTH:
        if (!(opts->op_arg[k] > 0.0 && opts->op_arg[k] < 1.0))
          return bg_fail(c, BG_E_ARG, "--kth on the GPU path takes 0 < val < 1 (0 is --min, 1 is --max)");
        [[fallthrough]];
      case BG_MAP_MAD:
      case BG_MAP_MEDIAN:  // order statistics of the window's scores, taken by the formatter
        need_ext = true;
        need |= NEED_WIN;
        break;
      case BG_MAP_VARIANCE: case BG_MAP_STDEV: case BG_MAP_CV:
        need_sum = true;
        need |= NEED_SQ;
        break;
      case BG_MAP_MIN_ELEMENT: case BG_MAP_MAX_ELEMENT: case BG_MAP_MIN_ELEMENT_RAND: case BG_MAP_MAX_ELEMENT_RAND:
        // the whole row is printed, and rows equal in score and coordinates are told
        // apart by their full_rest() (the set keeps the first added)
        if (!M->rest_off) return bg_fail(c, BG_E_ARG, "--min-element/--max-element need the map file loaded as BG_BED5_REST");
        [[fallthrough]];
      case BG_MAP_WMEAN:
        need_ext = true;
        need |= NEED_WIN;
        break;
      case BG_MAP_TMEAN: {
        const double lo = opts->op_arg[k], hi = opts->op_arg2[k];
        // Input.hpp:303-325 and the constructor's assertions (TrimmedMeanVisitor.hpp:62-73)
        if (!(lo >= 0 && lo <= 1 && hi >= 0 && hi <= 1 && lo + hi <= 1 + DBL_EPSILON))
          return bg_fail(c, BG_E_ARG, "--tmean Expect 0 <= low < hi <= 1 and (low + hi) <= 1.");
        need_ext = true;
        need |= NEED_WIN;
        tmean = true;
        break;
      }
      default: return bg_fail(c, BG_E_UNSUPPORTED, "bedmap operation not on the GPU path");
    }
  }
  if (need_sum) need |= NEED_SUM;
  if (need_ext) need |= NEED_EXT;
  if (need_sum || need_ext) mapfields = 5;  // score operations read the map as B5Rest
  // any --prec >= 0 (bedmap/src/Input.hpp:133-141): digits past the fast paths' 17 come from
  // the exact formatter (bg_decfmt.h)
  if (opts->precision < 0) return bg_fail(c, BG_E_ARG, "--prec must be >= 0");
  const int crit = opts->criterion;
  const bool faster = opts->faster != 0;
  // Input.hpp:349: --faster needs a symmetric criterion the sweep can run with
  if (faster && crit != BG_OVR_BP && crit != BG_OVR_RANGE && crit != BG_OVR_FRAC_BOTH && crit != BG_OVR_EXACT)
    return bg_fail(c, BG_E_ARG, "--faster compatible with --range, --bp-ovr, --fraction-both, and --exact only");
  double perc = 1.0;
  switch (crit) {
    case BG_OVR_BP:
      if (opts->overlap_bp < 1) return BG_E_ARG;
      break;
    case BG_OVR_RANGE:
      if (opts->range_bp < 1 || opts->range_bp > (uint64_t)BG_COORD_MASK) return BG_E_ARG;
      break;
    case BG_OVR_FRAC_REF: case BG_OVR_FRAC_MAP: case BG_OVR_FRAC_EITHER: case BG_OVR_FRAC_BOTH:
      if (!(opts->fraction > 0.0 && opts->fraction <= 1.0)) return BG_E_ARG;
      // PercentOverlapMapping's constructor (BedDistances.hpp:126-136), same host doubles
      perc = opts->fraction;
      while (perc > 1) perc /= 10.0;
      perc -= DBL_EPSILON;
      if (perc <= 0.0) perc = DBL_EPSILON;
      // at perc_ <= DBL_EPSILON Ref2Map is 0 for any pair not strictly apart (:147-150): rows
      // that only touch the reference row, or have no length, are in S(r) while the sweep's
      // deque still holds them: the windows are then the deque itself (map_deque_prep)
      break;
    case BG_OVR_EXACT: break;
    default: return BG_E_ARG;
  }
  if ((need & (NEED_SUM | NEED_EXT)) && !M->score)
    return bg_fail(c, BG_E_ARG, "score operations need the map file loaded as BG_BED5");
  // decimal scores: the running doubles are replayed in event order (map_running_sums)
  const bool decimal = need_sum && (!M->score_int || force_running);
  const bool tiny = !faster && crit >= BG_OVR_FRAC_REF && crit <= BG_OVR_FRAC_BOTH && perc <= DBL_EPSILON;
  const bool need_sq = (need & NEED_SQ) != 0;
  if (decimal && opts->shard)
    return bg_fail(c, BG_E_UNSUPPORTED, "decimal-score running sums span every chromosome: not on a chromosome shard");
  if (decimal) {
    if (!M->rest_off)
      return bg_fail(c, BG_E_ARG, "non-integer scores under --mean/--sum/--variance/--stdev/--cv need the map file loaded as BG_BED5_REST (equal rows are ordered by id and remainder)");
    need &= ~(NEED_SUM | NEED_SQ);
    need |= NEED_WIN;
  }
  BG_HIP(c, hipMemsetAsync(c->dstat, 0, sizeof(bg_dstatus), c->stream));
  const uint64_t n1 = R->n ? R->n : 1;
  bg_result* res = new bg_result();
  res->ctx = c;
  res->set = set;
  res->kind = RES_MAP;
  res->n = R->n;
  res->mopts = *opts;
  if (!res->mopts.multidelim[0]) strcpy(res->mopts.multidelim, ";");  // unset: the default
  res->tab = ref;
  res->single = ref == map;
  res->cnt = (int32_t*)bg_alloc(c, 4 * n1);
  if (need & NEED_SUM) res->isum = (int64_t*)bg_alloc(c, 8 * n1);
  if (need & NEED_EXT) {
    res->vmin = (double*)bg_alloc(c, 8 * n1);
    res->vmax = (double*)bg_alloc(c, 8 * n1);
  }
  if (need & NEED_BASES) res->bases = (uint64_t*)bg_alloc(c, 8 * n1);
  if (need & NEED_UNIQ) res->uniq = (uint32_t*)bg_alloc(c, 4 * n1);
  if (need & NEED_SQ) res->isq = (int64_t*)bg_alloc(c, 8 * n1);
  if (decimal) {
    res->dsum = (double*)bg_alloc(c, 8 * n1);
    if (need_sq) res->dsq = (double*)bg_alloc(c, 8 * n1);
    if (!res->dsum || (need_sq && !res->dsq)) {
      bg_result_free(res);
      return BG_E_NOMEM;
    }
  }
  if (faster) need |= NEED_WIN;  // the windows are the sweep's (bg_faster.hip), kept for every use
  if (need & NEED_WIN) {
    res->wlo = (uint64_t*)bg_alloc(c, 8 * n1);
    res->whi = (uint64_t*)bg_alloc(c, 8 * n1);
  }
  res->map_tab = map;
  res->mapfields = mapfields;
  res->perc = perc;
  if (!res->cnt || ((need & NEED_SUM) && !res->isum) || ((need & NEED_EXT) && (!res->vmin || !res->vmax)) ||
      ((need & NEED_BASES) && !res->bases) || ((need & NEED_UNIQ) && !res->uniq) ||
      ((need & NEED_WIN) && (!res->wlo || !res->whi)) || ((need & NEED_SQ) && !res->isq)) {
    bg_result_free(res);
    return BG_E_NOMEM;
  }
  // zero-length rows change the sweep window under Overlapping(0); RangedDist (--range)
  // treats them as ordinary rows
  if (faster) {
    const uint64_t m1 = M->n ? M->n : 1;
    res->zin = (int64_t*)bg_alloc(c, 8 * m1);
    res->zout = (int64_t*)bg_alloc(c, 8 * m1);
    int rf = (!res->zin || !res->zout) ? BG_E_NOMEM
                                       : bg_faster_windows(c, R, M, crit, (int64_t)opts->overlap_bp,
                                                           (int64_t)opts->range_bp, perc, ref == map, res->wlo,
                                                           res->whi, res->zin, res->zout);
    if (rf) {
      bg_result_free(res);
      return rf;
    }
  } else if (tiny || (crit != BG_OVR_RANGE && (R->has_zero_len || M->has_zero_len))) {
    int rz = ref == map ? map_zero_prep_single(c, R, res) : tiny ? map_deque_prep(c, R, M, res) : map_zero_prep(c, R, M, res);
    if (rz) {
      bg_result_free(res);
      return rz;
    }
  }
  MapArgs A;
  A.RS = R->ks;
  A.RE = R->ke;
  A.nr = R->n;
  A.MS = M->ks;
  A.ME = M->ke;
  A.SC = (need & (NEED_SUM | NEED_EXT)) ? M->score : nullptr;
  A.nm = M->n;
  A.L = M->maxlen > 0 ? M->maxlen : 1;  // longest map row (from the loader)
  A.lrows = LongRows{nullptr, nullptr, nullptr, 0, 0};
  // rows longer than BG_LONG_THR get per-length-class windows (bg_map_cands), so a few
  // chromosome-length rows do not widen every reference row's window; the zero-length
  // and running-double replays enumerate one contiguous window and keep the global bound
  if (M->maxlen > BG_LONG_THR && !res->zin && !decimal && !tmean && !faster) {
    int rl = map_long_rows(c, M, res);
    if (rl) {
      bg_result_free(res);
      return rl;
    }
    A.lrows = res->lrows;
    if (A.lrows.ncls) A.L = BG_LONG_THR;
  }
  A.ovr = (int64_t)opts->overlap_bp;
  A.range = (int64_t)opts->range_bp;
  A.touch = tiny ? 1 : 0;
  A.perc = perc;
  A.need = need;
  A.cnt = res->cnt;
  A.isum = res->isum;
  A.vmin = res->vmin;
  A.vmax = res->vmax;
  A.bases = res->bases;
  A.uniq = res->uniq;
  A.isq = res->isq;
  A.wlo = res->wlo;
  A.whi = res->whi;
  A.zin = res->zin;
  A.zout = res->zout;
  A.st = c->dstat;
  if (R->n) {
    const dim3 g(bg_blocks(R->n, BG_NT)), b(BG_NT);
#define BG_MAP_LAUNCH(K)                                                                   \
  do {                                                                                     \
    if (A.lrows.ncls) {                                                                    \
      if (A.zin) BG_LAUNCH(c, "k_map_ops", (k_map_ops<K, true, true>), g, b, A);           \
      else BG_LAUNCH(c, "k_map_ops", (k_map_ops<K, false, true>), g, b, A);                \
    } else {                                                                               \
      if (A.zin) BG_LAUNCH(c, "k_map_ops", (k_map_ops<K, true, false>), g, b, A);          \
      else BG_LAUNCH(c, "k_map_ops", (k_map_ops<K, false, false>), g, b, A);               \
    }                                                                                      \
  } while (0)
    switch (faster ? BG_OVR_FAST : crit) {
      case BG_OVR_FAST: BG_LAUNCH(c, "k_map_ops", (k_map_ops<BG_OVR_FAST, true, false>), g, b, A); break;
      case BG_OVR_BP: BG_MAP_LAUNCH(BG_OVR_BP); break;
      case BG_OVR_RANGE: BG_MAP_LAUNCH(BG_OVR_RANGE); break;
      case BG_OVR_FRAC_REF: BG_MAP_LAUNCH(BG_OVR_FRAC_REF); break;
      case BG_OVR_FRAC_MAP: BG_MAP_LAUNCH(BG_OVR_FRAC_MAP); break;
      case BG_OVR_FRAC_EITHER: BG_MAP_LAUNCH(BG_OVR_FRAC_EITHER); break;
      case BG_OVR_FRAC_BOTH: BG_MAP_LAUNCH(BG_OVR_FRAC_BOTH); break;
      default: BG_MAP_LAUNCH(BG_OVR_EXACT); break;
    }
#undef BG_MAP_LAUNCH
  }
  int rc = bg_hip_ok(c, hipGetLastError());
  // equal map rows are ordered by the reference's heap addresses (bg_heap.hip): replay them
  // when an operation can see such a tie (both modes: one file replays sweep overload 1)
  if (!rc && R->n && M->n) {
    bool want = false, all = false, echo = false, rest_ties = false;
    for (int k = 0; k < opts->n_ops; ++k) {
      const int op = opts->ops[k];
      // every window's address order: WeightedAverage sums in it; TrimmedMean and the *-rand
      // element operations order equal SCORES by address
      if (op == BG_MAP_WMEAN || op == BG_MAP_TMEAN || op == BG_MAP_MIN_ELEMENT_RAND || op == BG_MAP_MAX_ELEMENT_RAND)
        all = true;
      if (op == BG_MAP_ECHO_MAP || op == BG_MAP_ECHO_MAP_ID || op == BG_MAP_ECHO_MAP_SCORE ||
          op == BG_MAP_ECHO_MAP_SIZE || op == BG_MAP_ECHO_OVERLAP_SIZE)
        echo = true;  // GenomicAddressCompare: ties of (chrom, start, end)
      if (op >= BG_MAP_MIN_ELEMENT && op <= BG_MAP_MAX_ELEMENT_RAND) rest_ties = true;
    }
    if (decimal) rest_ties = true;  // CoordRestAddressCompare: ties of (start, end, full_rest)
    if (all) want = true;
    else if (echo || rest_ties) {
      bool any = false;
      rc = bg_heap_ties(c, M, mapfields, !echo, &any);
      want = any;
    }
    if (!rc && want) {
      if (opts->shard) rc = bg_fail(c, BG_E_UNSUPPORTED, "address-ordered ties span every chromosome: not on a chromosome shard");
      else {
        bg_heap_spec hs;
        hs.crit = crit;
        hs.faster = faster;
        hs.ovr = (int64_t)opts->overlap_bp;
        hs.range = (int64_t)opts->range_bp;
        hs.perc = perc;
        hs.skip_unmapped = opts->skip_unmapped != 0;
        hs.nops = opts->n_ops;
        hs.ops = opts->ops;
        rc = bg_heap_addr(c, set, R, M, mapfields, &hs, &res->maddr);
      }
    }
  }
  if (!rc && (decimal || tmean) && R->n) {
    EvArgs E;
    E.RS = R->ks;
    E.RE = R->ke;
    E.nr = R->n;
    E.MS = M->ks;
    E.ME = M->ke;
    E.SC = M->score;
    E.nm = M->n;
    E.wlo = res->wlo;
    E.whi = res->whi;
    E.ovr = A.ovr;
    E.range = A.range;
    E.perc = perc;
    E.text = M->text;
    E.rest_off = M->rest_off;
    E.rest_len = M->rest_len;
    E.mapfields = mapfields;
    E.addr = res->maddr;
    E.ro = nullptr;
    E.P = nullptr;
    E.PL = nullptr;
    E.zin = faster ? res->zin : nullptr;
    E.mz_in = faster ? nullptr : res->zin;  // the zero-length replay's windows (else null)
    E.mz_out = faster ? nullptr : res->zout;
    E.mz_exact = !faster && res->zin && (ref == map || tiny);
    uint32_t* ro = nullptr;
    ulonglong2* pk = nullptr;
    uint32_t* pl = nullptr;
    if (M->n && M->n < (1ull << 32)) {  // set order of every run of equal map starts
      ro = (uint32_t*)bg_alloc(c, 4 * M->n);
      pk = (ulonglong2*)bg_alloc(c, 16 * M->n);
      pl = (uint32_t*)bg_alloc(c, 4 * M->n);
      if (!ro || !pk || !pl) rc = BG_E_NOMEM;
      else {
        BG_LAUNCH(c, "k_ev_keys", k_ev_keys, dim3(bg_blocks(M->n, BG_NT)), dim3(BG_NT), E, pk, pl);
        rc = bg_hip_ok(c, hipGetLastError());
        E.P = pk;
        E.PL = pl;
        if (!rc) rc = ev_order(c, E, M, mapfields, ro);
        E.ro = ro;
      }
    }
    const int ecrit = faster ? BG_OVR_FAST : crit;
    if (!rc && decimal) rc = map_running_sums(c, ecrit, E, need_sq, res);
    if (!rc && tmean) {
      if (!M->rest_off)
        rc = bg_fail(c, BG_E_ARG, "--tmean needs the map file loaded as BG_BED5_REST (equal rows are ordered by id and remainder)");
      else
        rc = map_tmean(c, ecrit, E, res->cnt, opts, res);
    }
    if (ro || pk || pl) {
      (void)hipStreamSynchronize(c->stream);
      bg_release(c, ro);
      bg_release(c, pk);
      bg_release(c, pl);
    }
  }
  if (!rc) rc = bg_hip_ok(c, hipMemcpyAsync(c->hstat, c->dstat, sizeof(bg_dstatus), hipMemcpyDeviceToHost, c->stream));
  if (!rc) rc = bg_hip_ok(c, hipStreamSynchronize(c->stream));
  if (!rc && need_rrank && R->n) {  // printed-line ranks for --echo-ref-row-id
    res->rrank = (uint64_t*)bg_alloc(c, 8 * n1);
    if (!res->rrank) rc = BG_E_NOMEM;
    if (!rc) {
      BG_LAUNCH(c, "k_map_printed", k_map_printed, dim3(bg_blocks(R->n, BG_NT)), dim3(BG_NT), res->cnt,
                R->n, res->rrank);
      rc = bg_hip_ok(c, hipGetLastError());
    }
    if (!rc) rc = bg_scan_sum_u64(c, res->rrank, res->rrank, R->n, nullptr);
  }
  if (!rc && (c->hstat->flags & 4ULL) && !decimal) {
    // a window sum reached 2^53: the int64 sums are exact where the reference's doubles are
    // not; redo with the reference's running doubles
    bg_result_free(res);
    return map_impl(c, set, ref, map, opts, out, true);
  }
  if (rc) {
    bg_result_free(res);
    return rc;
  }
  *out = res;
  bg_mark(c, "map");
  return 0;
}
