// bg_setops.hip — K1..K4: the bedops sweep kernels on keyed SoA intervals.
//
// The reference walks the inputs with pull readers and strcmp on every comparison
// (applications/bed/bedops/src/Bedops.cpp:792-1243). Here every operation is a
// scan, a merge-path pass or a binary search over whole sorted arrays:
//
//  components(X)        = running-max merge of one start-sorted array: row i opens a
//                         component iff ks[i] > max(ke[0..i-1]); touching rows merge
//                         (mergeOverlap's `p1.end >= p2.start`, Bedops.cpp:864-886;
//                         nextMergeAllLines, :1186-1243)
//  merge_sorted(X, Y)   = stable merge path of two start-sorted arrays (k-way union)
//  intersect2(X, Y)     = every element of merge(X,Y) (ties: Y first) emits at most one
//                         piece: [x.s, min(x.e, y.e)) with y the last Y starting <= x.s,
//                         [y.s, min(y.e, x.e)) with x the last X starting < y.s; pieces
//                         of length 0 are never emitted (nextIntersectLine :1105-1181)
//  difference(R, O)     = merge of R by start with O by end (ties: O first): r emits
//                         [r.s, min(r.e, q.s)) unless covered, q = first O ending after
//                         r.s; o emits [o.e, min(r.e, next.s)) inside the last R starting
//                         before o.e. This reproduces nextDifferenceLine (:950-1018)
//                         including its zero-length-row behaviour.
//  element_of(rows, O)  = exact covered bp by two binary searches + prefix sums of
//                         component lengths, then the reference's double-precision
//                         test (:1094-1096)
// Memory access: every kernel reads its inputs coalesced. components() uses a
// wave-striped layout (lane l of wave w handles rows w*W + k*64 + l) with 64-lane
// max-scans and ballots; the merge-path kernels stage each 2048-element diagonal tile
// of both inputs in LDS first. Count pass and write pass share one device function
// (reduce-then-scan between them), so outputs are deterministic and exactly sized.
#include <climits>

#include "bg_internal.h"

#define CT_ITEMS 8                    // rows per lane per wave in components()
#define CT_WROWS (64 * CT_ITEMS)      // rows per wave
#define CT_TILE (BG_NT * CT_ITEMS)    // rows per workgroup (4 waves)
#define MP_ITEMS 4
#define MP_TILE (BG_NT * MP_ITEMS)    // merged elements per workgroup

__device__ __forceinline__ int64_t wave_max_all(int64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = max(v, (int64_t)__shfl_xor(v, d, 64));
  return v;
}

// ------------------------------- components ---------------------------------------
// max end of each components() tile; one workgroup covers TM_TILES tiles with 16-byte
// loads (16 in flight per thread)
#define TM_TILES 4
__global__ void __launch_bounds__(BG_NT) k_tile_max(const int64_t* __restrict__ E, uint64_t n,
                                                    uint32_t ntiles, int64_t* __restrict__ tmax) {
  __shared__ int64_t wm[TM_TILES][BG_NT / 64];
  const uint64_t base = (uint64_t)blockIdx.x * TM_TILES * CT_TILE;  // elements
  constexpr int NV = TM_TILES * CT_TILE / 2 / BG_NT;                 // vectors per thread
  int64_t m[TM_TILES];
#pragma unroll
  for (int q = 0; q < TM_TILES; ++q) m[q] = LLONG_MIN;
  if (base + (uint64_t)TM_TILES * CT_TILE <= n) {
    const longlong2* E2 = reinterpret_cast<const longlong2*>(E + base);
    longlong2 v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = E2[k * BG_NT + threadIdx.x];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int q = (k * BG_NT * 2) / CT_TILE;
      m[q] = max(m[q], max((int64_t)v[k].x, (int64_t)v[k].y));
    }
  } else {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int q = (k * BG_NT * 2) / CT_TILE;
      const uint64_t i = base + 2ull * (k * BG_NT + threadIdx.x);
      if (i < n) m[q] = max(m[q], E[i]);
      if (i + 1 < n) m[q] = max(m[q], E[i + 1]);
    }
  }
#pragma unroll
  for (int q = 0; q < TM_TILES; ++q) {
    const int64_t x = wave_max_all(m[q]);
    if (bg_lane() == 0) wm[q][bg_wave()] = x;
  }
  __syncthreads();
  if (threadIdx.x < TM_TILES) {
    const uint32_t t = blockIdx.x * TM_TILES + threadIdx.x;
    if (t < ntiles) {
      int64_t x = wm[threadIdx.x][0];
      for (int w = 1; w < BG_NT / 64; ++w) x = max(x, wm[threadIdx.x][w]);
      tmax[t] = x;
    }
  }
}

template <bool WRITE>
__global__ void __launch_bounds__(BG_NT) k_components(
    const int64_t* __restrict__ S, const int64_t* __restrict__ E, uint64_t n,
    const int64_t* __restrict__ carry, uint64_t* __restrict__ cnt, const uint64_t* __restrict__ off,
    int64_t* __restrict__ CS, int64_t* __restrict__ CE) {
  __shared__ int64_t wmax[BG_NT / 64];
  __shared__ uint32_t wcnt[BG_NT / 64];
  const int lane = bg_lane(), w = bg_wave();
  const uint64_t wbase = (uint64_t)blockIdx.x * CT_TILE + (uint64_t)w * CT_WROWS;
  int64_t vs[CT_ITEMS], ve[CT_ITEMS];
  int64_t lm = LLONG_MIN;
#pragma unroll
  for (int k = 0; k < CT_ITEMS; ++k) {
    const uint64_t i = wbase + (uint64_t)k * 64 + lane;
    const bool in = i < n;
    vs[k] = in ? S[i] : LLONG_MAX;
    ve[k] = in ? E[i] : LLONG_MIN;
    lm = max(lm, ve[k]);
  }
  lm = wave_max_all(lm);
  if (lane == 0) wmax[w] = lm;
  __syncthreads();
  int64_t run = carry[blockIdx.x];
  for (int q = 0; q < w; ++q) run = max(run, wmax[q]);
  uint64_t bal[CT_ITEMS];
  int64_t incl[CT_ITEMS];
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < CT_ITEMS; ++k) {
    const uint64_t i = wbase + (uint64_t)k * 64 + lane;
    const int64_t inc = wave_incl_scan(ve[k], OpMax());
    int64_t ex = __shfl_up(inc, 1, 64);
    if (lane == 0) ex = LLONG_MIN;
    const bool f = (i < n) && vs[k] > max(run, ex);
    incl[k] = max(run, inc);
    bal[k] = __ballot(f);
    c += __popcll(bal[k]);
    run = max(run, (int64_t)__shfl(inc, 63, 64));
  }
  if (lane == 0) wcnt[w] = c;
  __syncthreads();
  if (!WRITE) {
    if (threadIdx.x == 0) {
      uint64_t t = 0;
      for (int q = 0; q < BG_NT / 64; ++q) t += wcnt[q];
      cnt[blockIdx.x] = t;
    }
    return;
  }
  uint64_t q0 = off[blockIdx.x];
  for (int q = 0; q < w; ++q) q0 += wcnt[q];
  const uint64_t lt = (1ULL << lane) - 1, le = lt | (1ULL << lane);
  uint64_t before = 0;
#pragma unroll
  for (int k = 0; k < CT_ITEMS; ++k) {
    const uint64_t i = wbase + (uint64_t)k * 64 + lane;
    if (i < n) {
      if ((bal[k] >> lane) & 1ULL) CS[q0 + before + __popcll(bal[k] & lt)] = vs[k];
      bool next_opens;
      if (i + 1 >= n) next_opens = true;
      else if (lane < 63) next_opens = (bal[k] >> (lane + 1)) & 1ULL;
      else if (k + 1 < CT_ITEMS) next_opens = bal[k + 1] & 1ULL;
      else next_opens = S[i + 1] > incl[k];
      if (next_opens) CE[q0 + before + __popcll(bal[k] & le) - 1] = incl[k];
    }
    before += __popcll(bal[k]);
  }
}

// ------------------------------- merge (union of two lists) -----------------------
__global__ void __launch_bounds__(BG_NT) k_merge_sorted(const int64_t* __restrict__ XS,
                                                        const int64_t* __restrict__ XE, uint64_t nx,
                                                        const int64_t* __restrict__ YS,
                                                        const int64_t* __restrict__ YE, uint64_t ny,
                                                        int64_t* __restrict__ ZS,
                                                        int64_t* __restrict__ ZE) {
  const uint64_t d0 = ((uint64_t)blockIdx.x * BG_NT + threadIdx.x) * MP_ITEMS;
  const uint64_t nz = nx + ny;
  if (d0 >= nz) return;
  uint64_t i = merge_path_xfirst(XS, nx, YS, ny, d0), j = d0 - i;
  for (int k = 0; k < MP_ITEMS && d0 + k < nz; ++k) {
    const bool takex = i < nx && (j >= ny || XS[i] <= YS[j]);
    if (takex) { ZS[d0 + k] = XS[i]; ZE[d0 + k] = XE[i]; ++i; }
    else { ZS[d0 + k] = YS[j]; ZE[d0 + k] = YE[j]; ++j; }
  }
}

// ------------------------------- merge-path tiles ---------------------------------
// part[b] = number of X elements among the first min(b*MP_TILE, nx+ny) elements of the
// merge of X (key XK) and Y (key YK), ties Y first
__global__ void k_mp_partition(const int64_t* __restrict__ XK, uint64_t nx,
                               const int64_t* __restrict__ YK, uint64_t ny, uint32_t nparts,
                               uint64_t* __restrict__ part) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > nparts) return;
  const uint64_t d = min((uint64_t)b * MP_TILE, nx + ny);
  part[b] = merge_path_ystrict(XK, nx, YK, ny, d);
}

enum { MP_INTERSECT = 0, MP_DIFFERENCE = 1 };

// One 2048-element diagonal tile of merge(X, Y). LDS holds X[i0-1 .. i1) then
// Y[j0-1 .. j1] (+1 for difference's "next O start"); sentinels outside the arrays.
//   MP_INTERSECT : X, Y = component lists, keys = starts
//   MP_DIFFERENCE: X = reference components (key start), Y = other components (key end)
//   SEG (with WRITE): no count pass. The tile's pieces go to its own segment
//     [blockIdx.x * MP_TILE, + count) (a tile of MP_TILE merged elements yields at most
//     MP_TILE pieces), with the count in cnt[] and the printed bytes in bytes[] (name_len:
//     the set's chromosome name lengths): a segmented result (bg_result::nseg) that the
//     formatter reads in place.
static_assert(MP_TILE == BG_SEG_CAP, "segment capacity = merge-path tile");
template <int MODE, bool WRITE, bool SEG = false>
__global__ void __launch_bounds__(BG_NT) k_mp_tile(
    const int64_t* __restrict__ XS, const int64_t* __restrict__ XE, uint64_t nx,
    const int64_t* __restrict__ YS, const int64_t* __restrict__ YE, uint64_t ny,
    const uint64_t* __restrict__ part, uint64_t* __restrict__ cnt, const uint64_t* __restrict__ off,
    int64_t* __restrict__ OS, int64_t* __restrict__ OE, const uint32_t* __restrict__ name_len = nullptr,
    uint64_t* __restrict__ bytes = nullptr) {
  __shared__ int64_t ls_[MP_TILE + 4];
  __shared__ int64_t le_[MP_TILE + 4];
  __shared__ uint32_t shc[BG_NT / 64 + 1];
  const uint64_t nz = nx + ny;
  const uint64_t d0 = (uint64_t)blockIdx.x * MP_TILE;
  const uint64_t d1 = min(d0 + MP_TILE, nz);
  const uint64_t i0 = part[blockIdx.x], i1 = part[blockIdx.x + 1];
  const uint64_t j0 = d0 - i0, j1 = d1 - i1;
  const uint32_t nxl = (uint32_t)(i1 - i0), nyl = (uint32_t)(j1 - j0);
  const uint32_t xb = 0, yb = nxl + 1;  // LDS slots: X[i0-1+q] at xb+q, Y[j0-1+q] at yb+q
  for (uint32_t q = threadIdx.x; q < nxl + 1; q += BG_NT) {
    const int64_t gi = (int64_t)i0 - 1 + q;
    ls_[xb + q] = gi >= 0 ? XS[gi] : LLONG_MIN;
    le_[xb + q] = gi >= 0 ? XE[gi] : LLONG_MIN;
  }
  for (uint32_t q = threadIdx.x; q < nyl + 2; q += BG_NT) {
    const int64_t gj = (int64_t)j0 - 1 + q;
    const bool in = gj >= 0 && (uint64_t)gj < ny;
    ls_[yb + q] = in ? YS[gj] : (gj < 0 ? LLONG_MIN : LLONG_MAX);
    le_[yb + q] = in ? YE[gj] : (gj < 0 ? LLONG_MIN : LLONG_MAX);
  }
  __syncthreads();
  const int64_t* xk = ls_ + xb + 1;  // local X[0..nxl)
  const int64_t* yk = (MODE == MP_INTERSECT ? ls_ : le_) + yb + 1;
  int64_t ps[MP_ITEMS], pe[MP_ITEMS];
  uint32_t c = 0;
  const uint32_t dl = threadIdx.x * MP_ITEMS, dn = (uint32_t)(d1 - d0);
  if (dl < dn) {
    // local merge path on the LDS slices (ties: Y first)
    uint32_t lo = dl > nyl ? dl - nyl : 0, hi = dl < nxl ? dl : nxl;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (xk[mid] < yk[dl - 1 - mid]) lo = mid + 1;
      else hi = mid;
    }
    uint32_t i = lo, j = dl - lo;  // local indices; global = i0 + i, j0 + j
    for (int k = 0; k < MP_ITEMS && dl + k < dn; ++k) {
      const bool takex = i < nxl && (j >= nyl || xk[i] < yk[j]);
      if (MODE == MP_INTERSECT) {
        int64_t s, e, pend;
        if (takex) { s = ls_[xb + 1 + i]; e = le_[xb + 1 + i]; pend = le_[yb + j]; ++i; }
        else { s = ls_[yb + 1 + j]; e = le_[yb + 1 + j]; pend = le_[xb + i]; ++j; }
        const int64_t h = min(e, pend);
        if (h > s) { ps[c] = s; pe[c] = h; ++c; }
      } else {
        if (takex) {
          const int64_t a = ls_[xb + 1 + i], b = le_[xb + 1 + i];
          const int64_t qs = ls_[yb + 1 + j];  // first O ending after a (LLONG_MAX if none)
          if (qs >= b) { ps[c] = a; pe[c] = b; ++c; }
          else if (qs > a) { ps[c] = a; pe[c] = qs; ++c; }
          ++i;
        } else {
          if (i0 + i > 0) {
            const int64_t oe = le_[yb + 1 + j], rb = le_[xb + i];
            if (rb > oe) {
              const int64_t nxt = min(rb, ls_[yb + 2 + j]);
              ps[c] = oe; pe[c] = nxt; ++c;
            }
          }
          ++j;
        }
      }
    }
  }
  uint32_t btot;
  const uint32_t o = block_excl_scan(c, OpSum(), 0u, shc, &btot);
  if (!WRITE) {
    if (threadIdx.x == 0) cnt[blockIdx.x] = btot;
    return;
  }
  if (SEG) {  // printed bytes of the tile's pieces (the formatter's count pass, here)
    uint32_t nb = 0;
#pragma unroll
    for (int k = 0; k < MP_ITEMS; ++k)
      if (k < (int)c) nb += bg_ivl_len(name_len, ps[k], pe[k]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) nb += __shfl_xor(nb, d, 64);
    __syncthreads();  // shc reused
    if (bg_lane() == 0) shc[bg_wave()] = nb;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t tb = 0;
      for (int w = 0; w < BG_NT / 64; ++w) tb += shc[w];
      cnt[blockIdx.x] = btot;
      bytes[blockIdx.x] = tb;
    }
  }
  // stage the tile's pieces in LDS (the input slices are no longer read), then store them
  // with consecutive lanes on consecutive elements
  __syncthreads();
  for (uint32_t k = 0; k < c; ++k) { ls_[o + k] = ps[k]; le_[o + k] = pe[k]; }
  __syncthreads();
  const uint64_t q = SEG ? (uint64_t)blockIdx.x * MP_TILE : off[blockIdx.x];
  for (uint32_t k = threadIdx.x; k < btot; k += BG_NT) { OS[q + k] = ls_[k]; OE[q + k] = le_[k]; }
}

// ------------------------------- element-of ---------------------------------------
__global__ void __launch_bounds__(BG_NT) k_lengths(const int64_t* __restrict__ S,
                                                   const int64_t* __restrict__ E, uint64_t n,
                                                   uint64_t* __restrict__ L) {
  const uint64_t i = (uint64_t)blockIdx.x * BG_NT + threadIdx.x;
  if (i < n) L[i] = (uint64_t)(E[i] - S[i]);
}

// One thread per reference row; the workgroup first bounds the component range its rows
// can touch (two searches over the whole list), stages that slice of component starts and
// ends in LDS when it fits (it nearly always does: 256 consecutive rows span few
// components), and each row's own two searches run there instead of in L2.
#define EF_SLICE 1024
__device__ __forceinline__ uint32_t lds_lower(const int64_t* X, uint32_t lo, uint32_t hi, int64_t v) {
  while (lo < hi) {  // first k in [lo, hi) with X[k] >= v
    const uint32_t mid = (lo + hi) >> 1;
    if (X[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ uint32_t lds_upper(const int64_t* X, uint32_t lo, uint32_t hi, int64_t v) {
  while (lo < hi) {  // first k in [lo, hi) with X[k] > v
    const uint32_t mid = (lo + hi) >> 1;
    if (X[mid] <= v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// the first component of each k_element_flags block (one thread per block: every search in
// flight at once, instead of one search per resident 256-thread block while its other threads
// wait); the block finds the end of its range by a gallop from there (usually a few steps)
__global__ void __launch_bounds__(BG_NT) k_element_lo(const int64_t* __restrict__ RS,
                                                    const int64_t* __restrict__ OE_, uint64_t no,
                                                    uint64_t nblk, uint64_t* __restrict__ blo) {
  const uint64_t b = (uint64_t)blockIdx.x * BG_NT + threadIdx.x;
  if (b < nblk) blo[b] = upper_bound_i64(OE_, no, RS[b * BG_NT]);  // rows start at >= RS[b * BG_NT]
}
__global__ void __launch_bounds__(BG_NT) k_element_flags(
    const int64_t* __restrict__ RS, const int64_t* __restrict__ RE, uint64_t nr,
    const int64_t* __restrict__ OS_, const int64_t* __restrict__ OE_, uint64_t no,
    const uint64_t* __restrict__ P, double thres, int use_pct, int invert,
    uint8_t* __restrict__ flag, const uint32_t* __restrict__ name_len,
    const uint32_t* __restrict__ rest_len, uint16_t* __restrict__ blen,
    unsigned int* __restrict__ blen_ovf, const uint64_t* __restrict__ blo_) {
  __shared__ int64_t wmax[BG_NT / 64];
  __shared__ uint64_t bnd1;
  __shared__ int64_t xs[EF_SLICE], xe[EF_SLICE];
  const uint64_t r0 = (uint64_t)blockIdx.x * BG_NT;
  const uint64_t r = r0 + threadIdx.x;
  const bool live = r < nr;
  const int64_t s = live ? RS[r] : LLONG_MAX, e = live ? RE[r] : LLONG_MIN;
  const int64_t em = wave_max_all(e);
  if (bg_lane() == 0) wmax[bg_wave()] = em;
  const uint64_t blo = blo_[blockIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {  // first component starting at/after the block's largest end: a gallop
    int64_t m = wmax[0];
    for (int w = 1; w < BG_NT / 64; ++w) m = max(m, wmax[w]);
    uint64_t lo = blo, step = 1;  // OS_[k] < m for every k < lo
    while (lo < no && OS_[lo] < m) {
      const uint64_t nx = lo + step;
      if (nx >= no || OS_[nx] >= m) {
        bnd1 = lower_bound_in(OS_, lo + 1, nx < no ? nx : no, m);
        lo = ~0ull;
        break;
      }
      lo = nx + 1;
      step <<= 1;
    }
    if (lo != ~0ull) bnd1 = lo < no ? lo : no;
  }
  __syncthreads();
  const uint64_t bhi = max(blo, bnd1);
  const bool staged = bhi - blo <= EF_SLICE;  // block-uniform
  if (staged) {
    for (uint32_t i = threadIdx.x; i < bhi - blo; i += BG_NT) {
      xs[i] = OS_[blo + i];
      xe[i] = OE_[blo + i];
    }
    __syncthreads();
  }
  if (!live) return;
  // exact within [blo, bhi]: a row's first component ending after s is >= blo, and its
  // first component starting at/after e is <= bhi; a clamped lo == bhi means no overlap,
  // which decides like "nothing left" below (keep = invert)
  const uint32_t n = (uint32_t)(bhi - blo);
  const uint64_t lo = staged ? blo + lds_upper(xe, 0, n, s)
                             : upper_bound_in(OE_, blo, bhi, s);  // first component ending after s
  bool keep;
  if (lo >= no) {
    keep = invert;  // nothing left to be an element of (Bedops.cpp:1044-1048)
  } else {
    const uint64_t hi = staged ? blo + lds_lower(xs, (uint32_t)(lo - blo), n, e)
                               : lower_bound_in(OS_, blo, bhi, e);  // first component starting at/after e
    uint64_t ov = 0;
    if (lo < hi) {
      ov = P[hi] - P[lo];
      const int64_t slo = staged ? xs[lo - blo] : OS_[lo];
      const int64_t ehi = staged ? xe[hi - 1 - blo] : OE_[hi - 1];
      if (s > slo) ov -= (uint64_t)(s - slo);
      if (ehi > e) ov -= (uint64_t)(ehi - e);
    }
    const double rov = (double)ov, range = (double)(e - s);
    const bool is_el = use_pct ? (rov / range >= thres) : (rov >= thres);
    keep = invert ? !is_el : is_el;
  }
  flag[r] = keep ? 1 : 0;
  if (blen && keep) {  // the kept row's printed length "%s\t%lu\t%lu%s\n" (k_compact_rows_bytes)
    const uint32_t l = bg_ivl_len(name_len, s, e) + rest_len[r];
    if (l > 0xFFFFu) atomicOr(blen_ovf, 1u);
    blen[r] = (uint16_t)l;
  }
}

#define CF_ITEMS 16
#define CF_TILE (BG_NT * CF_ITEMS)
template <bool WRITE>
__global__ void __launch_bounds__(BG_NT) k_compact_flags(const uint8_t* __restrict__ flag,
                                                         uint64_t n, uint64_t* __restrict__ cnt,
                                                         const uint64_t* __restrict__ off,
                                                         uint64_t* __restrict__ rows) {
  __shared__ uint32_t wc[BG_NT / 64];
  const int lane = bg_lane(), w = bg_wave();
  const uint64_t wbase = (uint64_t)blockIdx.x * CF_TILE + (uint64_t)w * 64 * CF_ITEMS;
  uint64_t bal[CF_ITEMS];
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < CF_ITEMS; ++k) {
    const uint64_t i = wbase + (uint64_t)k * 64 + lane;
    bal[k] = __ballot(i < n && flag[i]);
    c += __popcll(bal[k]);
  }
  if (lane == 0) wc[w] = c;
  __syncthreads();
  if (!WRITE) {
    if (threadIdx.x == 0) cnt[blockIdx.x] = (uint64_t)wc[0] + wc[1] + wc[2] + wc[3];
    return;
  }
  uint64_t q = off[blockIdx.x];
  for (int v = 0; v < w; ++v) q += wc[v];
  const uint64_t lt = (1ULL << lane) - 1;
#pragma unroll
  for (int k = 0; k < CF_ITEMS; ++k) {
    if ((bal[k] >> lane) & 1ULL) rows[q + __popcll(bal[k] & lt)] = wbase + (uint64_t)k * 64 + lane;
    q += __popcll(bal[k]);
  }
}

// ------------------------------- intersect: zero-length pieces --------------------
// A file's zero-length piece [t, t) (an isolated zero-length row) never contributes to the
// set intersection, but nextIntersectLine (Bedops.cpp:1105-1181) prints it as "chr t t"
// when its stream reaches it in a particular state. The state between two calls is just
// one head piece per file, and after a call that printed [s, e) with marker file q it is
// canonical: every file's head is its first piece ending after s, except q's, which is its
// first piece ending after e (the final pass left each head overlapping [s, e); the
// marker's piece, the first one ending at e, was consumed, :1178). Zero-length pieces
// never change which non-empty pieces are printed (they only pop pieces that end at or
// before t, none of which can meet a piece on the far side of t), so: the non-empty
// output is the set intersection (k_mp_tile), and for every non-empty output O[m] that
// has a zero-length piece t with O[m-1].s < t <= O[m].s, one thread replays the calls
// from the canonical state after O[m-1] until the next non-empty print, which must be
// O[m], collecting the zero-length prints in call order. tests/model_setops.py holds the
// same construction; both are compared with oracle/bedops_oracle.c (next_intersect).
struct ZFile {
  const int64_t* s;
  const int64_t* e;
  uint64_t n;
};

// first index >= h with E[index] > v, galloping from h (heads move forward a little)
__device__ __forceinline__ uint64_t zi_pop(const int64_t* E, uint64_t n, uint64_t h, int64_t v) {
  if (h >= n || E[h] > v) return h;
  uint64_t lo = h + 1, step = 1;
  while (lo + step <= n && E[lo + step - 1] <= v) { lo += step; step <<= 1; }
  return upper_bound_in(E, lo, min(n, lo + step), v);
}

// k_zi_mark: flag[m] = 1 for the first output m starting at or after some zero-length piece
__global__ void __launch_bounds__(BG_NT) k_zi_mark(const int64_t* __restrict__ S,
                                                   const int64_t* __restrict__ E, uint64_t n,
                                                   const int64_t* __restrict__ OS, uint64_t no,
                                                   uint8_t* __restrict__ flag) {
  const uint64_t i = (uint64_t)blockIdx.x * BG_NT + threadIdx.x;
  if (i >= n) return;
  const int64_t t = S[i];
  if (E[i] != t) return;
  flag[lower_bound_i64(OS, no, t)] = 1;
}

// One thread per anchor m (from k_zi_mark): replay calls from the state after O[m-1]
// (the initial state for m == 0). COUNT: cnt[a] = zero-length prints. WRITE: store them
// at m + off[a] + k. H is per-thread scratch (nf heads); bad[0] != 0 flags an internal
// inconsistency (the replay did not reach O[m]) or the iteration bound.
template <bool WRITE>
__global__ void __launch_bounds__(BG_NT) k_zi_replay(
    const ZFile* __restrict__ F, int nf, const int64_t* __restrict__ OS,
    const int64_t* __restrict__ OE, uint64_t no, const uint64_t* __restrict__ anchors, uint64_t na,
    uint64_t* __restrict__ H, uint64_t* __restrict__ cnt, const uint64_t* __restrict__ off,
    int64_t* __restrict__ ZS, int64_t* __restrict__ ZE, uint64_t cap,
    unsigned long long* __restrict__ bad) {
  const uint64_t a = (uint64_t)blockIdx.x * BG_NT + threadIdx.x;
  if (a >= na) return;
  const uint64_t m = anchors[a];
  uint64_t* h = H + a * (uint64_t)nf;
  if (m == 0) {
    for (int f = 0; f < nf; ++f) h[f] = 0;
  } else {
    const int64_t s = OS[m - 1], e = OE[m - 1];
    int q = -1;
    for (int f = 0; f < nf; ++f) {
      h[f] = upper_bound_i64(F[f].e, F[f].n, s);
      if (q < 0 && h[f] < F[f].n && F[f].e[h[f]] == e) q = f;
    }
    if (q < 0) { atomicOr(bad, 1ULL); return; }
    h[q] += 1;
  }
  uint64_t k = 0, steps = 0;
  const uint64_t base = WRITE ? m + off[a] : 0;
  for (;;) {  // one iteration = one nextIntersectLine call
    bool stop = false;
    int mj = 0;
    for (int f = 0; f < nf && !stop; ++f) {
      if (h[f] >= F[f].n) stop = true;
      else if (f > 0 && F[f].s[h[f]] > F[mj].s[h[mj]]) mj = f;
    }
    if (stop) break;
    int64_t cs = F[mj].s[h[mj]], ce = F[mj].e[h[mj]];
    int marker = -1;
    int64_t minE = LLONG_MAX;
    for (int f = 0; f < nf;) {
      if (++steps > cap) { atomicOr(bad, 2ULL); return; }
      h[f] = zi_pop(F[f].e, F[f].n, h[f], cs);
      if (h[f] >= F[f].n) { stop = true; break; }
      const int64_t ps = F[f].s[h[f]], pe = F[f].e[h[f]];
      if (ps >= ce) {  // no overlap: restart from this piece (:1161-1168)
        cs = ps; ce = pe; marker = -1; minE = LLONG_MAX; f = 0;
        continue;
      }
      cs = max(cs, ps);
      ce = min(ce, pe);
      if (pe < minE) { minE = pe; marker = f; }
      ++f;
    }
    if (stop) break;
    h[marker] += 1;
    if (cs != ce) {  // the next non-empty print: must be O[m]
      if (m >= no || OS[m] != cs || OE[m] != ce) atomicOr(bad, 4ULL);
      break;
    }
    if (WRITE) { ZS[base + k] = cs; ZE[base + k] = ce; }
    ++k;
  }
  if (!WRITE) cnt[a] = k;
}

// O[m] -> position m + (zero-length prints anchored at or before m)
__global__ void __launch_bounds__(BG_NT) k_zi_place(const int64_t* __restrict__ OS,
                                                    const int64_t* __restrict__ OE, uint64_t no,
                                                    const uint64_t* __restrict__ anchors,
                                                    uint64_t na, const uint64_t* __restrict__ off,
                                                    int64_t* __restrict__ ZS,
                                                    int64_t* __restrict__ ZE) {
  const uint64_t m = (uint64_t)blockIdx.x * BG_NT + threadIdx.x;
  if (m >= no) return;
  uint64_t lo = 0, hi = na;  // anchors <= m
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (anchors[mid] <= m) lo = mid + 1;
    else hi = mid;
  }
  const uint64_t p = m + off[lo];
  ZS[p] = OS[m];
  ZE[p] = OE[m];
}

// =====================================================================================
// host drivers
// =====================================================================================
void ivl_free(bg_ctx* c, Ivl& v) {
  if (v.owned) {
    bg_release(c, v.s);
    bg_release(c, v.e);
    bg_release(c, v.seg_off);
    bg_release(c, v.seg_boff);
  }
  v = Ivl();
}

int ivl_alloc(bg_ctx* c, Ivl& v, uint64_t n) {
  v.n = n;
  v.s = (int64_t*)bg_alloc(c, 8 * (n ? n : 1));
  v.e = (int64_t*)bg_alloc(c, 8 * (n ? n : 1));
  v.owned = true;
  return (v.s && v.e) ? 0 : BG_E_NOMEM;
}

// k_compact_flags' write pass that also sums the kept rows' printed lengths (blen) per
// output format tile of BG_FMT_TILE rows: a wave's kept rows of one ballot are consecutive
// outputs spanning at most two tiles, lane 0 carries a running (tile, bytes) pair and adds
// it to tb[] when the tile changes (a few atomics per 1024 input rows)
__global__ void __launch_bounds__(BG_NT) k_compact_rows_bytes(const uint8_t* __restrict__ flag,
                                                              const uint16_t* __restrict__ blen, uint64_t n,
                                                              const uint64_t* __restrict__ off,
                                                              uint64_t* __restrict__ rows,
                                                              unsigned long long* __restrict__ tb) {
  __shared__ uint32_t wc[BG_NT / 64];
  const int lane = bg_lane(), w = bg_wave();
  const uint64_t wbase = (uint64_t)blockIdx.x * CF_TILE + (uint64_t)w * 64 * CF_ITEMS;
  uint64_t bal[CF_ITEMS];
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < CF_ITEMS; ++k) {
    const uint64_t i = wbase + (uint64_t)k * 64 + lane;
    bal[k] = __ballot(i < n && flag[i]);
    c += __popcll(bal[k]);
  }
  if (lane == 0) wc[w] = c;
  __syncthreads();
  uint64_t q = off[blockIdx.x];
  for (int v = 0; v < w; ++v) q += wc[v];
  const uint64_t lt = (1ULL << lane) - 1;
  uint64_t ct = ~0ULL, cs = 0;  // lane 0's open (tile, bytes)
#pragma unroll
  for (int k = 0; k < CF_ITEMS; ++k) {
    const uint64_t i = wbase + (uint64_t)k * 64 + lane;
    const bool mine = (bal[k] >> lane) & 1ULL;
    const uint64_t qi = q + __popcll(bal[k] & lt);
    uint32_t l = 0;
    if (mine) {
      rows[qi] = i;
      l = blen[i];
    }
    if (bal[k]) {
      const uint64_t t0 = q / BG_FMT_TILE;
      const bool hi = mine && qi / BG_FMT_TILE != t0;
      uint32_t s0 = hi ? 0u : l, s1 = hi ? l : 0u;
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        s0 += __shfl_xor(s0, d, 64);
        s1 += __shfl_xor(s1, d, 64);
      }
      if (lane == 0) {
        if (ct != t0) {
          if (ct != ~0ULL && cs) atomicAdd(&tb[ct], (unsigned long long)cs);
          ct = t0;
          cs = 0;
        }
        cs += s0;
        if (s1) {
          if (cs) atomicAdd(&tb[ct], (unsigned long long)cs);
          ct = t0 + 1;
          cs = s1;
        }
      }
    }
    q += __popcll(bal[k]);
  }
  if (lane == 0 && ct != ~0ULL && cs) atomicAdd(&tb[ct], (unsigned long long)cs);
}

// indices i with flag[i] != 0, in order (count -> scan -> write)
int bg_compact_flags(bg_ctx* c, const uint8_t* flag, uint64_t n, uint64_t** rows, uint64_t* total) {
  const unsigned nb = bg_blocks(n, CF_TILE);
  *rows = nullptr;
  return count_scan_write(
      c, nb,
      [&](uint64_t* cnt) {
        BG_LAUNCH(c, "k_compact_flags_count", k_compact_flags<false>, dim3(nb), dim3(BG_NT), flag,
                  n, cnt, (const uint64_t*)nullptr, (uint64_t*)nullptr);
      },
      [&](uint64_t* off, uint64_t tot) -> int {
        *rows = (uint64_t*)bg_alloc(c, 8 * (tot ? tot : 1));
        if (!*rows) return BG_E_NOMEM;
        if (nb)
          BG_LAUNCH(c, "k_compact_flags_write", k_compact_flags<true>, dim3(nb), dim3(BG_NT), flag,
                    n, (uint64_t*)nullptr, off, *rows);
        return 0;
      },
      total);
}

int bg_components(bg_ctx* c, const Ivl& in, Ivl& out) {
  const uint64_t n = in.n;
  if (n == 0) return ivl_alloc(c, out, 0);
  const unsigned nb = bg_blocks(n, CT_TILE);
  int64_t* carry = (int64_t*)bg_alloc(c, 8ull * nb);
  if (!carry) return BG_E_NOMEM;
  BG_LAUNCH(c, "k_tile_max", k_tile_max, dim3(bg_blocks(nb, TM_TILES)), dim3(BG_NT), in.e, n, nb,
            carry);
  BG_HIP(c, hipGetLastError());
  int rc = bg_scan_max_i64(c, carry, carry, nb, LLONG_MIN);
  if (rc) return rc;
  uint64_t total = 0;
  rc = count_scan_write(
      c, nb,
      [&](uint64_t* cnt) {
        BG_LAUNCH(c, "k_components_count", k_components<false>, dim3(nb), dim3(BG_NT), in.s, in.e,
                  n, carry, cnt, (const uint64_t*)nullptr, (int64_t*)nullptr, (int64_t*)nullptr);
      },
      [&](uint64_t* off, uint64_t tot) -> int {
        int r = ivl_alloc(c, out, tot);
        if (r) return r;
        BG_LAUNCH(c, "k_components_write", k_components<true>, dim3(nb), dim3(BG_NT), in.s, in.e,
                  n, carry, (uint64_t*)nullptr, off, out.s, out.e);
        return 0;
      },
      &total);
  bg_release(c, carry);
  return rc;
}

static int merge_sorted(bg_ctx* c, const Ivl& x, const Ivl& y, Ivl& z) {
  int rc = ivl_alloc(c, z, x.n + y.n);
  if (rc) return rc;
  if (x.n + y.n == 0) return 0;
  BG_LAUNCH(c, "k_merge_sorted", k_merge_sorted, dim3(bg_blocks(x.n + y.n, MP_TILE)), dim3(BG_NT),
            x.s, x.e, x.n, y.s, y.e, y.n, z.s, z.e);
  BG_HIP(c, hipGetLastError());
  return 0;
}

// merge-path tile operation over X and Y (MODE: intersect / difference). seg: the result
// is left segmented per tile with its printed byte counts (one pass, no count pass): for a
// result that goes straight to the formatter (bg_result::nseg)
template <int MODE>
static int mp_op(bg_ctx* c, const Ivl& x, const Ivl& y, Ivl& out, const char* cname,
                 const char* wname, const uint32_t* seg_names = nullptr) {
  const uint64_t nz = x.n + y.n;
  const unsigned nb = bg_blocks(nz, MP_TILE);
  if (nb == 0) return ivl_alloc(c, out, 0);
  uint64_t* part = (uint64_t*)bg_alloc(c, 8ull * (nb + 1));
  if (!part) return BG_E_NOMEM;
  const int64_t* yk = (MODE == MP_INTERSECT) ? y.s : y.e;
  BG_LAUNCH(c, "k_mp_partition", k_mp_partition, dim3(bg_blocks(nb + 1, 256)), dim3(256), x.s, x.n,
            yk, y.n, nb, part);
  BG_HIP(c, hipGetLastError());
  if (seg_names) {
    int rc = ivl_alloc(c, out, nz);
    out.seg_off = (uint64_t*)bg_alloc(c, 8ull * (nb + 1));
    out.seg_boff = (uint64_t*)bg_alloc(c, 8ull * (nb + 1));
    if (rc || !out.seg_off || !out.seg_boff) return BG_E_NOMEM;
    out.nseg = nb;
    BG_LAUNCH(c, wname, (k_mp_tile<MODE, true, true>), dim3(nb), dim3(BG_NT), x.s, x.e, x.n, y.s, y.e,
              y.n, part, out.seg_off, (const uint64_t*)nullptr, out.s, out.e, seg_names, out.seg_boff);
    BG_HIP(c, hipGetLastError());
    if ((rc = bg_scan_sum_u64(c, out.seg_off, out.seg_off, nb, out.seg_off + nb))) return rc;
    if ((rc = bg_scan_sum_u64(c, out.seg_boff, out.seg_boff, nb, out.seg_boff + nb))) return rc;
    // the piece count stays on the device: the formatter fetches it with the byte count after
    // its kernel (no host round trip in between)
    out.n = 0;
    out.seg_nz = nz;
    out.n_pending = true;
    bg_release(c, part);
    return 0;
  }
  uint64_t total = 0;
  int rc = count_scan_write(
      c, nb,
      [&](uint64_t* cnt) {
        BG_LAUNCH(c, cname, (k_mp_tile<MODE, false>), dim3(nb), dim3(BG_NT), x.s, x.e, x.n, y.s, y.e,
                  y.n, part, cnt, (const uint64_t*)nullptr, (int64_t*)nullptr, (int64_t*)nullptr);
      },
      [&](uint64_t* off, uint64_t tot) -> int {
        int r = ivl_alloc(c, out, tot);
        if (r) return r;
        BG_LAUNCH(c, wname, (k_mp_tile<MODE, true>), dim3(nb), dim3(BG_NT), x.s, x.e, x.n, y.s, y.e,
                  y.n, part, (uint64_t*)nullptr, off, out.s, out.e);
        return 0;
      },
      &total);
  bg_release(c, part);
  return rc;
}

Ivl bg_table_ivl(bg_table* T) {
  Ivl v;
  v.s = T->ks;
  v.e = T->ke;
  v.n = T->n;
  v.owned = false;
  return v;
}

int bg_table_components(bg_ctx* c, bg_table* T, Ivl& out) {
  if (T->is_set) {
    out = Ivl();
    out.s = T->cs;
    out.e = T->ce;
    out.n = T->nc;
    out.owned = false;
    return 0;
  }
  return bg_components(c, bg_table_ivl(T), out);
}

int bg_need_rows(bg_ctx* c, bg_set* set, const int* files, int nf, const char* what) {
  for (int k = 0; k < nf; ++k)
    if (set->t[files[k]]->is_set)
      return bg_fail(c, BG_E_ARG, std::string(what) + ": input " + std::to_string(files[k] + 1) +
                                      " was loaded as BG_BED3_SET (no rows kept)");
  return 0;
}

// components of the union of the given tables
int bg_union_components(bg_ctx* c, bg_set* set, const int* files, int nf, Ivl& out) {
  Ivl acc;
  int rc = bg_table_components(c, set->t[files[0]], acc);
  if (rc) return rc;
  for (int k = 1; k < nf; ++k) {
    Ivl ck, z, m;
    if ((rc = bg_table_components(c, set->t[files[k]], ck))) return rc;
    if ((rc = merge_sorted(c, acc, ck, z))) return rc;
    ivl_free(c, acc);
    ivl_free(c, ck);
    if ((rc = bg_components(c, z, m))) return rc;
    ivl_free(c, z);
    acc = m;
  }
  out = acc;
  return 0;
}

bg_result* bg_new_ivl_result(bg_ctx* c, bg_set* set, Ivl& v) {
  if (!v.owned && v.s) {  // a view of a table's set: the result gets its own copy
    Ivl w;
    if (ivl_alloc(c, w, v.n)) return nullptr;
    if (v.n) {
      if (hipMemcpyAsync(w.s, v.s, 8 * v.n, hipMemcpyDeviceToDevice, c->stream) != hipSuccess ||
          hipMemcpyAsync(w.e, v.e, 8 * v.n, hipMemcpyDeviceToDevice, c->stream) != hipSuccess) {
        ivl_free(c, w);
        return nullptr;
      }
    }
    v = w;
  }
  bg_result* r = new bg_result();
  r->ctx = c;
  r->set = set;
  r->kind = RES_IVL;
  r->n = v.n;
  r->s = v.s;
  r->e = v.e;
  r->nseg = v.nseg;
  r->seg_off = v.seg_off;
  r->seg_boff = v.seg_boff;
  r->seg_nz = v.seg_nz;
  r->n_pending = v.n_pending;
  v.owned = false;
  return r;
}

// segment t's pieces -> [seg_off[t], seg_off[t+1]) of contiguous s/e
__global__ void __launch_bounds__(BG_NT) k_seg_compact(const int64_t* __restrict__ S, const int64_t* __restrict__ E,
                                                       const uint64_t* __restrict__ seg_off, int64_t* __restrict__ CS,
                                                       int64_t* __restrict__ CE) {
  const uint64_t t = blockIdx.x, c0 = seg_off[t], n = seg_off[t + 1] - c0;
  for (uint64_t j = threadIdx.x; j < n; j += BG_NT) {
    CS[c0 + j] = S[t * BG_SEG_CAP + j];
    CE[c0 + j] = E[t * BG_SEG_CAP + j];
  }
}

int bg_result_resolve_n(bg_ctx* c, bg_result* r) {
  if (!r || !r->n_pending) return 0;
  const int rc = bg_fetch_u64(c, r->seg_off + r->nseg, &r->n);
  if (!rc) r->n_pending = false;
  return rc;
}

int bg_result_compact(bg_ctx* c, bg_result* r) {
  if (!r || r->kind != RES_IVL || !r->nseg) return 0;
  int rc = bg_result_resolve_n(c, r);
  if (rc) return rc;
  Ivl w;
  if (ivl_alloc(c, w, r->n)) {
    ivl_free(c, w);
    return BG_E_NOMEM;
  }
  BG_LAUNCH(c, "k_seg_compact", k_seg_compact, dim3((unsigned)r->nseg), dim3(BG_NT), r->s, r->e, r->seg_off,
            w.s, w.e);
  BG_HIP(c, hipGetLastError());
  BG_HIP(c, hipStreamSynchronize(c->stream));
  bg_release(c, r->s);
  bg_release(c, r->e);
  bg_release(c, r->seg_off);
  bg_release(c, r->seg_boff);
  r->s = w.s;
  r->e = w.e;
  r->nseg = 0;
  r->seg_off = r->seg_boff = nullptr;
  return 0;
}

int bg_check_files(bg_ctx* c, bg_set* set, const int* files, int nf, int minf) {
  if (!c || !set || !files || nf < minf) return BG_E_ARG;
  for (int k = 0; k < nf; ++k)
    if (files[k] < 0 || files[k] >= (int)set->t.size()) return BG_E_ARG;
  return 0;
}

extern "C" int bg_merge(bg_ctx* c, bg_set* set, const int* files, int nf, bg_result** out) {
  int rc = bg_check_files(c, set, files, nf, 1);
  if (rc) return rc;
  Ivl m;
  if ((rc = bg_union_components(c, set, files, nf, m))) return rc;
  *out = bg_new_ivl_result(c, set, m);
  if (!*out) return BG_E_NOMEM;
  bg_mark(c, "merge");
  return 0;
}

// the zero-length prints of nextIntersectLine (see k_zi_replay) merged into `acc`
static int intersect_zero_len(bg_ctx* c, const std::vector<Ivl>& F, Ivl& acc) {
  const int nf = (int)F.size();
  const uint64_t no = acc.n;
  uint8_t* flag = (uint8_t*)bg_alloc(c, no + 1);
  if (!flag) return BG_E_NOMEM;
  BG_HIP(c, hipMemsetAsync(flag, 0, no + 1, c->stream));
  uint64_t npieces = 0;
  for (const Ivl& f : F) {
    npieces += f.n;
    if (f.n)
      BG_LAUNCH(c, "k_zi_mark", k_zi_mark, dim3(bg_blocks(f.n, BG_NT)), dim3(BG_NT), f.s, f.e, f.n,
                acc.s, no, flag);
  }
  BG_HIP(c, hipGetLastError());
  uint64_t* anchors = nullptr;
  uint64_t na = 0;
  int rc = bg_compact_flags(c, flag, no + 1, &anchors, &na);
  bg_release(c, flag);
  if (rc) return rc;
  if (na == 0) {
    bg_release(c, anchors);
    return 0;
  }
  std::vector<ZFile> hf(nf);
  for (int f = 0; f < nf; ++f) hf[f] = ZFile{F[f].s, F[f].e, F[f].n};
  ZFile* dF = (ZFile*)bg_alloc(c, sizeof(ZFile) * nf);
  uint64_t* H = (uint64_t*)bg_alloc(c, 8ull * na * nf);
  uint64_t* cnt = (uint64_t*)bg_alloc(c, 8ull * (na + 1));
  uint64_t* bad = (uint64_t*)bg_alloc(c, 8);
  if (!dF || !H || !cnt || !bad) return BG_E_NOMEM;
  BG_HIP(c, hipMemcpyAsync(dF, hf.data(), sizeof(ZFile) * nf, hipMemcpyHostToDevice, c->stream));
  BG_HIP(c, hipMemsetAsync(bad, 0, 8, c->stream));
  // every loop iteration of a replay advances a head or restarts from a later piece
  const uint64_t cap = 8ull * (npieces + 16) * (uint64_t)(nf + 1);
  const unsigned nb = bg_blocks(na, BG_NT);
  BG_LAUNCH(c, "k_zi_replay_count", k_zi_replay<false>, dim3(nb), dim3(BG_NT), dF, nf, acc.s, acc.e,
            no, anchors, na, H, cnt, (const uint64_t*)nullptr, (int64_t*)nullptr, (int64_t*)nullptr,
            cap, (unsigned long long*)bad);
  BG_HIP(c, hipGetLastError());
  if ((rc = bg_scan_sum_u64(c, cnt, cnt, na, cnt + na))) return rc;
  uint64_t total = 0, hbad = 0;
  if ((rc = bg_fetch_u64(c, cnt + na, &total)) || (rc = bg_fetch_u64(c, bad, &hbad))) return rc;
  if (hbad)
    return bg_fail(c, BG_E_INTERNAL, "intersect: zero-length replay inconsistent (code " +
                                         std::to_string(hbad) + ")");
  Ivl out;
  if ((rc = ivl_alloc(c, out, no + total))) return rc;
  BG_LAUNCH(c, "k_zi_replay_write", k_zi_replay<true>, dim3(nb), dim3(BG_NT), dF, nf, acc.s, acc.e,
            no, anchors, na, H, (uint64_t*)nullptr, (const uint64_t*)cnt, out.s, out.e, cap,
            (unsigned long long*)bad);
  if (no)
    BG_LAUNCH(c, "k_zi_place", k_zi_place, dim3(bg_blocks(no, BG_NT)), dim3(BG_NT), acc.s, acc.e, no,
              anchors, na, (const uint64_t*)cnt, out.s, out.e);
  BG_HIP(c, hipGetLastError());
  BG_HIP(c, hipStreamSynchronize(c->stream));  // hf/dF copy and the scratch below
  bg_release(c, dF);
  bg_release(c, H);
  bg_release(c, cnt);
  bg_release(c, bad);
  bg_release(c, anchors);
  ivl_free(c, acc);
  acc = out;
  return 0;
}

extern "C" int bg_intersect(bg_ctx* c, bg_set* set, const int* files, int nf, bg_result** out) {
  int rc = bg_check_files(c, set, files, nf, 2);
  if (rc) return rc;
  // Each file's pieces (getNextFileMergedCoords); the non-empty output is the set
  // intersection, folded pairwise. Files with zero-length pieces add nextIntersectLine's
  // zero-length prints afterwards (intersect_zero_len).
  bool zero = false;
  std::vector<Ivl> comp(nf);
  for (int k = 0; k < nf; ++k) {
    zero = zero || set->t[files[k]]->has_zero_len;
    if ((rc = bg_table_components(c, set->t[files[k]], comp[k]))) return rc;
  }
  Ivl acc = comp[0];
  acc.owned = false;  // comp[0] keeps ownership
  for (int k = 1; k < nf; ++k) {
    Ivl p;
    // the last fold goes straight to the formatter, segmented (unless the zero-length
    // replay still reads it)
    const uint32_t* seg = (k + 1 == nf && !zero) ? set->d_name_len : nullptr;
    if ((rc = mp_op<MP_INTERSECT>(c, acc, comp[k], p, "k_intersect_count", "k_intersect_write", seg)))
      return rc;
    ivl_free(c, acc);
    acc = p;
  }
  if (zero && (rc = intersect_zero_len(c, comp, acc))) return rc;
  for (Ivl& v : comp) ivl_free(c, v);
  *out = bg_new_ivl_result(c, set, acc);
  bg_mark(c, "intersect");
  return 0;
}

extern "C" int bg_difference(bg_ctx* c, bg_set* set, int ref, const int* others, int no,
                             bg_result** out) {
  int rc = bg_check_files(c, set, others, no, 1);
  if (rc) return rc;
  if (ref < 0 || ref >= (int)set->t.size()) return BG_E_ARG;
  Ivl r, o, d;
  if ((rc = bg_table_components(c, set->t[ref], r))) return rc;
  if ((rc = bg_union_components(c, set, others, no, o))) return rc;
  if ((rc = mp_op<MP_DIFFERENCE>(c, r, o, d, "k_difference_count", "k_difference_write", set->d_name_len)))
    return rc;
  ivl_free(c, r);
  ivl_free(c, o);
  *out = bg_new_ivl_result(c, set, d);
  bg_mark(c, "difference");
  return 0;
}

extern "C" int bg_element_of(bg_ctx* c, bg_set* set, int ref, const int* others, int no,
                             double thres, int use_pct, int invert, bg_result** out) {
  int rc = bg_check_files(c, set, others, no, 1);
  if (rc) return rc;
  if (ref < 0 || ref >= (int)set->t.size()) return BG_E_ARG;
  bg_table* R = set->t[ref];
  if ((rc = bg_need_rows(c, set, &ref, 1, "element-of reference"))) return rc;
  Ivl o;
  if ((rc = bg_union_components(c, set, others, no, o))) return rc;
  uint64_t* P = (uint64_t*)bg_alloc(c, 8 * (o.n + 1));
  uint8_t* flag = (uint8_t*)bg_alloc(c, R->n ? R->n : 1);
  if (!P || !flag) return BG_E_NOMEM;
  // the kept rows' printed lengths, summed per format tile during the compaction (no
  // formatter count pass) when the table keeps its remainders (row results print them)
  uint16_t* blen = R->rest_len ? (uint16_t*)bg_alloc(c, 2 * (R->n ? R->n : 1)) : nullptr;
  unsigned int* ovf = blen ? (unsigned int*)bg_alloc(c, 4) : nullptr;
  if (blen && !ovf) return BG_E_NOMEM;
  if (ovf) BG_HIP(c, hipMemsetAsync(ovf, 0, 4, c->stream));
  if (o.n) {
    BG_LAUNCH(c, "k_lengths", k_lengths, dim3(bg_blocks(o.n, BG_NT)), dim3(BG_NT), o.s, o.e, o.n, P);
    BG_HIP(c, hipGetLastError());
  }
  if ((rc = bg_scan_sum_u64(c, P, P, o.n, P + o.n))) return rc;
  if (R->n) {
    const uint64_t nblk = bg_blocks(R->n, BG_NT);
    uint64_t* bnd = (uint64_t*)bg_alloc(c, 8 * nblk);
    if (!bnd) return BG_E_NOMEM;
    BG_LAUNCH(c, "k_element_lo", k_element_lo, dim3(bg_blocks(nblk, BG_NT)), dim3(BG_NT), R->ks, o.e, o.n, nblk,
              bnd);
    BG_HIP(c, hipGetLastError());
    BG_LAUNCH(c, "k_element_flags", k_element_flags, dim3((unsigned)nblk), dim3(BG_NT),
              R->ks, R->ke, R->n, o.s, o.e, o.n, P, thres, use_pct, invert, flag, set->d_name_len, R->rest_len,
              blen, ovf, (const uint64_t*)bnd);
    BG_HIP(c, hipGetLastError());
    bg_release(c, bnd);
  }
  uint64_t total = 0;
  uint64_t* rows = nullptr;
  uint64_t* tbytes = nullptr;
  if (!blen) {
    rc = bg_compact_flags(c, flag, R->n, &rows, &total);
  } else {
    const unsigned nb = bg_blocks(R->n, CF_TILE);
    rc = count_scan_write(
        c, nb,
        [&](uint64_t* cnt) {
          BG_LAUNCH(c, "k_compact_flags_count", k_compact_flags<false>, dim3(nb), dim3(BG_NT), flag, R->n, cnt,
                    (const uint64_t*)nullptr, (uint64_t*)nullptr);
        },
        [&](uint64_t* off, uint64_t tot) -> int {
          rows = (uint64_t*)bg_alloc(c, 8 * (tot ? tot : 1));
          const uint64_t nt = bg_blocks(tot, BG_FMT_TILE);
          tbytes = (uint64_t*)bg_alloc(c, 8 * (nt ? nt : 1));
          if (!rows || !tbytes) return BG_E_NOMEM;
          BG_HIP(c, hipMemsetAsync(tbytes, 0, 8 * (nt ? nt : 1), c->stream));
          if (nb)
            BG_LAUNCH(c, "k_compact_rows_bytes", k_compact_rows_bytes, dim3(nb), dim3(BG_NT), flag, blen, R->n,
                      off, rows, (unsigned long long*)tbytes);
          return 0;
        },
        &total);
    unsigned int h = 0;  // a line over 64 KiB: the formatter counts instead
    if (!rc) BG_HIP(c, hipMemcpyAsync(&h, ovf, 4, hipMemcpyDeviceToHost, c->stream));
    if (!rc) BG_HIP(c, hipStreamSynchronize(c->stream));
    if (h) {
      bg_release(c, tbytes);
      tbytes = nullptr;
    }
  }
  if (rc) return rc;
  bg_release(c, P);
  bg_release(c, flag);
  bg_release(c, blen);
  bg_release(c, ovf);
  ivl_free(c, o);
  bg_result* res = new bg_result();
  res->ctx = c;
  res->set = set;
  res->kind = RES_ROWS;
  res->n = total;
  res->rows = rows;
  res->tbytes = tbytes;
  res->tab = ref;
  *out = res;
  bg_mark(c, "element-of");
  return 0;
}
