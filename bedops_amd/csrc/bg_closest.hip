// bg_closest.hip — K6: closest-features <input-file> <query-file>.
//
// Reference: FeatDist::findDistances (applications/bed/closestfeats/src/ClosestFeature.cpp:
// 260-413) walks the sorted <input-file> rows ("ref" rows b) once; for each b it reads
// <query-file> rows ("candidates" c) through a BedReader whose LIFO cache
// (closestfeats/src/BedReader.hpp:55-80) gets back a list of rows the previous b kept.
// Which rows that cache keeps is NOT "every row that could still matter": a new best
// left empties it (ClosestFeature.cpp:300-304, :369-373), so a row that overlapped an
// earlier b and ends later than the new left is gone for every later b. The chosen
// left/right therefore depend on the history of the scan, not only on b (verified
// against the restatement in oracle/closest_oracle.c: a cache-free search differs on
// nested inputs). The GPU reproduces the sequential state machine exactly:
//
//   state between two ref rows = (file position fp, cached rows in pop order)
//
// - k_closest_chunks: one thread per chunk of CQ consecutive ref rows. Chunk 0 starts
//   from the true initial state. Chunk k > 0 starts SPECULATIVELY CW rows earlier, with
//   an empty cache and fp at the first candidate that starts within the longest
//   candidate length before that row (so every row the true cache may still hold is
//   read again), replays those CW rows without output, records the state it reached at
//   its first own row, then emits left/right for its rows and records its final state.
//   (Measured on random nested inputs with the Python replay of the oracle: 16 warm-up
//   rows reproduce the exact cache — content AND order — at ~100% of chunk starts.)
// - k_closest_check: chunk k is exact iff its recorded start state equals chunk k-1's
//   final state (and chunk k-1 is exact): induction from chunk 0.
// - k_closest_fix: chunks whose start differs from a stable predecessor's final state
//   re-run from that state; check again; after a few rounds any remainder is resolved by
//   one in-order pass (k_closest_serial), so the result is exact in every case.
// The row-by-row rules below follow ClosestFeature.cpp:284-401 line for line in meaning;
// getDistance :244-255 and the centroid proportion :226-239 use the same double
// arithmetic. Output (PrintAll / PrintShortest, Printers.hpp:46-205) is rendered by
// bg_format.hip from the per-row (left, right) candidate indices.
#include <climits>
#include <cstring>

#include "bg_internal.h"

#ifndef CQ_DEF
#define CQ_DEF 22  // ref rows per chunk (10M x 1B, round 6: 22 rows + 3 warm-up 16.5-16.7 ms, step 37.5-37.7; 20 + 4: 17.55; 24 + 4: 17.95; 16 or 28: 18.6;
                   // round 6: the 6.5K waves of 24-row chunks took 1.27 rounds of the 5 resident per SIMD;
                   // 3-8 warm-up rows, profiles/r04_closest_cq.txt)
#endif
#ifndef CW_DEF
#define CW_DEF 3   // speculative warm-up rows before a chunk (2: the fix-up pass dominates, step 42.5 ms)
#endif
#define CBACK 4096 // at most this many candidates before the warm-up row are re-read
#define CAP0 256   // initial capacity of the cache stack / kept list (x4 on overflow)
#define FIX_ROUNDS 8

struct ClArgs {
  const int64_t* qs;  // ref rows (<input-file>), keyed
  const int64_t* qe;
  uint64_t nq;
  const int64_t* cs;  // candidates (<query-file>), keyed
  const int64_t* ce;
  uint64_t nc;
  int overlaps;
  int64_t* left;
  int64_t* right;
  // per chunk k: slot 2k = start state (snapshot), slot 2k+1 = working / final state,
  // kl[k] = the per-row kept list; each holds `cap` candidate indices
  uint64_t* st_fp;
  uint32_t* st_n;
  uint32_t* st_c;  // cache stack per slot, bottom first (pop from the top = last)
  uint32_t* kl;
  uint32_t cap;
  uint32_t cq, cw;  // rows per chunk, warm-up rows
  int64_t lmax;  // longest candidate: a row still cached can start at most lmax earlier
  uint32_t nchunks;
  uint32_t* flag;
  uint32_t* nflag;
  uint32_t* overflow;
};

// The cache stack and the kept list of a chunk live in LDS, CL_D entries per thread (one
// column per thread: [entry][thread], so a wave's accesses stay in distinct banks), and
// spill to the chunk's global slot only when deeper: the stack keeps its top CL_D entries
// in a ring in LDS and moves the oldest to global memory on overflow; the kept list keeps
// its first CL_D entries in LDS. Global memory sees the state only at the two snapshots
// (after the warm-up, at the chunk's end) and on deep stacks (nested inputs).
#define CL_D 16
struct ClState {
  uint64_t fp;
  uint32_t n;   // stack depth
  uint32_t m;   // top entries resident in the LDS ring (entries [n - m, n))
  uint32_t* c;  // stack storage (global, `cap` entries): entries [0, n - m)
  uint32_t* l;  // this thread's LDS ring column (entry i at l[(i % CL_D) * BG_NT])
};
__device__ __forceinline__ void cl_push(ClState& S, uint32_t x) {
  if (S.m == CL_D) {  // spill the oldest ring entry
    const uint32_t i = S.n - S.m;
    S.c[i] = S.l[(i & (CL_D - 1)) * BG_NT];
    --S.m;
  }
  S.l[(S.n & (CL_D - 1)) * BG_NT] = x;
  ++S.n;
  ++S.m;
}
__device__ __forceinline__ uint32_t cl_pop(ClState& S) {
  --S.n;
  if (S.m) {
    --S.m;
    return S.l[(S.n & (CL_D - 1)) * BG_NT];
  }
  return S.c[S.n];
}
// entry i (from the bottom) without popping
__device__ __forceinline__ uint32_t cl_peek(const ClState& S, uint32_t i) {
  return i >= S.n - S.m ? S.l[(i & (CL_D - 1)) * BG_NT] : S.c[i];
}
// pop k entries
__device__ __forceinline__ void cl_drop(ClState& S, uint32_t k) {
  S.n -= k;
  S.m = S.m > k ? S.m - k : 0;
}
// the whole stack in global memory (snapshots, comparisons)
__device__ __forceinline__ void cl_flush(ClState& S) {
  for (uint32_t i = S.n - S.m; i < S.n; ++i) S.c[i] = S.l[(i & (CL_D - 1)) * BG_NT];
  S.m = 0;
}
struct ClKept {  // the per-row kept list: entries [0, CL_D) in LDS, the rest in global
  uint32_t* l;   // LDS column
  uint32_t* g;   // global overflow (`cap` entries)
  __device__ __forceinline__ void put(uint32_t i, uint32_t x) const {
    if (i < CL_D) l[i * BG_NT] = x;
    else g[i] = x;
  }
  __device__ __forceinline__ uint32_t get(uint32_t i) const { return i < CL_D ? l[i * BG_NT] : g[i]; }
};

#define D_MINUS LLONG_MIN
#define D_PLUS LLONG_MAX

// getDistance(c, b): ClosestFeature.cpp:244-255 on keyed coordinates
__device__ __forceinline__ int64_t cl_dist(int64_t cs, int64_t ce, int64_t bs, int64_t be) {
  const int64_t gc = cs >> BG_KEY_SHIFT, gb = bs >> BG_KEY_SHIFT;
  if (gc != gb) return gc < gb ? D_MINUS : D_PLUS;
  if (ce <= bs) return -((bs - ce) + 1);
  if (be <= cs) return (cs - be) + 1;
  return 0;
}

// replay ref rows [b0, b1) from state S; emit: write left/right. false on overflow.
//
// One candidate per iteration, in the order the reference reads them (the cache stack
// first, then the file). The reference's branch chain (ClosestFeature.cpp:284-401) is
// evaluated as flags: every case below sets some of
//   reset   : the kept list is emptied (a new best left)
//   keepL/R/C: the current left / right / this candidate is appended to the kept list,
//             always in that order
//   left, right, ld, rdist, lc (leftCached) updates, brk (the scan of b ends)
// and the updates are applied with selects: the lanes of a wave take different cases on
// almost every candidate, and a nested if-chain made each wave issue every case's
// exec-mask bookkeeping in turn (SALU-bound: ~700 scalar instructions per candidate).
//   case                                   reference lines
//   d = -inf (earlier chromosome)          skip                           :289-291
//   d < 0, d >= ld  (newleft)              reset; left = c                :300-305
//   d < 0, d <  ld  (dropL)                keepL(!lc); lc = 1             :306-309
//   d = +inf                               keepL; keepR; keepC; brk       :292-298
//   d > 0, d < rdist (firstR)              keepL; right = c; keepC; brk   :315-323
//   d > 0, else (farR)                     keepL; keepR; keepC; brk       :324-330
//   d = 0, overlaps, cs <= bs (hangL)      keepL unless ce[left] <= ce; left = c, ld = 0
//   d = 0, overlaps, be <= ce (hangR)      keepL; keepR; right = c, rdist = 0
//   d = 0, overlaps, inside: by the centroid proportion (:227-239, :355-388)
//   d = 0, no-overlaps (noov)              keepL (lc = 1); keepC          :389-397
__device__ bool cl_run(const ClArgs& A, uint64_t b0, uint64_t b1, ClState& S, const ClKept& kept,
                       bool emit) {
  const uint32_t cap = A.cap;
  // the next CPF file candidates, loaded ahead: the scan's loads are independent of its
  // decisions, so the file stream is software-pipelined (one candidate at a time each
  // lane waited an L2 round trip per candidate; lanes read disjoint regions)
  constexpr int CPF = 4;
  int64_t pcs[CPF], pce[CPF];
  const uint64_t nc1 = A.nc ? A.nc - 1 : 0;
#pragma unroll
  for (int i = 0; i < CPF; ++i) {
    const uint64_t j = min(S.fp + i, nc1);
    pcs[i] = A.nc ? A.cs[j] : 0;
    pce[i] = A.nc ? A.ce[j] : 0;
  }
  for (uint64_t b = b0; b < b1; ++b) {
    const int64_t bs = A.qs[b], be = A.qe[b];
    int64_t ld = D_MINUS, rdist = D_PLUS;
    int64_t left = -1, right = -1, lce = 0;  // lce = ce[left]
    bool lc = false;  // leftCached
    uint32_t nk = 0;  // the std::list "read" of findDistances
    bool ovf = false, eof = false;
#define KEEP(x)                         \
  do {                                  \
    if (nk == cap) ovf = true;          \
    else kept.put(nk++, (uint32_t)(x)); \
  } while (0)
    // one candidate through the reference's branch chain; true when the scan of b ends
    auto step = [&](int64_t c, int64_t cs, int64_t ce) -> bool {
      const int64_t d = cl_dist(cs, ce, bs, be);
      if (d == D_MINUS) return false;  // earlier chromosome: dropped
      const bool hasL = left >= 0, hasR = right >= 0;
      const bool plus = d == D_PLUS;
      const bool neg = d < 0;
      const bool pos = d > 0 && !plus;
      const bool newleft = neg && d >= ld;
      const bool dropL = neg && !newleft;
      const bool firstR = pos && d < rdist;
      const bool farR = pos && !firstR;
      const bool ovl = d == 0 && A.overlaps;
      const bool noov = d == 0 && !A.overlaps;
      const bool hangL = ovl && cs <= bs;
      const bool hangR = ovl && !hangL && be <= ce;
      const bool inside = ovl && !hangL && !hangR;
      bool half = false;
      {  // the reference's centroid test (ClosestFeature.cpp: prop = (cen + 1 - cs) / (ce - cs),
         // cen = (be - 1 + bs) / 2 as doubles, prop < 0.5) in exact integers (round 5; checked
         // against the double form, boundary cases included, tests/test_closest_model.py)
        const int64_t bsc = bs & BG_COORD_MASK, bec = be & BG_COORD_MASK;
        const int64_t csc = cs & BG_COORD_MASK, cec = ce & BG_COORD_MASK;
        half = inside && (2 * csc > bsc + bec - 1 || bsc + bec + 1 - 2 * csc < cec - csc);
      }
      const bool in_a = inside && ld == 0 && half;    // keepL(!lc), lc = 1, keepR, right = c
      const bool in_b = inside && ld == 0 && !half;   // keepL(!lc), lc = 1, keepC
      const bool in_c = inside && ld != 0 && !half;   // reset, left = c, ld = 0, lc = 0
      const bool in_d = inside && ld != 0 && half;    // keepL, keepR, right = c
      const bool reset = newleft || in_c;
      const bool keepL = hasL && !lc &&
                         (plus || firstR || farR || hangR || in_d || noov || dropL || in_a || in_b ||
                          (hangL && !(lce <= ce)));
      const bool keepR = hasR && (plus || farR || hangR || in_a || in_d);
      const bool keepC = plus || firstR || farR || in_b || noov;
      if (reset) {
        nk = 0;
        ovf = false;
      }
      if (keepL) KEEP(left);
      if (keepR) KEEP(right);
      if (keepC) KEEP(c);
      // lc: set to hasL when the scan moves on past the left, 1 when the left was cached,
      // cleared by a new left
      const bool lc_hasl = plus || firstR || farR || hangR || in_d;
      const bool lc_one = dropL || in_a || in_b || (noov && hasL);
      const bool lc_zero = newleft || hangL || in_c;
      lc = lc_zero ? false : (lc_one ? true : (lc_hasl ? hasL : lc));
      const bool setleft = newleft || hangL || in_c;
      left = setleft ? c : left;
      lce = setleft ? ce : lce;
      ld = newleft ? d : ((hangL || in_c) ? 0 : ld);
      const bool setright = firstR || hangR || in_a || in_d;
      right = setright ? c : right;
      rdist = firstR ? d : ((hangR || in_a || in_d) ? 0 : rdist);
      return plus || pos;
    };
    // the next file row (its keys from the look-ahead registers)
    auto advance = [&]() {
#pragma unroll
      for (int i = 0; i + 1 < CPF; ++i) {
        pcs[i] = pcs[i + 1];
        pce[i] = pce[i + 1];
      }
      const uint64_t j = min(S.fp + (CPF - 1), nc1);
      pcs[CPF - 1] = A.cs[j];
      pce[CPF - 1] = A.ce[j];
    };
    // The scan in three phases, each run by all lanes of a wave together (lanes whose scan
    // already ended idle), so a phase costs its longest lane, not the sum of every lane's
    // phases one after the other:
    //   A: the cached rows (popped in the reference's order);
    //   B: the file's run of rows that end at or before bs (d < 0, or an earlier chromosome,
    //      skipped): they change only (left, ld, lc) and the kept list, as the chain would:
    //        d >= ld (newleft): reset; left = c; ld = d; lc = 0
    //        d <  ld (dropL)  : keepL unless lc; lc = 1
    //      ~70% of the rows read on the benchmark's inputs, at a compare and a select each;
    //   C: the rest of the file through the chain, up to the row that ends the scan.
    bool brk = false;
    while (S.n && !brk) {  // A
      const int64_t c = cl_pop(S);
      brk = step(c, A.cs[c], A.ce[c]);
    }
    if (!brk) {  // B in closed form, the file's ends CB at a time
      // Over the run, the chain's effect is: every row whose end is >= the running maximum
      // (and >= the current left's, d >= ld) is a new left (reset), every other row a
      // dropL. So the left afterwards is the LAST row holding the run's largest end M when
      // M beats the current left, the kept list is reset there, and a row after it keeps
      // it (lc); otherwise the first row keeps the current left (unless cached) and lc = 1.
      // Only the ends are needed: CB of them per load, all in flight together (one row at a
      // time through the chain, round 3, waited an L2 round trip per row: 28.1 -> 19.0 ms;
      // CB = 16, 18.7 ms, costs registers)
      constexpr int CB = 8;
      const int64_t gb = bs >> BG_KEY_SHIFT;
      uint64_t j = S.fp, jend = A.nc;
      int64_t M = LLONG_MIN;
      uint64_t p = 0;
      bool any = false, after = false, end = false;
      while (!end && j < A.nc) {
        const uint64_t base = j & ~(uint64_t)(CB - 1);
        int64_t v[CB];
        if (base + CB <= A.nc) {
          const longlong2* q = reinterpret_cast<const longlong2*>(A.ce + base);
#pragma unroll
          for (int i = 0; i < CB / 2; ++i) {
            const longlong2 t = q[i];
            v[2 * i] = t.x;
            v[2 * i + 1] = t.y;
          }
        } else {
#pragma unroll
          for (int i = 0; i < CB; ++i) v[i] = base + i < A.nc ? A.ce[base + i] : LLONG_MAX;
        }
#pragma unroll
        for (int i = 0; i < CB; ++i) {
          const uint64_t x = base + i;
          if (end || x < j) continue;
          if (v[i] > bs) {  // (LLONG_MAX past the file: its end)
            end = true;
            jend = min(x, A.nc);
            continue;
          }
          if ((v[i] >> BG_KEY_SHIFT) != gb) continue;  // earlier chromosome: dropped
          any = true;
          if (v[i] >= M) {
            M = v[i];
            p = x;
            after = false;
          } else {
            after = true;
          }
        }
        j = base + CB;
      }
      S.fp = end ? jend : A.nc;
      if (any) {
        const int64_t d = -((bs - M) + 1);
        if (d >= ld) {
          nk = 0;
          ovf = false;
          left = (int64_t)p;
          lce = M;
          ld = d;
          lc = false;
          if (after) {
            KEEP(left);
            lc = true;
          }
        } else {
          if (left >= 0 && !lc) KEEP(left);
          lc = true;
        }
      }
#pragma unroll
      for (int i = 0; i < CPF; ++i) {  // the look-ahead registers from the new position
        const uint64_t q = min(S.fp + i, nc1);
        pcs[i] = A.nc ? A.cs[q] : 0;
        pce[i] = A.nc ? A.ce[q] : 0;
      }
    }
    while (!brk) {  // C
      if (S.fp >= A.nc) {
        eof = true;
        break;
      }
      const int64_t c = (int64_t)S.fp++;
      const int64_t cs = pcs[0], ce = pce[0];
      advance();
      brk = step(c, cs, ce);
    }
    if (eof && left >= 0 && !lc) KEEP(left);
    if (eof && right >= 0) KEEP(right);
#undef KEEP
    // BedReader::PushBack(list): the list comes back out in list order
    if (ovf || S.n + nk > cap) return false;
    for (uint32_t i = nk; i-- > 0;) cl_push(S, kept.get(i));
    if (emit) {
      A.left[b] = left;
      A.right[b] = right;
    }
  }
  return true;
}

__device__ __forceinline__ uint32_t* cl_slot(const ClArgs& A, uint64_t slot) {
  return A.st_c + slot * A.cap;
}
__device__ __forceinline__ void cl_copy(const ClArgs& A, uint64_t from, uint64_t to) {
  const uint32_t n = A.st_n[from];
  A.st_fp[to] = A.st_fp[from];
  A.st_n[to] = n;
  const uint32_t* x = cl_slot(A, from);
  uint32_t* y = cl_slot(A, to);
  for (uint32_t i = 0; i < n; ++i) y[i] = x[i];
}
__device__ __forceinline__ bool cl_same(const ClArgs& A, uint64_t x, uint64_t y) {
  if (A.st_fp[x] != A.st_fp[y] || A.st_n[x] != A.st_n[y]) return false;
  const uint32_t* a = cl_slot(A, x);
  const uint32_t* b = cl_slot(A, y);
  for (uint32_t i = 0; i < A.st_n[x]; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

__device__ __forceinline__ ClKept cl_kept(const ClArgs& A, uint32_t k, uint32_t* lk) {
  return ClKept{lk + threadIdx.x, A.kl + (uint64_t)k * A.cap};
}

// run chunk k's own rows from the state held in its working slot (global)
__device__ __forceinline__ void cl_own(const ClArgs& A, uint32_t k, uint32_t* ls, uint32_t* lk) {
  const uint64_t q0 = (uint64_t)k * A.cq, q1 = min(q0 + A.cq, A.nq);
  const uint64_t w = 2ull * k + 1;
  ClState S{A.st_fp[w], A.st_n[w], 0, cl_slot(A, w), ls + threadIdx.x};
  if (!cl_run(A, q0, q1, S, cl_kept(A, k, lk), true)) {
    atomicOr(A.overflow, 1u);
    S.fp = ~0ull - 1;  // a final state no successor starts from
    S.n = S.m = 0;
  }
  cl_flush(S);
  A.st_fp[w] = S.fp;
  A.st_n[w] = S.n;
}

#ifndef BG_CL_WAVES
#define BG_CL_WAVES
#endif
__global__ void __launch_bounds__(BG_NT) BG_CL_WAVES k_closest_chunks(ClArgs A) {
  __shared__ uint32_t ls[CL_D * BG_NT], lk[CL_D * BG_NT];
  const uint32_t k = blockIdx.x * BG_NT + threadIdx.x;
  if (k >= A.nchunks) return;
  const uint64_t q0 = (uint64_t)k * A.cq;
  const uint64_t w = 2ull * k + 1;
  ClState S{0, 0, 0, cl_slot(A, w), ls + threadIdx.x};
  if (k > 0) {
    const uint64_t qw = q0 - A.cw;
    // speculative start: every candidate that can still overlap row qw or anything
    // after it (starts within lmax before it), read afresh; the state converges to the
    // true one within a few rows (the check below proves it or triggers the fix-up)
    const uint64_t p = lower_bound_i64(A.cs, A.nc, A.qs[qw]);
    const uint64_t f = lower_bound_i64(A.cs, A.nc, A.qs[qw] - A.lmax - 1);
    S.fp = (p - f > CBACK) ? p - CBACK : f;
    if (!cl_run(A, qw, q0, S, cl_kept(A, k, lk), false)) {
      // speculation overflowed: leave this chunk to the fix-up
      A.st_fp[2ull * k] = ~0ull;  // a start state no predecessor ends in
      A.st_n[2ull * k] = 0;
      A.st_fp[w] = ~0ull - 1;
      A.st_n[w] = 0;
      return;
    }
  }
  cl_flush(S);
  A.st_fp[w] = S.fp;
  A.st_n[w] = S.n;
  cl_copy(A, w, 2ull * k);  // snapshot of the start state
  cl_own(A, k, ls, lk);
}

__global__ void k_closest_check(ClArgs A) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= A.nchunks) return;
  const bool bad = k > 0 && !cl_same(A, 2ull * k, 2ull * (k - 1) + 1);
  A.flag[k] = bad;
  if (bad) atomicAdd(A.nflag, 1u);
}

// re-run chunks whose predecessor is consistent (its final state is stable this round)
__global__ void __launch_bounds__(BG_NT) k_closest_fix(ClArgs A) {
  __shared__ uint32_t ls[CL_D * BG_NT], lk[CL_D * BG_NT];
  const uint32_t k = blockIdx.x * BG_NT + threadIdx.x;
  if (k == 0 || k >= A.nchunks || !A.flag[k] || A.flag[k - 1]) return;
  cl_copy(A, 2ull * (k - 1) + 1, 2ull * k);
  cl_copy(A, 2ull * k, 2ull * k + 1);
  cl_own(A, k, ls, lk);
}

// last resort: one in-order pass (exact for any input)
__global__ void __launch_bounds__(BG_NT) k_closest_serial(ClArgs A) {
  __shared__ uint32_t ls[CL_D * BG_NT], lk[CL_D * BG_NT];
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  for (uint32_t k = 1; k < A.nchunks; ++k) {
    if (cl_same(A, 2ull * k, 2ull * (k - 1) + 1)) continue;
    cl_copy(A, 2ull * (k - 1) + 1, 2ull * k);
    cl_copy(A, 2ull * k, 2ull * k + 1);
    cl_own(A, k, ls, lk);
  }
}

// one attempt at capacity A.cap; *ovf set if some state outgrew it
static int closest_pass(bg_ctx* c, ClArgs& A, bool* ovf) {
  *ovf = false;
  const uint64_t slots = 2ull * A.nchunks;
  A.st_fp = (uint64_t*)bg_alloc(c, 8 * slots);
  A.st_n = (uint32_t*)bg_alloc(c, 4 * slots);
  A.st_c = (uint32_t*)bg_alloc(c, 4ull * A.cap * slots);
  A.kl = (uint32_t*)bg_alloc(c, 4ull * A.cap * A.nchunks);
  A.flag = (uint32_t*)bg_alloc(c, 4ull * A.nchunks);
  A.nflag = (uint32_t*)bg_alloc(c, 8);
  A.overflow = A.nflag + 1;
  int rc = 0;
  if (!A.st_fp || !A.st_n || !A.st_c || !A.kl || !A.flag || !A.nflag) rc = BG_E_NOMEM;
  if (!rc) rc = bg_hip_ok(c, hipMemsetAsync(A.nflag, 0, 8, c->stream));
  if (!rc) {
    BG_LAUNCH(c, "k_closest_chunks", k_closest_chunks, dim3(bg_blocks(A.nchunks, BG_NT)),
              dim3(BG_NT), A);
    rc = bg_hip_ok(c, hipGetLastError());
  }
  uint32_t h[2] = {0, 0};
  for (int round = 0; !rc; ++round) {
    rc = bg_hip_ok(c, hipMemsetAsync(A.nflag, 0, 4, c->stream));
    if (rc) break;
    BG_LAUNCH(c, "k_closest_check", k_closest_check, dim3(bg_blocks(A.nchunks, 256)), dim3(256), A);
    rc = bg_hip_ok(c, hipMemcpyAsync(h, A.nflag, 8, hipMemcpyDeviceToHost, c->stream));
    if (!rc) rc = bg_hip_ok(c, hipStreamSynchronize(c->stream));
    if (rc || h[0] == 0 || h[1]) break;
    if (round == FIX_ROUNDS) {
      BG_LAUNCH(c, "k_closest_serial", k_closest_serial, dim3(1), dim3(BG_NT), A);
      rc = bg_hip_ok(c, hipGetLastError());
      if (!rc) rc = bg_hip_ok(c, hipMemcpyAsync(h, A.nflag, 8, hipMemcpyDeviceToHost, c->stream));
      if (!rc) rc = bg_hip_ok(c, hipStreamSynchronize(c->stream));
      break;  // the in-order pass leaves every chunk consistent
    }
    BG_LAUNCH(c, "k_closest_fix", k_closest_fix, dim3(bg_blocks(A.nchunks, BG_NT)), dim3(BG_NT), A);
    rc = bg_hip_ok(c, hipGetLastError());
  }
  *ovf = h[1] != 0;
  bg_release(c, A.st_fp);
  bg_release(c, A.st_n);
  bg_release(c, A.st_c);
  bg_release(c, A.kl);
  bg_release(c, A.flag);
  bg_release(c, A.nflag);
  return rc;
}

extern "C" int bg_closest(bg_ctx* c, bg_set* set, int ref, int query, const bg_closest_opts* o,
                          bg_result** out) {
  if (!c || !set || !o || !out || ref < 0 || query < 0 || ref >= (int)set->t.size() ||
      query >= (int)set->t.size())
    return BG_E_ARG;
  *out = nullptr;
  {
    const int f[2] = {ref, query};
    int rc0 = bg_need_rows(c, set, f, 2, "closest-features");
    if (rc0) return rc0;
  }
  bg_table* Q = set->t[ref];
  bg_table* C = set->t[query];
  if (!Q->rest_off || !C->rest_off)
    return bg_fail(c, BG_E_ARG, "closest-features needs both inputs loaded as BG_BED3_REST");
  if (C->n >= (1ull << 32))
    return bg_fail(c, BG_E_UNSUPPORTED, "more than 2^32 rows in <query-file>");
  bg_result* r = new bg_result();
  r->ctx = c;
  r->set = set;
  r->kind = RES_CLOSEST;
  r->tab = ref;
  r->tab2 = query;
  r->copts = *o;
  r->copts.delim[15] = 0;
  r->n = Q->n;
  const uint64_t n = Q->n ? Q->n : 1;
  r->left = (int64_t*)bg_alloc(c, 8 * n);
  r->right = (int64_t*)bg_alloc(c, 8 * n);
  if (!r->left || !r->right) { bg_result_free(r); return BG_E_NOMEM; }
  if (Q->n == 0) { *out = r; return 0; }

  ClArgs A;
  memset(&A, 0, sizeof(A));
  A.qs = Q->ks; A.qe = Q->ke; A.nq = Q->n;
  A.cs = C->ks; A.ce = C->ke; A.nc = C->n;
  A.overlaps = !o->no_overlaps;
  A.lmax = C->maxlen;
  A.left = r->left; A.right = r->right;
  A.cq = CQ_DEF;
  A.cw = CW_DEF;
  A.nchunks = (uint32_t)((Q->n + A.cq - 1) / A.cq);
  int rc = 0;
  // the reader cache of the reference can hold many rows on nested inputs: grow the
  // per-chunk state capacity until it fits (bounded by device memory)
  for (A.cap = CAP0;; A.cap *= 4) {
    bool ovf = false;
    rc = closest_pass(c, A, &ovf);
    if (rc || !ovf) break;
    if (3ull * 4ull * A.cap * A.nchunks * 4 > (64ull << 30)) {
      rc = bg_fail(c, BG_E_UNSUPPORTED, "closest-features: reader cache too deep for device memory");
      break;
    }
  }
  if (rc) { bg_result_free(r); return rc; }
  *out = r;
  return 0;
}
