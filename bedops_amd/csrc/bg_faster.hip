// bg_faster.hip — bedmap --faster: the sweep run with the criterion itself.
//
// Reference: with --faster, selectSweep (applications/bed/bedmap/src/Bedmap.cpp:728-745)
// calls the sweep with the criterion's distance dt instead of Overlapping(0) and the visitors
// derive from plain Visitor instead of BedBaseVisitor (SelectBase<true>, :579-583), so there is
// no fixWindow re-test: a reference row's window is exactly the sweep's deque.
//   two files, WindowSweep::sweep overload 2 (interfaces/src/algorithm/sweep/
//   WindowSweepImpl.cpp:168-256): per reference row r, pop the deque front while
//   dt.Map2Ref(front, r) < 0, then read map rows: dt.Ref2Map(r, m) == 0 joins the deque,
//   < 0 is cached (reading stops), > 0 is deleted unseen;
//   one file, overload 1 (:66-162; the Overlapping specialisation WindowSweepImpl.specialize.cpp
//   :40-138 hides rows shorter than the required overlap from the visitors): row i is the
//   reference when it is win[index]; the front is popped while Map2Ref(front, row i) < 0,
//   rows are read while Ref2Map(row i, b) == 0, and a reference past the deque's end
//   restarts the deque at the next unread row.
// Both loops decompose into two chains of one integer each:
//   phase 1, the read position after row i:  p_i = read_i(p_{i-1})  (reads never look at the
//            deque); a map row is decided by the first row i with p_i > m and joins the deque
//            iff Ref2Map(r_i, m) == 0 (phase 2, k_fs_added: zin[m] = i, else never);
//   phase 3, the front after row i's pops:   f_i = pop_i(f_{i-1}), over the rows that joined.
// Reference row i's window is then { m in [f_i, p_i) : m joined } (wlo = f, whi = p, zin), the
// form bg_map's kernels and the formatter already take for the zero-length replay.
// Each chain runs like bg_closest.hip's reader state: chunks of CQ rows, one thread each;
// chunk k > 0 starts CW rows early from a guess (the first map row the earlier rows could not
// have consumed / popped), records the state it reaches at its first own row, and is exact
// iff that equals chunk k-1's final state (induction from chunk 0, k_fs_check); the others
// re-run from their predecessor's state (k_fs_fix) and, after FS_ROUNDS, one in-order pass
// (k_fs_serial) makes every chunk exact. On inputs without nested rows (what --faster is
// documented for, docs/content/reference/set-operations/nested-elements.rst:62) the guesses
// hold at every chunk.
#include <climits>
#include <cstring>

#include "bg_internal.h"

#define FS_CQ 32
#define FS_CW 8
#define FS_BACK 4096  // a guessed front is at most this many rows before the read position
#define FS_ROUNDS 8

struct FsArgs {
  const int64_t* RS;
  const int64_t* RE;
  uint64_t nr;
  const int64_t* MS;  // map rows (single file: the same table as RS/RE)
  const int64_t* ME;
  uint64_t nm;
  int crit;
  int64_t ovr, range;
  double perc;
  int64_t L;           // longest map row
  const uint64_t* p;   // phase 3: the read position after each reference row (phase 1)
  const int64_t* zin;  // phase 3, two files: joined rows (zin != INT64_MAX)
  uint64_t* out;       // the chain's value after each reference row
  uint64_t* s0;        // per chunk: the state its first own row starts from
  uint64_t* s1;        // per chunk: the state after its last row
  uint32_t cq, cw, nchunks;
  uint32_t* flag;
  uint32_t* nflag;
};

// one reference row of the chain: y = the state before row i, returns the state after it
template <int PH, bool SINGLE>
__device__ __forceinline__ uint64_t fs_step(const FsArgs& A, uint64_t i, uint64_t y) {
  const int64_t rs = A.RS[i], re = A.RE[i];
  if (PH == 1) {
    uint64_t x = y;
    if (SINGLE) {  // a row past the deque's end restarts it: row i is read unconditionally
      if (x <= i) x = i + 1;
      while (x < A.nm && bg_fs_r2m(A.crit, A.ovr, A.range, A.perc, rs, re, A.MS[x], A.ME[x]) == 0) ++x;
    } else {
      while (x < A.nm && bg_fs_r2m(A.crit, A.ovr, A.range, A.perc, rs, re, A.MS[x], A.ME[x]) >= 0) ++x;
    }
    return x;
  }
  if (SINGLE) {
    const uint64_t fp = i ? A.p[i - 1] : 0;
    if (fp <= i) return i;  // the deque restarts at row i
    uint64_t f = y;  // pops stop at row i at the latest (Map2Ref(row, row) is never < 0)
    while (f < i && bg_fs_m2r(A.crit, A.ovr, A.range, A.perc, A.MS[f], A.ME[f], rs, re) < 0) ++f;
    return f;
  }
  const uint64_t pm = i ? A.p[i - 1] : 0;  // rows below pm were read by earlier rows
  uint64_t f = y;
  while (f < pm) {
    if (A.zin[f] != INT64_MAX && bg_fs_m2r(A.crit, A.ovr, A.range, A.perc, A.MS[f], A.ME[f], rs, re) >= 0)
      break;
    ++f;  // popped, or never joined
  }
  return f;
}

// the guessed state before row q (chunk warm-up starts). Phase 1: every map row starting
// before r_q.start has Ref2Map(r_q, m) >= 0 under each criterion, so any read position at
// or below the first row starting at r_q.start gives the same step. Phase 3: rows that end
// (plus the range) before r_q.start are poppable at r_q; the front is guessed at the first
// row that can still be in the deque, at most FS_BACK rows before the read position.
template <int PH, bool SINGLE>
__device__ __forceinline__ uint64_t fs_guess(const FsArgs& A, uint64_t q) {
  const int64_t rs = A.RS[q];
  if (PH == 1) return SINGLE ? q : lower_bound_i64(A.MS, A.nm, rs);
  const uint64_t pm = q ? A.p[q - 1] : 0;
  const uint64_t hi = SINGLE ? q : pm;
  uint64_t g = lower_bound_i64(A.MS, A.nm, rs - A.L - A.range - 1);
  if (hi > FS_BACK && g < hi - FS_BACK) g = hi - FS_BACK;
  return g < hi ? g : hi;
}

template <int PH, bool SINGLE>
__device__ __forceinline__ void fs_own(const FsArgs& A, uint32_t k, uint64_t y) {
  const uint64_t q0 = (uint64_t)k * A.cq, q1 = min(q0 + A.cq, A.nr);
  A.s0[k] = y;
  for (uint64_t i = q0; i < q1; ++i) {
    y = fs_step<PH, SINGLE>(A, i, y);
    A.out[i] = y;
  }
  A.s1[k] = y;
}

template <int PH, bool SINGLE>
__global__ void __launch_bounds__(BG_NT) k_fs_chunks(FsArgs A) {
  const uint32_t k = blockIdx.x * BG_NT + threadIdx.x;
  if (k >= A.nchunks) return;
  uint64_t y = 0;
  if (k > 0) {
    const uint64_t q0 = (uint64_t)k * A.cq, qw = q0 - A.cw;
    y = fs_guess<PH, SINGLE>(A, qw);
    for (uint64_t i = qw; i < q0; ++i) y = fs_step<PH, SINGLE>(A, i, y);
  }
  fs_own<PH, SINGLE>(A, k, y);
}

__global__ void k_fs_check(FsArgs A) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= A.nchunks) return;
  const bool bad = k > 0 && A.s0[k] != A.s1[k - 1];
  A.flag[k] = bad;
  if (bad) atomicAdd(A.nflag, 1u);
}

// re-run the chunks whose predecessor's final state is stable this round
template <int PH, bool SINGLE>
__global__ void __launch_bounds__(BG_NT) k_fs_fix(FsArgs A) {
  const uint32_t k = blockIdx.x * BG_NT + threadIdx.x;
  if (k == 0 || k >= A.nchunks || !A.flag[k] || A.flag[k - 1]) return;
  fs_own<PH, SINGLE>(A, k, A.s1[k - 1]);
}

// last resort: one in-order pass over the chunks (exact for any input)
template <int PH, bool SINGLE>
__global__ void k_fs_serial(FsArgs A) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  for (uint32_t k = 1; k < A.nchunks; ++k)
    if (A.s0[k] != A.s1[k - 1]) fs_own<PH, SINGLE>(A, k, A.s1[k - 1]);
}

// phase 2: which map rows join the deque (zin = the reference row they join at, else never)
// and, one file, which rows the visitors see at all (the Overlapping specialisation hides
// rows shorter than the required overlap); zout: no row leaves other than through the front
// range [f_i, p_i)
template <bool SINGLE>
__global__ void k_fs_added(FsArgs A, int64_t* __restrict__ zin, int64_t* __restrict__ zout) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= A.nm) return;
  const int64_t ms = A.MS[m], me = A.ME[m];
  bool in;
  int64_t at = 0;
  if (SINGLE) {
    in = A.crit != BG_OVR_BP || me - ms >= A.ovr;
  } else {
    const uint64_t i = upper_bound_i64((const int64_t*)A.out, A.nr, (int64_t)m);
    in = i < A.nr && bg_fs_r2m(A.crit, A.ovr, A.range, A.perc, A.RS[i], A.RE[i], ms, me) == 0;
    at = (int64_t)i;
  }
  zin[m] = in ? at : INT64_MAX;
  zout[m] = INT64_MAX;
}

template <int PH, bool SINGLE>
static int fs_chain(bg_ctx* c, FsArgs& A) {
  int rc = bg_hip_ok(c, hipMemsetAsync(A.nflag, 0, 8, c->stream));
  if (rc) return rc;
  BG_LAUNCH(c, "k_fs_chunks", (k_fs_chunks<PH, SINGLE>), dim3(bg_blocks(A.nchunks, BG_NT)), dim3(BG_NT), A);
  if ((rc = bg_hip_ok(c, hipGetLastError()))) return rc;
  for (int round = 0;; ++round) {
    uint64_t h = 0;  // (the counter is the low word of an 8-byte slot)
    if ((rc = bg_hip_ok(c, hipMemsetAsync(A.nflag, 0, 8, c->stream)))) return rc;
    BG_LAUNCH(c, "k_fs_check", k_fs_check, dim3(bg_blocks(A.nchunks, 256)), dim3(256), A);
    if ((rc = bg_fetch_u64(c, (const uint64_t*)A.nflag, &h))) return rc;
    if (h == 0) return 0;
    if (round == FS_ROUNDS) {
      BG_LAUNCH(c, "k_fs_serial", (k_fs_serial<PH, SINGLE>), dim3(1), dim3(64), A);
      return bg_hip_ok(c, hipGetLastError());
    }
    BG_LAUNCH(c, "k_fs_fix", (k_fs_fix<PH, SINGLE>), dim3(bg_blocks(A.nchunks, BG_NT)), dim3(BG_NT), A);
    if ((rc = bg_hip_ok(c, hipGetLastError()))) return rc;
  }
}

// bedmap --faster windows of every reference row of R over M (M == R: one file):
// wlo = f_i, whi = p_i, zin / zout as bg_map_live reads them (all device, R->n / M->n long)
int bg_faster_windows(bg_ctx* c, const bg_table* R, const bg_table* M, int crit, int64_t ovr, int64_t range,
                      double perc, bool single, uint64_t* wlo, uint64_t* whi, int64_t* zin, int64_t* zout) {
  const uint64_t nr = R->n, nm = M->n;
  if (!nr) return 0;
  FsArgs A;
  memset(&A, 0, sizeof(A));
  A.RS = R->ks;
  A.RE = R->ke;
  A.nr = nr;
  A.MS = M->ks;
  A.ME = M->ke;
  A.nm = nm;
  A.crit = crit;
  A.ovr = ovr;
  A.range = crit == BG_OVR_RANGE ? range : 0;
  A.perc = perc;
  A.L = M->maxlen > 0 ? M->maxlen : 1;
  A.cq = FS_CQ;
  A.cw = FS_CW;
  A.nchunks = (uint32_t)((nr + A.cq - 1) / A.cq);
  A.s0 = (uint64_t*)bg_alloc(c, 8ull * A.nchunks);
  A.s1 = (uint64_t*)bg_alloc(c, 8ull * A.nchunks);
  A.flag = (uint32_t*)bg_alloc(c, 4ull * A.nchunks + 16);
  A.nflag = A.flag + ((A.nchunks + 1) & ~1u);  // 8-byte aligned
  int rc = (!A.s0 || !A.s1 || !A.flag) ? BG_E_NOMEM : 0;
  if (!rc) {  // phase 1: the read positions (whi)
    A.out = whi;
    rc = single ? fs_chain<1, true>(c, A) : fs_chain<1, false>(c, A);
  }
  if (!rc && nm) {  // phase 2: rows that join the deque
    if (single) BG_LAUNCH(c, "k_fs_added", k_fs_added<true>, dim3(bg_blocks(nm, BG_NT)), dim3(BG_NT), A, zin, zout);
    else BG_LAUNCH(c, "k_fs_added", k_fs_added<false>, dim3(bg_blocks(nm, BG_NT)), dim3(BG_NT), A, zin, zout);
    rc = bg_hip_ok(c, hipGetLastError());
  }
  if (!rc) {  // phase 3: the fronts (wlo)
    A.p = whi;
    A.zin = zin;
    A.out = wlo;
    rc = single ? fs_chain<3, true>(c, A) : fs_chain<3, false>(c, A);
  }
  bg_release(c, A.s0);
  bg_release(c, A.s1);
  bg_release(c, A.flag);
  return rc;
}
