// bg_internal.h — shared internals of libbedgpu (host structs + gfx950 device helpers).
//
// Data layout in HBM: every parsed input is two int64 SoA columns
//   ks[i] = (chrom_id << 40) | start_i,   ke[i] = (chrom_id << 40) | end_i
// with chrom_id the rank of the chromosome name in strcmp order over the union of
// the inputs (the order every reference comparator uses: BedCompare.hpp:42-43).
// Coordinates are <= 999,999,999,999 < 2^40 (BEDOPS.Constants.hpp:36), so keyed
// intervals of different chromosomes never overlap or touch, and a whole
// multi-chromosome file is ONE sorted array: every sweep is a single global
// scan / merge-path pass with no per-chromosome segmentation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <unordered_map>
#include <thread>
#include <vector>

#include "../../include/bedgpu.h"

#define BG_KEY_SHIFT 40
#define BG_COORD_MASK ((1LL << BG_KEY_SHIFT) - 1)
#define BG_MAX_COORD 999999999999ULL
// the largest coordinate a keyed row holds: without --ec the reference reads any %lu
// (Bed.hpp:244-255) and prints it back, so coordinates above MAX_COORD_VALUE
// (BEDOPS.Constants.hpp:36) but below 2^40 are kept (only --ec rejects them, bg_check)
#define BG_KEY_COORD_MAX ((1ULL << BG_KEY_SHIFT) - 1)
#define BG_CHR_MAX 127

// ---------------------------------------------------------------------------------
// device status word: first error as (row << 8 | code), run-record counters
// ---------------------------------------------------------------------------------
struct bg_dstatus {
  unsigned long long first_bad;  // min over errors of (row << 8) | code; ~0 if none
  unsigned long long nruns;      // chromosome-run records appended by the parser
  unsigned long long nblank;     // blank lines seen
  unsigned long long flags;      // bit0: non-integer score, bit1: zero-length row, bit2: |sum|>=2^53
  long long maxlen;              // max (end - start) seen (bedmap window)
  unsigned long long stop_row;   // bedmap: first row where the reference throws (~0: none)
  unsigned long long pad[2];
  unsigned long long nbig;       // BED5 scores left to the exact big-number conversion (k_score_big)
};

// bedmap: map rows longer than thr, by length class (see bg_map_cands below)
#define BG_LONG_MAXC 30
struct LongRows {
  const uint64_t* idx;   // long rows' map indices, grouped by class, index order inside
  const int64_t* ls;     // their starts
  const uint64_t* coff;  // class c = [coff[c], coff[c + 1])
  int ncls;              // 0: no long rows (one range is exact)
  int64_t thr;
};

// bg_dstatus.flags bit: a formatter row rendered to another length than its count pass
// measured (its inputs changed between the passes); the result is refused, not written
#define BG_FMT_MISMATCH 64ULL

enum { ERR_PARSE = 1, ERR_CHROM = 2, ERR_RANGE = 3, ERR_UNSORTED = 4, ERR_BLANK = 5, ERR_SCORE = 6 };

// ---------------------------------------------------------------------------------
// host-side objects
// ---------------------------------------------------------------------------------
struct bg_buf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct bg_ctx {
  int device = 0;
  bool row_wide = false;  // bg_load: rows parsed by k_parse (a redo after BG_ROW_OVERFLOW)
  uint64_t big_need = 0;   // bg_load: capacity of the k_score_big list (a redo after it overflowed)
  uint64_t out_skip = 0;  // bytes write_device_ring still drops (bg_set_output_skip)
  int ncu = 256;  // compute units
  std::vector<std::pair<const void*, uint32_t>> resident;  // kernel -> resident BG_NT blocks
  // pinned host staging for the loader's small copies (async DMA, no bounce buffer):
  // chunks are kept for the context's lifetime, handed out by a bump pointer reset per call
  std::vector<std::pair<char*, size_t>> pin_chunks;
  size_t pin_chunk = 0, pin_used = 0;
  // staging ring for bulk host<->device copies (bg_ring_get): driver-allocated pinned slots,
  // so no user-pointer pages the kernel driver could invalidate under running kernels
  std::vector<char*> ring;
  char* ring_base = nullptr;  // the H2D slots' one allocation (ring[0 .. BG_RING_SLOTS) point into it)
  std::vector<hipEvent_t> ring_ev;
  std::thread ring_th;  // bg_open starts pinning the ring; its first use joins
  int ring_rc = 0;
  struct bg_pool* pool = nullptr;  // the ring's copy threads (bg_api.hip)
  hipStream_t pstream = nullptr;  // prefetch copies (bg_file_image_copy), fenced by slot events
  std::vector<hipEvent_t> copy_ev;  // bg_file_image_copy slots
  std::vector<hipEvent_t> order_ev;  // bg_copy_order: ctx's stream position a slot's copies wait for
  std::vector<char> order_set;
  std::mutex copy_mu;  // (also guards err_async)
  // errors raised on another host thread (the read-ahead copier, bg_file_image_copy) land in
  // err_async under copy_mu and move to err when bg_last_error is read on the owner's side;
  // only the thread that launches work may call bg_alloc / bg_release
  std::thread::id owner;
  std::string err_async;
  hipStream_t stream = nullptr;
  // side stream: a set input's post-parse passes (bg_load.hip) run there beside the next
  // input's parse; blocks released while it is in use wait in `deferred` until the join
  hipStream_t sstream = nullptr;
  hipEvent_t sfork = nullptr, sjoin = nullptr;
  bool defer_release = false;
  std::vector<bg_buf> deferred;
  std::string err;
  bg_dstatus* dstat = nullptr;  // device
  void* warm = nullptr;         // device scratch of the ring's warm-up copy
  bg_dstatus* hstat = nullptr;  // pinned host mirror
  // caching allocator: free blocks by size; live blocks -> their size (per context, so
  // contexts on different devices can be driven from different host threads)
  std::vector<bg_buf> free_list;
  std::unordered_map<void*, size_t> live;
  // stage timing
  bool stats = false;
  std::vector<std::pair<std::string, hipEvent_t>> marks;
  std::string stats_text;
  // kernel profiling
  std::string prof_filter;  // "" off, "*" all, else exact kernel name
  struct Pend { std::string name; hipEvent_t a, b; };
  std::vector<Pend> prof_pending;
  std::vector<hipEvent_t> prof_events;  // recycled
  struct KStat { double ms = 0; uint64_t calls = 0; };
  std::vector<std::pair<std::string, KStat>> prof;
};

struct bg_table {
  uint64_t n = 0;
  int kind = BG_BED3;
  int64_t* ks = nullptr;  // keyed starts (raw coordinates until keyed)
  int64_t* ke = nullptr;  // keyed ends
  // kept for BG_BED3_REST output: text + remainder span per row
  const char* text = nullptr;  // device text
  uint64_t nbytes = 0;
  char* own_text = nullptr;  // when the library copied host text in
  uint64_t* rest_off = nullptr;
  uint32_t* rest_len = nullptr;
  double* score = nullptr;  // BG_BED5
  bool score_int = true;     // every score is an integer (exact sums)
  bool has_zero_len = false; // some row has end == start
  int64_t maxlen = 0;        // max (end - start) over the rows (window bound for sweeps)
  // BG_BED3_SET: the file's merged set only (ks/ke stay null)
  bool is_set = false;
  int64_t* cs = nullptr;
  int64_t* ce = nullptr;
  uint64_t nc = 0;
  // chromosome runs (host, sorted by row): rows [row0[k], row0[k+1]) are chrom names[k]
  std::vector<uint64_t> run_row0;
  std::vector<std::string> run_name;
};

struct bg_set {
  bg_ctx* ctx = nullptr;
  std::vector<bg_table*> t;
  std::vector<std::string> names;  // global chromosome dictionary, strcmp order
  char* d_names = nullptr;         // packed names on device
  uint32_t* d_name_off = nullptr;  // offset of name g
  uint32_t* d_name_len = nullptr;
  uint32_t max_name_len = 0;
};

enum { RES_IVL = 0, RES_ROWS = 1, RES_MAP = 2, RES_CLOSEST = 3, RES_MULTI = 4 };

struct bg_result {
  bg_ctx* ctx = nullptr;
  bg_set* set = nullptr;
  int kind = RES_IVL;
  uint64_t n = 0;
  // RES_IVL: keyed intervals
  int64_t* s = nullptr;
  int64_t* e = nullptr;
  // RES_ROWS: selected row indices of table `tab`
  // RES_MULTI (--everything): s/e per output row, rows = device address of its verbatim
  // remainder, rlen = remainder length
  uint64_t* rows = nullptr;
  uint32_t* rlen = nullptr;
  bool rest_tab = false;  // RES_MULTI: a non-empty remainder is printed after a tab (sort-bed)
  bool own_set = false;   // the result owns its set (bg_sortbed)
  int tab = -1;
  // RES_MAP: per reference row columns
  int32_t* cnt = nullptr;    // rows in S(r) (Count, Indicator, --skip-unmapped)
  int64_t* isum = nullptr;   // exact integer score sum (Average, Sum)
  double* vmin = nullptr;    // Extreme (min / max score)
  double* vmax = nullptr;
  uint64_t* bases = nullptr; // OvrAggregate
  uint32_t* uniq = nullptr;  // OvrUnique (unsigned int, as the reference)
  int64_t* isq = nullptr;    // exact integer sum of squared scores (Variance, StdDev, CV)
  double* dsum = nullptr;    // decimal scores: the reference's running sum_ at each row
  double* dsq = nullptr;     //   and squareSum_ (bg_map.hip, k_mev_*), replacing isum / isq
  double* tmv[16] = {};      // --tmean ops[q]: TrimmedMean's value at each row (k_tm_replay)
  bool single = false;       // single-file mode (ref == map table)
  uint64_t* rrank = nullptr; // --echo-ref-row-id with --skip-unmapped: printed lines before row r
  uint64_t* wlo = nullptr;   // --echo-map*: candidate range [wlo, whi) of map rows per ref row
  uint64_t* whi = nullptr;
  LongRows lrows = {nullptr, nullptr, nullptr, 0, 0};  // bedmap: long map rows by class (owned)
  // zero-length rows in a bedmap input: map row m is in the sweep window of reference rows
  // [zin[m], zout[m]) only (bg_map.hip, k_mz_member); null otherwise
  int64_t* zin = nullptr;
  int64_t* zout = nullptr;
  // map row -> simulated heap address of the reference's row object, the tie-break of its
  // address-ordered sets (bg_heap.hip); null: row order (no tie an operation can see)
  int64_t* maddr = nullptr;
  int map_tab = -1;          // the map table
  int mapfields = 3;         // map row type printed by --echo-map (B3Rest / B4Rest / B5Rest)
  double perc = 1.0;         // PercentOverlapMapping::perc_ of the criterion
  bg_map_opts mopts;
  // RES_CLOSEST: per row of table `tab`, the chosen rows of table `tab2` (-1: NA)
  int64_t* left = nullptr;
  int64_t* right = nullptr;
  int tab2 = -1;
  bg_closest_opts copts;
  // rendered text
  char* text = nullptr;
  uint64_t nbytes = 0;
  bool formatted = false;
  bool stopped = false;      // the text ends where the reference throws (BG_E_VISITOR)
  uint64_t* toff = nullptr;  // byte offset of each 1024-row format tile (kept for spans)
  // RES_ROWS from bg_element_of: printed bytes of every BG_FMT_TILE-row format tile, summed
  // while the rows were compacted (the formatter's count pass, done already); null: count
  uint64_t* tbytes = nullptr;
  // RES_IVL straight from a merge-path tile kernel: s/e are SEGMENTED, segment t's pieces at
  // [t * BG_SEG_CAP, t * BG_SEG_CAP + seg_off[t+1] - seg_off[t]); seg_off / seg_boff are the
  // exclusive scans of the pieces and printed bytes per segment (nseg + 1 entries). The
  // formatter reads this layout directly; bg_result_compact makes s/e contiguous
  uint64_t nseg = 0;
  uint64_t* seg_off = nullptr;
  uint64_t* seg_boff = nullptr;
  uint64_t seg_nz = 0;     // pieces the segments can hold (the merged elements)
  bool n_pending = false;  // n is still only on the device (seg_off[nseg]): bg_result_resolve_n
};
// n of a segmented result fetched from the device when still pending
int bg_result_resolve_n(bg_ctx* c, bg_result* r);
// rows per format tile (bg_format.hip FT_TILE)
#define BG_FMT_TILE 512
// pieces per segment of a segmented RES_IVL (= the merge-path tile, bg_setops.hip)
#define BG_SEG_CAP 1024
// s/e of a segmented RES_IVL result made contiguous (no-op otherwise)
int bg_result_compact(bg_ctx* c, bg_result* r);

// workgroups of BG_NT threads of `kern` resident on the whole device at once (persistent
// grid size; occupancy query x compute units, cached per kernel)
uint32_t bg_resident_blocks(bg_ctx* c, const void* kern);

// pinned host scratch valid until the next bg_pin_reset (the caller syncs before reading
// device-to-host results); nullptr if pinned memory cannot be had
void bg_pin_reset(bg_ctx* c);
void* bg_pin_take(bg_ctx* c, size_t bytes);

// allocator / error helpers (bg_api.cpp)
void* bg_alloc(bg_ctx* c, size_t bytes);
void bg_release(bg_ctx* c, void* p);
// device blocks released to the context's pool on every exit path of a host function
struct BgHold {
  bg_ctx* c;
  std::vector<void*> p;
  explicit BgHold(bg_ctx* cc) : c(cc) {}
  template <class T>
  T* operator()(T* q) {
    p.push_back((void*)q);
    return q;
  }
  ~BgHold() {
    for (void* q : p) bg_release(c, q);
  }
};
int bg_fail(bg_ctx* c, int code, const std::string& msg);
int bg_hip_fail(bg_ctx* c, hipError_t e, const char* what);
void bg_mark(bg_ctx* c, const char* name);

// kernel profiling (bg_prof_enable): HIP events on the context stream around launches
// whose name matches the filter ("*" = all)
bool bg_prof_on(bg_ctx* c, const char* name);
void bg_prof_push(bg_ctx* c, const char* name, hipEvent_t a, hipEvent_t b);
hipEvent_t bg_prof_event(bg_ctx* c);

#define BG_LAUNCH(c, name, kern, grid, block, ...)                           \
  do {                                                                       \
    const bool _p = bg_prof_on((c), (name));                                 \
    hipEvent_t _a = nullptr, _b = nullptr;                                   \
    if (_p) { _a = bg_prof_event(c); hipEventRecord(_a, (c)->stream); }      \
    hipLaunchKernelGGL(kern, grid, block, 0, (c)->stream, __VA_ARGS__);      \
    if (_p) { _b = bg_prof_event(c); hipEventRecord(_b, (c)->stream);        \
              bg_prof_push((c), (name), _a, _b); }                           \
  } while (0)

#define BG_HIP(c, expr)                                  \
  do {                                                   \
    hipError_t _e = (expr);                              \
    if (_e != hipSuccess) return bg_hip_fail((c), _e, #expr); \
  } while (0)

// device-wide helpers (bg_scan.hip)
// exclusive prefix sum of n uint64 values (in may alias out); *total (device ptr,
// optional) receives the sum.
int bg_scan_sum_u64(bg_ctx* c, const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* d_total);
// exclusive prefix max of n int64 values with identity `init`
int bg_scan_max_i64(bg_ctx* c, const int64_t* in, int64_t* out, uint64_t n, int64_t init);
// copy one device uint64 to host (synchronises the stream)
int bg_fetch_u64(bg_ctx* c, const uint64_t* d, uint64_t* h);

// ---------------------------------------------------------------------------------
// keyed interval lists and the shared sweep building blocks (bg_setops.hip)
// ---------------------------------------------------------------------------------
struct Ivl {
  int64_t* s = nullptr;
  int64_t* e = nullptr;
  uint64_t n = 0;
  bool owned = false;
  // segmented layout (bg_result::nseg); owned with s/e
  uint64_t nseg = 0;
  uint64_t* seg_off = nullptr;
  uint64_t* seg_boff = nullptr;
  uint64_t seg_nz = 0;
  bool n_pending = false;
};
void ivl_free(bg_ctx* c, Ivl& v);
int ivl_alloc(bg_ctx* c, Ivl& v, uint64_t n);
Ivl bg_table_ivl(bg_table* T);
// the components of one table: a view of a BG_BED3_SET table's set, computed otherwise
int bg_table_components(bg_ctx* c, bg_table* T, Ivl& out);
// BG_E_ARG unless every listed table keeps its rows (not BG_BED3_SET)
int bg_need_rows(bg_ctx* c, bg_set* set, const int* files, int nf, const char* what);
// components (maximal touching-merged pieces) of one start-sorted list / of a union
int bg_components(bg_ctx* c, const Ivl& in, Ivl& out);
int bg_union_components(bg_ctx* c, bg_set* set, const int* files, int nf, Ivl& out);
bg_result* bg_new_ivl_result(bg_ctx* c, bg_set* set, Ivl& v);
int bg_check_files(bg_ctx* c, bg_set* set, const int* files, int nf, int minf);
int bg_compact_flags(bg_ctx* c, const uint8_t* flag, uint64_t n, uint64_t** rows, uint64_t* total);
// full_rest() of each listed map row copied to the host: row i's bytes are txt[off[i], off[i+1])
// (bg_heap.hip); strcmp order of two such byte strings
int bg_frest_gather(bg_ctx* c, const bg_table* M, int fields, const std::vector<uint64_t>& rows,
                    std::vector<char>& txt, std::vector<uint64_t>& off);
static inline bool bg_bytes_less(const char* a, uint64_t la, const char* b, uint64_t lb) {
  const int cmp = memcmp(a, b, la < lb ? la : lb);
  return cmp ? cmp < 0 : la < lb;
}
// stable ascending radix sort of uint64 keys with an optional uint32 payload (bg_sort.hip)
int bg_sort_u64(bg_ctx* c, uint64_t* keys, uint32_t* vals, uint64_t n);

// count pass -> scan -> allocate exact output -> write pass
template <typename CountFn, typename WriteFn>
static int count_scan_write(bg_ctx* c, unsigned nb, CountFn cf, WriteFn wf, uint64_t* total) {
  uint64_t* cnt = (uint64_t*)bg_alloc(c, 8ull * (nb ? nb : 1));
  uint64_t* d_tot = (uint64_t*)bg_alloc(c, 8);
  if (!cnt || !d_tot) return BG_E_NOMEM;
  if (nb) {
    cf(cnt);
    BG_HIP(c, hipGetLastError());
  }
  int rc = bg_scan_sum_u64(c, cnt, cnt, nb, d_tot);
  if (rc) return rc;
  if ((rc = bg_fetch_u64(c, d_tot, total))) return rc;
  bg_release(c, d_tot);
  if ((rc = wf(cnt, *total))) return rc;
  BG_HIP(c, hipGetLastError());
  bg_release(c, cnt);
  return 0;
}

// ---------------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------------
#define BG_NT 256  // threads per workgroup (4 waves of 64)

__device__ __forceinline__ int bg_lane() { return threadIdx.x & 63; }

// decimal digits of v: compares only, 32-bit ones when v fits (the common case)
__device__ __forceinline__ int dec_len_u64(uint64_t v) {
  if ((v >> 32) == 0) {
    const uint32_t w = (uint32_t)v;
    return 1 + (w >= 10u) + (w >= 100u) + (w >= 1000u) + (w >= 10000u) + (w >= 100000u) +
           (w >= 1000000u) + (w >= 10000000u) + (w >= 100000000u) + (w >= 1000000000u);
  }
  int l = 10;  // v >= 2^32 > 10^9
  uint64_t p = 10000000000ull;
#pragma unroll
  for (int k = 0; k < 10; ++k, p *= 10) l += v >= p;
  return l;
}
// printed bytes of an interval line "%s\t%lu\t%lu\n" (keys: chrom << BG_KEY_SHIFT | coord)
__device__ __forceinline__ uint32_t bg_ivl_len(const uint32_t* name_len, int64_t s, int64_t e) {
  const uint32_t g = (uint32_t)(s >> BG_KEY_SHIFT);
  return name_len[g] + 3u + (uint32_t)dec_len_u64((uint64_t)(s & BG_COORD_MASK)) +
         (uint32_t)dec_len_u64((uint64_t)(e & BG_COORD_MASK));
}
__device__ __forceinline__ int bg_wave() { return threadIdx.x >> 6; }

// inclusive wave (64-lane) scan
template <typename T, typename Op>
__device__ __forceinline__ T wave_incl_scan(T v, Op op) {
  const int lane = bg_lane();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    T u = __shfl_up(v, d, 64);
    if (lane >= d) v = op(v, u);
  }
  return v;
}

struct OpSum {
  template <typename T>
  __device__ __forceinline__ T operator()(T a, T b) const { return a + b; }
};
struct OpMax {
  template <typename T>
  __device__ __forceinline__ T operator()(T a, T b) const { return a > b ? a : b; }
};
struct OpMin {
  template <typename T>
  __device__ __forceinline__ T operator()(T a, T b) const { return a < b ? a : b; }
};

// DPP form of the most common scan (u32 sums: line starts, counts): row_shr 1/2/4/8 within
// 16-lane rows, row_bcast 15/31 across them; lanes with no source read 0
template <int CTRL, int RMASK, bool BC>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RMASK, 0xF, BC);
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, OpSum) {
  v += dpp32<0x111, 0xF, true>(v);
  v += dpp32<0x112, 0xF, true>(v);
  v += dpp32<0x114, 0xF, true>(v);
  v += dpp32<0x118, 0xF, true>(v);
  v += dpp32<0x142, 0xA, false>(v);
  v += dpp32<0x143, 0xC, false>(v);
  return v;
}

static inline int bg_hip_ok(bg_ctx* c, hipError_t e) {
  return e == hipSuccess ? 0 : bg_hip_fail(c, e, "HIP runtime call");
}

// Block (BG_NT threads) exclusive scan. `sh` must hold BG_NT/64 + 1 elements.
// Returns the exclusive prefix of this thread; *total gets the block aggregate.
template <typename T, typename Op>
__device__ __forceinline__ T block_excl_scan(T v, Op op, T identity, T* sh, T* total) {
  const int lane = bg_lane(), w = bg_wave();
  T inc = wave_incl_scan(v, op);
  if (lane == 63) sh[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    T run = identity;
#pragma unroll
    for (int i = 0; i < BG_NT / 64; ++i) {
      T x = sh[i];
      sh[i] = run;
      run = op(run, x);
    }
    sh[BG_NT / 64] = run;
  }
  __syncthreads();
  T wpre = sh[w];
  T excl = __shfl_up(inc, 1, 64);
  excl = (lane == 0) ? wpre : op(wpre, excl);
  *total = sh[BG_NT / 64];
  __syncthreads();  // sh may be reused by the caller
  return excl;
}

__device__ __forceinline__ bool bg_isws(uint8_t c) {
  // C-locale isspace minus '\n' (lines are split on '\n' first)
  return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f';
}

// number of elements of X among the first d of merge(X, Y) when X[i] goes first
// only if X[i] < Y[j] strictly (ties: Y first). X, Y sorted ascending.
__device__ __forceinline__ uint64_t merge_path_ystrict(const int64_t* X, uint64_t nx,
                                                       const int64_t* Y, uint64_t ny,
                                                       uint64_t d) {
  uint64_t lo = d > ny ? d - ny : 0, hi = d < nx ? d : nx;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (X[mid] < Y[d - 1 - mid]) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// same with X first on ties (X[i] <= Y[j])
__device__ __forceinline__ uint64_t merge_path_xfirst(const int64_t* X, uint64_t nx,
                                                      const int64_t* Y, uint64_t ny,
                                                      uint64_t d) {
  uint64_t lo = d > ny ? d - ny : 0, hi = d < nx ? d : nx;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (X[mid] <= Y[d - 1 - mid]) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// bedmap: is map row [ms, me) in S(r) of reference row [s, e)? (keys of one chromosome;
// criteria of data/bed/BedDistances.hpp, see bg_map.hip). Rows outside the sweep's
// Overlapping(0) window never are, except under --range (RangedDist sweeps too).
// BG_OVR_FAST (internal, never in bg_map_opts): bedmap --faster windows, whose members are
// the sweep's own deque (bg_faster.hip); every candidate in the window range is a member
// once bg_map_live has said it is in the deque
#define BG_OVR_FAST 99
__host__ __device__ __forceinline__ bool bg_map_in(int crit, int64_t ovr, int64_t range, double perc,
                                                   int64_t s, int64_t e, int64_t ms, int64_t me) {
  if (crit == BG_OVR_FAST) return true;
  if (crit == BG_OVR_RANGE) return (s < me) ? (e + range > ms) : (me + range > s);
  // Exact (:300-309) compares coordinates only: a zero-length row matches its equal (it can
  // be a window member only in one-file mode, where the row itself is in the deque)
  if (crit == BG_OVR_EXACT) return ms == s && me == e;
  // perc_ <= DBL_EPSILON: PercentOverlapMapping::Ref2Map is 0 for every pair not strictly
  // apart (:147-150), rows that only touch or have no length included (each fraction
  // variant reduces to that test then)
  if (crit != BG_OVR_BP && perc <= 2.220446049250313e-16) return !(e < ms || me < s);
  const int64_t ov = (e < me ? e : me) - (s > ms ? s : ms);
  if (ov <= 0) return false;
  if (crit == BG_OVR_BP) return ov >= ovr;
  // sz of BedDistances.hpp:160-174 is the overlap length for overlapping rows
  const bool fm = (double)ov / (double)(me - ms) >= perc;  // relative to the map row
  const bool fr = (double)ov / (double)(e - s) >= perc;    // relative to the ref row
  if (crit == BG_OVR_FRAC_MAP) return fm;
  if (crit == BG_OVR_FRAC_REF) return fr;
  if (crit == BG_OVR_FRAC_EITHER) return fm || fr;
  return fm && fr;
}

// bedmap --faster: the distance the sweep itself runs with is the criterion's (Bedmap.cpp:
// 287-290, 728-745; no BedBaseVisitor re-test). Ref2Map(a = reference row, b = map row) and
// Map2Ref(b, a) of data/bed/BedDistances.hpp, on keyed rows (chromosome ids are in strcmp
// order, so comparing keys compares chromosomes first):
//   Overlapping(ovr)  operator() :97-115, both directions the same function;
//   RangedDist(R)     operator() :57-64;
//   PercentOverlapBoth Ref2Map :262-272 over PercentOverlapMapping::Ref2Map :141-180 (the
//                     reference's double arithmetic), Map2Ref = -Ref2Map :278-281;
//   Exact             Ref2Map :300-309, Map2Ref = -Ref2Map :313-315.
// Overlapping's last tie (equal rows overlapping by less than ovr) compares heap addresses
// (:108-110); such a pair never satisfies the criterion, and whichever way the tie falls the
// sweep's deque ends up the same (the row is deleted now or when the next reference row
// passes it; no row it holds back could join the current window), so -1 is returned.
__host__ __device__ __forceinline__ int bg_fs_ovl(int64_t as, int64_t ae, int64_t bs, int64_t be, int64_t ovr) {
  const int64_t ca = as >> BG_KEY_SHIFT, cb = bs >> BG_KEY_SHIFT;
  if (ca != cb) return ca > cb ? 1 : -1;
  const int64_t mn = as > bs ? as : bs, mx = ae < be ? ae : be;
  if (mx > mn) {
    if (mx - mn >= ovr) return 0;
    if (as != bs) return as < bs ? -1 : 1;
    if (ae != be) return ae < be ? -1 : 1;
    return -1;
  }
  return as < bs ? -1 : 1;
}
__host__ __device__ __forceinline__ int bg_fs_ranged(int64_t as, int64_t ae, int64_t bs, int64_t be, int64_t d) {
  const int64_t ca = as >> BG_KEY_SHIFT, cb = bs >> BG_KEY_SHIFT;
  if (ca != cb) return ca > cb ? 1 : -1;
  if (as < be) return (ae + d > bs) ? 0 : -1;
  return (be + d > as) ? 0 : 1;
}
// PercentOverlapMapping::Ref2Map(ref = a, map = b)
__host__ __device__ __forceinline__ int bg_fs_pmap(int64_t as, int64_t ae, int64_t bs, int64_t be, double perc) {
  const int64_t ca = as >> BG_KEY_SHIFT, cb = bs >> BG_KEY_SHIFT;
  if (ca != cb) return ca > cb ? 1 : -1;
  if (ae < bs) return -1;
  if (be < as) return 1;
  if (perc <= 2.220446049250313e-16) return 0;
  const double tl = (double)(uint64_t)(be - bs);
  double sz;
  int dir;
  if (as <= bs) {
    sz = (double)(uint64_t)((ae >= be) ? be - bs : ae - bs);
    dir = -1;
  } else {
    sz = (double)(uint64_t)((ae >= be) ? be - as : ae - as);
    dir = 1;
  }
  return (sz / tl >= perc) ? 0 : dir;
}
__host__ __device__ __forceinline__ int bg_fs_r2m(int crit, int64_t ovr, int64_t range, double perc, int64_t rs,
                                                  int64_t re, int64_t ms, int64_t me) {
  switch (crit) {
    case BG_OVR_BP: return bg_fs_ovl(rs, re, ms, me, ovr);
    case BG_OVR_RANGE: return bg_fs_ranged(rs, re, ms, me, range);
    case BG_OVR_FRAC_BOTH: {
      const int v1 = bg_fs_pmap(rs, re, ms, me, perc);
      if (v1) return v1;
      return -bg_fs_pmap(ms, me, rs, re, perc);
    }
    default: {  // BG_OVR_EXACT
      const int64_t ca = rs >> BG_KEY_SHIFT, cb = ms >> BG_KEY_SHIFT;
      if (ca != cb) return ca < cb ? -1 : 1;
      if (rs != ms) return rs < ms ? -1 : 1;
      if (re != me) return re < me ? -1 : 1;
      return 0;
    }
  }
}
__host__ __device__ __forceinline__ int bg_fs_m2r(int crit, int64_t ovr, int64_t range, double perc, int64_t ms,
                                                  int64_t me, int64_t rs, int64_t re) {
  switch (crit) {
    case BG_OVR_BP: return bg_fs_ovl(ms, me, rs, re, ovr);
    case BG_OVR_RANGE: return bg_fs_ranged(ms, me, rs, re, range);
    default: return -bg_fs_r2m(crit, ovr, range, perc, rs, re, ms, me);
  }
}

// bedmap with zero-length rows: is map row m in reference row r's sweep window at all?
__device__ __forceinline__ bool bg_map_live(const int64_t* zin, const int64_t* zout, uint64_t r,
                                            uint64_t m) {
  return !zin || (zin[m] <= (int64_t)r && (int64_t)r < zout[m]);
}

// ---------------------------------------------------------------------------------
// bedmap candidate windows by row-length class. Map rows of length <= thr are searched in
// one start range [s - pad - thr + 1, e + pad); longer rows sit in per-class lists (class
// c: lengths in (thr << c, thr << (c + 1)]), each searched with its own bound, so one
// chromosome-length row no longer widens every reference row's window to its chromosome.
// The candidates are visited in map-row (start) order: a merge of the short range and the
// class ranges (the visitors that depend on order — bases-uniq, echo-map — see the same
// sequence as from one range).
__device__ __forceinline__ uint64_t bg_lb_range(const int64_t* A, uint64_t lo, uint64_t hi, int64_t v) {
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (A[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
template <typename F>
__device__ __forceinline__ void bg_map_cands(const int64_t* MS, const int64_t* ME, uint64_t lo, uint64_t hi,
                                             const LongRows& LR, int64_t s, int64_t e, int64_t pad, F f) {
  if (LR.ncls == 0) {  // f returns false to stop
    for (uint64_t m = lo; m < hi; ++m)
      if (!f(m)) return;
    return;
  }
  const int64_t g = s & ~BG_COORD_MASK;
  const int64_t khi = min(g + (1LL << BG_KEY_SHIFT), e + pad);
  uint64_t q[BG_LONG_MAXC], qe[BG_LONG_MAXC];
  for (int c = 0; c < LR.ncls; ++c) {
    const int64_t klo = max(g, s - pad - (LR.thr << (c + 1)) + 1);
    q[c] = bg_lb_range(LR.ls, LR.coff[c], LR.coff[c + 1], klo);
    qe[c] = bg_lb_range(LR.ls, q[c], LR.coff[c + 1], khi);
  }
  uint64_t m = lo;
  for (;;) {
    while (m < hi && ME[m] - MS[m] > LR.thr) ++m;  // long rows come from their class
    uint64_t best = m < hi ? m : ~0ULL;
    int bc = -1;
    for (int c = 0; c < LR.ncls; ++c)
      if (q[c] < qe[c] && LR.idx[q[c]] < best) { best = LR.idx[q[c]]; bc = c; }
    if (best == ~0ULL || !f(best)) break;
    if (bc < 0) ++m;
    else ++q[bc];
  }
}

// first index k in [0,n) with A[k] >= v (A sorted ascending); n if none
__device__ __forceinline__ uint64_t lower_bound_i64(const int64_t* A, uint64_t n, int64_t v) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (A[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// first index k in [lo, hi) with A[k] >= v (hi if none)
__device__ __forceinline__ uint64_t lower_bound_in(const int64_t* A, uint64_t lo, uint64_t hi,
                                                   int64_t v) {
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (A[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// first index k in [lo, hi) with A[k] > v (hi if none)
__device__ __forceinline__ uint64_t upper_bound_in(const int64_t* A, uint64_t lo, uint64_t hi,
                                                   int64_t v) {
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (A[mid] <= v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// first index k with A[k] > v
__device__ __forceinline__ uint64_t upper_bound_i64(const int64_t* A, uint64_t n, int64_t v) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (A[mid] <= v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// full_rest() of map row m (the third key of CoordRestAddressCompare, BedCompare.hpp:143-194)
// as up to two byte ranges of the resident text: B3Rest the remainder after `end`, B4Rest
// id + the remainder after it, B5Rest id + the remainder after the score (Bed.hpp:301, 537,
// 788; the score itself is not part of it)
__device__ __forceinline__ bool bg_frest_ws(char c) {
  return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f';
}
__device__ __forceinline__ void bg_frest(const char* text, const uint64_t* rest_off, const uint32_t* rest_len,
                                         int mapfields, uint64_t m, const char*& p1, uint32_t& l1,
                                         const char*& p2, uint32_t& l2) {
  const char* rp = text + rest_off[m];
  const uint32_t rl = rest_len[m];
  l2 = 0;
  p2 = rp;
  if (mapfields == 3) { p1 = rp; l1 = rl; return; }
  uint32_t i = 0;
  while (i < rl && bg_frest_ws(rp[i])) ++i;
  p1 = rp + i;
  if (mapfields == 4) { l1 = rl - i; return; }
  uint32_t j = i;
  while (j < rl && !bg_frest_ws(rp[j])) ++j;
  l1 = j - i;
  uint32_t k = j;
  while (k < rl && bg_frest_ws(rp[k])) ++k;
  while (k < rl && !bg_frest_ws(rp[k])) ++k;
  p2 = rp + k;
  l2 = rl - k;
}
// strcmp of the full_rest() strings of map rows a and b
__device__ __forceinline__ int bg_frest_cmp(const char* text, const uint64_t* rest_off, const uint32_t* rest_len,
                                            int mapfields, uint64_t a, uint64_t b) {
  const char *a1, *a2, *b1, *b2;
  uint32_t la1, la2, lb1, lb2;
  bg_frest(text, rest_off, rest_len, mapfields, a, a1, la1, a2, la2);
  bg_frest(text, rest_off, rest_len, mapfields, b, b1, lb1, b2, lb2);
  const uint32_t la = la1 + la2, lb = lb1 + lb2;
  for (uint32_t q = 0; q < la && q < lb; ++q) {
    const uint8_t x = (uint8_t)(q < la1 ? a1[q] : a2[q - la1]);
    const uint8_t y = (uint8_t)(q < lb1 ? b1[q] : b2[q - lb1]);
    if (x != y) return x < y ? -1 : 1;
  }
  return la == lb ? 0 : (la < lb ? -1 : 1);
}

__device__ __forceinline__ void bg_report(bg_dstatus* st, uint64_t row, int code) {
  atomicMin(&st->first_bad, (unsigned long long)((row << 8) | (uint64_t)code));
}

// bg_heap.hip: the reference's heap address of every map row (device array), and whether
// adjacent map rows tie on (start, end) [+ full_rest()]
// (the replayed run: the visitors' criterion and its parameters, --faster, --skip-unmapped and
// the operations in command-line order)
struct bg_heap_spec {
  int crit = 0;
  bool faster = false;
  int64_t ovr = 0, range = 0;
  double perc = 1.0;
  bool skip_unmapped = false;
  int nops = 0;
  const int* ops = nullptr;
};
int bg_heap_addr(bg_ctx* c, bg_set* set, const bg_table* R, const bg_table* M, int fields,
                 const bg_heap_spec* spec, int64_t** out);
// bedmap --faster windows (bg_faster.hip)
int bg_faster_windows(bg_ctx* c, const bg_table* R, const bg_table* M, int crit, int64_t ovr, int64_t range,
                      double perc, bool single, uint64_t* wlo, uint64_t* whi, int64_t* zin, int64_t* zout);
int bg_heap_ties(bg_ctx* c, const bg_table* M, int fields, bool rest, bool* any);
// the address of map row m (row order without a replay)
__device__ __forceinline__ int64_t bg_maddr(const int64_t* addr, uint64_t m) {
  return addr ? addr[m] : (int64_t)m;
}

static inline unsigned bg_blocks(uint64_t n, uint64_t per) { return (unsigned)((n + per - 1) / per); }
