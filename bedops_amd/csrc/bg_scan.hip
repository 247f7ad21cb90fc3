// bg_scan.hip — device-wide exclusive scans (sum / max) used between the two passes
// of every count-then-write kernel pair (reduce-then-scan; deterministic, no
// inter-workgroup hand-off inside a launch).
#include "bg_internal.h"

#ifndef SCAN_ITEMS
#define SCAN_ITEMS 4  // (16 -> 4: 4x the workgroups on the ~0.6M-entry tile arrays of the loaders)
#endif
#define SCAN_TILE (BG_NT * SCAN_ITEMS)

// (the reduction's order does not matter: striped, coalesced loads)
template <typename T, typename Op>
__global__ void __launch_bounds__(BG_NT) k_tile_reduce(const T* __restrict__ in, uint64_t n,
                                                       T* __restrict__ part, Op op, T identity) {
  __shared__ T sh[BG_NT / 64 + 1];
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + threadIdx.x;
  T acc = identity;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k)
    if (base + (uint64_t)k * BG_NT < n) acc = op(acc, in[base + (uint64_t)k * BG_NT]);
  T tot;
  (void)block_excl_scan(acc, op, identity, sh, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// exclusive scan of one tile, seeded by carry[blockIdx.x] (or identity)
template <typename T, typename Op>
__global__ void __launch_bounds__(BG_NT) k_tile_scan(const T* in, T* out, uint64_t n,
                                                     const T* __restrict__ carry, Op op,
                                                     T identity, T* d_total) {
  __shared__ T sh[BG_NT / 64 + 1];
  uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
  T v[SCAN_ITEMS];
  T acc = identity;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    v[k] = (base + k < n) ? in[base + k] : identity;
    acc = op(acc, v[k]);
  }
  T tot;
  T pre = block_excl_scan(acc, op, identity, sh, &tot);
  T c = carry ? carry[blockIdx.x] : identity;
  pre = op(c, pre);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    if (base + k < n) out[base + k] = pre;
    pre = op(pre, v[k]);
  }
  if (d_total && threadIdx.x == BG_NT - 1 && blockIdx.x == gridDim.x - 1) *d_total = pre;
}

template <typename T, typename Op>
static int scan_impl(bg_ctx* c, const T* in, T* out, uint64_t n, Op op, T identity,
                     T* d_total) {
  if (n == 0) {
    if (d_total) BG_HIP(c, hipMemsetAsync(d_total, 0, sizeof(T), c->stream));
    return 0;
  }
  unsigned nb = bg_blocks(n, SCAN_TILE);
  if (nb == 1) {
    BG_LAUNCH(c, "k_tile_scan", (k_tile_scan<T, Op>), dim3(1), dim3(BG_NT), in, out, n,
                       (const T*)nullptr, op, identity, d_total);
    BG_HIP(c, hipGetLastError());
    return 0;
  }
  T* part = (T*)bg_alloc(c, sizeof(T) * nb);
  if (!part) return BG_E_NOMEM;
  BG_LAUNCH(c, "k_tile_reduce", (k_tile_reduce<T, Op>), dim3(nb), dim3(BG_NT), in, n, part,
                     op, identity);
  BG_HIP(c, hipGetLastError());
  int rc = scan_impl<T, Op>(c, part, part, nb, op, identity, (T*)nullptr);
  if (rc) return rc;
  BG_LAUNCH(c, "k_tile_scan", (k_tile_scan<T, Op>), dim3(nb), dim3(BG_NT), in, out, n,
                     (const T*)part, op, identity, d_total);
  BG_HIP(c, hipGetLastError());
  bg_release(c, part);
  return 0;
}

int bg_scan_sum_u64(bg_ctx* c, const uint64_t* in, uint64_t* out, uint64_t n,
                    uint64_t* d_total) {
  return scan_impl<uint64_t, OpSum>(c, in, out, n, OpSum(), (uint64_t)0, d_total);
}

int bg_scan_max_i64(bg_ctx* c, const int64_t* in, int64_t* out, uint64_t n, int64_t init) {
  return scan_impl<int64_t, OpMax>(c, in, out, n, OpMax(), init, (int64_t*)nullptr);
}

int bg_fetch_u64(bg_ctx* c, const uint64_t* d, uint64_t* h) {
  BG_HIP(c, hipMemcpyAsync(h, d, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
  BG_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}
