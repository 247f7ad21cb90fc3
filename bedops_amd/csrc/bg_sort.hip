// bg_sort.hip — stable LSD radix sort of uint64 keys (+ optional uint32 payload).
//
// Used off the headline path: the breakpoint/event sort of --partition and --symmdiff
// and the re-sort of rows clamped at base 0 by --range padding (BedPadReader::getFirst,
// applications/bed/bedops/src/BedPadReader.hpp:194-277, a std::multiset keeps ties in
// input order, so the sort must be stable).
//
// One pass per 8-bit digit over tiles of RS_TILE keys:
//   k_rs_hist     per-tile digit histogram (LDS atomics) -> H[digit * ntiles + tile]
//   scan          exclusive prefix over H (digit-major), so H[d * nt + t] is where tile t's
//                 keys with digit d start in the output
//   k_rs_scatter  stable in-tile rank: items are taken in index order (round j covers
//                 elements j*RS_NT .. j*RS_NT+RS_NT-1 of the tile), each wave finds the
//                 lanes sharing its digit with 8 ballots, and per-digit running counts
//                 in LDS carry the rank across waves and rounds.
#include "bg_internal.h"

#define RS_NT 256
#define RS_ITEMS 8
#define RS_TILE (RS_NT * RS_ITEMS)

__global__ void __launch_bounds__(RS_NT) k_rs_hist(const uint64_t* __restrict__ K, uint64_t n,
                                                   int shift, uint64_t* __restrict__ H,
                                                   unsigned ntiles) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
#pragma unroll
  for (int j = 0; j < RS_ITEMS; ++j) {
    const uint64_t i = base + (uint64_t)j * RS_NT + threadIdx.x;
    if (i < n) atomicAdd(&h[(K[i] >> shift) & 255], 1u);
  }
  __syncthreads();
  H[(uint64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

template <bool VALS>
__global__ void __launch_bounds__(RS_NT) k_rs_scatter(const uint64_t* __restrict__ K,
                                                      const uint32_t* __restrict__ V, uint64_t n,
                                                      int shift, const uint64_t* __restrict__ H,
                                                      unsigned ntiles, uint64_t* __restrict__ KO,
                                                      uint32_t* __restrict__ VO) {
  __shared__ uint64_t dst[256];   // running output position of each digit
  __shared__ uint32_t wc[4][256];  // this round's per-wave digit counts
  const int lane = bg_lane(), w = bg_wave();
  dst[threadIdx.x] = H[(uint64_t)threadIdx.x * ntiles + blockIdx.x];
  for (int q = 0; q < 4; ++q) wc[q][threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int j = 0; j < RS_ITEMS; ++j) {
    const uint64_t i = base + (uint64_t)j * RS_NT + threadIdx.x;
    const bool ok = i < n;
    const uint64_t key = ok ? K[i] : 0;
    const uint32_t d = (uint32_t)(key >> shift) & 255u;
    uint64_t peer = __ballot(ok);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t m = __ballot((d >> b) & 1u);
      peer &= ((d >> b) & 1u) ? m : ~m;
    }
    const uint32_t below = (uint32_t)__popcll(peer & lt);
    if (ok && below == 0) wc[w][d] = (uint32_t)__popcll(peer);
    __syncthreads();
    if (ok) {
      uint64_t pos = dst[d] + below;
      for (int q = 0; q < w; ++q) pos += wc[q][d];
      KO[pos] = key;
      if (VALS) VO[pos] = V[i];
    }
    __syncthreads();
    const uint32_t t = threadIdx.x;  // one thread per digit advances the running count
    dst[t] += (uint64_t)wc[0][t] + wc[1][t] + wc[2][t] + wc[3][t];
    wc[0][t] = wc[1][t] = wc[2][t] = wc[3][t] = 0;
    __syncthreads();
  }
}

__global__ void k_rs_max(const uint64_t* __restrict__ K, uint64_t n, unsigned long long* out) {
  uint64_t m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    m = K[i] > m ? K[i] : m;
  m = wave_incl_scan(m, OpMax());
  if (bg_lane() == 63) atomicMax(out, (unsigned long long)m);
}

// Sorts keys[0, n) (and vals alongside, if given) ascending, stably. Only the digits
// below the highest set bit of the largest key are processed.
int bg_sort_u64(bg_ctx* c, uint64_t* keys, uint32_t* vals, uint64_t n) {
  if (n < 2) return 0;
  unsigned long long* d_max = (unsigned long long*)bg_alloc(c, 8);
  if (!d_max) return BG_E_NOMEM;
  BG_HIP(c, hipMemsetAsync(d_max, 0, 8, c->stream));
  BG_LAUNCH(c, "k_rs_max", k_rs_max, dim3(std::min<uint64_t>(bg_blocks(n, 256), 1024)), dim3(256),
            keys, n, d_max);
  BG_HIP(c, hipGetLastError());
  uint64_t mx = 0;
  int rc = bg_fetch_u64(c, (const uint64_t*)d_max, &mx);
  bg_release(c, d_max);
  if (rc) return rc;
  int bits = 0;
  while (bits < 64 && (mx >> bits) != 0) ++bits;
  const int passes = (bits + 7) / 8;
  if (passes == 0) return 0;
  const unsigned nt = bg_blocks(n, RS_TILE);
  uint64_t* H = (uint64_t*)bg_alloc(c, 8ull * 256 * nt);
  uint64_t* k2 = (uint64_t*)bg_alloc(c, 8 * n);
  uint32_t* v2 = vals ? (uint32_t*)bg_alloc(c, 4 * n) : nullptr;
  if (!H || !k2 || (vals && !v2)) return BG_E_NOMEM;
  uint64_t *ka = keys, *kb = k2;
  uint32_t *va = vals, *vb = v2;
  for (int p = 0; p < passes; ++p) {
    const int sh = 8 * p;
    BG_LAUNCH(c, "k_rs_hist", k_rs_hist, dim3(nt), dim3(RS_NT), ka, n, sh, H, nt);
    BG_HIP(c, hipGetLastError());
    if ((rc = bg_scan_sum_u64(c, H, H, 256ull * nt, nullptr))) return rc;
    if (vals)
      BG_LAUNCH(c, "k_rs_scatter", k_rs_scatter<true>, dim3(nt), dim3(RS_NT), ka, va, n, sh, H, nt,
                kb, vb);
    else
      BG_LAUNCH(c, "k_rs_scatter", k_rs_scatter<false>, dim3(nt), dim3(RS_NT), ka, va, n, sh, H,
                nt, kb, vb);
    BG_HIP(c, hipGetLastError());
    std::swap(ka, kb);
    std::swap(va, vb);
  }
  if (ka != keys) {  // odd number of passes: result is in the scratch buffers
    BG_HIP(c, hipMemcpyAsync(keys, ka, 8 * n, hipMemcpyDeviceToDevice, c->stream));
    if (vals) BG_HIP(c, hipMemcpyAsync(vals, va, 4 * n, hipMemcpyDeviceToDevice, c->stream));
  }
  bg_release(c, H);
  bg_release(c, k2);
  bg_release(c, v2);
  return 0;
}
