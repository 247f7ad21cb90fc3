// bg_load.hip — K0: BED text in HBM -> keyed int64 SoA columns, one text pass.
//
// Replaces the reference's per-line readers (fscanf "%s\t%lu\t%lu%*[^\n]s\n" + fgetc,
// interfaces/general-headers/data/bed/Bed.hpp:244-255,270-272; B3Rest :277-383;
// Bed5 :829-860; iterator EOF rule AllocateIterator_BED_starch.hpp:161-176).
// Accepted line grammar (one record per '\n'-terminated line):
//   [ws] chrom ws+ [+]digits ws+ [+]digits rest* '\n'
// ws = ' ' '\t' '\r' '\v' '\f'; rest = any bytes up to '\n' (kept verbatim for
// BG_BED3_REST: it starts right after the end digits, exactly like "%[^\n]").
// Bytes after the last '\n' are ignored (the reference drops an unterminated final
// line: !feof check). Lines outside the grammar are reported as BG_E_PARSE with the
// line number instead of reproducing fscanf's cross-line behaviour on garbage.
//
// Pipeline per input (tiles of 8 KiB; a tile owns the lines that START in it):
//   k_scout      '\n' count per tile + hash of the chromosome token of the tile's
//                first line                                        (text read 1x)
//   scan         row0[t] = '\n' before the tile = row index of its first owned line
//   k_boundary   tiles whose first token differs from the next tile's hold every
//                chromosome change; k_tile_runs lists the token changes inside them
//   host         run list per input (position, name), strcmp order check, global
//                dictionary over all inputs -> chromosome id per run
//   k_parse      per tile: text + halos staged in LDS, '\n' offsets by a block scan,
//                one thread per line: SWAR field masks + 8-digit SWAR decimal
//                conversion (bg_parse.h; byte path for anything else), run by
//                position, token hash check against the run, keys
//                ks = (chrom_id << 40) | start, ke = (chrom_id << 40) | end written
//                directly, in-tile sort check                     (text read 1x)
//   k_check_bounds  sort check across tile boundaries
#include <algorithm>
#include <cstring>
#include <map>

#include <type_traits>

#include "bg_internal.h"
#include "bg_parse.h"
#include "bg_strtod.h"

#define TT 8192   // tile bytes
#define HB 16     // halo before (we need the byte before the tile)
#define HA 256    // halo after (the tail of the tile's last line)
#define LBUF (HB + TT + HA + 32)
#define LCAP 1536  // lines per tile on the LDS path (>= TT / 6: shortest valid line)
#define REC_CAP (1u << 20)

__device__ __forceinline__ uint32_t nl_mask4(uint32_t w) {
  // bit 7 of each byte set iff that byte == '\n' (exact, no borrow artefacts)
  uint32_t x = w ^ 0x0A0A0A0Au;
  uint32_t nz = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;
  return ~nz & 0x80808080u;
}

// guarded 16-byte load of txt[base, base+16) (bytes outside [0, nbytes) read as 0)
__device__ __forceinline__ uint4 load16(const uint8_t* __restrict__ txt, int64_t base,
                                        uint64_t nbytes) {
  if (base >= 0 && (uint64_t)base + 16 <= nbytes) return *reinterpret_cast<const uint4*>(txt + base);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int k = 0; k < 16; ++k)
    if (base + k >= 0 && (uint64_t)(base + k) < nbytes)
      w[k >> 2] |= (uint32_t)txt[base + k] << (8 * (k & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// byte view of one tile: LDS copy of [lo, hi), global memory elsewhere (< nbytes)
struct TileText {
  const uint8_t* g;
  const uint8_t* l;
  int64_t lo, hi;
  uint64_t nb;
  __device__ __forceinline__ uint8_t at(int64_t p) const {
    return (p >= lo && p < hi) ? l[p - lo] : g[p];
  }
};

// A tile's bytes as registers: v0/v1 = this thread's 32 tile bytes, vh = one 16-byte
// piece of the halos (threads < (HA+32)/16: after the tile; the last thread: before it)
struct TileRegs {
  uint4 v0, v1, vh;
};
__device__ __forceinline__ void load_tile(const uint8_t* __restrict__ txt, uint64_t nb, int64_t t0,
                                          TileRegs& R) {
  const int64_t b = t0 + (int64_t)threadIdx.x * 32;
  R.v0 = load16(txt, b, nb);
  R.v1 = load16(txt, b + 16, nb);
  if (threadIdx.x < (HA + 32) / 16) R.vh = load16(txt, t0 + TT + (int64_t)threadIdx.x * 16, nb);
  else if (threadIdx.x == BG_NT - 1) R.vh = load16(txt, t0 - HB, nb);
}
// [t0-HB, t0+TT+HA) into LDS (zeros outside the text)
__device__ __forceinline__ void store_tile(uint8_t* buf, const TileRegs& R) {
  *reinterpret_cast<uint4*>(&buf[HB + threadIdx.x * 32]) = R.v0;
  *reinterpret_cast<uint4*>(&buf[HB + threadIdx.x * 32 + 16]) = R.v1;
  if (threadIdx.x < (HA + 32) / 16) *reinterpret_cast<uint4*>(&buf[HB + TT + threadIdx.x * 16]) = R.vh;
  else if (threadIdx.x == BG_NT - 1) *reinterpret_cast<uint4*>(&buf[0]) = R.vh;
}
// Stage [t0-HB, t0+TT+HA) into LDS (zeros outside the text). Each thread also returns
// its 32 tile bytes in registers.
__device__ __forceinline__ void stage_tile(const uint8_t* __restrict__ txt, uint64_t nb,
                                           int64_t t0, uint8_t* buf, uint4& v0, uint4& v1) {
  TileRegs R;
  load_tile(txt, nb, t0, R);
  store_tile(buf, R);
  v0 = R.v0;
  v1 = R.v1;
}

// token [tok, tok+len) of the line starting at p (leading ws skipped, stops at ws or
// '\n'); returns its hash; blank line -> len 0
__device__ __forceinline__ uint64_t line_token(const TileText& T, int64_t p, int64_t& tok,
                                               uint32_t& len) {
  while ((uint64_t)p < T.nb) {
    uint8_t ch = T.at(p);
    if (!bg_isws(ch)) break;
    ++p;
  }
  tok = p;
  uint64_t h = BGP_FNV_OFF;  // bgp_hash_words over zero-padded 32-bit words
  uint32_t n = 0, w = 0;
  while ((uint64_t)p < T.nb) {
    uint8_t ch = T.at(p);
    if (ch == '\n' || bg_isws(ch)) break;
    w |= (uint32_t)ch << (8 * (n & 3));
    ++n;
    if ((n & 3) == 0) { h = (h ^ w) * BGP_FNV_PRIME; w = 0; }
    ++p;
  }
  if (n & 3) h = (h ^ w) * BGP_FNV_PRIME;
  len = n;
  return (h ^ n) * BGP_FNV_PRIME;
}

// -------------------------------------------------------------------------------------
// k_scout: newline count + first '\n' offset per tile (pure streaming read)
// -------------------------------------------------------------------------------------
#define SCOUT_TILES 4  // tiles per workgroup: 8 x 16-B loads in flight per thread
__global__ void __launch_bounds__(BG_NT) k_scout(const uint8_t* __restrict__ txt, uint64_t nb,
                                                 uint32_t ntiles, uint64_t* __restrict__ cnt,
                                                 uint32_t* __restrict__ fnl) {
  __shared__ uint32_t shc[SCOUT_TILES][BG_NT / 64];
  __shared__ uint32_t shm[SCOUT_TILES][BG_NT / 64];
  uint4 v[SCOUT_TILES][2];
#pragma unroll
  for (int q = 0; q < SCOUT_TILES; ++q) {  // issue every load first
    const int64_t b = ((int64_t)blockIdx.x * SCOUT_TILES + q) * TT + (int64_t)threadIdx.x * 32;
    v[q][0] = load16(txt, b, nb);
    v[q][1] = load16(txt, b + 16, nb);
  }
#pragma unroll
  for (int q = 0; q < SCOUT_TILES; ++q) {
    const uint32_t w[8] = {v[q][0].x, v[q][0].y, v[q][0].z, v[q][0].w,
                           v[q][1].x, v[q][1].y, v[q][1].z, v[q][1].w};
    uint32_t c = 0, first = TT;
#pragma unroll
    for (int k = 7; k >= 0; --k) {
      const uint32_t m = nl_mask4(w[k]);
      c += __popc(m);
      if (m) first = threadIdx.x * 32 + 4 * k + (__ffs(m) - 1) / 8;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      c += __shfl_xor(c, d, 64);
      first = min(first, (uint32_t)__shfl_xor(first, d, 64));
    }
    if (bg_lane() == 0) { shc[q][bg_wave()] = c; shm[q][bg_wave()] = first; }
  }
  __syncthreads();
  if (threadIdx.x < SCOUT_TILES) {
    const uint32_t t = blockIdx.x * SCOUT_TILES + threadIdx.x;
    if (t < ntiles) {
      uint64_t s = 0;
      uint32_t f = TT;
      for (int w = 0; w < BG_NT / 64; ++w) { s += shc[threadIdx.x][w]; f = min(f, shm[threadIdx.x][w]); }
      cnt[t] = s;
      fnl[t] = f;
    }
  }
}


// line_token's hash of the line at ls from three aligned 16-byte loads, when the line
// starts with its token (no leading whitespace) of at most 16 bytes ending within 32
// bytes; false: the caller takes the byte loop
__device__ __forceinline__ bool token_hash_fast(const uint8_t* __restrict__ txt, uint64_t nb,
                                                int64_t ls, uint64_t& h) {
  const int64_t a = ls & ~15LL;
  if ((uint64_t)a + 48 > nb) return false;
  const uint4 x = *reinterpret_cast<const uint4*>(txt + a);
  const uint4 y = *reinterpret_cast<const uint4*>(txt + a + 16);
  const uint4 z = *reinterpret_cast<const uint4*>(txt + a + 32);
  const uint32_t d[12] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w, z.x, z.y, z.z, z.w};
  const uint32_t o = (uint32_t)(ls - a);  // 0..15
  const uint32_t wo = o >> 2, bo = o & 3;
  uint32_t W[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // bytes [ls, ls + 32) as dwords
    uint32_t lo = d[0], hi = d[1];
#pragma unroll
    for (int k = 1; k < 4; ++k)
      if (wo == (uint32_t)k) { lo = d[i + k]; hi = d[i + k + 1]; }
    if (wo == 0) { lo = d[i]; hi = d[i + 1]; }
    W[i] = bgp_align(lo, hi, bo);
  }
  uint32_t WS, DG;
  bgp_classify8(W, WS, DG);  // whitespace class includes '\n'
  if (WS & 1u) return false;  // leading whitespace or a blank line
  if (!(WS & 0x1FFFEu)) return false;  // token longer than 16 bytes (or no end in sight)
  const uint32_t len = bgp_ctz(WS);
  const uint64_t lo8 = (uint64_t)W[0] | ((uint64_t)W[1] << 32);
  const uint64_t hi8 = (uint64_t)W[2] | ((uint64_t)W[3] << 32);
  h = bgp_hash16(lo8, hi8, len);
  return true;
}

// first owned line of each tile and the hash of its chromosome token (one thread per
// tile, reads a few bytes). fnl: first '\n' per tile from k_scout, or nullptr: found here
// by a forward scan (BG_BED3_SET loads have no scout pass)
__global__ void k_tokhash(const uint8_t* __restrict__ txt, uint64_t nb, uint32_t ntiles,
                          const uint32_t* __restrict__ fnl, int64_t* __restrict__ fls,
                          uint64_t* __restrict__ fhash) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  const int64_t t0 = (int64_t)t * TT;
  uint32_t f = TT;
  if (fnl) {
    f = fnl[t];
  } else {
    const int64_t te = min((int64_t)nb, t0 + TT);
    for (int64_t q = t0; q < te; q += 16) {
      const uint4 v = load16(txt, q, nb);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      uint32_t hit = TT;
#pragma unroll
      for (int k = 3; k >= 0; --k) {
        const uint32_t m = nl_mask4(w[k]);
        if (m) hit = (uint32_t)(q - t0) + 4 * k + (__ffs(m) - 1) / 8;
      }
      if (hit < TT) { f = hit; break; }
    }
    if (f >= (uint32_t)(te - t0)) f = TT;
  }
  int64_t ls = -1;
  if (t0 == 0 || txt[t0 - 1] == '\n') ls = t0;
  else if (f + 1 < TT) ls = t0 + f + 1;
  if (ls >= 0 && (uint64_t)ls >= nb) ls = -1;
  uint64_t h = 0;
  if (ls >= 0 && !token_hash_fast(txt, nb, ls, h)) {
    TileText T{txt, txt, 0, 0, nb};  // global reads only
    int64_t tok;
    uint32_t len;
    h = line_token(T, ls, tok, len);
  }
  fls[t] = ls;
  fhash[t] = h;
}

// tile t may hold a chromosome change iff its first token differs from the next
// tile's (or either has no line start); tile 0 and the last tile always qualify
__global__ void k_boundary(const int64_t* __restrict__ fls, const uint64_t* __restrict__ fhash,
                           uint32_t ntiles, uint32_t* __restrict__ list, uint32_t* __restrict__ nlist) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  bool b = (t == 0) || (t + 1 == ntiles) || fls[t] < 0 || fls[t + 1] < 0 || fhash[t] != fhash[t + 1];
  if (b) list[atomicAdd(nlist, 1u)] = t;
}

// line starts of the tile (local offsets) -> LDS; returns the number of lines.
// has0: a line starts at the tile's first byte. Lines are the starts t0+ls[k].
__device__ __forceinline__ uint32_t tile_line_starts(const uint4& v0, const uint4& v1,
                                                     const uint8_t* buf, int64_t t0,
                                                     uint16_t* ls, uint32_t cap,
                                                     uint32_t* shs, bool& has0) {
  has0 = (t0 == 0) || buf[HB - 1] == '\n';
  const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  uint32_t nlg = 0;  // bit j: byte j of this thread's 32 is '\n'
#pragma unroll
  for (int k = 0; k < 8; ++k) nlg |= bgp_group4(nl_mask4(w[k])) << (4 * k);
  // a '\n' on the tile's last byte starts a line in the next tile
  if (threadIdx.x == BG_NT - 1) nlg &= 0x7FFFFFFFu;
  // exclusive sum of the newline counts over the block: one barrier (every thread adds up
  // the wave totals itself; the barrier at the end protects shs from its next use)
  const uint32_t inc = wave_incl_scan((uint32_t)__popc(nlg), OpSum());
  if (bg_lane() == 63) shs[bg_wave()] = inc;
  __syncthreads();
  uint32_t tot = 0, wpre = 0;
#pragma unroll
  for (int q = 0; q < BG_NT / 64; ++q) {
    const uint32_t x = shs[q];
    if (q < bg_wave()) wpre += x;
    tot += x;
  }
  uint32_t o = wpre + inc - (uint32_t)__popc(nlg) + (has0 ? 1u : 0u);
  if (threadIdx.x == 0 && has0) ls[0] = 0;
  for (uint32_t m = nlg; m; m &= m - 1) {  // one iteration per line start
    if (o < cap) ls[o] = (uint16_t)(threadIdx.x * 32 + bgp_ctz(m) + 1);
    ++o;
  }
  __syncthreads();
  return tot + (has0 ? 1u : 0u);
}

// end ('\n' position) of the line starting at p, searching from `from`; -1 if none
__device__ __forceinline__ int64_t find_nl(const TileText& T, int64_t from) {
  for (int64_t q = from; (uint64_t)q < T.nb; ++q)
    if (T.at(q) == '\n') return q;
  return -1;
}

// k_tile_runs: records (position, token hash, token bytes) of every line in a boundary
// tile whose token differs from the previous line's, plus the tile's first line and the
// next tile's first line. Grid-strided over the boundary list, whose length it reads on
// the device (no host round trip between k_boundary and this kernel).
// one chromosome-run record (copied to the host in one piece)
struct RunRec {
  int64_t pos;
  uint64_t hash;
  uint32_t len;
  uint32_t pad;
  char name[128];
};
__device__ __forceinline__ void put_record(const TileText& T, int64_t p, uint64_t h, int64_t tok,
                                           uint32_t len, uint32_t cap, RunRec* recs,
                                           uint32_t* nrec) {
  const uint32_t q = atomicAdd(nrec, 1u);
  if (q >= cap) return;  // the host reports the overflow
  recs[q].pos = p;
  recs[q].hash = h;
  recs[q].len = len;
  char* o = recs[q].name;
  const uint32_t n = len < 127 ? len : 127;
  for (uint32_t i = 0; i < n; ++i) o[i] = (char)T.at(tok + i);
  o[n] = 0;
}

__global__ void __launch_bounds__(BG_NT) k_tile_runs(
    const uint8_t* __restrict__ txt, uint64_t nb, const uint32_t* __restrict__ tiles,
    const uint32_t* __restrict__ ntiles_b, const int64_t* __restrict__ fls, uint32_t ntiles,
    uint32_t cap, RunRec* __restrict__ recs, uint32_t* __restrict__ nrec) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[LBUF];
  __shared__ uint16_t lst[TT + 1];
  __shared__ uint32_t shs[BG_NT / 64 + 1];
  const uint32_t nbd = *ntiles_b;
  for (uint32_t bi = blockIdx.x; bi < nbd; bi += gridDim.x) {
    const uint32_t t = tiles[bi];
    const int64_t t0 = (int64_t)t * TT;
    uint4 v0, v1;
    __syncthreads();  // the previous tile's readers are done with the LDS
    stage_tile(txt, nb, t0, buf, v0, v1);
    __syncthreads();
    bool has0;
    const uint32_t L = tile_line_starts(v0, v1, buf, t0, lst, TT + 1, shs, has0);
    TileText T{txt, buf, t0 - HB, t0 + TT + HA, nb};
    for (uint32_t k = threadIdx.x; k < L; k += BG_NT) {
      const int64_t p = t0 + lst[k];
      if ((uint64_t)p >= nb) continue;
      int64_t tok;
      uint32_t len;
      const uint64_t h = line_token(T, p, tok, len);
      bool rec = (k == 0);
      if (!rec) {
        int64_t ptok;
        uint32_t plen;
        rec = line_token(T, t0 + lst[k - 1], ptok, plen) != h;
      }
      if (rec) put_record(T, p, h, tok, len, cap, recs, nrec);
    }
    if (threadIdx.x == 0) {  // first line of the next tile that has one
      uint32_t u = t + 1;
      while (u < ntiles && fls[u] < 0) ++u;
      if (u < ntiles) {
        int64_t tok;
        uint32_t len;
        const uint64_t h = line_token(T, fls[u], tok, len);
        put_record(T, fls[u], h, tok, len, cap, recs, nrec);
      }
    }
  }
}

// -------------------------------------------------------------------------------------
// k_parse
// -------------------------------------------------------------------------------------
struct RunInfo {
  int64_t pos;    // byte position of the run's first line (ascending over runs)
  uint64_t hash;  // token hash (bgp_hash_words form)
  uint64_t tlo, thi;  // first 16 token bytes, zero padded (fast-path identity check)
  uint32_t tlen;  // token length
  int32_t gid;    // global chromosome id
};
struct RunTable {
  const RunInfo* info;
  uint64_t* row;  // out: row index of each run's first line
  uint32_t n;
};

__device__ __forceinline__ uint32_t run_of(const RunTable& R, int64_t p, uint32_t lo, uint32_t hi) {
  // last k in [lo, hi] with pos[k] <= p
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (R.info[mid].pos <= p) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ bool parse_u64(const TileText& T, int64_t& p, int64_t le, uint64_t& v) {
  if (p < le && T.at(p) == '+') ++p;
  int nd = 0;
  uint64_t x = 0;
  while (p < le) {
    const uint8_t ch = T.at(p);
    if (ch < '0' || ch > '9') break;
    if (nd < 19) x = x * 10 + (ch - '0');
    ++nd;
    ++p;
  }
  v = (nd > 13) ? ~0ULL : x;  // > 13 digits is always out of range
  return nd > 0;
}

// N * 2^e2 (N > 0) rounded to the nearest double, ties to even (normal range only: the
// callers' |exponents| keep it there)
__device__ __forceinline__ double round_u128(unsigned __int128 N, int e2) {
  const uint64_t hi = (uint64_t)(N >> 64), lo = (uint64_t)N;
  const int lz = hi ? __builtin_clzll(hi) : 64 + __builtin_clzll(lo);
  N <<= lz;  // top bit at 127
  e2 -= lz;
  uint64_t mant = (uint64_t)(N >> 75);  // 53 bits
  const unsigned __int128 rest = N & (((unsigned __int128)1 << 75) - 1), half = (unsigned __int128)1 << 74;
  if (rest > half || (rest == half && (mant & 1))) {
    ++mant;
    if (mant >> 53) {
      mant >>= 1;
      ++e2;
    }
  }
  return ldexp((double)mant, e2 + 75);
}
// m * 10^pw correctly rounded for what Clinger's fast path does not cover: m up to 2^64 and
// -26 <= pw <= 27. pw >= 0: m * 5^pw exactly in 128 bits, times 2^pw. pw < 0: m / 5^k * 2^-k
// with m scaled to 117 bits, so the quotient keeps >= 55 bits and the remainder is the
// sticky bit. false outside that range.
__device__ __forceinline__ bool decimal_exact(uint64_t m, int pw, double& out) {
  if (pw > 27 || pw < -26) return false;
  uint64_t f5 = 1;
  for (int k = 0; k < (pw < 0 ? -pw : pw); ++k) f5 *= 5;
  if (pw >= 0) {
    out = round_u128((unsigned __int128)m * f5, pw);
    return true;
  }
  const int s = 117 - (64 - __builtin_clzll(m));
  const unsigned __int128 num = (unsigned __int128)m << s;
  const unsigned __int128 q = num / f5, r = num - q * f5;
  out = round_u128((q << 1) | (r != 0 ? 1 : 0), -s - 1 + pw);
  return true;
}

// exact powers of ten (a table in constant memory: a local array indexed at run time is
// placed in scratch)
__constant__ double BG_P10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                  1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// strtod subset, correctly rounded where it accepts: [+-]digits[.digits][(e|E)[+-]digits]
// with <= 19 significant digits m and value m * 10^p, |p| <= 22 and m <= 2^53 (Clinger's
// fast path: one rounding of exact operands), p up to 37 when m * 10^(p-22) stays an exact
// integer <= 2^53, otherwise -26 <= p <= 27 by exact 128-bit arithmetic (decimal_exact:
// e.g. the 17 significant digits of %.17g / repr output). Integers up to 2^53 are flagged
// (exact sums). Any other valid number (up to BG_SD_DIGITS significant digits, any
// exponent) returns isint = -1: the caller lists it for k_score_big (bg_strtod.h). More
// digits, or anything that is not a plain decimal number -> ERR_SCORE.
// EXACT == false (k_parse_rv): what would take decimal_exact's 128-bit arithmetic is listed for
// k_score_big instead (isint -1: the same correctly rounded value; the 128-bit division's
// registers spilled in the row kernel's every wave)
template <bool EXACT = true>
__device__ __forceinline__ bool parse_score(const TileText& T, int64_t& p, int64_t le,
                                            double& out, int& isint) {
  bool neg = false;
  if (p < le && (T.at(p) == '+' || T.at(p) == '-')) neg = T.at(p++) == '-';
  uint64_t m = 0;
  int nd = 0, frac = 0, sig = 0;
  bool dot = false, big = false;
  while (p < le) {
    const uint8_t ch = T.at(p);
    if (ch == '.' && !dot) { dot = true; ++p; continue; }
    if (ch < '0' || ch > '9') break;
    ++nd;
    if (dot) ++frac;
    if (m != 0 || ch != '0') ++sig;
    if (sig <= 19) m = m * 10 + (ch - '0');
    else big = true;  // past 19 digits: k_score_big (up to BG_SD_DIGITS)
    ++p;
  }
  if (nd == 0 || sig > BG_SD_DIGITS) return false;
  int ex = 0;
  if (p < le && (T.at(p) == 'e' || T.at(p) == 'E')) {  // strtod takes the exponent only if digits follow
    int64_t q = p + 1;
    bool eneg = false;
    if (q < le && (T.at(q) == '+' || T.at(q) == '-')) eneg = T.at(q++) == '-';
    int ed = 0;
    while (q < le && T.at(q) >= '0' && T.at(q) <= '9') {
      if (ex < 10000) ex = ex * 10 + (T.at(q) - '0');
      ++ed;
      ++q;
    }
    if (ed == 0) return false;  // "1e" / "1e+": not a plain number for this path
    if (eneg) ex = -ex;
    p = q;
  }
  if (p < le && !bg_isws(T.at(p))) return false;  // junk after the number
  if (big) {  // a syntactically valid number for the exact conversion (isint -1)
    isint = -1;
    out = 0;
    return true;
  }
  int pw = ex - frac;  // value = m * 10^pw
  while (pw < 0 && m != 0 && m % 10 == 0) { m /= 10; ++pw; }  // trailing zeros
  const double* const P10 = BG_P10;
  if (m == 0) {
    isint = 1;
    out = neg ? -0.0 : 0.0;
    return true;
  }
  if (m > (1ULL << 53) || pw < -22) {  // outside Clinger's fast path: exact 128-bit rounding
    if (!EXACT || !decimal_exact(m, pw, out)) {  // beyond 128 bits: k_score_big
      isint = -1;
      out = 0;
      return true;
    }
    isint = 0;  // a fraction, or an integer above 2^53 (no exact int64 sums)
    if (neg) out = -out;
    return true;
  }
  if (pw < 0) {
    isint = 0;
    out = (double)m / P10[-pw];
  } else {
    if (pw > 22) {  // m * 10^(pw-22) exact and <= 2^53, then one rounding by 1e22
      uint64_t mm = m;
      int pp = pw;
      for (; pp > 22; --pp) {
        if (mm > (1ULL << 53) / 10) break;
        mm *= 10;
      }
      if (pp > 22) {  // not exact that way
        if (!EXACT || !decimal_exact(m, pw, out)) {
          isint = -1;
          out = 0;
          return true;
        }
        isint = 0;
        if (neg) out = -out;
        return true;
      }
      m = mm;
      pw = pp;
    }
    // an integer: exact sums need |value| <= 2^53
    uint64_t v = m;
    bool small = true;
    for (int k = 0; k < pw && small; ++k) {
      if (v > (1ULL << 53) / 10) small = false;
      else v *= 10;
    }
    isint = small ? 1 : 0;
    out = (double)m * P10[pw];
  }
  if (neg) out = -out;
  return true;
}

struct Line {
  int64_t tok;
  uint32_t toklen;
  uint64_t hash;
  uint64_t start, end;
  int64_t rest;
  double score;
  int err;
  int scoreint;  // 1: an integer <= 2^53; 0: other; -1: left to k_score_big
  int64_t spos;  // the score's first byte
};

// full grammar, byte by byte (fallback path and error reporting)
template <bool EXACT = true>
__device__ __forceinline__ void parse_line_slow(const TileText& T, int64_t ls, int64_t le, int kind,
                                             Line& L) {
  L.err = 0;
  L.scoreint = 1;
  L.score = 0;
  int64_t p = ls;
  while (p < le && bg_isws(T.at(p))) ++p;
  if (p == le) { L.err = ERR_BLANK; return; }
  {
    int64_t tk;
    uint32_t tl;
    L.hash = line_token(T, p, tk, tl);
    L.tok = tk;
    L.toklen = tl;
    p = tk + tl;
  }
  if (L.toklen > BG_CHR_MAX) { L.err = ERR_CHROM; return; }
  while (p < le && bg_isws(T.at(p))) ++p;
  if (!parse_u64(T, p, le, L.start)) { L.err = ERR_PARSE; return; }
  if (p < le && !bg_isws(T.at(p))) { L.err = ERR_PARSE; return; }
  while (p < le && bg_isws(T.at(p))) ++p;
  if (!parse_u64(T, p, le, L.end)) { L.err = ERR_PARSE; return; }
  L.rest = p;
  if (kind == BG_BED5) {
    if (p == le || !bg_isws(T.at(p))) { L.err = ERR_PARSE; return; }
    while (p < le && bg_isws(T.at(p))) ++p;
    const int64_t id = p;
    while (p < le && !bg_isws(T.at(p))) ++p;
    if (p == id) { L.err = ERR_PARSE; return; }
    while (p < le && bg_isws(T.at(p))) ++p;
    int isint = 1;
    L.spos = p;
    if (!parse_score<EXACT>(T, p, le, L.score, isint)) { L.err = ERR_SCORE; return; }
    L.scoreint = isint;
  }
}

// a score for k_score_big: (row, first byte) pairs; beyond the list's capacity the load
// refuses (finish_one)
__device__ __forceinline__ void big_push(bg_dstatus* st, uint64_t* big, uint32_t cap, uint64_t r, int64_t pos) {
  const unsigned long long q = atomicAdd(&st->nbig, 1ULL);
  if (q < cap) {
    big[2 * q] = r;
    big[2 * q + 1] = (uint64_t)pos;
  }
}

// the exact conversion of the listed scores (parse_score's isint -1: more than 19 significant
// digits or exponents past the 128-bit path), one thread per score; the syntax was checked
// by parse_score. st->flags bit 5: a score with more than BG_SD_DIGITS significant digits
__global__ void k_score_big(const uint8_t* __restrict__ txt, uint64_t nb, const uint64_t* __restrict__ big,
                            uint64_t n, double* __restrict__ score) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t r = big[2 * i];
  uint64_t p = big[2 * i + 1];
  bool neg = false;
  if (p < nb && (txt[p] == '+' || txt[p] == '-')) neg = txt[p++] == '-';
  uint8_t dg[BG_SD_DIGITS];
  int nd = 0, frac_after = 0;  // significant digits; fraction digits after the first significant one
  int lead_frac = 0;           // fraction digits before it (leading zeros after the point)
  bool dot = false;
  for (; p < nb; ++p) {
    const uint8_t ch = txt[p];
    if (ch == '.' && !dot) { dot = true; continue; }
    if (ch < '0' || ch > '9') break;
    if (nd == 0 && ch == '0') {
      if (dot) ++lead_frac;
      continue;
    }
    if (nd < BG_SD_DIGITS) dg[nd] = (uint8_t)(ch - '0');
    ++nd;
    if (dot) ++frac_after;
  }
  int ex = 0;
  if (p < nb && (txt[p] == 'e' || txt[p] == 'E')) {
    uint64_t q = p + 1;
    bool eneg = false;
    if (q < nb && (txt[q] == '+' || txt[q] == '-')) eneg = txt[q++] == '-';
    for (; q < nb && txt[q] >= '0' && txt[q] <= '9'; ++q)
      if (ex < 100000) ex = ex * 10 + (txt[q] - '0');
    if (eneg) ex = -ex;
  }
  int n10 = nd;
  while (n10 > 0 && n10 <= BG_SD_DIGITS && dg[n10 - 1] == 0) --n10;  // trailing zeros
  double v = 0;
  if (nd <= BG_SD_DIGITS && n10 > 0) {
    const int e = ex - lead_frac - frac_after + (nd - n10);  // exponent of the last kept digit
    strtod_big(dg, n10, e, false, v);
  }
  score[r] = neg ? -v : v;
}

// 16 bytes of LDS starting at byte offset q (q + 20 <= LBUF)
__device__ __forceinline__ void lds16(const uint8_t* buf, uint32_t q, uint64_t& lo, uint64_t& hi) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(buf + (q & ~3u));
  const uint32_t o = q & 3u;
  const uint32_t x0 = d[0], x1 = d[1], x2 = d[2], x3 = d[3], x4 = d[4];
  lo = (uint64_t)bgp_align(x0, x1, o) | ((uint64_t)bgp_align(x1, x2, o) << 32);
  hi = (uint64_t)bgp_align(x2, x3, o) | ((uint64_t)bgp_align(x3, x4, o) << 32);
}

// the 12 bytes of LDS ending at byte offset e (e >= 12, e + 4 <= LBUF)
__device__ __forceinline__ void lds12_end(const uint8_t* buf, uint32_t e, uint32_t& d1,
                                          uint32_t& d2, uint32_t& d3) {
  const uint32_t q = e - 12;
  const uint32_t* d = reinterpret_cast<const uint32_t*>(buf + (q & ~3u));
  const uint32_t o = q & 3u;
  const uint32_t x0 = d[0], x1 = d[1], x2 = d[2], x3 = d[3];
  d1 = bgp_align(x0, x1, o);
  d2 = bgp_align(x1, x2, o);
  d3 = bgp_align(x2, x3, o);
}

// 32-bit window of a per-tile class bitmap starting at local byte offset p (bit j of
// the result = byte p + j); m holds one 32-bit word per 32 tile bytes
__device__ __forceinline__ uint32_t mask_window(const uint32_t* m, uint32_t p) {
  const uint32_t w = p >> 5, b = p & 31;
  const uint64_t two = (uint64_t)m[w] | ((uint64_t)m[w + 1] << 32);
  return (uint32_t)(two >> b);
}

// fast path: fields from the tile's class bitmaps + LDS bytes -> true if decided.
// q: local offset of the line start inside the tile (0 <= q < TT). The chromosome token
// is returned as its first 16 bytes (zero padded) + length; tokens longer than 16 bytes
// take the byte path.
struct Fast {
  uint64_t start, end;
  uint64_t tlo, thi;
  uint32_t toklen;
  uint32_t rest;  // local offset (from the line start) of the rest
};
// 8 bytes of LDS starting at byte offset q
__device__ __forceinline__ uint64_t lds8(const uint8_t* buf, uint32_t q) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(buf + (q & ~3u));
  const uint32_t o = q & 3u;
  const uint32_t x0 = d[0], x1 = d[1], x2 = d[2];
  return (uint64_t)bgp_align(x0, x1, o) | ((uint64_t)bgp_align(x1, x2, o) << 32);
}
// short8: the caller only accepts tokens of <= 8 bytes (its run's token is that short), so
// 8 bytes of the token are read instead of 16
__device__ __forceinline__ bool parse_line_fast(const uint8_t* buf, const uint32_t* wsm,
                                                const uint32_t* dgm, uint32_t q, uint32_t len,
                                                Fast& L, bool short8 = false) {
  BgpFields F;
  const int r = bgp_fields_masks(mask_window(wsm, q), mask_window(dgm, q), len, F);
  if (r != 1) return false;  // blank lines and errors take the byte path (messages)
  const uint32_t toklen = F.a1 - F.a0;
  if (toklen > 16 || F.s1 - F.s0 > 12 || F.e1 - F.e0 > 12) return false;
  const uint32_t b = q + HB;  // LDS byte offset of the line start (>= HB = 16)
  uint32_t d1, d2, d3;
  lds12_end(buf, b + F.s1, d1, d2, d3);
  L.start = bgp_digits_r(d1, d2, d3, (int)(F.s1 - F.s0));
  lds12_end(buf, b + F.e1, d1, d2, d3);
  L.end = bgp_digits_r(d1, d2, d3, (int)(F.e1 - F.e0));
  uint64_t lo, hi;
  if (short8) {
    if (toklen > 8) return false;
    lo = lds8(buf, b + F.a0);
    hi = 0;
  } else {
    lds16(buf, b + F.a0, lo, hi);
  }
  if (toklen < 16) {
    if (toklen <= 8) {
      hi = 0;
      lo = toklen == 8 ? lo : (lo & ((1ull << (8 * toklen)) - 1));
    } else {
      hi &= (1ull << (8 * (toklen - 8))) - 1;
    }
  }
  L.tlo = lo;
  L.thi = hi;
  L.toklen = toklen;
  L.rest = F.e1;
  return true;
}

// parse_line_fast from the whitespace mask alone (k_parse_rv: the tile is classified for
// whitespace only, half the prologue's work): numbers end at whitespace and their bytes are
// checked to be digits while they are converted (bgp_fields_ws / bgp_digits_rc); a line this
// refuses takes the byte path, as in parse_line_fast
__device__ __forceinline__ bool parse_line_fast_ws(const uint8_t* buf, const uint32_t* wsm, uint32_t q,
                                                   uint32_t len, Fast& L, bool short8 = false) {
  BgpFields F;
  const int r = bgp_fields_ws(mask_window(wsm, q), len, F);
  if (r != 1) return false;
  const uint32_t toklen = F.a1 - F.a0;
  if (toklen > 16 || F.s1 - F.s0 > 12 || F.e1 - F.e0 > 12) return false;
  const uint32_t b = q + HB;
  bool ok = true;
  uint32_t d1, d2, d3;
  lds12_end(buf, b + F.s1, d1, d2, d3);
  L.start = bgp_digits_rc(d1, d2, d3, (int)(F.s1 - F.s0), ok);
  lds12_end(buf, b + F.e1, d1, d2, d3);
  L.end = bgp_digits_rc(d1, d2, d3, (int)(F.e1 - F.e0), ok);
  uint64_t lo, hi;
  if (short8) {
    if (toklen > 8) return false;
    lo = lds8(buf, b + F.a0);
    hi = 0;
  } else {
    lds16(buf, b + F.a0, lo, hi);
  }
  if (toklen < 16) {
    if (toklen <= 8) {
      hi = 0;
      lo = toklen == 8 ? lo : (lo & ((1ull << (8 * toklen)) - 1));
    } else {
      hi &= (1ull << (8 * (toklen - 8))) - 1;
    }
  }
  L.tlo = lo;
  L.thi = hi;
  L.toklen = toklen;
  L.rest = F.e1;
  return ok;
}

// BED5 fast path: "<ws> id <ws> score" after the end field, score a plain unsigned
// integer of <= 12 digits followed by whitespace or the line end (the common bedmap map
// file); anything else (signs, decimals, exponents, long fields) takes the byte path.
// q: local line start, len: line length, e1: end of the `end` digits (line-relative).
__device__ __forceinline__ bool parse_score_fast(const uint8_t* buf, const uint32_t* wsm,
                                                 const uint32_t* dgm, uint32_t q, uint32_t len,
                                                 uint32_t e1, double& score) {
  uint32_t WS = mask_window(wsm, q + e1), DG = mask_window(dgm, q + e1);
  const uint32_t l2 = len - e1;  // bytes from e1 to the line end
  if (l2 < 32) {                 // bytes past the line end act as whitespace
    const uint32_t endm = ~0u << l2;
    WS |= endm;
    DG &= ~endm;
  }
  if (!(WS & 1u)) return false;  // the end digits must be followed by whitespace
  const uint32_t NW = ~WS;
  if (!NW) return false;
  const uint32_t i0 = bgp_ctz(NW);  // id
  const uint32_t m1 = WS & (~0u << i0);
  if (!m1) return false;
  const uint32_t i1 = bgp_ctz(m1);
  if (i1 >= 31) return false;
  const uint32_t m2 = NW & (~0u << i1);
  if (!m2) return false;
  const uint32_t c0 = bgp_ctz(m2);  // score
  if (c0 >= l2 || !((DG >> c0) & 1u)) return false;
  const uint32_t m3 = ~DG & (~0u << c0);
  if (!m3) return false;
  const uint32_t c1 = bgp_ctz(m3);
  if (!((WS >> c1) & 1u) || c1 - c0 > 12) return false;  // digits end at whitespace / line end
  uint32_t d1, d2, d3;
  lds12_end(buf, q + HB + e1 + c1, d1, d2, d3);
  score = (double)bgp_digits_r(d1, d2, d3, (int)(c1 - c0));
  return true;
}

// runs that can occur in each tile of TB bytes: [runlo, runhi] by position
template <int TB = TT>
__global__ void k_run_range(RunTable R, uint32_t ntiles, uint32_t* __restrict__ runlo,
                            uint32_t* __restrict__ runhi) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  runlo[t] = run_of(R, (int64_t)t * TB, 0, R.n - 1);
  runhi[t] = run_of(R, (int64_t)t * TB + TB - 1, 0, R.n - 1);
}

// keys (+ rest span / score) of one parsed row; false if the chromosome does not match
// the run the row's position falls in (unsorted input)
__device__ __forceinline__ void emit_row(const RunTable& R, uint32_t run, int64_t ls, uint64_t r,
                                         uint64_t start, uint64_t end, int64_t* KS, int64_t* KE,
                                         bg_dstatus* st, int64_t& key, int64_t& mlen) {
  if (R.info[run].pos == ls) R.row[run] = r;
  if (end > BG_KEY_COORD_MAX || start > end) bg_report(st, r, ERR_RANGE);
  if (start == end) atomicOr(&st->flags, 2ULL);
  mlen = max(mlen, (int64_t)(end - start));
  const int64_t g = (int64_t)R.info[run].gid << BG_KEY_SHIFT;
  key = g | (int64_t)(start & BG_COORD_MASK);
  KS[r] = key;
  KE[r] = g | (int64_t)(end & BG_COORD_MASK);
}

// one tile staged in LDS with its class bitmaps
struct ParseBuf {
  __attribute__((aligned(16))) uint8_t buf[LBUF];
  uint32_t wsm[TT / 32 + HA / 32 + 1];  // class bitmaps: bit = byte
  uint32_t dgm[TT / 32 + HA / 32 + 1];
  uint32_t hnl;  // first '\n' in the halo after the tile (local offset)
};
// shared LDS of the parse kernels (NB staged tiles)
template <int NB>
struct ParseLdsT {
  ParseBuf b[NB];
  uint16_t lst[LCAP + 1];
  uint32_t shs[BG_NT / 64 + 1];
};

// the halo words of B's bitmaps start empty (LDS atomics in prologue_core), hnl unset
__device__ __forceinline__ void clear_halo(ParseBuf& B) {
  if (threadIdx.x == 0) B.hnl = ~0u;
  if (threadIdx.x < 2 * ((HA + 32) / 32)) {
    if (threadIdx.x < (HA + 32) / 32) B.wsm[TT / 32 + threadIdx.x] = 0;
    else B.dgm[TT / 32 + threadIdx.x - (HA + 32) / 32] = 0;
  }
}

// One tile's prologue once its bytes are in B.buf (and visible to every wave) and its
// halo words cleared: class bitmaps, line starts. v0/v1 = this thread's 32 tile bytes.
// Returns the number of owned lines L (> LCAP: error reported, caller returns); r0 = row
// of the first owned line; last_end = '\n' position ending the tile's last line.
__device__ __forceinline__ uint32_t prologue_core(const uint8_t* __restrict__ txt, uint64_t nb,
                                                  const uint64_t* __restrict__ row0, int64_t t0,
                                                  uint32_t tile, ParseBuf& B, uint16_t* lst,
                                                  uint32_t* shs, uint4 v0, uint4 v1, uint64_t& r0,
                                                  int64_t& last_end, bg_dstatus* st) {
  {  // classify this thread's 32 bytes once (SWAR), publish the masks
    const uint32_t W[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    uint32_t ws, dg;
    bgp_classify8(W, ws, dg);
    B.wsm[threadIdx.x] = ws;
    B.dgm[threadIdx.x] = dg;
  }
  {  // the halo after the tile, from its LDS copy: one dword per thread (72 threads), the
     // 4-bit groups merged into the mask words with LDS atomics
    constexpr uint32_t HD = (HA + 32) / 4;
    if (threadIdx.x < HD) {
      const uint32_t x = reinterpret_cast<const uint32_t*>(&B.buf[HB + TT])[threadIdx.x];
      uint32_t w4, d4;
      bgp_classify(x, w4, d4);
      const uint32_t sh = 4 * (threadIdx.x & 7);
      if (w4) atomicOr(&B.wsm[TT / 32 + threadIdx.x / 8], w4 << sh);
      if (d4) atomicOr(&B.dgm[TT / 32 + threadIdx.x / 8], d4 << sh);
      const uint32_t m = nl_mask4(x);
      if (m) atomicMin(&B.hnl, TT + 4 * threadIdx.x + (__ffs(m) - 1) / 8);
    }
  }
  bool has0;
  const uint32_t L = tile_line_starts(v0, v1, B.buf, t0, lst, LCAP + 1, shs, has0);
  r0 = (row0 ? row0[tile] : 0) + (has0 ? 0 : 1);  // row of the first owned line (if known)
  if (L > LCAP) {  // > LCAP lines in 8 KiB: some line is shorter than any valid record
    if (threadIdx.x == 0) bg_report(st, r0, ERR_PARSE);
    return L;
  }
  // end of the tile's last line: the tile's last byte, the halo, or further on
  TileText T{txt, B.buf, t0 - HB, t0 + TT + HA, nb};
  last_end = L == 0 ? -1
             : (B.buf[HB + TT - 1] == '\n') ? t0 + TT - 1
             : (B.hnl != ~0u ? t0 + B.hnl : find_nl(T, t0 + TT + HA + 32));
  return L;
}

// prologue of a tile loaded into registers (load_tile); the LDS must be free
template <int NB>
__device__ __forceinline__ uint32_t tile_prologue(const uint8_t* __restrict__ txt, uint64_t nb,
                                                  const uint64_t* __restrict__ row0, int64_t t0,
                                                  uint32_t tile, ParseLdsT<NB>& S, ParseBuf& B,
                                                  const TileRegs& TR, uint64_t& r0,
                                                  int64_t& last_end, bg_dstatus* st) {
  clear_halo(B);
  store_tile(B.buf, TR);
  __syncthreads();
  return prologue_core(txt, nb, row0, t0, tile, B, S.lst, S.shs, TR.v0, TR.v1, r0, last_end, st);
}

__global__ void __launch_bounds__(BG_NT) k_parse(
    const uint8_t* __restrict__ txt, uint64_t nb, uint64_t nrows, const uint64_t* __restrict__ row0,
    const uint32_t* __restrict__ runlo, const uint32_t* __restrict__ runhi,
    int kind, RunTable R, int64_t* __restrict__ KS, int64_t* __restrict__ KE,
    uint64_t* __restrict__ rest_off, uint32_t* __restrict__ rest_len, double* __restrict__ score,
    bg_dstatus* st, uint64_t* __restrict__ big, uint32_t bigcap) {
  __shared__ ParseLdsT<1> S;
  __shared__ int64_t lkey[LCAP];
  uint8_t* buf = S.b[0].buf;
  const uint16_t* lst = S.lst;
  const uint32_t* wsm = S.b[0].wsm;
  const uint32_t* dgm = S.b[0].dgm;
  const int64_t t0 = (int64_t)blockIdx.x * TT;
  const int64_t PENDING = LLONG_MIN + 1;  // lkey of a line left to the byte path
  uint64_t r0;
  int64_t last_end;
  TileRegs TR;
  load_tile(txt, nb, t0, TR);
  const uint32_t L = tile_prologue(txt, nb, row0, t0, blockIdx.x, S, S.b[0], TR, r0, last_end, st);
  if (L > LCAP) return;
  const uint32_t rl = runlo[blockIdx.x], rh = runhi[blockIdx.x];  // runs in this tile
  TileText T{txt, buf, t0 - HB, t0 + TT + HA, nb};
  int64_t mlen = 0;  // longest row of this thread (window bound of bedmap / closest)
  // hot loop: BED3 / BED3+rest lines decided by the masks; the rest is queued
  for (uint32_t k = threadIdx.x; k < L; k += BG_NT) {
    const int64_t ls = t0 + lst[k];
    const uint64_t r = r0 + k;
    int64_t key = LLONG_MIN;
    const int64_t le = (k + 1 < L) ? t0 + lst[k + 1] - 1 : last_end;
    // r >= nrows: the unterminated last line (dropped like the reference)
    if (r < nrows && le >= 0) {
      Fast F;
      const uint32_t run = (rl == rh) ? rl : run_of(R, ls, rl, rh);
      const RunInfo& I = R.info[run];
      double sc = 0;
      if (parse_line_fast(buf, wsm, dgm, lst[k], (uint32_t)(le - ls), F, I.tlen <= 8) &&
          F.toklen == I.tlen && F.tlo == I.tlo && F.thi == I.thi &&
          (kind != BG_BED5 ||
           parse_score_fast(buf, wsm, dgm, lst[k], (uint32_t)(le - ls), F.rest, sc))) {
        emit_row(R, run, ls, r, F.start, F.end, KS, KE, st, key, mlen);
        if (rest_off) {
          rest_off[r] = (uint64_t)(ls + F.rest);
          rest_len[r] = (uint32_t)(le - ls - F.rest);
        }
        if (score) score[r] = sc;
      } else {
        key = PENDING;
      }
    }
    lkey[k] = key;
  }
  // cold loop: the full grammar, byte by byte (BED5, long tokens, odd spacing, errors);
  // same line-to-thread mapping, so no barrier is needed before it
  for (uint32_t k = threadIdx.x; k < L; k += BG_NT) {
    if (lkey[k] != PENDING) continue;
    lkey[k] = LLONG_MIN;
    const int64_t ls = t0 + lst[k];
    const uint64_t r = r0 + k;
    const int64_t le = (k + 1 < L) ? t0 + lst[k + 1] - 1 : last_end;
    Line Ln;
    parse_line_slow(T, ls, le, kind, Ln);
    if (Ln.err) {
      if (Ln.err == ERR_BLANK) atomicAdd(&st->nblank, 1ULL);
      bg_report(st, r, Ln.err);
      KS[r] = KE[r] = 0;
      continue;
    }
    const uint32_t run = (rl == rh) ? rl : run_of(R, ls, rl, rh);
    if (Ln.hash != R.info[run].hash) {  // a chromosome outside the run order: unsorted input
      bg_report(st, r, ERR_UNSORTED);
      continue;
    }
    int64_t key;
    emit_row(R, run, ls, r, Ln.start, Ln.end, KS, KE, st, key, mlen);
    lkey[k] = key;
    if (rest_off) {
      rest_off[r] = (uint64_t)Ln.rest;
      rest_len[r] = (uint32_t)(le - Ln.rest);
    }
    if (score) {
      score[r] = Ln.score;
      if (Ln.scoreint <= 0) atomicOr(&st->flags, 1ULL);
      if (Ln.scoreint < 0) big_push(st, big, bigcap, r, Ln.spos);
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) mlen = max(mlen, (int64_t)__shfl_xor(mlen, d, 64));
  // the running max settles within the first blocks: atomics only when it grows
  if (bg_lane() == 0 && mlen > *(volatile long long*)&st->maxlen) atomicMax(&st->maxlen, (long long)mlen);
  __syncthreads();
  for (uint32_t k = threadIdx.x + 1; k < L; k += BG_NT)
    if (lkey[k] != LLONG_MIN && lkey[k - 1] != LLONG_MIN && lkey[k] < lkey[k - 1])
      bg_report(st, r0 + k, ERR_UNSORTED);
}

// sort order across tile boundaries: the first rows of each tile vs their predecessors
__global__ void k_check_bounds(const int64_t* __restrict__ KS, const uint64_t* __restrict__ row0,
                               uint32_t ntiles, uint64_t nrows, bg_dstatus* st) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  const uint64_t r = row0[t];
  for (uint64_t q = r; q < r + 2 && q < nrows; ++q)
    if (q > 0 && KS[q] < KS[q - 1]) bg_report(st, q, ERR_UNSORTED);
}

// -------------------------------------------------------------------------------------
// BG_BED3_SET: parse straight to the file's merged set (components), no row columns.
//
// The file's components are what every set operation reads (mergeOverlap /
// getNextFileMergedCoords, Bedops.cpp:792-814,865-886): row i opens a component iff
// ks[i] > max(ke[0..i-1]). k_parse_set_v parses a 4 KiB sub-tile (one line per lane per round
// of 64 lines, in line order), and with wave max-scans finds the sub-tile's LOCAL
// components (running max started at -inf), written to a staging area at the tile's
// first row index (a tile has at least as many rows as local components). k_set_count /
// k_set_write then apply the running max M of all earlier tiles: local components that
// start at or below M merge into the component open on entry (a prefix of them, the
// starts being increasing), the rest are global components. Row keys never reach HBM:
// per 100M-row file this writes ~0.5 GB of staged components instead of 1.6 GB of keys
// and drops the separate tile-max / components passes over those keys.
// -------------------------------------------------------------------------------------
struct SetTiles {
  int64_t* tmax;   // max ke of the tile's rows (LLONG_MIN: none)
  int64_t* tlast;  // max ks of the tile's rows (LLONG_MIN: none)
  uint64_t* base;  // staging index of the tile's first local component (= its first row)
  uint64_t* nloc;  // local components of the tile
  uint32_t* absorbed;  // local components merged into the component open on entry
  uint64_t* nrow;  // rows of the tile
  // staging form of the tile: >= 0, a tile inside one chromosome run whose local components
  // are staged as 32-bit coordinates (LCS/LCE of the tile's slots read as uint32, half the
  // bytes) under this key prefix; -1, 64-bit keys
  int64_t* gb;
};
// key of local component i of tile t (start: LCS, end: LCE), either staging form
__device__ __forceinline__ int64_t set_key(const int64_t* X, uint64_t b, int64_t gb, uint64_t i) {
  return gb >= 0 ? (gb | (int64_t)reinterpret_cast<const uint32_t*>(X + b)[i]) : X[b + i];
}

// one line -> keys; false if the line is not a row (dropped tail, blank, error: reported).
// Row numbers are not known here (no scout pass): errors are reported as row 0 and
// bg_load re-reads the input with its row columns to report the exact line.
// ONE: the tile lies inside one chromosome run (rl == rh), so the run and its token are
// workgroup-uniform (scalar loads, no per-lane run search)
template <bool ONE = false, bool WSO = false, typename BufT = ParseBuf>
__device__ __forceinline__ bool set_row(const BufT& B, const uint16_t* lst, const TileText& T,
                                        const RunTable& R, uint32_t rl, uint32_t rh, int64_t t0,
                                        uint32_t k, uint32_t L, int64_t last_end, int64_t& ks,
                                        int64_t& ke, bg_dstatus* st) {
  const int64_t ls = t0 + lst[k];
  const int64_t le = (k + 1 < L) ? t0 + lst[k + 1] - 1 : last_end;
  if (le < 0) return false;  // the unterminated last line (dropped, Bed.hpp:244-255 + feof)
  const uint32_t run = ONE ? rl : ((rl == rh) ? rl : run_of(R, ls, rl, rh));
  const RunInfo& I = R.info[run];
  uint64_t start, end;
  Fast F;
  bool fast;
  if constexpr (WSO) fast = parse_line_fast_ws(B.buf, B.wsm, lst[k], (uint32_t)(le - ls), F, I.tlen <= 8);
  else fast = parse_line_fast(B.buf, B.wsm, B.dgm, lst[k], (uint32_t)(le - ls), F, I.tlen <= 8);
  if (fast && F.toklen == I.tlen && F.tlo == I.tlo && F.thi == I.thi) {
    start = F.start;
    end = F.end;
  } else {
    Line Ln;
    parse_line_slow(T, ls, le, BG_BED3, Ln);
    if (Ln.err) {
      bg_report(st, 0, Ln.err);
      return false;
    }
    if (Ln.hash != I.hash) {  // a chromosome outside the run order: unsorted input
      bg_report(st, 0, ERR_UNSORTED);
      return false;
    }
    start = Ln.start;
    end = Ln.end;
  }
  if (end > BG_KEY_COORD_MAX || start > end) bg_report(st, 0, ERR_RANGE);
  if (start == end) atomicOr(&st->flags, 2ULL);
  const int64_t g = (int64_t)I.gid << BG_KEY_SHIFT;
  ks = g | (int64_t)(start & BG_COORD_MASK);
  ke = g | (int64_t)(end & BG_COORD_MASK);
  return true;
}

// 64-bit DPP lane moves and the wave-wide (64-lane) inclusive max scan built from them:
// row_shr 1/2/4/8 inside each 16-lane row, then row_bcast 15/31 across rows (gfx9 DPP;
// lanes with no source read 0, the identity of these unsigned scans)
template <int CTRL, int RMASK, bool BC>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, RMASK, 0xF, BC);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, RMASK, 0xF, BC);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t wave_incl_max_u64(uint64_t v) {
  v = max(v, dpp64<0x111, 0xF, true>(v));
  v = max(v, dpp64<0x112, 0xF, true>(v));
  v = max(v, dpp64<0x114, 0xF, true>(v));
  v = max(v, dpp64<0x118, 0xF, true>(v));
  v = max(v, dpp64<0x142, 0xA, false>(v));
  v = max(v, dpp64<0x143, 0xC, false>(v));
  return v;
}
__device__ __forceinline__ uint64_t wave_shr1_u64(uint64_t v) { return dpp64<0x138, 0xF, true>(v); }

// Keys inside the round loop are shifted by one, K = ks + 1 and E = ke + 1 (valid keys are
// >= 0), so 0 means "no row" and is the identity of every max below.
// BG_BED3_SET staging: local components of sub-tile t go to slots [t * SCAP_W, (t + 1) * SCAP_W).
// A sub-tile with more than SCAP_W (4 KiB of rows shorter than 16 bytes, almost all
// disjoint) sets BG_SET_OVERFLOW and bg_load re-reads that input with its row columns (BG_BED3).
#define BG_SET_OVERFLOW 8ULL  // bg_dstatus.flags bit
#define BG_ROW_OVERFLOW 16ULL  // k_parse_rv: a sub-tile of more than LCAP_R lines

__device__ __forceinline__ uint32_t wave_incl_max_u32(uint32_t v) {
  v = max(v, dpp32<0x111, 0xF, true>(v));
  v = max(v, dpp32<0x112, 0xF, true>(v));
  v = max(v, dpp32<0x114, 0xF, true>(v));
  v = max(v, dpp32<0x118, 0xF, true>(v));
  v = max(v, dpp32<0x142, 0xA, false>(v));
  v = max(v, dpp32<0x143, 0xC, false>(v));
  return v;
}
__device__ __forceinline__ uint32_t wave_incl_max_v(uint32_t v) { return wave_incl_max_u32(v); }
__device__ __forceinline__ uint64_t wave_incl_max_v(uint64_t v) { return wave_incl_max_u64(v); }
__device__ __forceinline__ uint32_t wave_shr1_v(uint32_t v) { return dpp32<0x138, 0xF, true>(v); }
__device__ __forceinline__ uint64_t wave_shr1_v(uint64_t v) { return wave_shr1_u64(v); }


// parse_score_fast from the whitespace mask alone: the score's bytes are checked to be
// digits while they are converted (bgp_digits_rc)
__device__ __forceinline__ bool parse_score_fast_ws(const uint8_t* buf, const uint32_t* wsm, uint32_t q,
                                                    uint32_t len, uint32_t e1, double& score, bool& isint) {
  uint32_t WS = mask_window(wsm, q + e1);
  const uint32_t l2 = len - e1;  // bytes from e1 to the line end
  if (l2 < 32) WS |= ~0u << l2;  // bytes past the line end act as whitespace
  if (!(WS & 1u)) return false;  // the end digits must be followed by whitespace
  const uint32_t NW = ~WS;
  if (!NW) return false;
  const uint32_t i0 = bgp_ctz(NW);  // id
  const uint32_t m1 = WS & (~0u << i0);
  if (!m1) return false;
  const uint32_t i1 = bgp_ctz(m1);
  if (i1 >= 31) return false;
  const uint32_t m2 = NW & (~0u << i1);
  if (!m2) return false;
  const uint32_t c0 = bgp_ctz(m2);  // score
  if (c0 >= l2) return false;
  const uint32_t m3 = WS & (~0u << c0);
  if (!m3) return false;
  const uint32_t c1 = bgp_ctz(m3);  // whitespace or the line end after the score
  uint32_t d1, d2, d3;
  bool ok = c1 - c0 <= 12;
  if (ok) {
    lds12_end(buf, q + HB + e1 + c1, d1, d2, d3);
    const uint64_t v = bgp_digits_rc(d1, d2, d3, (int)(c1 - c0), ok);
    score = (double)v;
    if (ok) return true;
  }
  // a decimal "<int digits>.<fraction digits>" (the common bedmap signal column): the value is
  // m / 10^f with m < 2^53 and f <= 12, one correctly rounded division of exact operands —
  // parse_score's result (Clinger's fast path), with its trailing-zero rule; a non-integer
  // clears `isint` (st->flags bit 0, as the byte path sets it). Anything else: the byte path.
  if (c1 - c0 > 20) return false;
  uint64_t lo, hi;
  lds16(buf, q + HB + e1 + c0, lo, hi);
  const uint64_t x = lo ^ 0x2e2e2e2e2e2e2e2eull, y = hi ^ 0x2e2e2e2e2e2e2e2eull;
  const uint64_t zx = (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
  const uint64_t zy = (y - 0x0101010101010101ull) & ~y & 0x8080808080808080ull;
  if (!zx && !zy) return false;
  const uint32_t dot = zx ? (uint32_t)__builtin_ctzll(zx) / 8 : 8 + (uint32_t)__builtin_ctzll(zy) / 8;
  const uint32_t ni = dot, nf = c1 - c0 - dot - 1;  // integer / fraction digits
  if (ni < 1 || ni > 12 || nf < 1 || nf > 12 || ni + nf > 19 || dot >= c1 - c0) return false;
  ok = true;
  lds12_end(buf, q + HB + e1 + c0 + dot, d1, d2, d3);
  const uint64_t vi = bgp_digits_rc(d1, d2, d3, (int)ni, ok);
  lds12_end(buf, q + HB + e1 + c1, d1, d2, d3);
  const uint64_t vf = bgp_digits_rc(d1, d2, d3, (int)nf, ok);
  if (!ok) return false;
  const double* const P10 = BG_P10;
  uint64_t m = vi * (uint64_t)P10[nf] + vf;
  int pw = -(int)nf;
  while (pw < 0 && m != 0 && m % 10 == 0) {
    m /= 10;
    ++pw;
  }
  if (m > (1ULL << 53)) return false;
  if (m == 0 || pw == 0) {  // "0.000", "12.000": integers (parse_score: isint, +0.0)
    score = (double)m;
    return true;
  }
  score = (double)m / P10[-pw];
  isint = false;
  return true;
}

// ---- BG_BED3_SET: one wavefront per 4 KiB sub-tile -------------------------------------
// A tile of TW = 4 KiB owned by ONE wave (64 lanes x 64 bytes): every exchange between lines
// (line-start counts, the per-round max of ends, the last key, the opening counts) is a DPP
// step or a readlane into a scalar register, and the workgroup barriers compile to nothing
// (the workgroup is one wave). Sub-tile u stages its local components in slots
// [u * SCAP_W, u * SCAP_W + SCAP_W) and has its own SetTiles entry: k_set_count /
// k_set_write treat sub-tiles as tiles. (Rounds 2-4 kernels with 8 KiB tiles of 128/256
// threads and the round-4 wave kernel measured 1.51 / 1.23 / 1.19 ms per file against 0.92
// for k_parse_set_v and were removed in round 6.)
#define TW 4096
#define SCAP_W 256
#define LCAP_W 512  // lines per sub-tile (4 KiB of lines averaging >= 8 bytes; more: refused)

__device__ __forceinline__ uint32_t wave_readlane(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t wave_readlane(uint64_t v, int l) {
  return ((uint64_t)wave_readlane((uint32_t)(v >> 32), l) << 32) | wave_readlane((uint32_t)v, l);
}

// the rounds of one sub-tile: 64 lines per round, one per lane, in line order (V as
// k_parse_rv's rows). kl: K (+1 form) of the sub-tile's largest row key.
template <typename V, typename LdsT>
__device__ __forceinline__ void set_rounds_w(const LdsT& S, const TileText& T, const RunTable& R,
                                             uint32_t rl, uint32_t rh, int64_t t0, uint32_t L,
                                             int64_t last_end, int64_t gbase, uint64_t base,
                                             int64_t* __restrict__ LCS, int64_t* __restrict__ LCE,
                                             uint64_t& nc, V& carry_e, V& kl, bg_dstatus* st) {
  constexpr bool NARROW = sizeof(V) == 4;
  const int lane = threadIdx.x;
  const uint64_t lt = (1ULL << lane) - 1;
  V carry_k = 0;
  const uint32_t rounds = (L + 63) / 64;
  for (uint32_t j = 0; j < rounds; ++j) {
    const uint32_t k = j * 64 + lane;
    int64_t ks = 0, ke = 0;
    const bool valid = k < L && set_row<NARROW, true>(S, S.lst, T, R, rl, rh, t0, k, L, last_end, ks, ke, st);
    V K = 0, E = 0;
    if (valid) {
      if (NARROW) {
        const uint64_t ce = (uint64_t)(ke & BG_COORD_MASK) + 1;
        if (ce >= 0xFFFFFFFFull) atomicOr(&st->flags, BG_SET_OVERFLOW);
        K = (V)((uint64_t)(ks & BG_COORD_MASK) + 1);
        E = (V)ce;
      } else {
        K = (V)ks + 1;
        E = (V)ke + 1;
      }
    }
    const V ie = wave_incl_max_v(E);
    const V pk = wave_shr1_v(K);  // with every lane active: a DPP move reads 0 from a masked lane
    const V prevK = lane ? pk : carry_k;
    if (valid && prevK && K < prevK) bg_report(st, 0, ERR_UNSORTED);
    const V ex_e = max(carry_e, wave_shr1_v(ie));
    const bool open = valid && K > ex_e;
    const uint64_t bal = __ballot(open);
    const uint64_t pos = nc + __popcll(bal & lt);
    if (open && pos < SCAP_W) {
      if (NARROW) {
        reinterpret_cast<uint32_t*>(LCS + base)[pos] = (uint32_t)(K - 1);
        if (pos > 0) reinterpret_cast<uint32_t*>(LCE + base)[pos - 1] = (uint32_t)(ex_e - 1);
      } else {
        LCS[base + pos] = ks;
        if (pos > 0) LCE[base + pos - 1] = gbase | (int64_t)(ex_e - 1);
      }
    }
    if (j + 1 == rounds) {  // the largest K: the last line's, or the one before when the last
                            // line is the file's dropped unterminated tail
      const int ll = (int)(L - 1 - j * 64);
      const V k1 = wave_readlane(K, ll);
      kl = k1 ? k1 : (ll > 0 ? wave_readlane(K, ll - 1) : carry_k);
    }
    carry_e = max(carry_e, wave_readlane(ie, 63));
    carry_k = wave_readlane(K, 63);
    nc += (uint64_t)__popcll(bal);
  }
}


// ---- k_parse_set_v (round 5): the set parse with a lean common path ---------------------
// The SQ counters of round 4's wave kernel (profiles/r04_sq_k_parse_set_w.txt: 1294 VALU + 504
// SALU per 4 KiB wave) and its ISA (64-bit address arithmetic, compares and masks, guarded
// byte-loop loads, funnel shifts for every unaligned LDS word) set what this kernel removes.
// On the common path — a
// sub-tile inside one chromosome run (rl == rh) whose lines are "<token> <start> <end>[...]"
// within their first 32 bytes, the token the run's, both numbers of at most 9 digits —
// every step is 32-bit:
//  - the global loads are unguarded when the sub-tile and its halos lie inside the text (a
//    wave-uniform test; only the file's first and last sub-tiles take load16);
//  - '\n' classes two dwords per multiply (the whitespace gather of bgp_ws8);
//  - lst[L] holds the last line's end, so a line's start and end come from ONE unaligned
//    32-bit LDS read of lst[k], lst[k+1];
//  - fields from the transitions of the line's whitespace window (starts = non-ws after ws,
//    ends = ws after non-ws: three ffbl + clear-lowest each) instead of a chain of masks;
//  - the window, the token and each number's last 12 bytes read from LDS as aligned dwords
//    funnelled by alignbyte (ldsu*: unaligned ds_reads stalled the LDS pipe);
//  - a number of <= 9 digits converts with two byte dot products per dword and 24-bit
//    multiply-adds (< 10^9 < 2^32);
//  - the token compared under the run's length mask (uniform).
// Any other line (longer fields, signs, errors, the dropped unterminated tail) takes set_row,
// the full grammar, in its own lane; sub-tiles over a chromosome change run set_rounds_w.

// v_ffbl_b32 itself: the lowest set bit's index, 0xFFFFFFFF for 0 (no select for the zero case)
__device__ __forceinline__ uint32_t ffbl_hw(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// Byte classes without v_mul_lo_u32 (a quarter-rate instruction): bit 7 of each byte is the
// byte's flag, v_bitop3_b32 merges the SWAR terms (truth tables as f(0xF0, 0xCC, 0xAA) over
// the operands S0, S1, S2), and byte dot products gather the flags of two dwords into 8 bits.
#define BOP3_A 0xF0u
#define BOP3_B 0xCCu
#define BOP3_C 0xAAu
// whitespace {' ', 0x09..0x0D} (bgp_ws80 in 7 operations)
__device__ __forceinline__ uint32_t ws80_v(uint32_t x) {
  const uint32_t lo7 = x & 0x7F7F7F7Fu;
  const uint32_t nz20 = (lo7 ^ 0x20202020u) + 0x7F7F7F7Fu;  // bit 7: byte != ' '
  const uint32_t ge9 = lo7 + 0x77777777u, ge14 = lo7 + 0x72727272u;
  const uint32_t f = __builtin_amdgcn_bitop3_b32(nz20, ge9, ge14, (~BOP3_A | (BOP3_B & ~BOP3_C)) & 0xFFu);
  return __builtin_amdgcn_bitop3_b32(f, x, 0x80808080u, (BOP3_A & ~BOP3_B & BOP3_C) & 0xFFu);
}
// '\n' (nl_mask4 in 3 operations; bit 7 of x ^ 0x0A is bit 7 of x)
__device__ __forceinline__ uint32_t nl80_v(uint32_t x) {
  const uint32_t t = __builtin_amdgcn_bitop3_b32(x, 0x0A0A0A0Au, 0x7F7F7F7Fu, ((BOP3_A ^ BOP3_B) & BOP3_C) & 0xFFu) +
                     0x7F7F7F7Fu;
  return __builtin_amdgcn_bitop3_b32(t, x, 0x80808080u, (~BOP3_A & ~BOP3_B & BOP3_C) & 0xFFu);
}
// bit-7 flags of two dwords -> their 8 flags (a's bytes, then b's) times 128
__device__ __forceinline__ uint32_t gather8x128(uint32_t fa, uint32_t fb) {
  return __builtin_amdgcn_udot4(fb, 0x80402010u, __builtin_amdgcn_udot4(fa, 0x08040201u, 0u, false), false);
}
// 32 bytes -> whitespace mask and '\n' mask (bit j = byte j)
__device__ __forceinline__ void classify32(const uint4 a, const uint4 b, uint32_t& ws, uint32_t& nl) {
  const uint32_t w0 = gather8x128(ws80_v(a.x), ws80_v(a.y)), w1 = gather8x128(ws80_v(a.z), ws80_v(a.w));
  const uint32_t w2 = gather8x128(ws80_v(b.x), ws80_v(b.y)), w3 = gather8x128(ws80_v(b.z), ws80_v(b.w));
  ws = (w0 >> 7) | (w1 << 1) | (w2 << 9) | (w3 << 17);
  const uint32_t n0 = gather8x128(nl80_v(a.x), nl80_v(a.y)), n1 = gather8x128(nl80_v(a.z), nl80_v(a.w));
  const uint32_t n2 = gather8x128(nl80_v(b.x), nl80_v(b.y)), n3 = gather8x128(nl80_v(b.z), nl80_v(b.w));
  nl = (n0 >> 7) | (n1 << 1) | (n2 << 9) | (n3 << 17);
}
// 16 bytes -> 16-bit masks
__device__ __forceinline__ void classify16(const uint4 a, uint32_t& ws, uint32_t& nl) {
  ws = (gather8x128(ws80_v(a.x), ws80_v(a.y)) >> 7) | (gather8x128(ws80_v(a.z), ws80_v(a.w)) << 1);
  nl = (gather8x128(nl80_v(a.x), nl80_v(a.y)) >> 7) | (gather8x128(nl80_v(a.z), nl80_v(a.w)) << 1);
}

struct LdsU3 {
  uint32_t x, y, z;
};
// unaligned LDS reads as aligned dwords + alignbyte (one extra ds_read per window, no
// LDS_UNALIGNED_STALL: k_parse_set_v 0.99 -> 0.92 ms, round 5, against unaligned ds_reads)
template <int N>
__device__ __forceinline__ void lds_words(const void* p, uint32_t* o) {
  // (the aligned address by pointer arithmetic on p, not an integer round trip: the compiler
  // keeps p's LDS address space and emits ds_read, not flat loads)
  const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
  const uint32_t* d = reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(p) - sh);
  uint32_t w[N + 1];
#pragma unroll
  for (int i = 0; i <= N; ++i) w[i] = d[i];
#pragma unroll
  for (int i = 0; i < N; ++i) o[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
}
__device__ __forceinline__ uint32_t ldsu32(const void* p) {
  uint32_t o[1];
  lds_words<1>(p, o);
  return o[0];
}
__device__ __forceinline__ uint2 ldsu64(const void* p) {
  uint32_t o[2];
  lds_words<2>(p, o);
  return make_uint2(o[0], o[1]);
}
__device__ __forceinline__ LdsU3 ldsu96(const void* p) {
  uint32_t o[3];
  lds_words<3>(p, o);
  return LdsU3{o[0], o[1], o[2]};
}
__device__ __forceinline__ uint4 ldsu128(const void* p) {
  uint32_t o[4];
  lds_words<4>(p, o);
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// (every sub-tile is staged in LDS: reading interior sub-tiles' line bytes from the text
// itself was timed within +-3% but read 4.21 GB per launch against 2.95 GB staged, round 5)
// the value of a number of L (1..9) digits whose last digit is the high byte of D.z (the 12
// bytes D end at the number's end); ok cleared when one of its bytes is not a digit
__device__ __forceinline__ uint32_t digits9(const LdsU3 D, uint32_t L, bool& ok) {
  const uint32_t u = 8u * (12u - L);                // bits before the number: 24..88
  const uint32_t sh = ~0u << (u & 31u);
  const uint32_t m1 = u < 32u ? sh : 0u;
  const uint32_t m2 = u < 32u ? ~0u : (u < 64u ? sh : 0u);
  const uint32_t m3 = u < 64u ? ~0u : sh;
  const uint32_t x1 = (D.x ^ 0x30303030u) & m1;     // digit values; bytes before the number 0
  const uint32_t x2 = (D.y ^ 0x30303030u) & m2;
  const uint32_t x3 = (D.z ^ 0x30303030u) & m3;
  const uint32_t bad = (x1 | ((x1 & 0x7F7F7F7Fu) + 0x76767676u)) | (x2 | ((x2 & 0x7F7F7F7Fu) + 0x76767676u)) |
                       (x3 | ((x3 & 0x7F7F7F7Fu) + 0x76767676u));
  ok = ok && (bad & 0x80808080u) == 0;
  // 10 * b0 + b1 and 10 * b2 + b3 of a dword by byte dot products; L <= 9: x1 holds one digit
  // (24-bit multiplies: full rate, every operand < 2^24)
  const uint32_t v2 = __builtin_amdgcn_udot4(x2, 0x010A0000u, __umul24(__builtin_amdgcn_udot4(x2, 0x0000010Au, 0u, false), 100u), false);
  const uint32_t v3 = __builtin_amdgcn_udot4(x3, 0x010A0000u, __umul24(__builtin_amdgcn_udot4(x3, 0x0000010Au, 0u, false), 100u), false);
  return __umul24(__umul24(x1 >> 24, 10000u) + v2, 10000u) + v3;
}

// k_parse_set_v's LDS: a 32-byte halo after the sub-tile (+32 bytes of padding the fast
// path's reads may touch) instead of 256, and at most 384 lines per 4 KiB (lines averaging
// under 10.7 bytes report ERR_PARSE and the load is redone with row columns): 5470 bytes
// instead of 5984, 29 waves per CU instead of 26 (LDS-bound residency). A last line whose
// '\n' lies past the halo is found by find_nl_wave (1 KiB per step).
#define HA_V 32
#define LCAP_V 384
struct ParseLdsV {
  __attribute__((aligned(16))) uint8_t buf[HB + TW + HA_V + 32];
  uint32_t wsm[TW / 32 + (HA_V + 32) / 32 + 1];
  uint16_t lst[LCAP_V + 1];
};

// first '\n' at or after `from` (-1: none before the end of the text), one wave, 1 KiB a step
__device__ __forceinline__ int64_t find_nl_wave(const uint8_t* __restrict__ txt, uint64_t nb, int64_t from) {
  const int lane = threadIdx.x & 63;
  for (int64_t b = from; b >= 0 && (uint64_t)b < nb; b += 1024) {
    const uint4 x = load16(txt, b + 16 * lane, nb);  // bytes past the text read as 0
    const uint32_t m = (gather8x128(nl80_v(x.x), nl80_v(x.y)) >> 7) | (gather8x128(nl80_v(x.z), nl80_v(x.w)) << 1);
    const uint64_t bal = __ballot(m != 0);
    if (bal) {
      const int f = __builtin_ctzll(bal);
      return b + 16 * f + __builtin_ctz(wave_readlane(m, f));
    }
  }
  return -1;
}

// what set_row / set_rounds_w read a sub-tile's lines through: its bytes from offset t0 - HB,
// whitespace masks and line starts (LDS)
struct SubView {
  const uint8_t* buf;
  const uint32_t* wsm;
  const uint16_t* lst;
};

// the sub-tile's bytes as registers: 64 per lane, and 16 of the halos (lanes < HL: after the
// sub-tile, lane 63: the 16 bytes before it); unguarded when the sub-tile and its halos lie
// inside the text (wave-uniform), load16 otherwise
#define HL_W ((HA_V + 32) / 16)
struct SubRegs {
  uint4 v[4];
  uint4 vh;
};
// (HAX: the staged halo after the sub-tile, + 32 bytes; k_parse_rv stages more than HA_V)
template <int HAX = HA_V>
__device__ __forceinline__ void load_sub(const uint8_t* __restrict__ txt, uint64_t nb, int64_t t0, SubRegs& R) {
  constexpr int HL = (HAX + 32) / 16;
  static_assert(HL % 2 == 0 && HL < 63, "halo lanes");
  const int lane = threadIdx.x & 63;
  uint4* const v = R.v;
  uint4& vh = R.vh;
  vh = make_uint4(0, 0, 0, 0);
  if (t0 >= HB && (uint64_t)t0 + TW + HAX + 32 <= nb) {  // wave-uniform: no guards
    const uint4* p = reinterpret_cast<const uint4*>(txt + t0) + 4 * lane;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = p[i];
    if (lane < HL) vh = reinterpret_cast<const uint4*>(txt + t0 + TW)[lane];
    else if (lane == 63) vh = *reinterpret_cast<const uint4*>(txt + t0 - HB);
  } else {
    const int64_t b = t0 + 64 * lane;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = load16(txt, b + 16 * i, nb);
    if (lane < HL) vh = load16(txt, t0 + TW + 16 * lane, nb);
    else if (lane == 63) vh = load16(txt, t0 - HB, nb);
  }
}

// LDS order inside one wave (k_parse_rv: two waves per workgroup, each with its own LDS
// block): the wave's LDS operations complete in order, so a code-motion barrier suffices
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// prologue of k_parse_set_v: prologue_w from the registers of load_sub, with the cheaper
// '\n' classes and lst[L] = the last line's end + 1 (0xFFFF: none or out of reach).
// ROWS (k_parse_rv): more than CAP lines set BG_ROW_OVERFLOW (the load is redone with
// k_parse) instead of ERR_PARSE, and the waves of the workgroup do not wait for each other
template <typename LdsT = ParseLdsV, uint32_t CAP = LCAP_V, bool ROWS = false, int HAX = HA_V>
__device__ __forceinline__ uint32_t prologue_v(const uint8_t* __restrict__ txt, uint64_t nb, int64_t t0,
                                               const SubRegs& R, LdsT& S, int64_t& last_end,
                                               bg_dstatus* st) {
  constexpr int HL = (HAX + 32) / 16;
  const int lane = threadIdx.x & 63;
  const uint4* const v = R.v;
  const uint4 vh = R.vh;
#pragma unroll
  for (int i = 0; i < 4; ++i) *reinterpret_cast<uint4*>(&S.buf[HB + 64 * lane + 16 * i]) = v[i];
  if (lane < HL) *reinterpret_cast<uint4*>(&S.buf[HB + TW + 16 * lane]) = vh;
  else if (lane == 63) *reinterpret_cast<uint4*>(&S.buf[0]) = vh;
  uint32_t w0, w1, n0, n1, hw, hm;
  classify32(v[0], v[1], w0, n0);
  classify32(v[2], v[3], w1, n1);
  classify16(vh, hw, hm);
  *reinterpret_cast<uint2*>(&S.wsm[2 * lane]) = make_uint2(w0, w1);
  {
    const uint32_t hn = __shfl_down(hw, 1, 64);
    if (lane < HL && !(lane & 1)) S.wsm[TW / 32 + lane / 2] = hw | (hn << 16);
    if (lane == HL) S.wsm[TW / 32 + HL / 2] = 0;
  }
  if (lane >= HL) hm = 0;
  const uint64_t hb = __ballot(hm != 0);
  int64_t hnl = -1;
  if (hb) {
    const int f = __builtin_ctzll(hb);
    hnl = TW + 16 * f + __builtin_ctz(wave_readlane(hm, f));
  }
  const bool has0 = t0 == 0 || (wave_readlane(vh.w, 63) >> 24) == '\n';
  const bool endnl = (wave_readlane(v[3].w, 63) >> 24) == '\n';
  if (lane == 63) n1 &= 0x7FFFFFFFu;
  const uint32_t cnt = (uint32_t)(__popc(n0) + __popc(n1));
  const uint32_t inc = wave_incl_scan(cnt, OpSum());
  const uint32_t L = wave_readlane(inc, 63) + (has0 ? 1u : 0u);
  if (L > CAP) {
    if (lane == 0) {
      if (ROWS) atomicOr(&st->flags, BG_ROW_OVERFLOW);
      else bg_report(st, 0, ERR_PARSE);
    }
    return L;
  }
  uint32_t o = inc - cnt + (has0 ? 1u : 0u);
  if (lane == 0 && has0) S.lst[0] = 0;
  for (uint32_t m = n0; m; m &= m - 1) S.lst[o++] = (uint16_t)(64 * lane + bgp_ctz(m) + 1);
  for (uint32_t m = n1; m; m &= m - 1) S.lst[o++] = (uint16_t)(64 * lane + 32 + bgp_ctz(m) + 1);
  if (ROWS) wave_lds_sync();
  else __syncthreads();  // (one wave: orders the LDS writes above before the reads below)
  last_end = L == 0 ? -1 : endnl ? t0 + TW - 1 : (hnl >= 0 ? t0 + hnl : find_nl_wave(txt, nb, t0 + TW + HAX + 32));
  if (lane == 0) {
    const int64_t d = last_end - t0 + 1;
    S.lst[L] = (last_end >= 0 && d < 0xFFFF) ? (uint16_t)d : (uint16_t)0xFFFF;
  }
  if (ROWS) wave_lds_sync();
  else __syncthreads();
  return L;
}

__device__ __forceinline__ uint32_t sgpr(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// the rounds of a one-run sub-tile (32-bit coordinates under the key prefix, set_rounds_w's
// staging); TOK16: the run's token is 9..16 bytes
template <bool TOK16>
__device__ __forceinline__ void set_rounds_v(const uint8_t* __restrict__ txt, const ParseLdsV& S,
                                             const SubView& SV, const TileText& T, const RunTable& R,
                                             uint32_t rl, int64_t t0, uint32_t L, int64_t last_end,
                                             uint64_t base, int64_t* __restrict__ LCS,
                                             int64_t* __restrict__ LCE, uint64_t& nc, uint32_t& carry_e,
                                             uint32_t& kl, bg_dstatus* st) {
  const int lane = threadIdx.x;
  const uint64_t lt = (1ULL << lane) - 1;
  // the run's token and the mask of its bytes, in SGPRs (readfirstlane: the stores below may
  // alias R.info as far as the compiler knows, and it would reload the token every round
  // behind an s_waitcnt vmcnt(0) that also waits for those stores)
  const RunInfo& I = R.info[rl];
  const uint32_t tlen = sgpr(I.tlen);
  const uint64_t tm = tlen >= 8 ? ~0ull : ((1ull << (8 * tlen)) - 1);
  const uint64_t tm2 = tlen >= 16 ? ~0ull : (tlen <= 8 ? 0ull : ((1ull << (8 * (tlen - 8))) - 1));
  const uint32_t tk0 = sgpr((uint32_t)I.tlo), tk1 = sgpr((uint32_t)(I.tlo >> 32));
  const uint32_t tk2 = sgpr((uint32_t)I.thi), tk3 = sgpr((uint32_t)(I.thi >> 32));
  const uint32_t tm0 = sgpr((uint32_t)tm), tm1 = sgpr((uint32_t)(tm >> 32)), tm2l = sgpr((uint32_t)tm2),
                 tm2h = sgpr((uint32_t)(tm2 >> 32));
  uint32_t* const S32 = reinterpret_cast<uint32_t*>(LCS + base);
  uint32_t* const E32 = reinterpret_cast<uint32_t*>(LCE + base);
  uint32_t carry_k = 0, nc32 = (uint32_t)nc;
  const uint32_t rounds = (L + 63) / 64;
  for (uint32_t j = 0; j < rounds; ++j) {
    const uint32_t k = j * 64 + lane;
    const bool act = k < L;
    const uint32_t pr = ldsu32(&S.lst[act ? k : 0]);
    const uint32_t q = pr & 0xFFFFu, qn = pr >> 16;
    const uint32_t len = qn - q - 1;  // bytes before the line's '\n'
    uint32_t WS;
    {
      const uint2 two = ldsu64(&S.wsm[q >> 5]);
      WS = __builtin_amdgcn_alignbit(two.y, two.x, q & 31u);
    }
    WS |= len < 32u ? (~0u << (len & 31u)) : 0u;  // bytes past the line end act as whitespace
    const uint32_t NW = ~WS, NW1 = NW << 1;
    uint32_t Ts = NW & ~NW1, Te = WS & NW1;    // field starts, field ends
    const uint32_t a0 = ffbl_hw(Ts);
    Ts &= Ts - 1;
    const uint32_t s0 = ffbl_hw(Ts);
    Ts &= Ts - 1;
    const uint32_t e0 = ffbl_hw(Ts);
    const uint32_t a1 = ffbl_hw(Te);
    Te &= Te - 1;
    const uint32_t s1 = ffbl_hw(Te);
    Te &= Te - 1;
    const uint32_t e1 = ffbl_hw(Te);
    // the third field ends inside the window (so do the others); short numbers; the token's
    // length; the line has an end (lst[L] != 0xFFFF)
    // (tokens past 16 bytes: compared in full by set_row's hash, not by the 16-byte prefix)
    bool ok = act && tlen <= 16u && e1 <= 31u && qn != 0xFFFFu && (a1 - a0) == tlen && (s1 - s0) <= 9u &&
              (e1 - e0) <= 9u;
    const uint8_t* lb = &SV.buf[HB + q];  // the line's bytes (LDS)
    {
      uint32_t dif;
      if (TOK16) {
        const uint4 t = ldsu128(lb + (a0 & 31u));
        dif = ((t.x ^ tk0) & tm0) | ((t.y ^ tk1) & tm1) | ((t.z ^ tk2) & tm2l) | ((t.w ^ tk3) & tm2h);
      } else {
        const uint2 t = ldsu64(lb + (a0 & 31u));
        dif = ((t.x ^ tk0) & tm0) | ((t.y ^ tk1) & tm1);
      }
      ok = ok && dif == 0;
    }
    uint32_t start = digits9(ldsu96(lb + (s1 & 31u) - 12), (s1 - s0) & 15u, ok);
    uint32_t end = digits9(ldsu96(lb + (e1 & 31u) - 12), (e1 - e0) & 15u, ok);
    bool valid = ok;
    if (act && !ok) {  // the full grammar (and its errors), this lane only
      int64_t ks = 0, ke = 0;
      valid = set_row<true, true>(SV, S.lst, T, R, rl, rl, t0, k, L, last_end, ks, ke, st);
      start = (uint32_t)(ks & BG_COORD_MASK);
      end = (uint32_t)(ke & BG_COORD_MASK);
      if (valid && (uint64_t)(ke & BG_COORD_MASK) + 1 >= 0xFFFFFFFFull) atomicOr(&st->flags, BG_SET_OVERFLOW);
    } else if (ok) {
      if (start > end) bg_report(st, 0, ERR_RANGE);
      if (start == end) atomicOr(&st->flags, 2ULL);
    }
    const uint32_t K = valid ? start + 1 : 0u, E = valid ? end + 1 : 0u;
    const uint32_t ie = wave_incl_max_u32(E);
    const uint32_t pk = wave_shr1_v(K);
    const uint32_t prevK = lane ? pk : carry_k;
    if (valid && prevK && K < prevK) bg_report(st, 0, ERR_UNSORTED);
    const uint32_t ex_e = max(carry_e, wave_shr1_v(ie));
    const bool open = valid && K > ex_e;
    const uint64_t bal = __ballot(open);
    const uint32_t pos = nc32 + (uint32_t)__popcll(bal & lt);
    if (open && pos < SCAP_W) {
      S32[pos] = K - 1;
      if (pos > 0) E32[pos - 1] = ex_e - 1;
    }
    if (j + 1 == rounds) {
      const int ll = (int)(L - 1 - j * 64);
      const uint32_t k1 = wave_readlane(K, ll);
      kl = k1 ? k1 : (ll > 0 ? wave_readlane(K, ll - 1) : carry_k);
    }
    carry_e = max(carry_e, wave_readlane(ie, 63));
    carry_k = wave_readlane(K, 63);
    nc32 += (uint32_t)__popcll(bal);
  }
  nc = nc32;
}

// one sub-tile from its registers
__device__ __forceinline__ void parse_sub_v(const uint8_t* __restrict__ txt, uint64_t nb, uint32_t u,
                                            const SubRegs& V, ParseLdsV& S,
                                            const uint32_t* __restrict__ runlo,
                                            const uint32_t* __restrict__ runhi, const RunTable& R,
                                            int64_t* __restrict__ LCS, int64_t* __restrict__ LCE,
                                            const SetTiles& TS, bg_dstatus* st) {
  const int64_t t0 = (int64_t)u * TW;
  const uint64_t base = (uint64_t)u * SCAP_W;
  int64_t last_end = -1;
  const uint32_t L = prologue_v(txt, nb, t0, V, S, last_end, st);
  if (L > LCAP_V) {
    if (threadIdx.x == 0) {
      TS.tmax[u] = TS.tlast[u] = LLONG_MIN;
      TS.base[u] = base;
      TS.nloc[u] = 0;
      TS.nrow[u] = 0;
      TS.gb[u] = -1;
    }
    return;
  }
  const uint32_t rl = runlo[u], rh = runhi[u];
  const SubView SV{S.buf, S.wsm, S.lst};
  const TileText T{txt, SV.buf, t0 - HB, t0 + TW + HA_V, nb};
  uint64_t nc = 0, cmax = 0, kmax = 0;
  int64_t gbase = 0;
  if (rl == rh) {
    gbase = (int64_t)R.info[rl].gid << BG_KEY_SHIFT;
    uint32_t ce = 0, kl = 0;
    const bool tok16 = R.info[rl].tlen > 8;
    if (tok16)
      set_rounds_v<true>(txt, S, SV, T, R, rl, t0, L, last_end, base, LCS, LCE, nc, ce, kl, st);
    else
      set_rounds_v<false>(txt, S, SV, T, R, rl, t0, L, last_end, base, LCS, LCE, nc, ce, kl, st);
    cmax = ce;
    kmax = kl;
  } else {
    set_rounds_w<uint64_t, SubView>(SV, T, R, rl, rh, t0, L, last_end, 0, base, LCS, LCE, nc, cmax, kmax, st);
  }
  if (threadIdx.x == 0) {
    if (nc > SCAP_W) {
      atomicOr(&st->flags, BG_SET_OVERFLOW);
      nc = 0;
    }
    if (nc > 0) {
      if (rl == rh) reinterpret_cast<uint32_t*>(LCE + base)[nc - 1] = (uint32_t)(cmax - 1);
      else LCE[base + nc - 1] = gbase | (int64_t)(cmax - 1);
    }
    TS.gb[u] = (rl == rh) ? gbase : -1;
    TS.tmax[u] = cmax ? (gbase | (int64_t)(cmax - 1)) : LLONG_MIN;
    TS.tlast[u] = kmax ? (gbase | (int64_t)(kmax - 1)) : LLONG_MIN;
    TS.base[u] = base;
    TS.nloc[u] = nc;
    TS.nrow[u] = L - ((L > 0 && last_end < 0) ? 1 : 0);
  }
}

// one wave per sub-tile
// (106 SGPRs: 6 waves per SIMD by SGPRs, 7 by LDS. Caps of 96 or 80 SGPRs, 7 waves, measured
// the same 0.92-0.93 ms, round 6: occupancy is not what bounds it; an L2 prefetch of a later
// sub-tile, round 5, measured neutral)
__global__ void __launch_bounds__(64) k_parse_set_v(
    const uint8_t* __restrict__ txt, uint64_t nb, uint32_t nsub,
    const uint32_t* __restrict__ runlo, const uint32_t* __restrict__ runhi, RunTable R,
    int64_t* __restrict__ LCS, int64_t* __restrict__ LCE, SetTiles TS, bg_dstatus* st) {
  __shared__ ParseLdsV S;
  SubRegs V;
  const uint32_t u = blockIdx.x;
  load_sub(txt, nb, (int64_t)u * TW, V);
  parse_sub_v(txt, nb, u, V, S, runlo, runhi, R, LCS, LCE, TS, st);
}

// ---- k_parse_rv (round 6): the row parse in k_parse_set_v's shape -----------------------
// Row columns (keys, rest spans, scores) for bedmap, closest-features and the row side of the
// element operations. A workgroup of two waves owns one 8 KiB tile (the scout's row0 unit);
// wave h parses sub-tile h (4 KiB) with k_parse_set_v's prologue and lean common path: on a
// one-run sub-tile a line "<token> <start> <end>..." whose three fields end inside its first 32
// bytes, the token the run's and both numbers <= 9 digits, is read from the whitespace
// transitions, the token compared in SGPRs and the numbers converted by digits9. BED5 scores
// then take parse_score_fast_ws (integers, "<int>.<frac>"); every other line takes
// the per-line path (parse_line_fast_ws, then the full grammar) in its own lane. Same outputs
// and error reports as k_parse (round 5's k_parse_n, 8 KiB tiles of 128 threads with a shared
// front end, measured 15.8 / 10.5 / 3.1 ms against 11.8 / 8.2 / 2.1 ms for this kernel on the
// closest, bedmap and element-of row files and was removed). The only exchange between the waves: wave 0's line
// count (wave 1's first row) and the keys on either side of the sub-tile edge (sort check).
#ifndef LCAP_R
#define LCAP_R 512  // lines per 4 KiB sub-tile (lines averaging >= 8 bytes; more: redone with k_parse)
#endif
// a 224-byte halo (+32) after the sub-tile, so that the lines crossing its end are staged for
// the score path too (with k_parse_set_v's 32 bytes, one BED5 sub-tile in seven sent a lane to
// the byte path)
#ifndef HA_R
#define HA_R 224
#endif
struct ParseLdsR {
  __attribute__((aligned(16))) uint8_t buf[HB + TW + HA_R + 32];
  uint32_t wsm[TW / 32 + (HA_R + 32) / 32 + 1];
  uint16_t lst[LCAP_R + 1];
};

__device__ __forceinline__ int64_t wave_shr1_i64(int64_t v) {
  return (int64_t)(((uint64_t)wave_shr1_v((uint32_t)((uint64_t)v >> 32)) << 32) | wave_shr1_v((uint32_t)v));
}

// the BED5 score after the end field ("<ws>id<ws>score", then whitespace or the line end) from
// the whitespace window at the end field's end (p = q + e1): an integer of <= 9 digits by the
// window's transitions and digits9; anything else parse_score_fast_ws, then the byte path
__device__ __forceinline__ bool score_fast_v(const ParseLdsR& S, uint32_t q, uint32_t len, uint32_t e1, double& sc) {
  const uint32_t p = q + e1, l2 = len - e1;
  uint32_t WS;
  {
    const uint2 two = ldsu64(&S.wsm[p >> 5]);
    WS = __builtin_amdgcn_alignbit(two.y, two.x, p & 31u);
  }
  WS |= l2 < 32u ? (~0u << (l2 & 31u)) : 0u;
  const uint32_t NW = ~WS, NW1 = NW << 1;
  uint32_t Ts = NW & ~NW1, Te = WS & NW1;
  Ts &= Ts - 1;  // (the id's start)
  const uint32_t c0 = ffbl_hw(Ts);
  Te &= Te - 1;  // (the id's end)
  const uint32_t c1 = ffbl_hw(Te);
  bool ok = c1 <= 31u && (c1 - c0) <= 9u && (WS & 1u);
  const uint32_t v = digits9(ldsu96(&S.buf[HB + p + (c1 & 31u) - 12]), (c1 - c0) & 15u, ok);
  sc = (double)v;
  return ok;
}

// one line on the per-line path (the run by position, parse_line_fast_ws, else the
// full grammar); key: the row's start key (LLONG_MIN: not a row)
template <bool REST, bool SCORE>
__device__ __forceinline__ void row_line_general(const ParseLdsR& S, const TileText& T, const RunTable& R,
                                                 uint32_t rl, uint32_t rh, int64_t t0, uint32_t q, int64_t ls,
                                                 int64_t le, uint64_t r, int64_t* __restrict__ KS,
                                                 int64_t* __restrict__ KE, uint64_t* __restrict__ rest_off,
                                                 uint32_t* __restrict__ rest_len, double* __restrict__ score,
                                                 bg_dstatus* st, uint64_t* __restrict__ big, uint32_t bigcap,
                                                 int64_t& key, int64_t& mlen, bool& nonint) {
  Fast F;
  const uint32_t run = (rl == rh) ? rl : run_of(R, ls, rl, rh);
  const RunInfo& I = R.info[run];
  const uint32_t len = (uint32_t)(le - ls);
  double sc = 0;
  bool isint = true;
  // (scores are read up to the line's end: only lines ending inside the staged halo)
  if (parse_line_fast_ws(S.buf, S.wsm, q, len, F, I.tlen <= 8) && F.toklen == I.tlen && F.tlo == I.tlo &&
      F.thi == I.thi &&
      (!SCORE || (le - t0 <= TW + HA_R && parse_score_fast_ws(S.buf, S.wsm, q, len, F.rest, sc, isint)))) {
    nonint |= !isint;
    emit_row(R, run, ls, r, F.start, F.end, KS, KE, st, key, mlen);
    if (REST) {
      rest_off[r] = (uint64_t)(ls + F.rest);
      rest_len[r] = len - F.rest;
    }
    if (SCORE) score[r] = sc;
    return;
  }
  Line Ln;
  parse_line_slow<false>(T, ls, le, SCORE ? BG_BED5 : BG_BED3, Ln);
  if (Ln.err) {
    if (Ln.err == ERR_BLANK) atomicAdd(&st->nblank, 1ULL);
    bg_report(st, r, Ln.err);
    KS[r] = KE[r] = 0;
  } else if (Ln.hash != I.hash) {  // a chromosome outside the run order: unsorted input
    bg_report(st, r, ERR_UNSORTED);
  } else {
    emit_row(R, run, ls, r, Ln.start, Ln.end, KS, KE, st, key, mlen);
    if (REST) {
      rest_off[r] = (uint64_t)Ln.rest;
      rest_len[r] = (uint32_t)(le - Ln.rest);
    }
    if (SCORE) {
      score[r] = Ln.score;
      if (Ln.scoreint <= 0) atomicOr(&st->flags, 1ULL);
      if (Ln.scoreint < 0) big_push(st, big, bigcap, r, Ln.spos);
    }
  }
}

// the rounds of one sub-tile (64 lines per round, one per lane, in line order); kf / kl: the
// keys of its first and last line (LLONG_MIN: not a row)
template <bool REST, bool SCORE>
__device__ __forceinline__ void row_rounds_v(const ParseLdsR& S, const TileText& T, const RunTable& R,
                                             uint32_t rl, uint32_t rh, int64_t t0, uint32_t L, int64_t last_end,
                                             uint64_t r0, uint64_t nrows, int64_t* __restrict__ KS,
                                             int64_t* __restrict__ KE, uint64_t* __restrict__ rest_off,
                                             uint32_t* __restrict__ rest_len, double* __restrict__ score,
                                             bg_dstatus* st, uint64_t* __restrict__ big, uint32_t bigcap,
                                             int64_t& kf, int64_t& kl, int64_t& mlen, bool& nonint) {
  const int lane = threadIdx.x & 63;
  const bool one = rl == rh;  // (wave-uniform)
  // the run's token, mask, first line and key prefix in SGPRs (as set_rounds_v)
  const RunInfo& I = R.info[rl];
  const uint32_t tlen = sgpr(I.tlen);
  const uint64_t tm = tlen >= 8 ? ~0ull : ((1ull << (8 * tlen)) - 1);
  const uint64_t tm2 = tlen >= 16 ? ~0ull : (tlen <= 8 ? 0ull : ((1ull << (8 * (tlen - 8))) - 1));
  const uint32_t tk0 = sgpr((uint32_t)I.tlo), tk1 = sgpr((uint32_t)(I.tlo >> 32));
  const uint32_t tk2 = sgpr((uint32_t)I.thi), tk3 = sgpr((uint32_t)(I.thi >> 32));
  const uint32_t tm0 = sgpr((uint32_t)tm), tm1 = sgpr((uint32_t)(tm >> 32)), tm2l = sgpr((uint32_t)tm2),
                 tm2h = sgpr((uint32_t)(tm2 >> 32));
  const int64_t pos0 = (int64_t)(((uint64_t)sgpr((uint32_t)((uint64_t)I.pos >> 32)) << 32) | sgpr((uint32_t)I.pos));
  const int64_t gbase = (int64_t)sgpr((uint32_t)I.gid) << BG_KEY_SHIFT;
  const bool tok16 = tlen > 8;
  int64_t carry = LLONG_MIN;
  kf = kl = LLONG_MIN;
  const uint32_t rounds = (L + 63) / 64;
  for (uint32_t j = 0; j < rounds; ++j) {
    const uint32_t k = j * 64 + lane;
    const bool act = k < L;
    const uint32_t pr = ldsu32(&S.lst[act ? k : 0]);
    const uint32_t q = pr & 0xFFFFu, qn = pr >> 16;
    const int64_t ls = t0 + q;
    const int64_t le = (k + 1 < L) ? t0 + qn - 1 : last_end;
    const uint64_t r = r0 + k;
    // le < 0 / r >= nrows: the unterminated last line (dropped like the reference)
    const bool live = act && r < nrows && le >= 0;
    const uint32_t len = live ? (uint32_t)(le - ls) : 0u;
    int64_t key = LLONG_MIN;
    bool ok = false;
    uint32_t start = 0, end = 0, e1 = 0;
    double sc = 0;
    bool isint = true;
    if (one) {
      uint32_t WS;
      {
        const uint2 two = ldsu64(&S.wsm[q >> 5]);
        WS = __builtin_amdgcn_alignbit(two.y, two.x, q & 31u);
      }
      WS |= len < 32u ? (~0u << (len & 31u)) : 0u;  // bytes past the line end act as whitespace
      const uint32_t NW = ~WS, NW1 = NW << 1;
      uint32_t Ts = NW & ~NW1, Te = WS & NW1;  // field starts, field ends
      const uint32_t a0 = ffbl_hw(Ts);
      Ts &= Ts - 1;
      const uint32_t s0 = ffbl_hw(Ts);
      Ts &= Ts - 1;
      const uint32_t e0 = ffbl_hw(Ts);
      const uint32_t a1 = ffbl_hw(Te);
      Te &= Te - 1;
      const uint32_t s1 = ffbl_hw(Te);
      Te &= Te - 1;
      e1 = ffbl_hw(Te);
      ok = live && tlen <= 16u && e1 <= 31u && (a1 - a0) == tlen && (s1 - s0) <= 9u && (e1 - e0) <= 9u;
      const uint8_t* lb = &S.buf[HB + q];
      {
        uint32_t dif;
        if (tok16) {
          const uint4 t = ldsu128(lb + (a0 & 31u));
          dif = ((t.x ^ tk0) & tm0) | ((t.y ^ tk1) & tm1) | ((t.z ^ tk2) & tm2l) | ((t.w ^ tk3) & tm2h);
        } else {
          const uint2 t = ldsu64(lb + (a0 & 31u));
          dif = ((t.x ^ tk0) & tm0) | ((t.y ^ tk1) & tm1);
        }
        ok = ok && dif == 0;
      }
      start = digits9(ldsu96(lb + (s1 & 31u) - 12), (s1 - s0) & 15u, ok);
      end = digits9(ldsu96(lb + (e1 & 31u) - 12), (e1 - e0) & 15u, ok);
      if (SCORE) ok = ok && le - t0 <= TW + HA_R && score_fast_v(S, q, len, e1, sc);
    }
    if (ok) {
      if (start > end) bg_report(st, r, ERR_RANGE);
      if (start == end) atomicOr(&st->flags, 2ULL);
      mlen = max(mlen, (int64_t)end - (int64_t)start);
      if (ls == pos0) R.row[rl] = r;
      key = gbase | (int64_t)start;
      KS[r] = key;
      KE[r] = gbase | (int64_t)end;
      if (REST) {
        rest_off[r] = (uint64_t)(ls + e1);
        rest_len[r] = len - e1;
      }
      if (SCORE) {
        score[r] = sc;
        nonint |= !isint;
      }
    } else if (live) {
      row_line_general<REST, SCORE>(S, T, R, rl, rh, t0, q, ls, le, r, KS, KE, rest_off, rest_len, score, st,
                                    big, bigcap, key, mlen, nonint);
    }
    // sort order: each line against the one before it (the lane before, or lane 63 of the
    // previous round)
    const int64_t pk = wave_shr1_i64(key);
    const int64_t prev = lane ? pk : carry;
    if (key != LLONG_MIN && prev != LLONG_MIN && key < prev) bg_report(st, r, ERR_UNSORTED);
    if (j == 0) kf = (int64_t)wave_readlane((uint64_t)key, 0);
    if (j + 1 == rounds) kl = (int64_t)wave_readlane((uint64_t)key, (int)(L - 1 - j * 64));
    carry = (int64_t)wave_readlane((uint64_t)key, 63);
  }
}

// (at least 6 waves per SIMD: <= 80 VGPRs. The BED5 variants then spill 28-40 bytes of values
// only the byte path reloads; capped at 5 waves they spill nothing and measured slower, bedmap
// 21.8 -> 22.1 ms, round 6)
template <bool REST, bool SCORE>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(6, 8))) k_parse_rv(
    const uint8_t* __restrict__ txt, uint64_t nb, uint64_t nrows, const uint64_t* __restrict__ row0,
    const uint32_t* __restrict__ runlo, const uint32_t* __restrict__ runhi, RunTable R,
    int64_t* __restrict__ KS, int64_t* __restrict__ KE, uint64_t* __restrict__ rest_off,
    uint32_t* __restrict__ rest_len, double* __restrict__ score, bg_dstatus* st, uint64_t* __restrict__ big,
    uint32_t bigcap) {
  __shared__ ParseLdsR SS[2];
  __shared__ uint32_t xl[2];
  __shared__ int64_t xk[2][2];  // [wave][first line, last line] keys
  // (h through readfirstlane: the compiler does not know a wave's threads share threadIdx.x >> 6,
  // and everything derived from it — the sub-tile, its runs, its row base — would take VGPRs)
  const int lane = threadIdx.x & 63, h = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t u = 2 * blockIdx.x + h;  // sub-tile
  const int64_t t0 = (int64_t)u * TW;
  const bool inside = (uint64_t)t0 < nb;  // (the file's last tile may hold one sub-tile)
  ParseLdsR& S = SS[h];
  int64_t last_end = -1;
  uint32_t L = 0;
  if (inside) {
    SubRegs V;
    load_sub<HA_R>(txt, nb, t0, V);
    L = prologue_v<ParseLdsR, LCAP_R, true, HA_R>(txt, nb, t0, V, S, last_end, st);
  }
  if (lane == 0) xl[h] = L;
  __syncthreads();
  const uint32_t L0 = xl[0];
  if (L0 > LCAP_R || xl[1] > LCAP_R) return;  // (BG_ROW_OVERFLOW: the load is redone with k_parse)
  // the first owned line's row: newlines before the tile (+1 when the tile opens mid-line);
  // wave 1's follows wave 0's L0 lines
  const int64_t tt = (int64_t)blockIdx.x * TT;
  const bool has0 = tt == 0 || SS[0].buf[HB - 1] == '\n';
  const uint64_t r0 = row0[blockIdx.x] + (has0 ? 0 : 1) + (h ? L0 : 0);
  int64_t mlen = 0, kf = LLONG_MIN, kl = LLONG_MIN;
  bool nonint = false;
  if (L > 0) {
    const TileText T{txt, S.buf, t0 - HB, t0 + TW + HA_R, nb};
    row_rounds_v<REST, SCORE>(S, T, R, runlo[u], runhi[u], t0, L, last_end, r0, nrows, KS, KE, rest_off,
                              rest_len, score, st, big, bigcap, kf, kl, mlen, nonint);
  }
  if (__ballot(nonint) && lane == 0) atomicOr(&st->flags, 1ULL);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) mlen = max(mlen, (int64_t)__shfl_xor(mlen, d, 64));
  if (lane == 0 && mlen > *(volatile long long*)&st->maxlen) atomicMax(&st->maxlen, (long long)mlen);
  if (lane == 0) {
    xk[h][0] = kf;
    xk[h][1] = kl;
  }
  __syncthreads();
  if (h == 1 && lane == 0 && L0 > 0 && L > 0) {  // wave 1's first line vs wave 0's last
    const int64_t a = xk[0][1], b = xk[1][0];
    if (a != LLONG_MIN && b != LLONG_MIN && b < a) bg_report(st, r0, ERR_UNSORTED);
  }
}


// per tile: sort check against the nearest earlier tile with rows (every tile is sorted
// inside, or has reported it), how many local components the running max M of the
// earlier tiles absorbs (mex = exclusive prefix max of tmax; the local starts increase,
// so they are a prefix: a gallop from the front, usually 0 or 1 steps), and the tile's
// rows summed into st->pad[1] (one atomic per workgroup)
__global__ void __launch_bounds__(BG_NT) k_set_count(const int64_t* __restrict__ LCS, SetTiles TS,
                                                     const int64_t* __restrict__ mex,
                                                     uint32_t ntiles, uint64_t* __restrict__ cnt,
                                                     bg_dstatus* st, uint32_t u0) {
  __shared__ unsigned long long srows[BG_NT / 64];
  const uint32_t t = u0 + blockIdx.x * blockDim.x + threadIdx.x;  // (tiles [u0, ntiles))
  uint64_t rows = 0;
  if (t < ntiles) {
    const uint64_t b = TS.base[t], n = TS.nloc[t];
    const int64_t gb = TS.gb[t];
    rows = TS.nrow[t];
    const int64_t first = n ? set_key(LCS, b, gb, 0) : 0;
    if (n > 0 && t > 0) {
      uint32_t u = t - 1;
      while (u > 0 && TS.tlast[u] == LLONG_MIN) --u;  // tiles without rows (lines > 8 KiB)
      if (first < TS.tlast[u]) bg_report(st, 0, ERR_UNSORTED);  // first row < an earlier row
    }
    const int64_t M = mex[t];
    uint64_t a = 0;
    if (n && first <= M) {
      uint64_t step = 1;  // gallop, then bisect
      while (a + step < n && set_key(LCS, b, gb, a + step) <= M) {
        a += step;
        step <<= 1;
      }
      uint64_t lo = a + 1, hi = min(n, a + step);  // first local index in [lo, hi) with key > M
      while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (set_key(LCS, b, gb, mid) <= M) lo = mid + 1;
        else hi = mid;
      }
      a = lo;
    }
    TS.absorbed[t] = (uint32_t)a;
    cnt[t] = n - a;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) rows += __shfl_xor(rows, d, 64);
  if (bg_lane() == 0) srows[bg_wave()] = rows;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long r = 0;
    for (int q = 0; q < BG_NT / 64; ++q) r += srows[q];
    if (r) atomicAdd((unsigned long long*)&st->pad[1], r);
  }
}

// one wave per tile: global components of the tile -> CS/CE at its offset. CE[g] is the
// running max just before component g+1 opens, written by the tile holding that opening
// (the last one by the last tile).
#define SW_TILES 64  // tiles per k_set_write workgroup
// (a range [u0, ntiles) of a file's tiles: off[] holds the range's exclusive offsets and
// *carry the components of the tiles before u0; the file's last tile is nlast - 1, whose
// workgroup also writes the file's component count to *total)
__global__ void __launch_bounds__(BG_NT) k_set_write(const int64_t* __restrict__ LCS,
                                                     const int64_t* __restrict__ LCE, SetTiles TS,
                                                     const int64_t* __restrict__ mex,
                                                     const uint64_t* __restrict__ off,
                                                     uint32_t ntiles, int64_t* __restrict__ CS,
                                                     int64_t* __restrict__ CE, uint32_t u0, uint32_t nlast,
                                                     const uint64_t* __restrict__ carry,
                                                     unsigned long long* __restrict__ total_out) {
  // SW_TILES tiles per workgroup, their surviving components flattened over all threads
  // (element e -> its tile by a search of the LDS prefix of counts): every load of a
  // workgroup is independent, instead of a wave waiting on one tile's descriptor first
  __shared__ uint32_t cpre[SW_TILES + 1];
  __shared__ uint64_t src[SW_TILES], dst[SW_TILES];
  __shared__ uint32_t sab[SW_TILES];       // absorbed local components (the first survivor's index)
  __shared__ int64_t sgb[SW_TILES];        // staging form (SetTiles::gb)
  __shared__ int64_t first_end[SW_TILES];  // CE value before the tile's first global component
  const uint32_t t0 = u0 + blockIdx.x * SW_TILES;
  const uint32_t nt = min((uint32_t)SW_TILES, ntiles - t0);
  const uint64_t cy = carry ? *carry : 0;
  uint32_t c = 0;
  if (threadIdx.x < nt) {
    const uint32_t t = t0 + threadIdx.x;
    const uint64_t b = TS.base[t], n = TS.nloc[t], a = TS.absorbed[t];
    const int64_t M = mex[t], gb = TS.gb[t];
    c = (uint32_t)(n - a);
    src[threadIdx.x] = b;
    sab[threadIdx.x] = (uint32_t)a;
    sgb[threadIdx.x] = gb;
    dst[threadIdx.x] = cy + off[t];
    first_end[threadIdx.x] = (c > 0) ? max(M, a > 0 ? set_key(LCE, b, gb, a - 1) : LLONG_MIN) : 0;
    if (t + 1 == nlast) {  // the last component ends at the running max of everything
      const uint64_t total = cy + off[t] + c;
      if (total > 0) CE[total - 1] = max(M, TS.tmax[t]);
      if (total_out) *total_out = total;
    }
  }
  // exclusive scan of c over the first wave (SW_TILES == 64)
  if (threadIdx.x < 64) {
    const uint32_t inc = wave_incl_scan(c, OpSum());
    cpre[threadIdx.x + 1] = inc;
    if (threadIdx.x == 0) cpre[0] = 0;
  }
  __syncthreads();
  const uint32_t tot = cpre[nt];
  for (uint32_t e = threadIdx.x; e < tot; e += BG_NT) {
    uint32_t lo = 0, hi = nt - 1;  // last q with cpre[q] <= e
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (cpre[mid] <= e) lo = mid;
      else hi = mid - 1;
    }
    const uint32_t j = e - cpre[lo];
    const uint64_t g = dst[lo] + j, b = src[lo], i = sab[lo] + j;
    const int64_t gb = sgb[lo];
    CS[g] = set_key(LCS, b, gb, i);
    if (g > 0) CE[g - 1] = j == 0 ? first_end[lo] : set_key(LCE, b, gb, i - 1);
  }
}

// -------------------------------------------------------------------------------------
// blank lines. The reference reads rows with fscanf("%s\t%lu\t%lu...") + fgetc
// (Bed.hpp:244-255): after a row's '\n' the next %s skips every whitespace byte, so lines of
// only whitespace (and a line's leading whitespace) are never seen. The loaders split on '\n',
// so a load that meets a blank line (ERR_BLANK) is redone on the text with those bytes removed:
// byte p goes iff it is whitespace or '\n' and the last '\n' before p comes after the last
// other byte before p (at the start of the text: both "before" values are below every
// position, the '\n' one higher). One wave per 4 KiB tile, 64 bytes per lane.
// -------------------------------------------------------------------------------------
constexpr uint32_t BK_T = 4096;

// per tile: its last '\n' (-1: none) and its last byte that is neither '\n' nor whitespace
// (-2: none), the identities of the exclusive max-scans that follow
__global__ void __launch_bounds__(BG_NT) k_blank_marks(const uint8_t* __restrict__ txt, uint64_t nb,
                                                       uint32_t nt, int64_t* __restrict__ tnl,
                                                       int64_t* __restrict__ tns) {
  const uint32_t lane = threadIdx.x & 63, t = blockIdx.x * (BG_NT / 64) + (threadIdx.x >> 6);
  if (t >= nt) return;
  const uint64_t b0 = (uint64_t)t * BK_T + 64ull * lane;
  int64_t lnl = -1, lns = -2;
  for (uint32_t k = 0; k < 64 && b0 + k < nb; ++k) {
    const uint8_t ch = txt[b0 + k];
    if (ch == '\n') lnl = (int64_t)(b0 + k);
    else if (!bg_isws(ch)) lns = (int64_t)(b0 + k);
  }
  for (int d = 32; d >= 1; d >>= 1) {
    lnl = max(lnl, (int64_t)__shfl_xor(lnl, d, 64));
    lns = max(lns, (int64_t)__shfl_xor(lns, d, 64));
  }
  if (lane == 0) {
    tnl[t] = lnl;
    tns[t] = lns;
  }
}

// count pass (out == nullptr: kept bytes per tile into cnt) or write pass (kept bytes to
// out + off[t]); xnl/xns: the exclusive max-scans of k_blank_marks' values
__global__ void __launch_bounds__(BG_NT) k_blank_pack(const uint8_t* __restrict__ txt, uint64_t nb,
                                                      uint32_t nt, const int64_t* __restrict__ xnl,
                                                      const int64_t* __restrict__ xns,
                                                      uint64_t* __restrict__ cnt,
                                                      const uint64_t* __restrict__ off,
                                                      uint8_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63, t = blockIdx.x * (BG_NT / 64) + (threadIdx.x >> 6);
  if (t >= nt) return;
  const uint64_t b0 = (uint64_t)t * BK_T + 64ull * lane;
  int64_t lnl = -1, lns = -2;  // this lane's own marks, then the lanes before it
  for (uint32_t k = 0; k < 64 && b0 + k < nb; ++k) {
    const uint8_t ch = txt[b0 + k];
    if (ch == '\n') lnl = (int64_t)(b0 + k);
    else if (!bg_isws(ch)) lns = (int64_t)(b0 + k);
  }
  for (int d = 1; d < 64; d <<= 1) {  // inclusive max-scan over the lanes
    const int64_t a = __shfl_up(lnl, d, 64), b = __shfl_up(lns, d, 64);
    if (lane >= (uint32_t)d) {
      lnl = max(lnl, a);
      lns = max(lns, b);
    }
  }
  int64_t cnl = __shfl_up(lnl, 1, 64), cns = __shfl_up(lns, 1, 64);
  if (lane == 0) cnl = -1, cns = -2;
  cnl = max(cnl, xnl[t]);
  cns = max(cns, xns[t]);
  const int64_t snl = cnl, sns = cns;
  uint32_t keep = 0;
  for (uint32_t k = 0; k < 64 && b0 + k < nb; ++k) {
    const uint8_t ch = txt[b0 + k];
    const bool sp = ch == '\n' || bg_isws(ch);
    keep += !(sp && cnl > cns);
    if (ch == '\n') cnl = (int64_t)(b0 + k);
    else if (!sp) cns = (int64_t)(b0 + k);
  }
  uint32_t pre = keep;  // inclusive sum over the lanes
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t a = __shfl_up(pre, d, 64);
    if (lane >= (uint32_t)d) pre += a;
  }
  if (!out) {
    if (lane == 63) cnt[t] = pre;
    return;
  }
  uint64_t o = off[t] + pre - keep;
  cnl = snl;
  cns = sns;
  for (uint32_t k = 0; k < 64 && b0 + k < nb; ++k) {
    const uint8_t ch = txt[b0 + k];
    const bool sp = ch == '\n' || bg_isws(ch);
    if (!(sp && cnl > cns)) out[o++] = ch;
    if (ch == '\n') cnl = (int64_t)(b0 + k);
    else if (!sp) cns = (int64_t)(b0 + k);
  }
}

// -------------------------------------------------------------------------------------
// host side
// -------------------------------------------------------------------------------------

// the device text txt[0, nb) without its blank lines (k_blank_*): *out (bg_alloc'ed, nbytes
// + 16), *nout bytes
static int strip_blank_lines(bg_ctx* c, const uint8_t* txt, uint64_t nb, char** out, uint64_t* nout) {
  *out = nullptr;
  *nout = 0;
  const uint32_t nt = (uint32_t)bg_blocks(nb, BK_T);
  char* o = (char*)bg_alloc(c, nb + 16);
  int64_t* w = (int64_t*)bg_alloc(c, 32ull * (nt ? nt : 1) + 16);
  if (!o || !w) {
    bg_release(c, o);
    bg_release(c, w);
    return BG_E_NOMEM;
  }
  int64_t *tnl = w, *tns = w + nt, *xnl = w + 2ull * nt, *xns = w + 3ull * nt;
  uint64_t* cnt = (uint64_t*)tnl;  // (tnl is dead once scanned)
  uint64_t* tot = (uint64_t*)(w + 4ull * nt);
  int rc = 0;
  if (nt) {
    const dim3 g(bg_blocks(nt, BG_NT / 64));
    hipLaunchKernelGGL(k_blank_marks, g, dim3(BG_NT), 0, c->stream, txt, nb, nt, tnl, tns);
    rc = bg_hip_ok(c, hipGetLastError());
    if (!rc) rc = bg_scan_max_i64(c, tnl, xnl, nt, -1);
    if (!rc) rc = bg_scan_max_i64(c, tns, xns, nt, -2);
    if (!rc) {
      hipLaunchKernelGGL(k_blank_pack, g, dim3(BG_NT), 0, c->stream, txt, nb, nt, (const int64_t*)xnl,
                         (const int64_t*)xns, cnt, (const uint64_t*)nullptr, (uint8_t*)nullptr);
      rc = bg_hip_ok(c, hipGetLastError());
    }
    if (!rc) rc = bg_scan_sum_u64(c, cnt, cnt, nt, tot);
    if (!rc) {
      hipLaunchKernelGGL(k_blank_pack, g, dim3(BG_NT), 0, c->stream, txt, nb, nt, (const int64_t*)xnl,
                         (const int64_t*)xns, (uint64_t*)nullptr, (const uint64_t*)cnt, (uint8_t*)o);
      rc = bg_hip_ok(c, hipGetLastError());
    }
    if (!rc) rc = bg_fetch_u64(c, tot, nout);
  }
  bg_release(c, w);
  if (rc) {
    bg_release(c, o);
    *nout = 0;
    return rc;
  }
  *out = o;
  return 0;
}

static const char* kind_name(int k) {
  return (k == BG_BED5 || k == BG_BED5_REST) ? "BED5" : (k == BG_BED3_REST ? "BED3+rest" : "BED3");
}

static int report_status(bg_ctx* c, int file, const bg_dstatus& h) {
  if (h.first_bad == ~0ULL) return 0;
  uint64_t row = h.first_bad >> 8;
  int code = (int)(h.first_bad & 0xff);
  char msg[256];
  const char* what = "";
  int rc = BG_E_PARSE;
  switch (code) {
    case ERR_PARSE: what = "malformed BED line (expected: chrom<tab>start<tab>end...)"; break;
    case ERR_CHROM: what = "chromosome name longer than 127 characters"; rc = BG_E_CHROM; break;
    case ERR_RANGE: what = "coordinate out of range (end < start or >= 2^40)"; rc = BG_E_RANGE; break;
    case ERR_UNSORTED: what = "input is not sorted (use sort-bed)"; rc = BG_E_UNSORTED; break;
    case ERR_BLANK: what = "blank line inside the data is not supported by the GPU loader"; rc = BG_E_BLANK; break;
    case ERR_SCORE: what = "score column is not a plain decimal number"; rc = BG_E_UNSUPPORTED; break;
  }
  snprintf(msg, sizeof(msg), "input %d, data line %llu: %s", file + 1,
           (unsigned long long)row + 1, what);
  return bg_fail(c, rc, msg);
}

// per-input loader state between the phases
struct LoadState {
  const uint8_t* txt = nullptr;
  uint64_t nb = 0;
  uint32_t ntiles = 0;
  uint32_t rc = 0;             // record capacity
  uint64_t* row0 = nullptr;    // tile row offsets (device)
  uint64_t* cnt = nullptr;
  int64_t* fls = nullptr;
  uint64_t* fhash = nullptr;
  uint32_t* fnl = nullptr;
  uint32_t* blist = nullptr;
  RunRec* recs = nullptr;      // run records (device)
  std::vector<int64_t> run_pos;
  std::vector<uint64_t> run_hash;
  // host copy of the records (pinned staging)
  const RunRec* hrec = nullptr;
  uint32_t nrec = 0;
  uint64_t* hrow = nullptr;  // pinned: run -> first row (row loads)
  // phase 3
  std::vector<RunInfo> info;
  RunInfo* d_info = nullptr;
  uint64_t* d_row = nullptr;
  uint32_t* rlo = nullptr;
  uint32_t* rhi = nullptr;
  uint32_t nrows_run = 0;  // runs whose first row comes back (row loads)
  // BG_BED3_SET staging
  int64_t* lcs = nullptr;
  int64_t* lce = nullptr;
  int64_t* tmax = nullptr;
  int64_t* tlast = nullptr;
  int64_t* mex = nullptr;
  int64_t* sex = nullptr;
  uint64_t* tbase = nullptr;
  uint64_t* nloc = nullptr;
  uint64_t* tcnt = nullptr;
  uint32_t* absorbed = nullptr;
  int64_t* tgb = nullptr;
  uint32_t set_nt = 0;  // staging units of a BG_BED3_SET parse whose merge passes are pending
  // BED5: scores for k_score_big, (row, first byte) pairs
  uint64_t* big = nullptr;
  uint32_t bigcap = 0;
  bool blank = false;  // a run record of a whitespace-only line (runs_one)
};

static void release_state(bg_ctx* c, LoadState& S) {
  for (void* p : {(void*)S.row0, (void*)S.cnt, (void*)S.fls, (void*)S.fhash, (void*)S.fnl,
                  (void*)S.blist, (void*)S.recs,
                  (void*)S.d_info, (void*)S.d_row, (void*)S.rlo, (void*)S.rhi, (void*)S.lcs,
                  (void*)S.lce, (void*)S.tmax, (void*)S.tlast, (void*)S.mex, (void*)S.sex,
                  (void*)S.tbase, (void*)S.nloc, (void*)S.tcnt, (void*)S.absorbed,
                  (void*)S.tgb, (void*)S.big})
    bg_release(c, p);
  S = LoadState();
}

// work on the side stream (sstream) from the ctx stream's current position: side_begin
// points c->stream at it, side_end records sjoin there and points c->stream back. Blocks
// released meanwhile wait in c->deferred until side_join (the side stream may still use them).
static int side_begin(bg_ctx* c, hipStream_t& main) {
  if (!c->sstream) {
    if (hipStreamCreateWithFlags(&c->sstream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->sfork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->sjoin, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      return bg_fail(c, BG_E_HIP, "side stream creation failed");
    }
  }
  BG_HIP(c, hipEventRecord(c->sfork, c->stream));
  BG_HIP(c, hipStreamWaitEvent(c->sstream, c->sfork, 0));
  c->defer_release = true;
  main = c->stream;
  c->stream = c->sstream;
  return 0;
}
static void side_end(bg_ctx* c, hipStream_t main) {
  (void)hipEventRecord(c->sjoin, c->sstream);  // (on errors too: side_join waits for what was queued)
  c->stream = main;
}
static int side_join(bg_ctx* c) {
  if (!c->defer_release) return 0;
  int rc = bg_hip_ok(c, hipStreamWaitEvent(c->stream, c->sjoin, 0));
  c->defer_release = false;
  for (auto& b : c->deferred) c->free_list.push_back(b);
  c->deferred.clear();
  return rc;
}

// the scout pass: k_scout + the row offsets' scan (run on the side stream beside the run
// discovery and the previous input's parse, it measured no faster: bedmap 21.93 -> 22.23 ms,
// the parse slowed by as much as the scout was hidden, round 6)
static int scout_pass(bg_ctx* c, LoadState& S, uint64_t* ctr) {
  const uint32_t nt = S.ntiles;
  BG_LAUNCH(c, "k_scout", k_scout, dim3(bg_blocks(nt, SCOUT_TILES)), dim3(BG_NT), S.txt, S.nb, nt,
            S.cnt, S.fnl);
  BG_HIP(c, hipGetLastError());
  return bg_scan_sum_u64(c, S.cnt, S.row0, nt, &ctr[0]);
}

// phase 1 (no host round trip): text to HBM, scout, row offsets, chromosome-run records.
// ctr[0] = rows, ctr[1] = boundary tiles (u32), ctr[2] = run records (u32)
static int scout_one(bg_ctx* c, const bg_input& in, bg_table* T, LoadState& S, uint64_t* ctr) {
  T->kind = in.kind;
  const uint8_t* txt;
  if (in.on_device) {
    if (((uintptr_t)in.data & 15) != 0) return bg_fail(c, BG_E_ARG, "device text must be 16-byte aligned");
    txt = (const uint8_t*)in.data;
  } else {
    T->own_text = (char*)bg_alloc(c, in.nbytes + 16);
    if (!T->own_text) return BG_E_NOMEM;
    if (in.nbytes)
      BG_HIP(c, hipMemcpyAsync(T->own_text, in.data, in.nbytes, hipMemcpyHostToDevice, c->stream));
    txt = (const uint8_t*)T->own_text;
  }
  T->text = (const char*)txt;
  T->nbytes = in.nbytes;
  S.txt = txt;
  S.nb = in.nbytes;
  S.ntiles = in.nbytes ? bg_blocks(in.nbytes, TT) : 0;
  if (S.ntiles == 0) return 0;
  const uint32_t nt = S.ntiles;
  // a boundary tile records at most one entry per line (+1)
  S.rc = (uint32_t)std::min<uint64_t>(REC_CAP, (uint64_t)nt * (TT / 6 + 2) + 16);
  const bool set = in.kind == BG_BED3_SET;  // no row numbers: no scout pass
  // row loads: the scout pass counts every tile's lines first (k_scout, a streaming read at
  // ~6 TB/s) for the rows' numbers (a decoupled look-back inside round 5's row parse instead measured
  // 2x slower in round 5: bedmap 50M x 500M k_parse 11.4 -> 20.7 ms)
  const bool scout = !set;
  if (scout) {
    S.row0 = (uint64_t*)bg_alloc(c, 8ull * nt);
    S.cnt = (uint64_t*)bg_alloc(c, 8ull * nt);
    S.fnl = (uint32_t*)bg_alloc(c, 4ull * nt);
    if (!S.row0 || !S.cnt || !S.fnl) return BG_E_NOMEM;
  }
  S.fls = (int64_t*)bg_alloc(c, 8ull * nt);
  S.fhash = (uint64_t*)bg_alloc(c, 8ull * nt);
  S.blist = (uint32_t*)bg_alloc(c, 4ull * nt);
  S.recs = (RunRec*)bg_alloc(c, sizeof(RunRec) * (size_t)S.rc);
  if (!S.fls || !S.fhash || !S.blist || !S.recs)
    return BG_E_NOMEM;
  if (scout) {
    int rc = scout_pass(c, S, ctr);
    if (rc) return rc;
  }
  BG_LAUNCH(c, "k_tokhash", k_tokhash, dim3(bg_blocks(nt, 256)), dim3(256), txt, S.nb, nt, scout ? S.fnl : nullptr,
            S.fls, S.fhash);
  BG_HIP(c, hipGetLastError());
  uint32_t* nbound = reinterpret_cast<uint32_t*>(&ctr[1]);
  uint32_t* nrec = reinterpret_cast<uint32_t*>(&ctr[2]);
  BG_LAUNCH(c, "k_boundary", k_boundary, dim3(bg_blocks(nt, 256)), dim3(256), S.fls, S.fhash, nt,
            S.blist, nbound);
  BG_HIP(c, hipGetLastError());
  BG_LAUNCH(c, "k_tile_runs", k_tile_runs, dim3(std::min<uint32_t>(nt, 1024)), dim3(BG_NT), txt,
            S.nb, S.blist, nbound, S.fls, nt, S.rc, S.recs, nrec);
  BG_HIP(c, hipGetLastError());
  return 0;
}

// phase 2 (host): the records of one input -> its chromosome runs, strcmp order checked
static int runs_one(bg_ctx* c, int idx, const bg_input& in, bg_table* T, LoadState& S) {
  const uint32_t nr = S.nrec;
  const RunRec* H = S.hrec;
  std::vector<uint32_t> ord(nr);
  for (uint32_t k = 0; k < nr; ++k) ord[k] = k;
  std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return H[a].pos < H[b].pos; });
  T->run_name.clear();
  S.run_pos.clear();
  S.run_hash.clear();
  int64_t last_pos = -1;
  uint64_t last_hash = 0;
  for (uint32_t k : ord) {  // runs: records by position, consecutive duplicates removed
    if (!S.run_pos.empty() && (last_pos == H[k].pos || last_hash == H[k].hash)) continue;
    if (H[k].len > BG_CHR_MAX) return bg_fail(c, BG_E_CHROM, "chromosome name longer than 127 characters");
    if (H[k].len == 0) {  // a whitespace-only line opens a tile: bg_load strips such lines
      S.blank = true;
      return bg_fail(c, BG_E_BLANK, "blank line");
    }
    last_pos = H[k].pos;
    last_hash = H[k].hash;
    S.run_pos.push_back(H[k].pos);
    S.run_hash.push_back(H[k].hash);
    T->run_name.emplace_back(H[k].name, strnlen(H[k].name, 128));
  }
  for (size_t k = 1; k < T->run_name.size(); ++k) {
    if (strcmp(T->run_name[k - 1].c_str(), T->run_name[k].c_str()) >= 0) {
      char msg[400];
      snprintf(msg, sizeof(msg),
               "input %d: chromosome '%s' follows '%s' (%s input is not sorted per sort-bed)",
               idx + 1, T->run_name[k].c_str(), T->run_name[k - 1].c_str(), kind_name(in.kind));
      return bg_fail(c, BG_E_UNSORTED, msg);
    }
  }
  return 0;
}

// run table of one input on the device (+ the runs each tile can hold)
// (tb: the tile size the per-tile run ranges are for; TW for k_parse_set_v's sub-tiles)
static int upload_runs(bg_ctx* c, bg_table* T, LoadState& S,
                       const std::map<std::string, int32_t>& gid, RunTable& R, int tb = TT) {
  const uint32_t ntr = tb == TT ? S.ntiles : (uint32_t)bg_blocks(S.nb, (uint64_t)tb);
  const uint32_t nr = (uint32_t)S.run_pos.size();
  RunInfo* info = (RunInfo*)bg_pin_take(c, sizeof(RunInfo) * nr);
  if (!info) {
    S.info.resize(nr);
    info = S.info.data();
  }
  for (uint32_t k = 0; k < nr; ++k) {
    RunInfo& I = info[k];
    const std::string& nm = T->run_name[k];
    I.pos = S.run_pos[k];
    I.hash = S.run_hash[k];
    I.tlen = (uint32_t)nm.size();
    uint8_t tb[16] = {0};
    memcpy(tb, nm.data(), std::min<size_t>(16, nm.size()));
    memcpy(&I.tlo, tb, 8);
    memcpy(&I.thi, tb + 8, 8);
    I.gid = gid.at(nm);
  }
  S.d_info = (RunInfo*)bg_alloc(c, sizeof(RunInfo) * nr);
  S.d_row = (uint64_t*)bg_alloc(c, 8ull * nr);
  S.rlo = (uint32_t*)bg_alloc(c, 4ull * ntr);
  S.rhi = (uint32_t*)bg_alloc(c, 4ull * ntr);
  if (!S.d_info || !S.d_row || !S.rlo || !S.rhi) return BG_E_NOMEM;
  BG_HIP(c, hipMemcpyAsync(S.d_info, info, sizeof(RunInfo) * nr, hipMemcpyHostToDevice, c->stream));
  BG_HIP(c, hipMemsetAsync(S.d_row, 0xff, 8ull * nr, c->stream));
  R = RunTable{S.d_info, S.d_row, nr};
  if (tb == TT)
    BG_LAUNCH(c, "k_run_range", k_run_range<TT>, dim3(bg_blocks(ntr, 256)), dim3(256), R, ntr, S.rlo, S.rhi);
  else
    BG_LAUNCH(c, "k_run_range", k_run_range<TW>, dim3(bg_blocks(ntr, 256)), dim3(256), R, ntr, S.rlo, S.rhi);
  BG_HIP(c, hipGetLastError());
  return 0;
}

// phase 3 (no host round trip): keyed parse with the global dictionary
static int parse_one(bg_ctx* c, const bg_input& in, bg_table* T, LoadState& S,
                     const std::map<std::string, int32_t>& gid, bg_dstatus* st) {
  const uint64_t na = T->n ? T->n : 1;
  T->ks = (int64_t*)bg_alloc(c, 8 * na);
  T->ke = (int64_t*)bg_alloc(c, 8 * na);
  if (!T->ks || !T->ke) return BG_E_NOMEM;
  if (in.kind == BG_BED3_REST || in.kind == BG_BED5_REST) {
    T->rest_off = (uint64_t*)bg_alloc(c, 8 * na);
    T->rest_len = (uint32_t*)bg_alloc(c, 4 * na);
    if (!T->rest_off || !T->rest_len) return BG_E_NOMEM;
  }
  if (in.kind == BG_BED5 || in.kind == BG_BED5_REST) {
    T->score = (double*)bg_alloc(c, 8 * na);
    if (!T->score) return BG_E_NOMEM;
  }
  const uint32_t nr = (uint32_t)S.run_pos.size();
  if (S.ntiles == 0 || T->n == 0 || nr == 0) return 0;
  // k_parse_rv (two waves per tile, run ranges per 4 KiB sub-tile) unless the load is a redo
  // with k_parse (a sub-tile of more than LCAP_R lines: BG_ROW_OVERFLOW)
  const bool rv = !c->row_wide;
  RunTable R;
  int rc = upload_runs(c, T, S, gid, R, rv ? TW : TT);
  if (rc) return rc;
  // scores past the loader's fast paths (parse_score: isint -1) go to k_score_big (finish_one);
  // the list holds 2^20 (BEDGPU_BIGCAP) unless a load that overflowed it is being redone with
  // the count it found (c->big_need)
  if (T->score) {
    static const uint64_t cap0 = [] {
      const char* e = getenv("BEDGPU_BIGCAP");
      return e ? (uint64_t)std::max(1, atoi(e)) : (uint64_t)(1u << 20);
    }();
    S.bigcap = (uint32_t)std::min<uint64_t>(T->n, std::max<uint64_t>(cap0, c->big_need));
    S.big = (uint64_t*)bg_alloc(c, 16ull * (S.bigcap ? S.bigcap : 1));
    if (!S.big) return BG_E_NOMEM;
  }
  const int kind = in.kind == BG_BED5_REST ? BG_BED5 : in.kind;
  if (rv) {
#define BG_ROWV(RE, SC)                                                                                    \
  BG_LAUNCH(c, "k_parse", (k_parse_rv<RE, SC>), dim3(S.ntiles), dim3(128), S.txt, S.nb, T->n, S.row0, S.rlo, \
            S.rhi, R, T->ks, T->ke, T->rest_off, T->rest_len, T->score, st, S.big, S.bigcap)
    const bool re = T->rest_off != nullptr, sc = kind == BG_BED5;
    if (re && sc) BG_ROWV(true, true);
    else if (re) BG_ROWV(true, false);
    else if (sc) BG_ROWV(false, true);
    else BG_ROWV(false, false);
#undef BG_ROWV
  } else {
    BG_LAUNCH(c, "k_parse", k_parse, dim3(S.ntiles), dim3(BG_NT), S.txt, S.nb, T->n, S.row0, S.rlo, S.rhi, kind, R,
              T->ks, T->ke, T->rest_off, T->rest_len, T->score, st, S.big, S.bigcap);
  }
  BG_HIP(c, hipGetLastError());
  BG_LAUNCH(c, "k_check_bounds", k_check_bounds, dim3(bg_blocks(S.ntiles, 256)), dim3(256), T->ks,
            S.row0, S.ntiles, T->n, st);
  BG_HIP(c, hipGetLastError());
  S.nrows_run = nr;  // copied back after every input's parse is queued
  return 0;
}

// phase 3 for BG_BED3_SET: parse -> staged local components -> global components
// (T->cs/T->ce, capacity = rows; the count lands in st->pad[0] and comes back with the
// statuses)
static int parse_set_one(bg_ctx* c, bg_table* T, LoadState& S,
                         const std::map<std::string, int32_t>& gid, bg_dstatus* st) {
  T->is_set = true;
  const uint32_t nr = (uint32_t)S.run_pos.size();
  const uint32_t nt = (uint32_t)bg_blocks(S.nb, (uint64_t)TW);  // staging units: 4 KiB sub-tiles
  const uint64_t cap = nt ? (uint64_t)nt * SCAP_W : 1;  // components <= staged slots
  T->cs = (int64_t*)bg_alloc(c, 8 * cap);
  T->ce = (int64_t*)bg_alloc(c, 8 * cap);
  if (!T->cs || !T->ce) return BG_E_NOMEM;
  if (nt == 0 || nr == 0) return 0;
  RunTable R;
  int rc = upload_runs(c, T, S, gid, R, TW);
  if (rc) return rc;
  S.lcs = (int64_t*)bg_alloc(c, 8 * cap);
  S.lce = (int64_t*)bg_alloc(c, 8 * cap);
  S.tmax = (int64_t*)bg_alloc(c, 8ull * nt);
  S.tlast = (int64_t*)bg_alloc(c, 8ull * nt);
  S.mex = (int64_t*)bg_alloc(c, 8ull * nt);
  S.tbase = (uint64_t*)bg_alloc(c, 8ull * nt);
  S.nloc = (uint64_t*)bg_alloc(c, 8ull * nt);
  S.tcnt = (uint64_t*)bg_alloc(c, 8ull * nt);
  S.absorbed = (uint32_t*)bg_alloc(c, 4ull * nt);
  S.tgb = (int64_t*)bg_alloc(c, 8ull * nt);
  S.cnt = (uint64_t*)bg_alloc(c, 8ull * nt);  // rows per tile
  if (!S.lcs || !S.lce || !S.tmax || !S.tlast || !S.mex || !S.tbase || !S.nloc ||
      !S.tcnt || !S.absorbed || !S.cnt || !S.tgb)
    return BG_E_NOMEM;
  SetTiles TS{S.tmax, S.tlast, S.tbase, S.nloc, S.absorbed, S.cnt, S.tgb};
  BG_LAUNCH(c, "k_parse_set", k_parse_set_v, dim3(nt), dim3(64), S.txt, S.nb, nt, S.rlo, S.rhi, R,
            S.lcs, S.lce, TS, st);
  BG_HIP(c, hipGetLastError());
  S.set_nt = nt;  // parse_set_merge follows
  return 0;
}

// the passes after k_parse_set: the running max of earlier tiles (mex), the absorbed local
// components and each tile's count (k_set_count), their offsets (scanned in place; the total
// to st->pad[0]) — set_merge_count — and the final component columns (k_set_write,
// set_merge_write). bg_load runs an input's count passes on the side stream beside the next
// input's parse, and its k_set_write (bandwidth-bound) on the side stream only once that
// parse has finished, beside the next input's own merge passes: run beside the parse it took
// the parse from 0.85 to 0.98 ms (round 6)
static int set_merge_count(bg_ctx* c, LoadState& S, bg_dstatus* st) {
  const uint32_t nt = S.set_nt;
  SetTiles TS{S.tmax, S.tlast, S.tbase, S.nloc, S.absorbed, S.cnt, S.tgb};
  int rc;
  if ((rc = bg_scan_max_i64(c, S.tmax, S.mex, nt, LLONG_MIN))) return rc;
  BG_LAUNCH(c, "k_set_count", k_set_count, dim3(bg_blocks(nt, BG_NT)), dim3(BG_NT), S.lcs, TS,
            (const int64_t*)S.mex, nt, S.tcnt, st, 0u);
  BG_HIP(c, hipGetLastError());
  return bg_scan_sum_u64(c, S.tcnt, S.tcnt, nt, (uint64_t*)&st->pad[0]);
}
static int set_merge_write(bg_ctx* c, bg_table* T, LoadState& S) {
  const uint32_t nt = S.set_nt;
  S.set_nt = 0;
  SetTiles TS{S.tmax, S.tlast, S.tbase, S.nloc, S.absorbed, S.cnt, S.tgb};
  BG_LAUNCH(c, "k_set_write", k_set_write, dim3(bg_blocks(nt, SW_TILES)), dim3(BG_NT), S.lcs,
            S.lce, TS, (const int64_t*)S.mex, (const uint64_t*)S.tcnt, nt, T->cs, T->ce, 0u, nt,
            (const uint64_t*)nullptr, (unsigned long long*)nullptr);
  BG_HIP(c, hipGetLastError());
  return 0;
}
static int parse_set_merge(bg_ctx* c, bg_table* T, LoadState& S, bg_dstatus* st) {
  const int rc = set_merge_count(c, S, st);
  return rc ? rc : set_merge_write(c, T, S);
}

// the side stream from the ctx stream's current position: count passes (write == false) or
// the deferred k_set_write (write == true)
static int set_merge_side(bg_ctx* c, bg_table* T, LoadState& S, bg_dstatus* st, bool write) {
  hipStream_t main;
  int rc = side_begin(c, main);
  if (rc) return rc;
  rc = write ? set_merge_write(c, T, S) : set_merge_count(c, S, st);
  side_end(c, main);
  return rc;
}

// after phase 3: per-input status, flags and the run -> row table
static int finish_one(bg_ctx* c, int idx, const bg_input& in, bg_table* T, LoadState& S,
                      const bg_dstatus& h) {
  T->run_row0.assign(1, 0);
  if (T->is_set) {  // errors / overflow were handled by bg_load (re-read with row columns)
    T->n = h.pad[1];
    T->nc = h.pad[0];
    T->has_zero_len = (h.flags & 2ULL) != 0;
    T->run_row0.push_back(T->n);
    if (S.ntiles == 0 || T->n == 0) T->run_name.clear();
    return 0;
  }
  if (S.ntiles == 0 || T->n == 0 || S.run_pos.empty()) {
    T->run_name.clear();
    return 0;
  }
  int rc = report_status(c, idx, h);
  if (rc) return rc;
  if (h.nbig) {  // scores past the fast paths: exact big-number conversion (bg_strtod.h)
    if (h.nbig > S.bigcap || !T->score)  // (bg_load redoes a load whose list overflowed)
      return bg_fail(c, BG_E_UNSUPPORTED, "too many scores needing the exact big-number conversion");
    BG_LAUNCH(c, "k_score_big", k_score_big, dim3(bg_blocks(h.nbig, 64)), dim3(64), S.txt, S.nb, S.big, h.nbig,
              T->score);
    rc = bg_hip_ok(c, hipGetLastError());
    if (rc) return rc;
  }
  if ((in.kind == BG_BED5 || in.kind == BG_BED5_REST) && (h.flags & 1ULL)) T->score_int = false;
  T->has_zero_len = (h.flags & 2ULL) != 0;
  T->maxlen = h.maxlen;
  // a trailing run may own only the dropped unterminated last line: no rows
  uint32_t nkeep = S.hrow ? S.nrows_run : 0;
  while (nkeep > 0 && S.hrow[nkeep - 1] == ~0ULL) --nkeep;
  T->run_name.resize(nkeep);
  T->run_row0.clear();
  for (uint32_t k = 0; k < nkeep; ++k) T->run_row0.push_back(S.hrow[k]);
  T->run_row0.push_back(T->n);
  return 0;
}

static int build_dictionary(bg_ctx* c, bg_set* s, std::map<std::string, int32_t>& gid,
                            std::string& packed, std::vector<uint32_t>& off,
                            std::vector<uint32_t>& len) {
  std::vector<std::string> all;
  for (bg_table* T : s->t)
    for (auto& nm : T->run_name) all.push_back(nm);
  std::sort(all.begin(), all.end(),
            [](const std::string& a, const std::string& b) { return strcmp(a.c_str(), b.c_str()) < 0; });
  all.erase(std::unique(all.begin(), all.end()), all.end());
  if (all.size() >= (1u << 22)) return bg_fail(c, BG_E_UNSUPPORTED, "too many chromosomes");
  s->names = all;
  for (size_t k = 0; k < all.size(); ++k) gid[all[k]] = (int32_t)k;
  off.assign(all.size() + 1, 0);
  len.assign(all.size() + 1, 0);
  for (size_t k = 0; k < all.size(); ++k) {
    off[k] = (uint32_t)packed.size();
    len[k] = (uint32_t)all[k].size();
    s->max_name_len = std::max<uint32_t>(s->max_name_len, len[k]);
    packed += all[k];
  }
  // one device block: names (16-B padded) | offsets | lengths, one copy from pinned staging
  const size_t nbn = (packed.size() + 16) & ~(size_t)15, nbo = 4 * off.size(), blk = nbn + 2 * nbo;
  s->d_names = (char*)bg_alloc(c, blk);
  if (!s->d_names) return BG_E_NOMEM;
  s->d_name_off = (uint32_t*)(s->d_names + nbn);
  s->d_name_len = (uint32_t*)(s->d_names + nbn + nbo);
  char* h = (char*)bg_pin_take(c, blk);
  std::vector<char> hv;
  if (!h) {
    hv.resize(blk);
    h = hv.data();
  }
  memcpy(h, packed.data(), packed.size());
  memcpy(h + nbn, off.data(), nbo);
  memcpy(h + nbn + nbo, len.data(), nbo);
  BG_HIP(c, hipMemcpyAsync(s->d_names, h, blk, hipMemcpyHostToDevice, c->stream));
  if (!hv.empty()) BG_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

// Two host round trips per call, whatever the number of inputs: run-record counts (with the
// first records), final statuses (a third, for the rest of the records, only past REC_SPEC).
#include <chrono>
static double hp_now() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define HP(tag) do { if (hp) fprintf(stderr, "hp %-10s %9.1f\n", tag, hp_now() - hp0); } while (0)
extern "C" int bg_load(bg_ctx* c, int n, const bg_input* inputs, bg_set** out) {
  static const bool hp = getenv("BEDGPU_HOSTPROF") != nullptr;
  const double hp0 = hp ? hp_now() : 0;
  if (!c || n <= 0 || !inputs || !out) return BG_E_ARG;
  *out = nullptr;
  bg_set* s = new bg_set();
  s->ctx = c;
  std::vector<LoadState> st(n);
  // per input: 8 counters (phase 1) + one status block (phase 3)
  uint64_t* ctr = (uint64_t*)bg_alloc(c, 64ull * n);
  bg_dstatus* dst = (bg_dstatus*)bg_alloc(c, sizeof(bg_dstatus) * n);
  bg_pin_reset(c);
  uint64_t* hctr = (uint64_t*)bg_pin_take(c, 64ull * n);
  bg_dstatus* hst = (bg_dstatus*)bg_pin_take(c, sizeof(bg_dstatus) * n);
  std::string packed;
  std::vector<uint32_t> off, len;
  std::map<std::string, int32_t> gid;
  int rc = (!ctr || !dst || !hctr || !hst) ? BG_E_NOMEM : 0;
  HP("alloc");
  if (!rc) rc = bg_hip_ok(c, hipMemsetAsync(ctr, 0, 64ull * n, c->stream));
  HP("memset");
  for (int i = 0; i < n && !rc; ++i) {
    s->t.push_back(new bg_table());
    rc = scout_one(c, inputs[i], s->t[i], st[i], ctr + 8ull * i);
  }
  HP("scout");
  // round trip 1: rows and record counts of every input, with the first REC_SPEC records
  // of each copied along speculatively (a genome's inputs have a few dozen: round trip 2,
  // the rest of the records, is then skipped)
  constexpr uint32_t REC_SPEC = 256;
  std::vector<RunRec*> spec(n, nullptr);
  for (int i = 0; i < n && !rc; ++i) {
    const uint32_t k = std::min<uint32_t>(REC_SPEC, st[i].rc);
    if (!st[i].ntiles || !k) continue;
    spec[i] = (RunRec*)bg_pin_take(c, sizeof(RunRec) * k);
    if (spec[i]) rc = bg_hip_ok(c, hipMemcpyAsync(spec[i], st[i].recs, sizeof(RunRec) * k, hipMemcpyDeviceToHost, c->stream));
  }
  if (!rc) rc = bg_hip_ok(c, hipMemcpyAsync(hctr, ctr, 64ull * n, hipMemcpyDeviceToHost, c->stream));
  if (!rc) rc = bg_hip_ok(c, hipStreamSynchronize(c->stream));
  HP("rt1");
  bool rt2 = false;
  for (int i = 0; i < n && !rc; ++i) {
    LoadState& S = st[i];
    s->t[i]->n = S.ntiles ? hctr[8ull * i] : 0;
    const uint32_t nr = (uint32_t)hctr[8ull * i + 2];
    if (nr > S.rc) { rc = bg_fail(c, BG_E_UNSUPPORTED, "too many chromosome changes in one input"); break; }
    S.nrec = nr;
    if (!nr) continue;
    if (spec[i] && nr <= REC_SPEC) {
      S.hrec = spec[i];
      continue;
    }
    RunRec* h = (RunRec*)bg_pin_take(c, sizeof(RunRec) * nr);
    if (!h) { rc = BG_E_NOMEM; break; }
    S.hrec = h;
    rt2 = true;
    rc = bg_hip_ok(c, hipMemcpyAsync(h, S.recs, sizeof(RunRec) * nr, hipMemcpyDeviceToHost, c->stream));
  }
  // round trip 2: the run records (only when an input has more than REC_SPEC)
  HP("rec_copy");
  if (!rc && rt2) rc = bg_hip_ok(c, hipStreamSynchronize(c->stream));
  HP("rt2");
  for (int i = 0; i < n && !rc; ++i) rc = runs_one(c, i, inputs[i], s->t[i], st[i]);
  bg_mark(c, "scout");
  if (!rc) rc = build_dictionary(c, s, gid, packed, off, len);
  if (!rc) {
    for (int i = 0; i < n; ++i) {
      memset(&hst[i], 0, sizeof(bg_dstatus));
      hst[i].first_bad = ~0ULL;
    }
    rc = bg_hip_ok(c, hipMemcpyAsync(dst, hst, sizeof(bg_dstatus) * n, hipMemcpyHostToDevice, c->stream));
  }
  HP("dict");
  // each set input's count passes on the side stream beside the next input's parse, its
  // k_set_write there once that parse is done (the last input's passes in line)
  int pending = -1;  // a set input whose k_set_write waits for the next parse
  for (int i = 0; i < n && !rc; ++i) {
    rc = inputs[i].kind == BG_BED3_SET ? parse_set_one(c, s->t[i], st[i], gid, dst + i)
                                       : parse_one(c, inputs[i], s->t[i], st[i], gid, dst + i);
    if (!rc && pending >= 0) {
      rc = set_merge_side(c, s->t[pending], st[pending], dst + pending, true);
      pending = -1;
    }
    if (!rc && st[i].set_nt) {
      if (i + 1 < n) {
        rc = set_merge_side(c, s->t[i], st[i], dst + i, false);
        pending = i;
      } else {
        rc = parse_set_merge(c, s->t[i], st[i], dst + i);
      }
    }
  }
  if (!rc && pending >= 0) rc = set_merge_side(c, s->t[pending], st[pending], dst + pending, true);
  {
    const int rj = side_join(c);  // (on errors too: the side stream's blocks return to the pool)
    if (!rc) rc = rj;
  }
  HP("parse_q");
  // round trip 3: statuses and run rows of every input (pageable copies block the host,
  // so they are issued only once all parses are queued)
  for (int i = 0; i < n && !rc; ++i)
    if (st[i].nrows_run) {
      st[i].hrow = (uint64_t*)bg_pin_take(c, 8ull * st[i].nrows_run);
      if (!st[i].hrow) { rc = BG_E_NOMEM; break; }
      rc = bg_hip_ok(c, hipMemcpyAsync(st[i].hrow, st[i].d_row, 8ull * st[i].nrows_run,
                                       hipMemcpyDeviceToHost, c->stream));
    }
  // (the status init above was read by the device before this copy overwrites it: stream order)
  if (!rc) rc = bg_hip_ok(c, hipMemcpyAsync(hst, dst, sizeof(bg_dstatus) * n, hipMemcpyDeviceToHost, c->stream));
  if (!rc) rc = bg_hip_ok(c, hipStreamSynchronize(c->stream));
  const bool hst_valid = rc == 0;
  HP("rt3");
  // a BG_BED3_SET input with an error (its exact line is not known) or a staging overflow:
  // the whole load is redone with that input's row columns (BG_BED3)
  bool redo = false, wide = false, setredo = false;
  for (int i = 0; i < n && !rc; ++i)
    if (inputs[i].kind == BG_BED3_SET && st[i].ntiles &&
        (hst[i].first_bad != ~0ULL || (hst[i].flags & BG_SET_OVERFLOW)))
      redo = setredo = true;
  // a row input with a sub-tile of more lines than k_parse_rv holds: redone with k_parse
  for (int i = 0; i < n && !rc; ++i)
    if (inputs[i].kind != BG_BED3_SET && st[i].ntiles && (hst[i].flags & BG_ROW_OVERFLOW)) redo = wide = true;
  // a row input with more long scores than its k_score_big list holds: redone with room for all
  uint64_t bigneed = 0;
  for (int i = 0; i < n && !rc; ++i)
    if (inputs[i].kind != BG_BED3_SET && st[i].ntiles && hst[i].first_bad == ~0ULL && hst[i].nbig > st[i].bigcap)
      bigneed = std::max<uint64_t>(bigneed, hst[i].nbig);
  if (bigneed) redo = true;
  for (int i = 0; i < n && !rc && !redo; ++i) rc = finish_one(c, i, inputs[i], s->t[i], st[i], hst[i]);
  // blank lines (k_blank_*): the load is redone on the texts without them, which then belong
  // to the new set
  std::vector<char*> stripped;
  std::vector<bg_input> unblank;
  if (rc == BG_E_BLANK) {
    rc = 0;
    bool changed = false;
    stripped.assign(n, nullptr);
    unblank.assign(inputs, inputs + n);
    for (int i = 0; i < n && !rc; ++i) {
      const bool b = st[i].blank || (hst_valid && (hst[i].nblank || (hst[i].first_bad != ~0ULL &&
                                                                    (hst[i].first_bad & 0xff) == ERR_BLANK)));
      if (!st[i].ntiles || !b) continue;
      uint64_t nb2 = 0;
      rc = strip_blank_lines(c, st[i].txt, st[i].nb, &stripped[i], &nb2);
      if (!rc) unblank[i] = bg_input{stripped[i], nb2, 1, inputs[i].kind};
      if (!rc && nb2 != st[i].nb) changed = true;
    }
    if (!rc && !changed) rc = BG_E_BLANK;  // (cannot happen: a stripped text has no blank line)
    if (rc) {
      for (char* p : stripped) bg_release(c, p);
      unblank.clear();
    }
  }
  if (rc) (void)hipStreamSynchronize(c->stream);  // pending copies use the pinned staging
  for (auto& S : st) release_state(c, S);
  bg_release(c, ctr);
  bg_release(c, dst);
  if (!rc && !unblank.empty()) {
    bg_set_free(s);
    const int rc2 = bg_load(c, n, unblank.data(), out);
    for (int i = 0; i < n; ++i) {
      if (!stripped[i]) continue;
      if (rc2 == 0) (*out)->t[i]->own_text = stripped[i];
      else bg_release(c, stripped[i]);
    }
    return rc2;
  }
  if (rc || redo) {
    bg_set_free(s);
    if (rc) return rc;
    std::vector<bg_input> rows(inputs, inputs + n);
    for (auto& in : rows)
      if (setredo && in.kind == BG_BED3_SET) in.kind = BG_BED3;
    const bool w0 = c->row_wide;
    const uint64_t b0 = c->big_need;
    if (wide) c->row_wide = true;
    if (bigneed) c->big_need = std::max(b0, bigneed);
    const int rc2 = bg_load(c, n, rows.data(), out);
    c->row_wide = w0;
    c->big_need = b0;
    return rc2;
  }
  for (bg_table* T : s->t)  // keep every column non-null for empty inputs
    if (T->is_set) {
      if (!T->cs) {
        T->cs = (int64_t*)bg_alloc(c, 8);
        T->ce = (int64_t*)bg_alloc(c, 8);
      }
    } else if (!T->ks) {
      T->ks = (int64_t*)bg_alloc(c, 8);
      T->ke = (int64_t*)bg_alloc(c, 8);
    }
  bg_mark(c, "parse");
  *out = s;
  return 0;
}

extern "C" int bg_set_rows(const bg_set* s, int i, uint64_t* rows) {
  if (!s || i < 0 || i >= (int)s->t.size() || !rows) return BG_E_ARG;
  *rows = s->t[i]->n;
  return 0;
}

extern "C" void bg_set_free(bg_set* s) {
  if (!s) return;
  bg_ctx* c = s->ctx;
  for (bg_table* T : s->t) {
    bg_release(c, T->ks);
    bg_release(c, T->ke);
    bg_release(c, T->cs);
    bg_release(c, T->ce);
    bg_release(c, T->own_text);
    bg_release(c, T->rest_off);
    bg_release(c, T->rest_len);
    bg_release(c, T->score);
    delete T;
  }
  bg_release(c, s->d_names);  // (offsets and lengths live in the same block)
  delete s;
}
