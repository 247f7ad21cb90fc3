// bg_sortbed.hip — sort-bed on the GPU: every line of the inputs, sorted.
//
// Reference: applications/bed/sort-bed/src (Sort.cpp:41-234, SortDetails.cpp:536-1118,
// Structures.hpp:45-86). The reference reads each line with its own field grammar
// (SortDetails.cpp:625-781: tab or space separators in the first three fields, digits
// only, <= 12 digits, end > start, headers "browser"/"track"/"#"/"@" only before the first
// data line of each file, blank lines skipped), keeps chrom / start / end and the rest of
// the line after the whitespace that follows `end` ("\t%[^\n]", none when empty), sorts
// chromosomes by strcmp (lexCompareBedData :1202-1208) and each chromosome's rows by
// (start, end, rest strcmp, no rest first) (bcd_cmp), and prints
// "%s\t%ld\t%ld" + ("\t%s\n" | "\n") (printBed :1120-1140).
//
// GPU form:
//   k_sb_count / k_sb_starts  line starts of each input (newlines per 4 KiB tile, scan,
//                             write) into one array of absolute device addresses
//   k_sb_first                per input, the first line that is not blank and not a header
//                             candidate (headers are skipped only before it)
//   k_sb_parse                one thread per line: the reference's checks in its order
//                             (first failing line by atomicMin on (line << 8 | code)),
//                             fields of the data lines, a 64-bit hash of the chromosome
//   dictionary                data lines sorted by hash (radix), one name per distinct hash
//                             to the host, ranked by strcmp, ranks looked up per line and
//                             every line's name compared with its representative's
//   sort                      stable LSD radix: by end, then by (rank << 40 | start)
//   sb_order_ties             runs of equal (chromosome, start, end): ordered by the rest
//                             (strcmp; no rest first) by rounds of radix refinement on
//                             8-byte rest chunks (k_sb_tflag/tgather/trid/tpick/tput)
// The output is a RES_MULTI result (chrom/start/end keys + the rest's address and length)
// whose rest is printed after a tab.
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "bg_internal.h"

#define SB_TILE 4096

enum {
  SB_OK = 0,
  SB_LEADING_WS = 1,   // "Row begins with a tab or space"
  SB_NO_TAB = 2,       // "No tabs/spaces found"
  SB_CHROM_LONG = 3,   // "Chromosome name too long"
  SB_NO_START_SEP = 4, // "No tabs/spaces found after the start coordinate"
  SB_START_LONG = 5,   // "Start coordinate is too large. Max decimal digits"
  SB_START_EMPTY = 6,  // "Consecutive tabs and/or spaces between chromosome and start"
  SB_START_NONNUM = 7, // "Non-numeric start coordinate"
  SB_NO_EOL = 8,       // "No end of line found"
  SB_END_LONG = 9,     // "End coordinate is too large. Max decimal digits"
  SB_END_EMPTY = 10,   // "Extra tab and/or space found in between start and end"
  SB_END_NONNUM = 11,  // "Non-numeric end coordinate"
  SB_END_LE_START = 12,// "Genomic end coordinate is less than (or equal to) start"
  SB_ID_LONG = 13,     // "ID field too long"
  SB_ROW_LONG = 14,    // "BED row length exceeds capacity"
};
#define SB_CHR_MAX 127
#define SB_ID_MAX 16383
#define SB_LINE_MAX (127 + 16383 + 8 * 131072 + 2 * 12)  // TOKENS_MAX_LENGTH

// newlines at positions p < n - 1 (each starts a line at p + 1) per tile
__global__ void __launch_bounds__(BG_NT) k_sb_count(const char* __restrict__ t, uint64_t n,
                                                    uint64_t* __restrict__ cnt) {
  __shared__ uint32_t ws[BG_NT / 64];
  const uint64_t b0 = (uint64_t)blockIdx.x * SB_TILE;
  uint32_t c = 0;
  for (uint32_t q = threadIdx.x; q < SB_TILE; q += BG_NT) {
    const uint64_t p = b0 + q;
    c += (p + 1 < n && t[p] == '\n') ? 1u : 0u;
  }
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if (bg_lane() == 0) ws[bg_wave()] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = (uint64_t)ws[0] + ws[1] + ws[2] + ws[3];
}

// line starts (absolute addresses), in order; S[base] = the text's first byte
__global__ void __launch_bounds__(BG_NT) k_sb_starts(const char* __restrict__ t, uint64_t n,
                                                     const uint64_t* __restrict__ off,
                                                     uint64_t* __restrict__ S) {
  __shared__ uint32_t wc[BG_NT / 64];
  const uint64_t b0 = (uint64_t)blockIdx.x * SB_TILE;
  uint64_t q0 = off[blockIdx.x] + 1;
  const int lane = bg_lane(), w = bg_wave();
  if (blockIdx.x == 0 && threadIdx.x == 0) S[0] = (uint64_t)t;
  for (uint32_t j = 0; j < SB_TILE; j += BG_NT) {  // rounds of BG_NT bytes, in order
    const uint64_t p = b0 + j + threadIdx.x;
    const bool f = p + 1 < n && t[p] == '\n';
    const uint64_t bal = __ballot(f);
    if (lane == 0) wc[w] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint64_t pos = q0 + __popcll(bal & ((1ULL << lane) - 1));
    for (int v = 0; v < w; ++v) pos += wc[v];
    if (f) S[pos] = (uint64_t)(t + p + 1);
    q0 += (uint64_t)wc[0] + wc[1] + wc[2] + wc[3];
    __syncthreads();
  }
}

__device__ __forceinline__ bool sb_hdr(const char* p, uint64_t len) {
  auto pre = [&](const char* w, uint64_t k) {
    if (len < k) return false;
    for (uint64_t i = 0; i < k; ++i)
      if (p[i] != w[i]) return false;
    return true;
  };
  return pre("browser", 7) || pre("track", 5) || pre("#", 1) || pre("@", 1);
}

struct SbLines {
  const uint64_t* S;  // line start addresses (all inputs)
  const uint64_t* E;  // line end (address of its '\n', or of the text end)
  const uint8_t* TM;  // 1: the line ends with '\n' (0: the unterminated last line)
  const uint32_t* F;  // input of each line
  const uint64_t* L0; // first line index of each input
  uint64_t n;
};

// line ends (the '\n' of the line, or the text end for an unterminated last line) and inputs
__global__ void k_sb_ends(const uint64_t* __restrict__ S, uint64_t a, uint64_t b, uint64_t tend,
                          int last_nl, uint32_t f, uint64_t* __restrict__ E, uint8_t* __restrict__ TM,
                          uint32_t* __restrict__ F) {
  const uint64_t i = a + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b) return;
  F[i] = f;
  const bool last = i + 1 == b;
  E[i] = last ? tend - (last_nl ? 1 : 0) : S[i + 1] - 1;
  TM[i] = (!last || last_nl) ? 1 : 0;
}

__global__ void k_sb_iota(uint32_t* __restrict__ o, uint64_t n) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) o[j] = (uint32_t)j;
}

// per input: the first line that is neither blank nor a header candidate
__global__ void k_sb_first(SbLines A, unsigned long long* __restrict__ first) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.n) return;
  const char* p = (const char*)A.S[i];
  const uint64_t len = A.E[i] - A.S[i];
  if (len == 0 || sb_hdr(p, len)) return;
  atomicMin(&first[A.F[i]], (unsigned long long)i);
}

struct SbOut {
  uint8_t* flag;     // 1: a data line
  uint64_t* h;       // chromosome hash
  uint64_t* tok;     // chromosome token address
  uint32_t* toklen;
  int64_t* start;
  int64_t* end;
  uint64_t* rest;    // rest address (no rest: length 0)
  uint32_t* restlen;
};

__device__ __forceinline__ bool sb_ws(char c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r';
}

// one line through the reference's checks (SortDetails.cpp:625-781), in its order
__global__ void k_sb_parse(SbLines A, const unsigned long long* __restrict__ first, SbOut O,
                           unsigned long long* __restrict__ err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.n) return;
  O.flag[i] = 0;
  const char* p = (const char*)A.S[i];
  const uint64_t len = A.E[i] - A.S[i];
  const bool term = A.TM[i] != 0;  // else the unterminated last line
  int code = SB_OK;
  if (len == 0) return;  // a blank line
  if (len + 1 >= SB_LINE_MAX) code = SB_ROW_LONG;
  else if (p[0] == ' ' || p[0] == '\t') code = SB_LEADING_WS;
  else if (i < first[A.F[i]] && sb_hdr(p, len)) return;  // a header before the first row
  uint64_t c1 = 0, s0 = 0, s1 = 0, e1 = 0;
  if (!code) {
    while (c1 < len && p[c1] != '\t' && p[c1] != ' ') ++c1;
    if (c1 == len) code = SB_NO_TAB;
    else if (c1 > SB_CHR_MAX) code = SB_CHROM_LONG;
  }
  if (!code) {
    s0 = c1 + 1;
    s1 = s0;
    while (s1 < len && p[s1] != '\t' && p[s1] != ' ') ++s1;
    if (s1 == len) code = SB_NO_START_SEP;
    else if (s1 - s0 > 12) code = SB_START_LONG;
    else if (s1 == s0) code = SB_START_EMPTY;
    else
      for (uint64_t q = s0; q < s1; ++q)
        if (p[q] < '0' || p[q] > '9') { code = SB_START_NONNUM; break; }
  }
  if (!code) {
    e1 = s1 + 1;
    while (e1 < len && p[e1] != '\t' && p[e1] != ' ') ++e1;
    if (e1 == len && !term) code = SB_NO_EOL;  // no separator and no '\n' after end
    else if (e1 - (s1 + 1) > 12) code = SB_END_LONG;
    else if (e1 == s1 + 1) code = SB_END_EMPTY;
    else
      for (uint64_t q = s1 + 1; q < e1; ++q)
        if (p[q] < '0' || p[q] > '9') { code = SB_END_NONNUM; break; }
  }
  int64_t sv = 0, ev = 0;
  uint64_t r0 = len;
  if (!code) {
    for (uint64_t q = s0; q < s1; ++q) sv = sv * 10 + (p[q] - '0');
    for (uint64_t q = s1 + 1; q < e1; ++q) ev = ev * 10 + (p[q] - '0');
    if (ev <= sv) code = SB_END_LE_START;
  }
  if (!code) {
    r0 = e1;
    while (r0 < len && sb_ws(p[r0])) ++r0;  // "\t%[^\n]": whitespace skipped, then the rest
    if (r0 < len) {
      uint64_t q = r0;
      while (q < len && p[q] != '\t' && p[q] != ' ') ++q;
      if (q - r0 > SB_ID_MAX) code = SB_ID_LONG;
    }
  }
  if (code) {
    atomicMin(err, (unsigned long long)((i << 8) | (uint64_t)code));
    return;
  }
  uint64_t h = 1469598103934665603ULL;  // FNV-1a of the chromosome token
  for (uint64_t q = 0; q < c1; ++q) h = (h ^ (uint8_t)p[q]) * 1099511628211ULL;
  O.flag[i] = 1;
  O.h[i] = h;
  O.tok[i] = (uint64_t)p;
  O.toklen[i] = (uint32_t)c1;
  O.start[i] = sv;
  O.end[i] = ev;
  O.rest[i] = (uint64_t)(p + r0);
  O.restlen[i] = (uint32_t)(len - r0);
}

// the data lines, compacted: hash keys (for the dictionary sort) and the line index payload
__global__ void k_sb_gather_hash(const uint64_t* __restrict__ idx, uint64_t n,
                                 const uint64_t* __restrict__ h, uint64_t* __restrict__ key,
                                 uint32_t* __restrict__ val) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  key[j] = h[idx[j]];
  val[j] = (uint32_t)j;
}

// 1 where a run of equal hashes starts
__global__ void k_sb_uniq(const uint64_t* __restrict__ key, uint64_t n, uint8_t* __restrict__ f) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) f[j] = (j == 0 || key[j] != key[j - 1]) ? 1 : 0;
}

// one row per distinct hash: (hash, data-line ordinal, token address, token length)
__global__ void k_sb_reps(const uint64_t* __restrict__ upos, uint64_t nu, const uint64_t* __restrict__ key,
                          const uint32_t* __restrict__ val, const uint64_t* __restrict__ idx,
                          const uint64_t* __restrict__ tok, const uint32_t* __restrict__ toklen,
                          uint64_t* __restrict__ out) {
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nu) return;
  const uint64_t p = upos[u], d = val[p], i = idx[d];
  out[4 * u] = key[p];
  out[4 * u + 1] = d;
  out[4 * u + 2] = tok[i];
  out[4 * u + 3] = toklen[i];
}
__global__ void k_sb_names(const uint64_t* __restrict__ info, uint64_t nu, const uint64_t* __restrict__ off,
                           char* __restrict__ dst) {
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nu) return;
  const char* src = (const char*)info[4 * u + 2];
  for (uint64_t q = 0; q < info[4 * u + 3]; ++q) dst[off[u] + q] = src[q];
}

// data line -> chromosome rank (binary search of its hash among the representatives);
// its token must equal the representative's (a 64-bit hash collision fails the sort)
__global__ void k_sb_rank(const uint64_t* __restrict__ idx, uint64_t nd, const uint64_t* __restrict__ h,
                          const uint64_t* __restrict__ tok, const uint32_t* __restrict__ toklen,
                          const uint64_t* __restrict__ uh, const uint32_t* __restrict__ urank,
                          const uint64_t* __restrict__ urep, uint64_t nu, uint32_t* __restrict__ rank,
                          unsigned long long* __restrict__ bad) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nd) return;
  const uint64_t i = idx[j], x = h[i];
  uint64_t lo = 0, hi = nu;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (uh[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  const uint64_t r = idx[urep[lo]];
  bool same = toklen[r] == toklen[i];
  const char *a = (const char*)tok[i], *b = (const char*)tok[r];
  for (uint32_t q = 0; same && q < toklen[i]; ++q) same = a[q] == b[q];
  if (!same) atomicOr(bad, 1ULL);
  rank[j] = urank[lo];
}

__global__ void k_sb_key(const uint64_t* __restrict__ idx, const uint32_t* __restrict__ ord,
                         uint64_t nd, const int64_t* __restrict__ val, const uint32_t* __restrict__ rank,
                         bool with_rank, uint64_t* __restrict__ key) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nd) return;
  const uint32_t d = ord[j];
  const uint64_t v = (uint64_t)val[idx[d]];
  key[j] = with_rank ? (((uint64_t)rank[d] << BG_KEY_SHIFT) | v) : v;
}

// rest a < rest b by bcd_cmp: no rest first, else strcmp
__device__ __forceinline__ bool sb_rest_less(const uint64_t* R, const uint32_t* RL, uint64_t a,
                                             uint64_t b) {
  const uint32_t la = RL[a], lb = RL[b];
  if (la == 0 || lb == 0) return la == 0 && lb != 0;
  const uint8_t *x = (const uint8_t*)R[a], *y = (const uint8_t*)R[b];
  const uint32_t m = la < lb ? la : lb;
  for (uint32_t q = 0; q < m; ++q)
    if (x[q] != y[q]) return x[q] < y[q];
  return la < lb;
}

// Runs of equal (chromosome, start, end) are ordered by their rests (bcd_cmp: no rest first,
// else strcmp) in rounds of radix refinement, so a run of any length costs O(run) per round:
// round q sorts the rows still tied on (key, end, rest bytes [0, 8q)) by rest bytes
// [8q, 8q + 8) inside their run (stable radix by that chunk, then by run id), until no row is
// tied or every tied rest is exhausted (then the rows are identical).
// rest bytes [8q, 8q + 8) of row i, big-endian, zero-padded (no rest: 0, first)
__device__ __forceinline__ uint64_t sb_chunk(const uint64_t* R, const uint32_t* RL, uint64_t i, uint32_t q) {
  const uint32_t l = RL[i];
  const uint8_t* p = (const uint8_t*)R[i];
  uint64_t v = 0;
  for (uint32_t b = 0; b < 8; ++b) {
    const uint32_t o = 8 * q + b;
    v = (v << 8) | (o < l ? p[o] : 0u);
  }
  return v;
}
__device__ __forceinline__ bool sb_same(const uint64_t* k1, const uint64_t* idx, const int64_t* endv,
                                        const uint64_t* R, const uint32_t* RL, const uint32_t* ord, uint64_t a,
                                        uint64_t b, uint32_t q) {
  if (k1[a] != k1[b]) return false;
  const uint64_t ia = idx[ord[a]], ib = idx[ord[b]];
  if (endv[ia] != endv[ib]) return false;
  for (uint32_t z = 0; z < q; ++z)
    if (sb_chunk(R, RL, ia, z) != sb_chunk(R, RL, ib, z)) return false;
  return true;
}
// tied[j]: row j shares its run with a neighbour; start[j]: it opens a run; more[j]: a tied
// row whose rest goes past byte 8q (another round can still split the run)
__global__ void k_sb_tflag(const uint64_t* __restrict__ k1, const uint64_t* __restrict__ idx,
                           const int64_t* __restrict__ endv, const uint64_t* __restrict__ R,
                           const uint32_t* __restrict__ RL, const uint32_t* __restrict__ ord, uint64_t nd,
                           uint32_t q, uint64_t* __restrict__ tied, uint64_t* __restrict__ start,
                           unsigned long long* __restrict__ more) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nd) return;
  const bool prev = j > 0 && sb_same(k1, idx, endv, R, RL, ord, j, j - 1, q);
  const bool next = j + 1 < nd && sb_same(k1, idx, endv, R, RL, ord, j, j + 1, q);
  const bool t = prev || next;
  tied[j] = t;
  start[j] = t && !prev;
  if (t && RL[idx[ord[j]]] > 8 * q) atomicOr(more, 1ULL);
}
__global__ void k_sb_tgather(const uint64_t* __restrict__ tied, const uint64_t* __restrict__ pos,
                             const uint64_t* __restrict__ start, const uint64_t* __restrict__ rid,
                             const uint64_t* __restrict__ idx,
                             const uint64_t* __restrict__ R, const uint32_t* __restrict__ RL,
                             const uint32_t* __restrict__ ord, uint64_t nd, uint32_t q, uint64_t* __restrict__ P,
                             uint64_t* __restrict__ K, uint32_t* __restrict__ V, uint64_t* __restrict__ RID) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nd || !tied[j]) return;
  const uint64_t k = pos[j];
  P[k] = j;
  K[k] = sb_chunk(R, RL, idx[ord[j]], q);
  V[k] = (uint32_t)k;
  RID[k] = rid[j] + start[j];  // run starts up to and including j: one id per run
}
__global__ void k_sb_trid(const uint64_t* __restrict__ RID, const uint32_t* __restrict__ V, uint64_t m,
                          uint64_t* __restrict__ K) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < m) K[t] = RID[V[t]];
}
// the t-th row in (run, chunk) order takes the t-th tied position
__global__ void k_sb_tpick(const uint64_t* __restrict__ P, const uint32_t* __restrict__ V, uint64_t m,
                           const uint32_t* __restrict__ ord, uint32_t* __restrict__ tmp) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < m) tmp[t] = ord[P[V[t]]];
}
__global__ void k_sb_tput(const uint64_t* __restrict__ P, uint64_t m, const uint32_t* __restrict__ tmp,
                          uint32_t* __restrict__ ord) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < m) ord[P[t]] = tmp[t];
}
static int sb_order_ties(bg_ctx* c, const uint64_t* key, const uint64_t* idx, const int64_t* endv, const uint64_t* R,
                         const uint32_t* RL, uint64_t nd, uint32_t* ord) {
  uint64_t* tied = (uint64_t*)bg_alloc(c, 8 * (nd + 1));
  uint64_t* start = (uint64_t*)bg_alloc(c, 8 * (nd + 1));
  uint64_t* pos = (uint64_t*)bg_alloc(c, 8 * (nd + 1));
  uint64_t* rid = (uint64_t*)bg_alloc(c, 8 * (nd + 1));
  unsigned long long* more = (unsigned long long*)bg_alloc(c, 8);
  if (!tied || !start || !pos || !rid || !more) return BG_E_NOMEM;
  int rc = 0;
  for (uint32_t q = 0; !rc; ++q) {
    BG_HIP(c, hipMemsetAsync(more, 0, 8, c->stream));
    BG_LAUNCH(c, "k_sb_tflag", k_sb_tflag, dim3(bg_blocks(nd, BG_NT)), dim3(BG_NT), key, idx, endv, R, RL, ord, nd, q,
              tied, start, more);
    BG_HIP(c, hipGetLastError());
    uint64_t m = 0, hm = 0;
    if ((rc = bg_scan_sum_u64(c, tied, pos, nd, pos + nd)) || (rc = bg_fetch_u64(c, pos + nd, &m))) break;
    if ((rc = bg_fetch_u64(c, (const uint64_t*)more, &hm))) break;
    if (m == 0 || !hm) break;  // nothing tied, or every tied rest already compared in full
    if ((rc = bg_scan_sum_u64(c, start, rid, nd, nullptr))) break;  // run starts before each row
    uint64_t* P = (uint64_t*)bg_alloc(c, 8 * m);
    uint64_t* K = (uint64_t*)bg_alloc(c, 8 * m);
    uint32_t* V = (uint32_t*)bg_alloc(c, 4 * m);
    uint64_t* RID = (uint64_t*)bg_alloc(c, 8 * m);
    uint32_t* tmp = (uint32_t*)bg_alloc(c, 4 * m);
    if (!P || !K || !V || !RID || !tmp) rc = BG_E_NOMEM;
    const dim3 gm(bg_blocks(m, BG_NT));
    if (!rc) {
      BG_LAUNCH(c, "k_sb_tgather", k_sb_tgather, dim3(bg_blocks(nd, BG_NT)), dim3(BG_NT), tied, pos, start, rid,
                idx, R, RL, ord, nd, q, P, K, V, RID);
      rc = bg_sort_u64(c, K, V, m);  // stable: by this chunk
    }
    if (!rc) {
      BG_LAUNCH(c, "k_sb_trid", k_sb_trid, gm, dim3(BG_NT), RID, V, m, K);
      rc = bg_sort_u64(c, K, V, m);  // stable: by run, keeping the chunk order inside it
    }
    if (!rc) {
      BG_LAUNCH(c, "k_sb_tpick", k_sb_tpick, gm, dim3(BG_NT), P, V, m, ord, tmp);
      BG_LAUNCH(c, "k_sb_tput", k_sb_tput, gm, dim3(BG_NT), P, m, tmp, ord);
      rc = bg_hip_ok(c, hipGetLastError());
    }
    for (void* x : {(void*)P, (void*)K, (void*)V, (void*)RID, (void*)tmp}) bg_release(c, x);
  }
  for (void* x : {(void*)tied, (void*)start, (void*)pos, (void*)rid, (void*)more}) bg_release(c, x);
  return rc;
}

__global__ void k_sb_emit(const uint32_t* __restrict__ ord, const uint64_t* __restrict__ idx,
                          const uint32_t* __restrict__ rank, uint64_t nd,
                          const int64_t* __restrict__ S, const int64_t* __restrict__ E,
                          const uint64_t* __restrict__ R, const uint32_t* __restrict__ RL,
                          int64_t* __restrict__ OS, int64_t* __restrict__ OE,
                          uint64_t* __restrict__ OR, uint32_t* __restrict__ ORL) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nd) return;
  const uint32_t d = ord[j];
  const uint64_t i = idx[d];
  const int64_t g = (int64_t)rank[d] << BG_KEY_SHIFT;
  OS[j] = g | S[i];
  OE[j] = g | E[i];
  OR[j] = R[i];
  ORL[j] = RL[i];
}

extern "C" int bg_sortbed(bg_ctx* c, int nin, const bg_input* in, bg_result** out,
                          bg_sortbed_error* err) {
  if (!c || nin < 1 || !in || !out || !err) return BG_E_ARG;
  *out = nullptr;
  memset(err, 0, sizeof(*err));
  bg_bind(c);
  bg_set* set = new bg_set();
  set->ctx = c;
  auto fail = [&](int rc) {
    bg_set_free(set);
    return rc;
  };
  // the texts on the device (the set owns copies of host inputs; rests point into them)
  std::vector<const char*> txt(nin);
  std::vector<uint64_t> nb(nin);
  for (int f = 0; f < nin; ++f) {
    bg_table* T = new bg_table();
    set->t.push_back(T);
    nb[f] = in[f].nbytes;
    if (in[f].on_device) {
      txt[f] = (const char*)in[f].data;
    } else {
      T->own_text = (char*)bg_alloc(c, nb[f] + 64);
      if (!T->own_text) return fail(BG_E_NOMEM);
      if (nb[f]) BG_HIP(c, hipMemcpyAsync(T->own_text, in[f].data, nb[f], hipMemcpyHostToDevice, c->stream));
      txt[f] = T->own_text;
    }
  }
  // line starts per input
  std::vector<uint64_t> L0(nin + 1, 0);
  std::vector<uint64_t*> cnts(nin, nullptr);
  uint64_t* d_tot = (uint64_t*)bg_alloc(c, 8ull * nin);
  if (!d_tot) return fail(BG_E_NOMEM);
  for (int f = 0; f < nin; ++f) {
    const unsigned nt = bg_blocks(nb[f], SB_TILE);
    cnts[f] = (uint64_t*)bg_alloc(c, 8ull * (nt + 1));
    if (!cnts[f]) return fail(BG_E_NOMEM);
    if (nt) BG_LAUNCH(c, "k_sb_count", k_sb_count, dim3(nt), dim3(BG_NT), txt[f], nb[f], cnts[f]);
    int rc = bg_scan_sum_u64(c, cnts[f], cnts[f], nt, d_tot + f);
    if (rc) return fail(rc);
  }
  std::vector<uint64_t> nnl(nin, 0);
  BG_HIP(c, hipMemcpyAsync(nnl.data(), d_tot, 8ull * nin, hipMemcpyDeviceToHost, c->stream));
  BG_HIP(c, hipStreamSynchronize(c->stream));
  for (int f = 0; f < nin; ++f) L0[f + 1] = L0[f] + (nb[f] ? nnl[f] + 1 : 0);
  const uint64_t nl = L0[nin];
  const uint64_t nl1 = nl ? nl : 1;
  uint64_t* S = (uint64_t*)bg_alloc(c, 8 * (nl1 + 1));
  uint64_t* Eaddr = (uint64_t*)bg_alloc(c, 8 * nl1);
  uint32_t* F = (uint32_t*)bg_alloc(c, 4 * nl1);
  uint64_t* dL0 = (uint64_t*)bg_alloc(c, 8ull * (nin + 1));
  unsigned long long* first = (unsigned long long*)bg_alloc(c, 8ull * nin);
  unsigned long long* derr = (unsigned long long*)bg_alloc(c, 16);
  if (!S || !Eaddr || !F || !dL0 || !first || !derr) return fail(BG_E_NOMEM);
  for (int f = 0; f < nin; ++f) {
    const unsigned nt = bg_blocks(nb[f], SB_TILE);
    if (nt) BG_LAUNCH(c, "k_sb_starts", k_sb_starts, dim3(nt), dim3(BG_NT), txt[f], nb[f], cnts[f], S + L0[f]);
  }
  // line ends and inputs: E[i] = S[i+1] - 1 inside an input, its text end for the last line
  {
    std::vector<uint64_t> hL0(L0.begin(), L0.end());
    BG_HIP(c, hipMemcpyAsync(dL0, hL0.data(), 8ull * (nin + 1), hipMemcpyHostToDevice, c->stream));
    BG_HIP(c, hipMemsetAsync(first, 0xff, 8ull * nin, c->stream));
    BG_HIP(c, hipMemsetAsync(derr, 0xff, 16, c->stream));
    BG_HIP(c, hipStreamSynchronize(c->stream));
  }
  uint8_t* TM = (uint8_t*)bg_alloc(c, nl1);
  if (!TM) return fail(BG_E_NOMEM);
  for (int f = 0; f < nin; ++f) {
    const uint64_t a = L0[f], b = L0[f + 1];
    if (a == b) continue;
    char lastc = 0;
    BG_HIP(c, hipMemcpyAsync(&lastc, txt[f] + nb[f] - 1, 1, hipMemcpyDeviceToHost, c->stream));
    BG_HIP(c, hipStreamSynchronize(c->stream));
    BG_LAUNCH(c, "k_sb_ends", k_sb_ends, dim3(bg_blocks(b - a, BG_NT)), dim3(BG_NT), S, a, b,
              (uint64_t)(txt[f] + nb[f]), lastc == '\n' ? 1 : 0, (uint32_t)f, Eaddr, TM, F);
  }
  SbLines A{S, Eaddr, TM, F, dL0, nl};
  SbOut O;
  O.flag = (uint8_t*)bg_alloc(c, nl1);
  O.h = (uint64_t*)bg_alloc(c, 8 * nl1);
  O.tok = (uint64_t*)bg_alloc(c, 8 * nl1);
  O.toklen = (uint32_t*)bg_alloc(c, 4 * nl1);
  O.start = (int64_t*)bg_alloc(c, 8 * nl1);
  O.end = (int64_t*)bg_alloc(c, 8 * nl1);
  O.rest = (uint64_t*)bg_alloc(c, 8 * nl1);
  O.restlen = (uint32_t*)bg_alloc(c, 4 * nl1);
  if (!O.flag || !O.h || !O.tok || !O.toklen || !O.start || !O.end || !O.rest || !O.restlen)
    return fail(BG_E_NOMEM);
  if (nl) {
    BG_LAUNCH(c, "k_sb_first", k_sb_first, dim3(bg_blocks(nl, BG_NT)), dim3(BG_NT), A, first);
    BG_LAUNCH(c, "k_sb_parse", k_sb_parse, dim3(bg_blocks(nl, BG_NT)), dim3(BG_NT), A, first, O, derr);
    BG_HIP(c, hipGetLastError());
  }
  uint64_t herr = ~0ULL;
  BG_HIP(c, hipMemcpyAsync(&herr, derr, 8, hipMemcpyDeviceToHost, c->stream));
  BG_HIP(c, hipStreamSynchronize(c->stream));
  if (herr != ~0ULL) {  // the first failing line in input order
    const uint64_t li = herr >> 8;
    int f = 0;
    while (f + 1 < nin && L0[f + 1] <= li) ++f;
    err->input = f;
    err->line = li - L0[f] + 1;  // 1-based physical line of that input
    err->code = (int)(herr & 0xff);
    return fail(bg_fail(c, BG_E_PARSE, "sort-bed: bad input line"));
  }
  // data lines
  uint64_t* idx = nullptr;
  uint64_t nd = 0;
  int rc = bg_compact_flags(c, O.flag, nl, &idx, &nd);
  if (rc) return fail(rc);
  const uint64_t nd1 = nd ? nd : 1;
  // dictionary: distinct chromosome names, ranked by strcmp on the host
  uint64_t* key = (uint64_t*)bg_alloc(c, 8 * nd1);
  uint32_t* val = (uint32_t*)bg_alloc(c, 4 * nd1);
  uint8_t* uf = (uint8_t*)bg_alloc(c, nd1);
  uint32_t* rank = (uint32_t*)bg_alloc(c, 4 * nd1);
  if (!key || !val || !uf || !rank) return fail(BG_E_NOMEM);
  std::vector<std::string> names;
  if (nd) {
    BG_LAUNCH(c, "k_sb_gather_hash", k_sb_gather_hash, dim3(bg_blocks(nd, BG_NT)), dim3(BG_NT), idx, nd,
              O.h, key, val);
    if ((rc = bg_sort_u64(c, key, val, nd))) return fail(rc);
    BG_LAUNCH(c, "k_sb_uniq", k_sb_uniq, dim3(bg_blocks(nd, BG_NT)), dim3(BG_NT), key, nd, uf);
    uint64_t* upos = nullptr;
    uint64_t nu = 0;
    if ((rc = bg_compact_flags(c, uf, nd, &upos, &nu))) return fail(rc);
    // ranks go into the key above bit 40 (rank << BG_KEY_SHIFT | start): as the loader
    // (bg_load.hip), at most 2^22 - 1 names keep the keys positive and distinct
    if (nu >= (1ull << 22)) return fail(bg_fail(c, BG_E_UNSUPPORTED, "too many chromosomes"));
    // representatives: hash, data-line ordinal, token address / length, then the names
    uint64_t* rinfo = (uint64_t*)bg_alloc(c, 8 * 4 * nu);
    if (!rinfo) return fail(BG_E_NOMEM);
    BG_LAUNCH(c, "k_sb_reps", k_sb_reps, dim3(bg_blocks(nu, BG_NT)), dim3(BG_NT), upos, nu, key, val, idx,
              O.tok, O.toklen, rinfo);
    std::vector<uint64_t> hi(4 * nu);
    BG_HIP(c, hipMemcpyAsync(hi.data(), rinfo, 8 * 4 * nu, hipMemcpyDeviceToHost, c->stream));
    BG_HIP(c, hipStreamSynchronize(c->stream));
    std::vector<uint64_t> hh(nu), noff(nu + 1, 0);
    std::vector<uint32_t> hval(nu);
    for (uint64_t u = 0; u < nu; ++u) {
      hh[u] = hi[4 * u];
      hval[u] = (uint32_t)hi[4 * u + 1];
      noff[u + 1] = noff[u] + hi[4 * u + 3];
    }
    char* dn = (char*)bg_alloc(c, noff[nu] + 1);
    uint64_t* dnoff = (uint64_t*)bg_alloc(c, 8 * (nu + 1));
    if (!dn || !dnoff) return fail(BG_E_NOMEM);
    BG_HIP(c, hipMemcpyAsync(dnoff, noff.data(), 8 * (nu + 1), hipMemcpyHostToDevice, c->stream));
    BG_LAUNCH(c, "k_sb_names", k_sb_names, dim3(bg_blocks(nu, BG_NT)), dim3(BG_NT), rinfo, nu, dnoff, dn);
    std::string packed_names(noff[nu], '\0');
    if (noff[nu]) BG_HIP(c, hipMemcpyAsync(&packed_names[0], dn, noff[nu], hipMemcpyDeviceToHost, c->stream));
    BG_HIP(c, hipStreamSynchronize(c->stream));
    names.resize(nu);
    for (uint64_t u = 0; u < nu; ++u) names[u] = packed_names.substr(noff[u], noff[u + 1] - noff[u]);
    bg_release(c, rinfo);
    bg_release(c, dn);
    bg_release(c, dnoff);
    std::vector<uint32_t> ord(nu);
    for (uint64_t u = 0; u < nu; ++u) ord[u] = (uint32_t)u;
    std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
      return strcmp(names[a].c_str(), names[b].c_str()) < 0;
    });
    std::vector<uint32_t> urank(nu);
    for (uint64_t r = 0; r < nu; ++r) urank[ord[r]] = (uint32_t)r;
    std::vector<std::string> sorted(nu);
    for (uint64_t r = 0; r < nu; ++r) sorted[r] = names[ord[r]];
    names = sorted;
    uint64_t* d_uh = (uint64_t*)bg_alloc(c, 8 * nu);
    uint32_t* d_ur = (uint32_t*)bg_alloc(c, 4 * nu);
    uint64_t* d_rep = (uint64_t*)bg_alloc(c, 8 * nu);
    unsigned long long* bad = (unsigned long long*)bg_alloc(c, 8);
    if (!d_uh || !d_ur || !d_rep || !bad) return fail(BG_E_NOMEM);
    std::vector<uint64_t> rep(nu);
    for (uint64_t u = 0; u < nu; ++u) rep[u] = hval[u];
    BG_HIP(c, hipMemcpyAsync(d_uh, hh.data(), 8 * nu, hipMemcpyHostToDevice, c->stream));
    BG_HIP(c, hipMemcpyAsync(d_ur, urank.data(), 4 * nu, hipMemcpyHostToDevice, c->stream));
    BG_HIP(c, hipMemcpyAsync(d_rep, rep.data(), 8 * nu, hipMemcpyHostToDevice, c->stream));
    BG_HIP(c, hipMemsetAsync(bad, 0, 8, c->stream));
    BG_LAUNCH(c, "k_sb_rank", k_sb_rank, dim3(bg_blocks(nd, BG_NT)), dim3(BG_NT), idx, nd, O.h, O.tok,
              O.toklen, d_uh, d_ur, d_rep, nu, rank, bad);
    uint64_t hbad = 0;
    BG_HIP(c, hipMemcpyAsync(&hbad, bad, 8, hipMemcpyDeviceToHost, c->stream));
    BG_HIP(c, hipStreamSynchronize(c->stream));
    if (hbad) return fail(bg_fail(c, BG_E_INTERNAL, "sort-bed: 64-bit chromosome hash collision"));
    bg_release(c, d_uh);
    bg_release(c, d_ur);
    bg_release(c, d_rep);
    bg_release(c, bad);
    bg_release(c, upos);
  }
  // the set's dictionary (names in strcmp order) for the formatter
  {
    std::string packed;
    std::vector<uint32_t> off(names.size() + 1, 0), len(names.size() + 1, 0);
    for (size_t k = 0; k < names.size(); ++k) {
      off[k] = (uint32_t)packed.size();
      len[k] = (uint32_t)names[k].size();
      set->max_name_len = std::max<uint32_t>(set->max_name_len, len[k]);
      packed += names[k];
    }
    set->names = names;
    const size_t nbn = (packed.size() + 16) & ~(size_t)15, nbo = 4 * off.size(), blk = nbn + 2 * nbo;
    set->d_names = (char*)bg_alloc(c, blk);
    if (!set->d_names) return fail(BG_E_NOMEM);
    set->d_name_off = (uint32_t*)(set->d_names + nbn);
    set->d_name_len = (uint32_t*)(set->d_names + nbn + nbo);
    std::vector<char> h(blk, 0);
    memcpy(h.data(), packed.data(), packed.size());
    memcpy(h.data() + nbn, off.data(), nbo);
    memcpy(h.data() + nbn + nbo, len.data(), nbo);
    BG_HIP(c, hipMemcpyAsync(set->d_names, h.data(), blk, hipMemcpyHostToDevice, c->stream));
    BG_HIP(c, hipStreamSynchronize(c->stream));
  }
  // sort: stable LSD by end, then by (rank << 40 | start)
  uint32_t* ord = val;  // reuse: data-line ordinals in sorted order
  if (nd) {
    BG_LAUNCH(c, "k_sb_iota", k_sb_iota, dim3(bg_blocks(nd, BG_NT)), dim3(BG_NT), ord, nd);
    BG_LAUNCH(c, "k_sb_key", k_sb_key, dim3(bg_blocks(nd, BG_NT)), dim3(BG_NT), idx, ord, nd, O.end, rank,
              false, key);
    if ((rc = bg_sort_u64(c, key, ord, nd))) return fail(rc);
    BG_LAUNCH(c, "k_sb_key", k_sb_key, dim3(bg_blocks(nd, BG_NT)), dim3(BG_NT), idx, ord, nd, O.start, rank,
              true, key);
    if ((rc = bg_sort_u64(c, key, ord, nd))) return fail(rc);
    if ((rc = sb_order_ties(c, key, idx, O.end, O.rest, O.restlen, nd, ord))) return fail(rc);
  }
  bg_result* r = new bg_result();
  r->ctx = c;
  r->set = set;
  r->kind = RES_MULTI;
  r->n = nd;
  r->rest_tab = true;
  r->s = (int64_t*)bg_alloc(c, 8 * nd1);
  r->e = (int64_t*)bg_alloc(c, 8 * nd1);
  r->rows = (uint64_t*)bg_alloc(c, 8 * nd1);
  r->rlen = (uint32_t*)bg_alloc(c, 4 * nd1);
  r->own_set = true;
  if (!r->s || !r->e || !r->rows || !r->rlen) {
    bg_result_free(r);
    return BG_E_NOMEM;
  }
  if (nd)
    BG_LAUNCH(c, "k_sb_emit", k_sb_emit, dim3(bg_blocks(nd, BG_NT)), dim3(BG_NT), ord, idx, rank, nd, O.start,
              O.end, O.rest, O.restlen, r->s, r->e, r->rows, r->rlen);
  BG_HIP(c, hipGetLastError());
  BG_HIP(c, hipStreamSynchronize(c->stream));
  for (void* p : {(void*)S, (void*)Eaddr, (void*)F, (void*)dL0, (void*)first, (void*)derr, (void*)O.flag,
                  (void*)O.h, (void*)O.tok, (void*)O.toklen, (void*)O.start, (void*)O.end, (void*)O.rest,
                  (void*)O.restlen, (void*)idx, (void*)key, (void*)val, (void*)uf, (void*)rank, (void*)d_tot,
                  (void*)TM})
    bg_release(c, p);
  for (auto p : cnts) bg_release(c, p);
  *out = r;
  bg_mark(c, "sort-bed");
  return 0;
}
