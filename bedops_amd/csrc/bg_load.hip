// bg_load.hip — K0: BED text in HBM -> keyed int64 SoA columns.
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
// Pipeline (per input):
//   k_nl_count   tiles of 4 KiB: '\n' count + last '\n' offset per tile   (text read 1x)
//   scans        row0[t] = sum of counts before t; prevnl[t] = last '\n' before t
//   k_parse      per tile: text (+256 B halo) staged in LDS, '\n' offsets found
//                with a wave/block scan, one thread per line parses
//                chrom/start/end(/id/score), writes raw start/end, records
//                chromosome-change rows and sort-order violations   (text read 1x)
//   host         chromosome dictionary (strcmp order over all inputs), run checks
//   k_key        ks/ke = (chrom_id << 40) | coordinate, in place, range checks
#include <algorithm>
#include <cstring>
#include <map>

#include "bg_internal.h"

#define TXT_TILE 4096
#define TXT_HALO 256
#define RUN_CAP (1u << 20)

__device__ __forceinline__ uint32_t nl_mask4(uint32_t w) {
  // bit 7 of each byte set iff that byte == '\n' (exact, no borrow artefacts)
  uint32_t x = w ^ 0x0A0A0A0Au;
  uint32_t nz = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;
  return ~nz & 0x80808080u;
}

// guarded 16-byte load of txt[base, base+16) (bytes >= nbytes read as 0)
__device__ __forceinline__ uint4 load16(const uint8_t* __restrict__ txt, uint64_t base,
                                        uint64_t nbytes) {
  if (base + 16 <= nbytes) return *reinterpret_cast<const uint4*>(txt + base);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int k = 0; k < 16; ++k)
    if (base + k < nbytes) w[k >> 2] |= (uint32_t)txt[base + k] << (8 * (k & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ void __launch_bounds__(BG_NT) k_nl_count(const uint8_t* __restrict__ txt,
                                                    uint64_t nbytes, uint64_t* __restrict__ cnt,
                                                    int64_t* __restrict__ lastnl) {
  __shared__ uint64_t shc[BG_NT / 64 + 1];
  __shared__ int64_t shm[BG_NT / 64 + 1];
  const uint64_t base = (uint64_t)blockIdx.x * TXT_TILE + (uint64_t)threadIdx.x * 16;
  uint4 v = load16(txt, base, nbytes);
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint64_t c = 0;
  int64_t last = -1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t m = nl_mask4(w[k]);
    c += __popc(m);
    if (m) last = (int64_t)(base + 4 * k + (31 - __clz(m)) / 8);
  }
  uint64_t tc;
  int64_t tm;
  (void)block_excl_scan(c, OpSum(), (uint64_t)0, shc, &tc);
  (void)block_excl_scan(last, OpMax(), (int64_t)-1, shm, &tm);
  if (threadIdx.x == 0) {
    cnt[blockIdx.x] = tc;
    lastnl[blockIdx.x] = tm;
  }
}

// byte view of one tile: LDS copy of [lo, hi), global memory elsewhere
struct TileText {
  const uint8_t* g;
  const uint8_t* l;
  int64_t lo, hi;
  __device__ __forceinline__ uint8_t at(int64_t p) const {
    return (p >= lo && p < hi) ? l[p - lo] : g[p];
  }
};

struct LineFields {
  int64_t tok;     // chrom token offset
  int32_t toklen;
  uint64_t start, end;
  int64_t rest;    // offset of the first byte after the end digits
  double score;
  int32_t err;     // 0 ok, ERR_*
  int32_t scoreint;
};

__device__ __forceinline__ bool parse_u64(const TileText& T, int64_t& p, int64_t le,
                                          uint64_t& v) {
  if (p < le && T.at(p) == '+') ++p;
  int nd = 0;
  uint64_t x = 0;
  while (p < le) {
    uint8_t ch = T.at(p);
    if (ch < '0' || ch > '9') break;
    if (nd < 19) x = x * 10 + (ch - '0');
    ++nd;
    ++p;
  }
  v = (nd > 13) ? ~0ULL : x;  // > 13 digits is always out of range
  return nd > 0;
}

// strtod subset, exact where it claims to be: [+-]digits[.digits] with <= 19
// significant digits; integers are flagged (scoreint). Anything else -> ERR_SCORE.
__device__ __forceinline__ bool parse_score(const TileText& T, int64_t& p, int64_t le,
                                            double& out, int& isint) {
  bool neg = false;
  if (p < le && (T.at(p) == '+' || T.at(p) == '-')) neg = T.at(p++) == '-';
  uint64_t m = 0;
  int nd = 0, frac = 0, sig = 0;
  bool dot = false, fracnz = false;
  while (p < le) {
    uint8_t ch = T.at(p);
    if (ch == '.' && !dot) { dot = true; ++p; continue; }
    if (ch < '0' || ch > '9') break;
    ++nd;
    if (dot) {
      ++frac;
      if (ch != '0') fracnz = true;
    }
    if (m != 0 || ch != '0') ++sig;
    if (sig <= 19) m = m * 10 + (ch - '0');
    else return false;
    ++p;
  }
  if (nd == 0 || sig > 19) return false;
  if (p < le && !bg_isws(T.at(p))) return false;  // exponent / junk: not on the GPU path
  isint = !fracnz;
  if (!fracnz) {
    // drop the zero fraction digits, value is m / 10^frac exactly an integer
    for (int k = 0; k < frac; ++k) m /= 10;
    if (m > (1ULL << 53)) return false;
    out = neg ? -(double)m : (double)m;
    return true;
  }
  // Clinger fast path: exact when m < 2^53 and 10^frac exactly representable
  if (m > (1ULL << 53) || frac > 22) return false;
  double d = (double)m, s = 1.0;
  for (int k = 0; k < frac; ++k) s *= 10.0;  // exact for frac <= 22
  out = d / s;
  if (neg) out = -out;
  return true;
}

__device__ __forceinline__ void parse_line(const TileText& T, int64_t ls, int64_t le, int kind,
                                           LineFields& L) {
  L.err = 0;
  L.scoreint = 1;
  L.score = 0;
  int64_t p = ls;
  while (p < le && bg_isws(T.at(p))) ++p;
  if (p == le) { L.err = ERR_BLANK; return; }
  L.tok = p;
  while (p < le && !bg_isws(T.at(p))) ++p;
  L.toklen = (int32_t)(p - L.tok);
  if (L.toklen > BG_CHR_MAX) { L.err = ERR_CHROM; return; }
  while (p < le && bg_isws(T.at(p))) ++p;
  if (!parse_u64(T, p, le, L.start)) { L.err = ERR_PARSE; return; }
  while (p < le && bg_isws(T.at(p))) ++p;
  if (!parse_u64(T, p, le, L.end)) { L.err = ERR_PARSE; return; }
  L.rest = p;
  if (kind == BG_BED5) {
    if (p == le || !bg_isws(T.at(p))) { L.err = ERR_PARSE; return; }
    while (p < le && bg_isws(T.at(p))) ++p;
    int64_t id = p;
    while (p < le && !bg_isws(T.at(p))) ++p;
    if (p == id) { L.err = ERR_PARSE; return; }
    while (p < le && bg_isws(T.at(p))) ++p;
    int isint = 1;
    if (!parse_score(T, p, le, L.score, isint)) { L.err = ERR_SCORE; return; }
    L.scoreint = isint;
  }
}

// chrom token + start of the line [ls, le) (used for the previous-line comparison)
__device__ __forceinline__ int parse_head(const TileText& T, int64_t ls, int64_t le,
                                          int64_t& tok, int32_t& toklen, uint64_t& start) {
  int64_t p = ls;
  while (p < le && bg_isws(T.at(p))) ++p;
  if (p == le) return ERR_BLANK;
  tok = p;
  while (p < le && !bg_isws(T.at(p))) ++p;
  toklen = (int32_t)(p - tok);
  while (p < le && bg_isws(T.at(p))) ++p;
  if (!parse_u64(T, p, le, start)) return ERR_PARSE;
  return 0;
}

__global__ void __launch_bounds__(BG_NT) k_parse(
    const uint8_t* __restrict__ txt, uint64_t nbytes, const uint64_t* __restrict__ cnt,
    const uint64_t* __restrict__ row0, const int64_t* __restrict__ prevnl, int kind,
    uint64_t* __restrict__ S, uint64_t* __restrict__ E, uint64_t* __restrict__ rest_off,
    uint32_t* __restrict__ rest_len, double* __restrict__ score, uint64_t* __restrict__ run_row,
    uint64_t* __restrict__ run_tok, uint32_t* __restrict__ run_len, bg_dstatus* st) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[TXT_HALO + TXT_TILE];
  __shared__ uint16_t nlpos[TXT_TILE];
  __shared__ uint32_t shs[BG_NT / 64 + 1];
  const uint64_t t = blockIdx.x;
  const int64_t t0 = (int64_t)(t * TXT_TILE);
  const uint64_t lines = cnt[t];
  if (lines == 0) return;  // uniform per block
  const int64_t lo = t0 >= TXT_HALO ? t0 - TXT_HALO : 0;
  // stage [lo, t0 + TILE) in LDS
  {
    const uint64_t b = (uint64_t)t0 + (uint64_t)threadIdx.x * 16;
    uint4 v = load16(txt, b, nbytes);
    *reinterpret_cast<uint4*>(&buf[TXT_HALO + threadIdx.x * 16]) = v;
    if (threadIdx.x < TXT_HALO / 16 && t0 >= TXT_HALO) {
      uint4 h = load16(txt, (uint64_t)lo + threadIdx.x * 16, nbytes);
      *reinterpret_cast<uint4*>(&buf[threadIdx.x * 16]) = h;
    }
    // newline offsets of this thread's 16 bytes, compacted by a block scan
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t m[4], c = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      m[k] = nl_mask4(w[k]);
      c += __popc(m[k]);
    }
    uint32_t tot;
    uint32_t o = block_excl_scan(c, OpSum(), 0u, shs, &tot);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t mm = m[k];
      while (mm) {
        int bit = __ffs(mm) - 1;
        nlpos[o++] = (uint16_t)(threadIdx.x * 16 + 4 * k + bit / 8);
        mm &= mm - 1;
      }
    }
  }
  __syncthreads();
  TileText T;
  T.g = txt;
  T.l = (t0 >= TXT_HALO) ? buf : buf + TXT_HALO;
  T.lo = lo;
  T.hi = t0 + TXT_TILE;
  const int64_t pnl = prevnl[t];  // '\n' before this tile (-1: none)
  const uint64_t r0 = row0[t];
  for (uint64_t j = threadIdx.x; j < lines; j += BG_NT) {
    const int64_t le = t0 + nlpos[j];
    const int64_t ls = (j == 0 ? pnl : t0 + (int64_t)nlpos[j - 1]) + 1;
    const uint64_t r = r0 + j;
    LineFields L;
    parse_line(T, ls, le, kind, L);
    if (L.err) {
      if (L.err == ERR_BLANK) atomicAdd(&st->nblank, 1ULL);
      bg_report(st, r, L.err);
      S[r] = E[r] = 0;
      continue;
    }
    S[r] = L.start;
    E[r] = L.end;
    if (rest_off) {
      rest_off[r] = (uint64_t)L.rest;
      rest_len[r] = (uint32_t)(le - L.rest);
    }
    if (score) {
      score[r] = L.score;
      if (!L.scoreint) atomicOr(&st->flags, 1ULL);
    }
    bool newrun = (r == 0);
    if (r > 0) {
      const int64_t ple = ls - 1;  // previous line's '\n'
      int64_t pls;
      if (j >= 2) pls = t0 + (int64_t)nlpos[j - 2] + 1;
      else if (j == 1) pls = pnl + 1;
      else {
        int64_t q = ple - 1;
        while (q >= 0 && T.at(q) != '\n') --q;
        pls = q + 1;
      }
      int64_t ptok = 0;
      int32_t ptoklen = 0;
      uint64_t pstart = 0;
      int perr = parse_head(T, pls, ple, ptok, ptoklen, pstart);
      if (perr) {
        newrun = true;  // the previous line is itself reported
      } else {
        bool same = (ptoklen == L.toklen);
        for (int32_t k = 0; same && k < L.toklen; ++k) same = T.at(ptok + k) == T.at(L.tok + k);
        if (!same) newrun = true;
        else if (L.start < pstart) bg_report(st, r, ERR_UNSORTED);
      }
    }
    if (newrun) {
      unsigned long long k = atomicAdd(&st->nruns, 1ULL);
      if (k < RUN_CAP) {
        run_row[k] = r;
        run_tok[k] = (uint64_t)L.tok;
        run_len[k] = (uint32_t)L.toklen;
      }
    }
  }
}

// gather the chromosome tokens of the run records into fixed 128-byte slots
__global__ void k_gather_tokens(const uint8_t* __restrict__ txt, const uint64_t* run_tok,
                                const uint32_t* run_len, uint64_t nruns, char* out) {
  uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nruns) return;
  uint32_t n = run_len[k];
  for (uint32_t i = 0; i < 128; ++i) out[k * 128 + i] = (i < n) ? (char)txt[run_tok[k] + i] : 0;
}

// ks/ke: raw -> (gid << 40) | coord, in place; run_row0 has nruns+1 entries
__global__ void __launch_bounds__(BG_NT) k_key(int64_t* __restrict__ S, int64_t* __restrict__ E,
                                               uint64_t n, const uint64_t* __restrict__ run_row0,
                                               const int32_t* __restrict__ run_gid,
                                               uint32_t nruns, bg_dstatus* st) {
  const uint64_t r = (uint64_t)blockIdx.x * BG_NT + threadIdx.x;
  if (r >= n) return;
  uint32_t lo = 0, hi = nruns;  // last k with run_row0[k] <= r
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (run_row0[mid] <= r) lo = mid;
    else hi = mid;
  }
  const int64_t g = (int64_t)run_gid[lo] << BG_KEY_SHIFT;
  const uint64_t s = (uint64_t)S[r], e = (uint64_t)E[r];
  if (e > BG_MAX_COORD || s > e) bg_report(st, r, ERR_RANGE);
  if (s == e) atomicOr(&st->flags, 2ULL);
  S[r] = g | (int64_t)(s & BG_COORD_MASK);
  E[r] = g | (int64_t)(e & BG_COORD_MASK);
}

// ---------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------
static const char* kind_name(int k) {
  return k == BG_BED5 ? "BED5" : (k == BG_BED3_REST ? "BED3+rest" : "BED3");
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
    case ERR_RANGE: what = "coordinate out of range (end < start or > 999999999999)"; rc = BG_E_RANGE; break;
    case ERR_UNSORTED: what = "input is not sorted (use sort-bed)"; rc = BG_E_UNSORTED; break;
    case ERR_BLANK: what = "blank line inside the data is not supported by the GPU loader"; rc = BG_E_BLANK; break;
    case ERR_SCORE: what = "score column is not a plain decimal number"; rc = BG_E_UNSUPPORTED; break;
  }
  snprintf(msg, sizeof(msg), "input %d, data line %llu: %s", file + 1,
           (unsigned long long)row + 1, what);
  return bg_fail(c, rc, msg);
}

static int parse_one(bg_ctx* c, int idx, const bg_input& in, bg_table* T) {
  T->kind = in.kind;
  // text into HBM
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
  const uint64_t nb = in.nbytes;
  const unsigned ntiles = nb ? bg_blocks(nb, TXT_TILE) : 0;
  if (ntiles == 0) {  // empty input: valid, zero rows; keep every column non-null
    T->n = 0;
    T->ks = (int64_t*)bg_alloc(c, 8);
    T->ke = (int64_t*)bg_alloc(c, 8);
    if (in.kind == BG_BED3_REST) {
      T->rest_off = (uint64_t*)bg_alloc(c, 8);
      T->rest_len = (uint32_t*)bg_alloc(c, 4);
    }
    if (in.kind == BG_BED5) T->score = (double*)bg_alloc(c, 8);
    T->run_row0.assign(1, 0);
    return 0;
  }
  uint64_t* cnt = (uint64_t*)bg_alloc(c, 8ull * ntiles);
  uint64_t* row0 = (uint64_t*)bg_alloc(c, 8ull * ntiles);
  int64_t* lastnl = (int64_t*)bg_alloc(c, 8ull * ntiles);
  int64_t* prevnl = (int64_t*)bg_alloc(c, 8ull * ntiles);
  uint64_t* d_rows = (uint64_t*)bg_alloc(c, 8);
  if (!cnt || !row0 || !lastnl || !prevnl || !d_rows) return BG_E_NOMEM;
  BG_LAUNCH(c, "k_nl_count", k_nl_count, dim3(ntiles), dim3(BG_NT), txt, nb, cnt, lastnl);
  BG_HIP(c, hipGetLastError());
  int rc = bg_scan_sum_u64(c, cnt, row0, ntiles, d_rows);
  if (rc) return rc;
  rc = bg_scan_max_i64(c, lastnl, prevnl, ntiles, -1);
  if (rc) return rc;
  uint64_t rows = 0;
  if ((rc = bg_fetch_u64(c, d_rows, &rows))) return rc;
  T->n = rows;
  const uint64_t na = rows ? rows : 1;
  T->ks = (int64_t*)bg_alloc(c, 8 * na);
  T->ke = (int64_t*)bg_alloc(c, 8 * na);
  if (!T->ks || !T->ke) return BG_E_NOMEM;
  if (in.kind == BG_BED3_REST) {
    T->rest_off = (uint64_t*)bg_alloc(c, 8 * na);
    T->rest_len = (uint32_t*)bg_alloc(c, 4 * na);
    if (!T->rest_off || !T->rest_len) return BG_E_NOMEM;
  }
  if (in.kind == BG_BED5) {
    T->score = (double*)bg_alloc(c, 8 * na);
    if (!T->score) return BG_E_NOMEM;
  }
  uint64_t* run_row = (uint64_t*)bg_alloc(c, 8ull * RUN_CAP);
  uint64_t* run_tok = (uint64_t*)bg_alloc(c, 8ull * RUN_CAP);
  uint32_t* run_len = (uint32_t*)bg_alloc(c, 4ull * RUN_CAP);
  if (!run_row || !run_tok || !run_len) return BG_E_NOMEM;
  BG_HIP(c, hipMemsetAsync(c->dstat, 0, sizeof(bg_dstatus), c->stream));
  BG_HIP(c, hipMemsetAsync(&c->dstat->first_bad, 0xff, 8, c->stream));
  if (rows) {
    BG_LAUNCH(c, "k_parse", k_parse, dim3(ntiles), dim3(BG_NT), txt, nb, cnt, row0,
                       prevnl, in.kind, (uint64_t*)T->ks, (uint64_t*)T->ke, T->rest_off,
                       T->rest_len, T->score, run_row, run_tok, run_len, c->dstat);
    BG_HIP(c, hipGetLastError());
  }
  BG_HIP(c, hipMemcpyAsync(c->hstat, c->dstat, sizeof(bg_dstatus), hipMemcpyDeviceToHost, c->stream));
  BG_HIP(c, hipStreamSynchronize(c->stream));
  bg_dstatus h = *c->hstat;
  if ((rc = report_status(c, idx, h))) return rc;
  if (h.nruns > RUN_CAP) return bg_fail(c, BG_E_UNSUPPORTED, "more than 2^20 chromosome runs in one input");
  if (in.kind == BG_BED5 && (h.flags & 1ULL)) T->score_int = false;
  // fetch run records
  const uint64_t nr = h.nruns;
  std::vector<uint64_t> rr(nr);
  std::vector<char> names(nr * 128);
  if (nr) {
    char* d_names = (char*)bg_alloc(c, nr * 128);
    if (!d_names) return BG_E_NOMEM;
    BG_LAUNCH(c, "k_gather_tokens", k_gather_tokens, dim3(bg_blocks(nr, 256)), dim3(256), txt,
                       run_tok, run_len, nr, d_names);
    BG_HIP(c, hipGetLastError());
    BG_HIP(c, hipMemcpyAsync(rr.data(), run_row, 8 * nr, hipMemcpyDeviceToHost, c->stream));
    BG_HIP(c, hipMemcpyAsync(names.data(), d_names, nr * 128, hipMemcpyDeviceToHost, c->stream));
    BG_HIP(c, hipStreamSynchronize(c->stream));
    bg_release(c, d_names);
  }
  std::vector<uint64_t> order(nr);
  for (uint64_t k = 0; k < nr; ++k) order[k] = k;
  std::sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return rr[a] < rr[b]; });
  T->run_row0.clear();
  T->run_name.clear();
  for (uint64_t k : order) {
    T->run_row0.push_back(rr[k]);
    T->run_name.emplace_back(&names[k * 128], strnlen(&names[k * 128], 128));
  }
  for (size_t k = 1; k < T->run_name.size(); ++k) {
    if (strcmp(T->run_name[k - 1].c_str(), T->run_name[k].c_str()) >= 0) {
      char msg[320];
      snprintf(msg, sizeof(msg),
               "input %d, data line %llu: chromosome '%s' follows '%s' (%s input is not sorted "
               "per sort-bed)",
               idx + 1, (unsigned long long)T->run_row0[k] + 1, T->run_name[k].c_str(),
               T->run_name[k - 1].c_str(), kind_name(in.kind));
      return bg_fail(c, BG_E_UNSORTED, msg);
    }
  }
  T->run_row0.push_back(rows);
  bg_release(c, run_row);
  bg_release(c, run_tok);
  bg_release(c, run_len);
  bg_release(c, cnt);
  bg_release(c, row0);
  bg_release(c, lastnl);
  bg_release(c, prevnl);
  bg_release(c, d_rows);
  return 0;
}

int bg_key_tables(bg_ctx* c, bg_set* s) {
  // global dictionary: union of names, strcmp order
  std::vector<std::string> all;
  for (bg_table* T : s->t)
    for (auto& nm : T->run_name) all.push_back(nm);
  std::sort(all.begin(), all.end(),
            [](const std::string& a, const std::string& b) { return strcmp(a.c_str(), b.c_str()) < 0; });
  all.erase(std::unique(all.begin(), all.end()), all.end());
  if (all.size() >= (1u << 22)) return bg_fail(c, BG_E_UNSUPPORTED, "too many chromosomes");
  s->names = all;
  std::map<std::string, int32_t> gid;
  for (size_t k = 0; k < all.size(); ++k) gid[all[k]] = (int32_t)k;
  // packed names on device
  std::vector<uint32_t> off(all.size() + 1, 0), len(all.size() + 1, 0);
  std::string packed;
  for (size_t k = 0; k < all.size(); ++k) {
    off[k] = (uint32_t)packed.size();
    len[k] = (uint32_t)all[k].size();
    s->max_name_len = std::max<uint32_t>(s->max_name_len, len[k]);
    packed += all[k];
  }
  s->d_names = (char*)bg_alloc(c, packed.size() + 16);
  s->d_name_off = (uint32_t*)bg_alloc(c, 4 * off.size());
  s->d_name_len = (uint32_t*)bg_alloc(c, 4 * len.size());
  if (!s->d_names || !s->d_name_off || !s->d_name_len) return BG_E_NOMEM;
  if (!packed.empty())
    BG_HIP(c, hipMemcpyAsync(s->d_names, packed.data(), packed.size(), hipMemcpyHostToDevice, c->stream));
  BG_HIP(c, hipMemcpyAsync(s->d_name_off, off.data(), 4 * off.size(), hipMemcpyHostToDevice, c->stream));
  BG_HIP(c, hipMemcpyAsync(s->d_name_len, len.data(), 4 * len.size(), hipMemcpyHostToDevice, c->stream));
  BG_HIP(c, hipMemsetAsync(c->dstat, 0, sizeof(bg_dstatus), c->stream));
  BG_HIP(c, hipMemsetAsync(&c->dstat->first_bad, 0xff, 8, c->stream));
  std::vector<uint64_t*> tmp_rows;
  std::vector<int32_t*> tmp_gid;
  for (size_t f = 0; f < s->t.size(); ++f) {
    bg_table* T = s->t[f];
    if (T->n == 0) continue;
    const uint32_t nr = (uint32_t)T->run_name.size();
    std::vector<int32_t> g(nr);
    for (uint32_t k = 0; k < nr; ++k) g[k] = gid[T->run_name[k]];
    uint64_t* d_r0 = (uint64_t*)bg_alloc(c, 8ull * (nr + 1));
    int32_t* d_g = (int32_t*)bg_alloc(c, 4ull * nr);
    if (!d_r0 || !d_g) return BG_E_NOMEM;
    // copies are from pageable vectors: make them synchronous w.r.t. the host below
    BG_HIP(c, hipMemcpyAsync(d_r0, T->run_row0.data(), 8ull * (nr + 1), hipMemcpyHostToDevice, c->stream));
    BG_HIP(c, hipMemcpyAsync(d_g, g.data(), 4ull * nr, hipMemcpyHostToDevice, c->stream));
    BG_LAUNCH(c, "k_key", k_key, dim3(bg_blocks(T->n, BG_NT)), dim3(BG_NT), T->ks, T->ke,
                       T->n, d_r0, d_g, nr, c->dstat);
    BG_HIP(c, hipGetLastError());
    BG_HIP(c, hipMemcpyAsync(c->hstat, c->dstat, sizeof(bg_dstatus), hipMemcpyDeviceToHost, c->stream));
    BG_HIP(c, hipStreamSynchronize(c->stream));
    bg_release(c, d_r0);
    bg_release(c, d_g);
    int rc = report_status(c, (int)f, *c->hstat);
    if (rc) return rc;
    T->has_zero_len = (c->hstat->flags & 2ULL) != 0;
    BG_HIP(c, hipMemsetAsync(&c->dstat->flags, 0, 8, c->stream));
  }
  return 0;
}

extern "C" int bg_load(bg_ctx* c, int n, const bg_input* inputs, bg_set** out) {
  if (!c || n <= 0 || !inputs || !out) return BG_E_ARG;
  *out = nullptr;
  bg_set* s = new bg_set();
  s->ctx = c;
  for (int i = 0; i < n; ++i) {
    bg_table* T = new bg_table();
    s->t.push_back(T);
    int rc = parse_one(c, i, inputs[i], T);
    if (rc) { bg_set_free(s); return rc; }
  }
  bg_mark(c, "parse");
  int rc = bg_key_tables(c, s);
  if (rc) { bg_set_free(s); return rc; }
  bg_mark(c, "key");
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
    bg_release(c, T->own_text);
    bg_release(c, T->rest_off);
    bg_release(c, T->rest_len);
    bg_release(c, T->score);
    delete T;
  }
  bg_release(c, s->d_names);
  bg_release(c, s->d_name_off);
  bg_release(c, s->d_name_len);
  delete s;
}
