// bg_check.hip — f3: `--ec` input validation on the GPU.
//
// Reference: Bed::bed_check_iterator (interfaces/general-headers/data/bed/
// BedCheckIterator.hpp): every line read with std::getline (Ext::ByLine) goes through
// check() — the row grammar of bg_check.h, headers allowed only before the first row
// (:215-228 skip them there, :238-246 reject them later), then the order checks against
// the previous row and end > start (:594-624); the first failing line throws
// "in <file>\n<message>\nSee row: <line number>".
// GPU form: two passes over 8 KiB tiles, one thread per line (found from each thread's
// 32 bytes and a block scan of newline counts on top of per-tile counts): pass 1 finds the
// first non-header line F; pass 2 checks every line (a line after F also re-reads the line
// before it for the order checks — stateless, so all lines check in parallel) and keeps
// the smallest (line << 8 | code) with one atomicMin. Pass 3 (failures only) returns that
// line's byte range; bg_check_message() words the reference's message from it on the host.
#include <climits>
#include <cstdio>
#include <cstring>

#include "bg_internal.h"
#include "bg_check.h"

#define CK_TILE 8192

__global__ void __launch_bounds__(BG_NT) k_ck_count(const char* __restrict__ t, uint64_t nb,
                                                    uint64_t* __restrict__ cnt) {
  __shared__ uint32_t sh[BG_NT / 64];
  const uint64_t b = (uint64_t)blockIdx.x * CK_TILE + (uint64_t)threadIdx.x * 32;
  uint32_t c = 0;
  for (uint32_t i = 0; i < 32; ++i) c += (b + i < nb && t[b + i] == '\n');
  c = wave_incl_scan(c, OpSum());
  if (bg_lane() == 63) sh[bg_wave()] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

struct CkArgs {
  const char* t;
  uint64_t nb;
  const uint64_t* base;  // newlines before each tile (exclusive scan)
  int nfields, has_rest, nest;
  uint64_t* first_data;  // pass 1 out / pass 2 in: first non-header line (1-based)
  unsigned long long* key;  // pass 2 out: min (line << 8 | code)
  uint64_t target;       // pass 3: the failing line
  uint64_t* range;       // pass 3 out: [start, end) of the line and of the line before
};

__device__ __forceinline__ uint64_t ck_line_end(const char* t, uint64_t nb, uint64_t p) {
  while (p < nb && t[p] != '\n') ++p;
  return p;
}

template <int PASS>
__device__ __forceinline__ void ck_one(const CkArgs& A, uint64_t row, uint64_t ls) {
  const uint64_t le = ck_line_end(A.t, A.nb, ls);
  if (PASS == 3) {
    if (row != A.target) return;
    uint64_t ps = ls;
    if (ls > 0) {
      ps = ls - 1;
      while (ps > 0 && A.t[ps - 1] != '\n') --ps;
    }
    A.range[0] = ls;
    A.range[1] = le;
    A.range[2] = ps;
    A.range[3] = ls > 0 ? ls - 1 : ls;
    return;
  }
  BgcRow R;
  const int code = bgc_line(A.t + ls, (uint32_t)min(le - ls, (uint64_t)UINT_MAX), A.nfields,
                            A.has_rest, R);
  if (PASS == 1) {
    if (code != BGC_HEADER) atomicMin((unsigned long long*)A.first_data, (unsigned long long)row);
    return;
  }
  const uint64_t F = *A.first_data;
  int err = BGC_OK;
  if (code == BGC_HEADER) {
    if (row > F) err = BGC_HEADER_LATE;
  } else if (code != BGC_OK) {
    err = code;
  } else if (row > F) {  // the previous line is a row: F <= row - 1
    uint64_t ps = ls - 1;
    while (ps > 0 && A.t[ps - 1] != '\n') --ps;
    BgcRow P;
    const uint32_t pn = (uint32_t)(ls - 1 - ps);
    if (bgc_line(A.t + ps, pn, A.nfields, A.has_rest, P) == BGC_OK)
      err = bgc_order(A.t + ps, pn, P, A.t + ls, (uint32_t)(le - ls), R, A.has_rest, A.nest);
  } else if (R.end <= R.start) {
    err = BGC_END_LE_START;
  }
  if (err) atomicMin(A.key, ((unsigned long long)row << 8) | (unsigned long long)err);
}

// one workgroup per tile; line g + 2 starts after the file's newline number g (0-based)
template <int PASS>
__global__ void __launch_bounds__(BG_NT) k_ck_lines(CkArgs A) {
  __shared__ uint32_t sh[BG_NT / 64];
  const uint64_t b = (uint64_t)blockIdx.x * CK_TILE + (uint64_t)threadIdx.x * 32;
  uint32_t m = 0;
  for (uint32_t i = 0; i < 32; ++i) m |= (b + i < A.nb && A.t[b + i] == '\n') ? (1u << i) : 0u;
  const uint32_t c = (uint32_t)__popc(m);
  const uint32_t inc = wave_incl_scan(c, OpSum());
  if (bg_lane() == 63) sh[bg_wave()] = inc;
  __syncthreads();
  uint64_t g = A.base[blockIdx.x] + inc - c;
  for (int q = 0; q < bg_wave(); ++q) g += sh[q];
  if (blockIdx.x == 0 && threadIdx.x == 0 && A.nb > 0) ck_one<PASS>(A, 1, 0);
  for (uint32_t x = m; x; x &= x - 1, ++g) {
    const uint64_t p = b + __builtin_ctz(x) + 1;
    if (p < A.nb) ck_one<PASS>(A, g + 2, p);
  }
}

extern "C" int bg_check(bg_ctx* c, const bg_input* in, int nfields, int has_rest,
                        bg_check_result* out) {
  if (!c || !in || !out || nfields < 3 || nfields > 6) return BG_E_ARG;
  memset(out, 0, sizeof(*out));
  const uint64_t nb = in->nbytes;
  if (nb == 0) return 0;
  const char* t = (const char*)in->data;
  char* dt = nullptr;
  if (!in->on_device) {
    dt = (char*)bg_alloc(c, nb);
    if (!dt) return BG_E_NOMEM;
    BG_HIP(c, hipMemcpyAsync(dt, in->data, nb, hipMemcpyHostToDevice, c->stream));
    t = dt;
  }
  const uint64_t nt = (nb + CK_TILE - 1) / CK_TILE;
  uint64_t* base = (uint64_t*)bg_alloc(c, 8 * nt);
  uint64_t* w = (uint64_t*)bg_alloc(c, 8 * 8);  // first_data, key, range[4]
  if (!base || !w) return BG_E_NOMEM;
  CkArgs A;
  A.t = t;
  A.nb = nb;
  A.base = base;
  A.nfields = nfields;
  A.has_rest = has_rest & 1;
  A.nest = (has_rest & BG_CHECK_NEST) != 0;
  A.first_data = w;
  A.key = (unsigned long long*)(w + 1);
  A.target = 0;
  A.range = w + 2;
  BG_HIP(c, hipMemsetAsync(w, 0xff, 16, c->stream));
  BG_LAUNCH(c, "k_ck_count", k_ck_count, dim3((unsigned)nt), dim3(BG_NT), t, nb, base);
  int rc = bg_scan_sum_u64(c, base, base, nt, nullptr);
  if (rc) return rc;
  BG_LAUNCH(c, "k_ck_lines<1>", k_ck_lines<1>, dim3((unsigned)nt), dim3(BG_NT), A);
  BG_LAUNCH(c, "k_ck_lines<2>", k_ck_lines<2>, dim3((unsigned)nt), dim3(BG_NT), A);
  BG_HIP(c, hipGetLastError());
  uint64_t h[2];
  BG_HIP(c, hipMemcpyAsync(h, w, 16, hipMemcpyDeviceToHost, c->stream));
  BG_HIP(c, hipStreamSynchronize(c->stream));
  if (h[1] != ~0ULL) {
    out->row = h[1] >> 8;
    out->code = (int)(h[1] & 0xff);
    A.target = out->row;
    BG_LAUNCH(c, "k_ck_lines<3>", k_ck_lines<3>, dim3((unsigned)nt), dim3(BG_NT), A);
    BG_HIP(c, hipGetLastError());
    uint64_t r[4];
    BG_HIP(c, hipMemcpyAsync(r, w + 2, 32, hipMemcpyDeviceToHost, c->stream));
    BG_HIP(c, hipStreamSynchronize(c->stream));
    out->line_off = r[0];
    out->line_len = r[1] - r[0];
    out->prev_off = r[2];
    out->prev_len = r[3] - r[2];
  }
  bg_release(c, base);
  bg_release(c, w);
  if (dt) bg_release(c, dt);
  bg_mark(c, "check");
  return 0;
}

// the reference's wording (BedCheckIterator.hpp:326-624) of `code` for `line`
extern "C" int bg_check_message(const char* line, uint64_t len, int code, int nfields, int has_rest,
                                char* buf, uint64_t cap) {
  if (!buf || cap == 0) return BG_E_ARG;
  BgcRow R;
  has_rest &= 1;
  if (line) (void)bgc_line(line, (uint32_t)len, nfields, has_rest, R);
  else R.bad = 0;
  char ch[2] = {(char)R.bad, 0};
  const char* m = nullptr;
  char tmp[512];
  switch (code) {
    case BGC_EMPTY: m = "Empty line found."; break;
    case BGC_CHR_SPACE: m = "First column should not have spaces.  Consider 'chr1' vs. 'chr1 '.  These are different names.\nsort-bed can correct this for you."; break;
    case BGC_CHR_TAB0: m = "First column name should not start with a tab."; break;
    case BGC_NO_TABS: m = "No tabs found in BED row."; break;
    case BGC_CHR_LONG:
      snprintf(tmp, sizeof(tmp), "Chromosome name does not fit in MAXCHROMSIZE chars.\nIncrease TOKEN_CHR_MAX_LENGTH in BEDOPS.Constants.hpp and recompile BEDOPS.\nMAXCHROMSIZE = %u; Size given = %u", BGC_MAXCHROMSIZE, R.bad);
      m = tmp;
      break;
    case BGC_S_TABS: m = "Two or more consecutive tabs.  No start coordinate."; break;
    case BGC_S_NEG: m = "Start coordinate cannot be < 0: "; break;
    case BGC_S_SPACE: m = "Start coordinate may not contain a space: "; break;
    case BGC_S_CHAR: snprintf(tmp, sizeof(tmp), "Start coordinate contains non-numeric character: %s", ch); m = tmp; break;
    case BGC_S_NOTAB: m = "No tabs after start coordinate."; break;
    case BGC_S_DIGITS: case BGC_E_DIGITS: m = "Sanity check failure - start coordinate has too many digits as defined by MAX_DEC_INTEGERS in BEDOPS.Constants.hpp"; break;
    case BGC_S_MAX: case BGC_E_MAX: m = "Sanity check failure - start coordinate is more than allowed by MAX_COORD_VALUE in BEDOPS.Constants.hpp"; break;
    case BGC_E_TABS: m = "Two or more consecutive tabs.  No end coordinate."; break;
    case BGC_E_NEG: m = "End coordinate cannot be < 0: "; break;
    case BGC_E_SPACE: m = "End coordinate may not contain a space: "; break;
    case BGC_E_CHAR: snprintf(tmp, sizeof(tmp), "End coordinate contains non-numeric character: %s", ch); m = tmp; break;
    case BGC_ONLY3: snprintf(tmp, sizeof(tmp), "Only 3 columns given.  Require at least %d", nfields); m = tmp; break;
    case BGC_ID_TABS: m = "Two or more consecutive tabs.  No ID field."; break;
    case BGC_ID_SPACE: m = "ID field may not contain a space."; break;
    case BGC_ONLY4: snprintf(tmp, sizeof(tmp), "Only 4 columns given.  Require at least %d", nfields); m = tmp; break;
    case BGC_ID_EMPTY: m = "Fourth (id) column is empty."; break;
    case BGC_ID_LONG:
      snprintf(tmp, sizeof(tmp), "ID field does not fit in MAXCHROMSIZE chars.\nIncrease TOKEN_ID_MAX_LENGTH in BEDOPS.Constants.hpp and recompile BEDOPS.\nMAXIDSIZE = %u; Size given = %u", BGC_MAXIDSIZE, R.bad);
      m = tmp;
      break;
    case BGC_M_TABS: m = "Two or more consecutive tabs.  No measurement given."; break;
    case BGC_M_DOTS: m = "More than one decimal point in measurement field."; break;
    case BGC_M_DOTEXP: m = "Bad decimal point - part of exponent."; break;
    case BGC_M_EXPS: m = "Measurement value contains non-numeric character (multiple 'E' or 'e' characters detected)."; break;
    case BGC_M_SPACE: m = "Measurement value may not contain a space."; break;
    case BGC_M_SIGNPOS: m = "Measurement value has '-' or '+' in wrong place."; break;
    case BGC_M_SIGNS: m = "Measurement value has multiple '-' and/or '+' characters."; break;
    case BGC_M_SIGNEXP: m = "Measurement value has bad '-' in the exponent."; break;
    case BGC_M_CHAR: snprintf(tmp, sizeof(tmp), "Measurement value contains non-numeric character: %s", ch); m = tmp; break;
    case BGC_ONLY5: snprintf(tmp, sizeof(tmp), "Only 5 columns given.  Require at least %d", nfields); m = tmp; break;
    case BGC_M_EMPTY: m = "Fifth (measure) column is empty."; break;
    case BGC_M_ENDMINUS: m = "Measurement value ends with a '-'."; break;
    case BGC_ST_TABS: m = "Two or more consecutive tabs.  No strand information given."; break;
    case BGC_ST_CHAR: snprintf(tmp, sizeof(tmp), "Strand (6th) column must be '+' or '-' (with no spaces).  Received: %s\nsort-bed can correct this for you.", ch); m = tmp; break;
    case BGC_ST_TWO: m = "Two or more consecutive '+' or '-'s detected."; break;
    case BGC_ST_EMPTY: m = "Sixth (strand) column is empty."; break;
    case BGC_REST_LONG:
      snprintf(tmp, sizeof(tmp), "The 'rest' of the input row (everything beyond the first %d fields) cannot fit into MAXRESTSIZE chars.\nIncrease TOKEN_REST_MAX_LENGTH in BEDOPS.Constants.hpp and recompile BEDOPS.\nMAXRESTSIZE = %u; Size given = %u", nfields, BGC_MAXRESTSIZE, R.bad);
      m = tmp;
      break;
    case BGC_UNSORTED_CHR: m = "Bed file not properly sorted by first column."; break;
    case BGC_UNSORTED_START: m = "Bed file not properly sorted by start coordinates."; break;
    case BGC_UNSORTED_END: m = "Bed file not properly sorted by end coordinates when start coordinates are identical."; break;
    case BGC_UNSORTED_REST: m = "Bed file not sorted by information following the 3rd column (columns 1-3 equal to previous row)."; break;
    case BGC_END_LE_START: m = "End coordinates must be greater than start coordinates."; break;
    case BGC_HEADER_LATE: m = "Header found but should be at top of file."; break;
    case BGC_NESTED: m = "Fully nested component found."; break;
    default: return BG_E_ARG;
  }
  snprintf(buf, cap, "%s", m);
  return 0;
}
