/*
 * bedgen — deterministic synthetic sorted BED3/BED5 generator.
 *
 * Re-implements the survey generator spec of SURVEY.md Appendix D exactly, so the
 * files (and the reference outputs whose sha256 prefixes the survey recorded) can
 * be reproduced on any box without the reference:
 *   - splitmix64 stream seeded with `seed`; call k uses state seed + (k+1)*gamma,
 *     so every contig can be generated independently (jump-ahead) and in parallel;
 *   - 25 GRCh38 primary contigs in strcmp order (or chr1 only);
 *   - per contig: n = (uint64)(N*(len/total)+0.5); n starts ~ next()%(len-80),
 *     sorted; n lengths 1+next()%80; lengths sorted inside runs of equal starts;
 *   - BED3 "chrom\tstart\tend\n"; BED5 "chrom\tstart\tend\tid<i>\t<next()%1000>\n"
 *     with the score draws after all start/length draws of that contig.
 *
 * Library entry: bedgen_buffer(); CLI: bedgen N seed [--bed5] [--chr1] > out.bed
 * Build: gcc -O3 -fopenmp -shared -fPIC (see Makefile).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define GAMMA 0x9e3779b97f4a7c15ULL

static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
/* value of the k-th (0-based) draw of a stream seeded with `seed` */
static inline uint64_t draw(uint64_t seed, uint64_t k) { return mix64(seed + (k + 1) * GAMMA); }

typedef struct { const char* name; uint64_t len; } contig_t;
static const contig_t HG38[25] = {
  {"chr1", 248956422}, {"chr10", 133797422}, {"chr11", 135086622}, {"chr12", 133275309},
  {"chr13", 114364328}, {"chr14", 107043718}, {"chr15", 101991189}, {"chr16", 90338345},
  {"chr17", 83257441}, {"chr18", 80373285}, {"chr19", 58617616}, {"chr2", 242193529},
  {"chr20", 64444167}, {"chr21", 46709983}, {"chr22", 50818468}, {"chr3", 198295559},
  {"chr4", 190214555}, {"chr5", 181538259}, {"chr6", 170805979}, {"chr7", 159345973},
  {"chr8", 145138636}, {"chr9", 138394717}, {"chrM", 16569}, {"chrX", 156040895},
  {"chrY", 57227415}};

/* LSD radix sort of uint32 keys (2 x 16-bit passes) */
static void radix_sort_u32(uint32_t* a, uint32_t* tmp, uint64_t n) {
  uint64_t* cnt = (uint64_t*)calloc(65536, sizeof(uint64_t));
  for (int pass = 0; pass < 2; ++pass) {
    int sh = pass * 16;
    memset(cnt, 0, 65536 * sizeof(uint64_t));
    for (uint64_t i = 0; i < n; ++i) cnt[(a[i] >> sh) & 0xffff]++;
    uint64_t s = 0;
    for (int b = 0; b < 65536; ++b) { uint64_t c = cnt[b]; cnt[b] = s; s += c; }
    for (uint64_t i = 0; i < n; ++i) tmp[cnt[(a[i] >> sh) & 0xffff]++] = a[i];
    memcpy(a, tmp, n * sizeof(uint32_t));
  }
  free(cnt);
}

static inline int u64_len(uint64_t v) { int l = 1; while (v >= 10) { v /= 10; ++l; } return l; }
static inline char* put_u64(char* p, uint64_t v) {
  char buf[24]; int l = 0;
  do { buf[l++] = (char)('0' + v % 10); v /= 10; } while (v);
  while (l) *p++ = buf[--l];
  return p;
}

typedef struct {
  int c;             /* contig index */
  uint64_t n;        /* rows */
  uint32_t* start;
  uint8_t* length;
  uint32_t* score;   /* BED5 only */
} cgen_t;

/* Number of contigs and their names/lengths (for sharding by chromosome). */
int bedgen_ncontigs(void) { return 25; }
const char* bedgen_contig_name(int c) { return (c >= 0 && c < 25) ? HG38[c].name : ""; }
uint64_t bedgen_contig_len(int c) { return (c >= 0 && c < 25) ? HG38[c].len : 0; }

/* Generate the rows of the contigs selected by `mask` (bit c = contig c) of the
 * file described by (N, seed, mode, chr1_only): identical bytes to the matching
 * contig sections of the full file, thanks to the jump-ahead stream. */
int bedgen_buffer_subset(uint64_t N, uint64_t seed, int mode, int chr1_only, uint64_t mask,
                         char** out, uint64_t* out_len, uint64_t* out_rows);

/* Generate a whole file into a malloc'ed buffer. mode: 3 = BED3, 5 = BED5,
 * 6 = BED5 with decimal scores ("<d>.<ddd>": draw % 100000 / 1000; not in SURVEY App. D).
 * Returns 0 on success; *out must be freed with bedgen_free(). */
int bedgen_buffer(uint64_t N, uint64_t seed, int mode, int chr1_only,
                  char** out, uint64_t* out_len, uint64_t* out_rows) {
  return bedgen_buffer_subset(N, seed, mode, chr1_only, ~0ULL, out, out_len, out_rows);
}

int bedgen_buffer_subset(uint64_t N, uint64_t seed, int mode, int chr1_only, uint64_t mask,
                         char** out, uint64_t* out_len, uint64_t* out_rows) {
  int nc = chr1_only ? 1 : 25;
  double total = 0;
  for (int c = 0; c < nc; ++c) total += (double)HG38[c].len;
  cgen_t* g = (cgen_t*)calloc((size_t)nc, sizeof(cgen_t));
  uint64_t* base = (uint64_t*)calloc((size_t)nc + 1, sizeof(uint64_t));
  uint64_t rows = 0;
  for (int c = 0; c < nc; ++c) {
    g[c].c = c;
    g[c].n = (uint64_t)((double)N * ((double)HG38[c].len / total) + 0.5);
    base[c + 1] = base[c] + g[c].n * (mode >= 5 ? 3 : 2);
  }
  for (int c = 0; c < nc; ++c) { /* unselected contigs keep their draw offsets, emit nothing */
    if (!((mask >> c) & 1ULL)) g[c].n = 0;
    rows += g[c].n;
  }
  /* draws + sorting, one contig per task */
  #pragma omp parallel for schedule(dynamic, 1)
  for (int c = 0; c < nc; ++c) {
    uint64_t n = g[c].n, k = base[c];
    uint64_t span = HG38[c].len - 80;
    uint32_t* st = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
    uint32_t* tmp = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
    uint8_t* ln = (uint8_t*)malloc(n ? n : 1);
    for (uint64_t i = 0; i < n; ++i) st[i] = (uint32_t)(draw(seed, k++) % span);
    radix_sort_u32(st, tmp, n);
    for (uint64_t i = 0; i < n; ++i) ln[i] = (uint8_t)(1 + draw(seed, k++) % 80);
    /* sort lengths within runs of equal starts (insertion sort: runs are tiny) */
    for (uint64_t i = 0; i < n;) {
      uint64_t j = i + 1;
      while (j < n && st[j] == st[i]) ++j;
      for (uint64_t a = i + 1; a < j; ++a) {
        uint8_t v = ln[a]; uint64_t b = a;
        while (b > i && ln[b - 1] > v) { ln[b] = ln[b - 1]; --b; }
        ln[b] = v;
      }
      i = j;
    }
    free(tmp);
    g[c].start = st; g[c].length = ln;
    if (mode >= 5) {
      uint32_t* sc = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
      for (uint64_t i = 0; i < n; ++i) sc[i] = (uint32_t)(draw(seed, k++) % (mode == 6 ? 100000 : 1000));
      g[c].score = sc;
    }
  }
  /* text layout: chunk rows, size pass, prefix, write pass */
  const uint64_t CH = 1u << 20;
  uint64_t nchunks = 0;
  for (int c = 0; c < nc; ++c) nchunks += (g[c].n + CH - 1) / CH;
  int* ck_c = (int*)malloc((nchunks ? nchunks : 1) * sizeof(int));
  uint64_t* ck_r0 = (uint64_t*)malloc((nchunks ? nchunks : 1) * sizeof(uint64_t));
  uint64_t* ck_off = (uint64_t*)calloc(nchunks + 1, sizeof(uint64_t));
  uint64_t q = 0;
  for (int c = 0; c < nc; ++c)
    for (uint64_t r = 0; r < g[c].n; r += CH) { ck_c[q] = c; ck_r0[q] = r; ++q; }
  #pragma omp parallel for schedule(dynamic, 1)
  for (uint64_t t = 0; t < nchunks; ++t) {
    const cgen_t* G = &g[ck_c[t]];
    uint64_t r1 = ck_r0[t] + CH < G->n ? ck_r0[t] + CH : G->n;
    uint64_t nl = strlen(HG38[G->c].name), bytes = 0;
    for (uint64_t i = ck_r0[t]; i < r1; ++i) {
      uint64_t s = G->start[i], e = s + G->length[i];
      bytes += nl + 1 + (uint64_t)u64_len(s) + 1 + (uint64_t)u64_len(e) + 1;
      if (mode == 5) bytes += 3 + (uint64_t)u64_len(i) + 1 + (uint64_t)u64_len(G->score[i]);
      if (mode == 6) bytes += 3 + (uint64_t)u64_len(i) + 1 + (uint64_t)u64_len(G->score[i] / 1000) + 4;
    }
    ck_off[t + 1] = bytes;
  }
  for (uint64_t t = 0; t < nchunks; ++t) ck_off[t + 1] += ck_off[t];
  uint64_t total_bytes = ck_off[nchunks];
  char* buf = (char*)malloc(total_bytes ? total_bytes : 1);
  if (!buf) return -1;
  #pragma omp parallel for schedule(dynamic, 1)
  for (uint64_t t = 0; t < nchunks; ++t) {
    const cgen_t* G = &g[ck_c[t]];
    uint64_t r1 = ck_r0[t] + CH < G->n ? ck_r0[t] + CH : G->n;
    const char* nm = HG38[G->c].name; size_t nl = strlen(nm);
    char* p = buf + ck_off[t];
    for (uint64_t i = ck_r0[t]; i < r1; ++i) {
      uint64_t s = G->start[i], e = s + G->length[i];
      memcpy(p, nm, nl); p += nl; *p++ = '\t';
      p = put_u64(p, s); *p++ = '\t'; p = put_u64(p, e);
      if (mode == 5) {
        *p++ = '\t'; *p++ = 'i'; *p++ = 'd'; p = put_u64(p, i);
        *p++ = '\t'; p = put_u64(p, G->score[i]);
      }
      if (mode == 6) {
        const uint32_t f = G->score[i] % 1000;
        *p++ = '\t'; *p++ = 'i'; *p++ = 'd'; p = put_u64(p, i);
        *p++ = '\t'; p = put_u64(p, G->score[i] / 1000);
        *p++ = '.'; *p++ = (char)('0' + f / 100); *p++ = (char)('0' + f / 10 % 10); *p++ = (char)('0' + f % 10);
      }
      *p++ = '\n';
    }
  }
  for (int c = 0; c < nc; ++c) { free(g[c].start); free(g[c].length); free(g[c].score); }
  free(g); free(base); free(ck_c); free(ck_r0); free(ck_off);
  *out = buf; *out_len = total_bytes;
  if (out_rows) *out_rows = rows;
  return 0;
}

void bedgen_free(char* p) { free(p); }

#ifdef BEDGEN_MAIN
int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: bedgen N seed [--bed5] [--chr1]\n");
    return 1;
  }
  uint64_t N = strtoull(argv[1], 0, 10), seed = strtoull(argv[2], 0, 10);
  int mode = 3, chr1 = 0;
  for (int i = 3; i < argc; ++i) {
    if (!strcmp(argv[i], "--bed5")) mode = 5;
    if (!strcmp(argv[i], "--bed5-decimal")) mode = 6;
    else if (!strcmp(argv[i], "--chr1")) chr1 = 1;
  }
  char* buf; uint64_t len, rows;
  if (bedgen_buffer(N, seed, mode, chr1, &buf, &len, &rows)) return 1;
  size_t off = 0;
  while (off < len) {
    size_t w = fwrite(buf + off, 1, len - off > (1u << 26) ? (1u << 26) : len - off, stdout);
    if (!w) return 1;
    off += w;
  }
  bedgen_free(buf);
  return 0;
}
#endif
