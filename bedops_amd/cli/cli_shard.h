/*
 * cli_shard.h — multi-GPU runs of the C front-ends (BEDGPU_DEVICES=0,1,...).
 *
 * The reference scales out by running one process per chromosome (`--chrom`,
 * docs/content/reference/set-operations/bedops.rst:721-726) and concatenating the
 * outputs in chromosome order. Here one process drives every listed GPU:
 *   1. each input's chromosome runs (byte ranges) are found by bisection over its sorted
 *      text — the idea of find_bed_range (interfaces/general-headers/algorithm/bed/
 *      FindBedRange.hpp:67-188): O(chromosomes x log(bytes)) line probes, no full scan;
 *   2. chromosomes go to devices by longest-processing-time on their bytes in all inputs;
 *   3. each device receives only its chromosomes' bytes, copied from the input files'
 *      mappings (bg_file_image: page-cache pages, nothing read whole into or pinned in host
 *      memory) through its context's pinned ring over its own link, and runs load ->
 *      operation -> format on its own host thread;
 *   4. stdout a regular file: each device writes its chromosomes' text spans straight to
 *      their offsets in the output (D2H over its own link, pwrite), so the output leaves
 *      over every device's link at once; otherwise (pipes) bg_group_gather reassembles the
 *      texts on device 0 in strcmp chromosome order over RCCL and device 0 streams them.
 * Inputs that are not regular files (stdin, pipes), inputs the host checks cannot split
 * cleanly (blank or out-of-order chromosome lines), a group that cannot be opened (fewer
 * GPUs than listed, RCCL unavailable) and any error inside a shard fall back to the
 * one-device path, so error messages and their line numbers are the single-device ones.
 */
#ifndef BEDOPS_AMD_CLI_SHARD_H
#define BEDOPS_AMD_CLI_SHARD_H

#include <pthread.h>

#include "cli_common.h"

#define SHARD_MAX_DEV 64
#define BG_CHR_NAME_CAP 128 /* chromosome names are at most 127 bytes (BEDOPS.Constants.hpp:32) */

typedef struct {
  char name[BG_CHR_NAME_CAP];
  uint64_t a, b; /* byte range [a, b) of the file */
} crun_t;

typedef struct {
  crun_t* r;
  int n, cap;
} cruns_t;

static int env_devices(int* dev, int cap) {
  const char* s = getenv("BEDGPU_DEVICES");
  if (!s || !*s) return 0;
  int n = 0;
  while (*s && n < cap) {
    char* e;
    long v = strtol(s, &e, 10);
    if (e == s || v < 0) return 0;
    dev[n++] = (int)v;
    s = e;
    if (*s == ',') ++s;
    else if (*s) return 0;
  }
  return n;
}

static uint64_t sh_line_start(const char* t, uint64_t p) {
  while (p > 0 && t[p - 1] != '\n') --p;
  return p;
}
static uint64_t sh_next_line(const char* t, uint64_t n, uint64_t p) {
  while (p < n && t[p] != '\n') ++p;
  return p < n ? p + 1 : n;
}
static int sh_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }
/* the chromosome token of the line starting at p (fscanf "%s" skips leading blanks) */
static int sh_token(const char* t, uint64_t n, uint64_t p, char* out) {
  while (p < n && sh_ws(t[p])) ++p;
  uint64_t q = p;
  while (q < n && t[q] != '\n' && !sh_ws(t[q])) ++q;
  if (q == p || q - p >= BG_CHR_NAME_CAP) return -1;
  memcpy(out, t + p, q - p);
  out[q - p] = 0;
  return 0;
}
static int sh_push(cruns_t* R, const char* nm, uint64_t a, uint64_t b) {
  if (R->n && !strcmp(R->r[R->n - 1].name, nm) && R->r[R->n - 1].b == a) {
    R->r[R->n - 1].b = b;
    return 0;
  }
  if (R->n == R->cap) {
    R->cap = R->cap ? 2 * R->cap : 64;
    R->r = (crun_t*)realloc(R->r, (size_t)R->cap * sizeof(crun_t));
    if (!R->r) return -1;
  }
  strcpy(R->r[R->n].name, nm);
  R->r[R->n].a = a;
  R->r[R->n].b = b;
  R->n++;
  return 0;
}
/* [a, b): a at a line start, b at a line start or n */
static int sh_runs_rec(const char* t, uint64_t n, uint64_t a, uint64_t b, cruns_t* R, int depth) {
  char ta[BG_CHR_NAME_CAP], tb[BG_CHR_NAME_CAP];
  if (depth > 200) return -1;
  const uint64_t lb = sh_line_start(t, b - 1);
  if (sh_token(t, n, a, ta) || sh_token(t, n, lb, tb)) return -1;
  if (!strcmp(ta, tb)) return sh_push(R, ta, a, b);
  uint64_t mid = sh_next_line(t, n, a + (b - a) / 2);
  if (mid >= b) mid = lb;
  if (mid <= a) mid = sh_next_line(t, n, a);
  if (mid <= a || mid >= b) return -1;
  if (sh_runs_rec(t, n, a, mid, R, depth + 1)) return -1;
  return sh_runs_rec(t, n, mid, b, R, depth + 1);
}
/* the chromosome runs of one sorted text; -1 when it cannot be split by names alone */
static int sh_find_runs(const char* t, uint64_t n, cruns_t* R) {
  R->n = 0;
  if (n == 0) return 0;
  if (sh_runs_rec(t, n, 0, n, R, 0)) return -1;
  for (int k = 1; k < R->n; ++k)
    if (strcmp(R->r[k - 1].name, R->r[k].name) >= 0) return -1; /* not in strcmp order */
  return 0;
}

/* one device's work: load its shard texts, run the operation, format */
typedef int (*shard_op_fn)(void* arg, bg_ctx* ctx, bg_set* set, bg_result** out);

typedef struct {
  bg_ctx* ctx;
  int nf;
  const bg_input* proto; /* kinds */
  const bg_file_image* fm; /* the input files' mappings */
  const cruns_t* runs;   /* per file */
  const int* owner;      /* global chromosome -> device */
  char (*gnames)[BG_CHR_NAME_CAP];
  int ngc, dev;
  shard_op_fn op;
  void* oparg;
  /* out */
  void** dtext;    /* per file: shard text on the device */
  bg_set* set;
  bg_result* res;
  const char* text;
  uint64_t nbytes;
  uint64_t *off, *len; /* per global chromosome */
  int rc;
} shard_job_t;

static int sh_gindex(char (*g)[BG_CHR_NAME_CAP], int n, const char* nm) {
  int lo = 0, hi = n;
  while (lo < hi) {
    int mid = (lo + hi) / 2;
    int v = strcmp(g[mid], nm);
    if (v == 0) return mid;
    if (v < 0) lo = mid + 1;
    else hi = mid;
  }
  return -1;
}

static void* shard_worker(void* p) {
  shard_job_t* J = (shard_job_t*)p;
  J->rc = bg_bind(J->ctx);
  if (J->rc) return NULL;
  bg_input* in = (bg_input*)calloc((size_t)J->nf, sizeof(bg_input));
  for (int f = 0; f < J->nf && !J->rc; ++f) {
    const cruns_t* R = &J->runs[f];
    const void** parts = (const void**)calloc((size_t)R->n + 1, sizeof(void*));
    uint64_t* lens = (uint64_t*)calloc((size_t)R->n + 1, sizeof(uint64_t));
    int np = 0;
    for (int k = 0; k < R->n; ++k) {
      const int g = sh_gindex(J->gnames, J->ngc, R->r[k].name);
      if (g < 0 || J->owner[g] != J->dev) continue;
      parts[np] = J->fm[f].data + R->r[k].a;
      lens[np++] = R->r[k].b - R->r[k].a;
    }
    uint64_t tot = 0;
    J->rc = bg_device_gather_host(J->ctx, np, parts, lens, &J->dtext[f], &tot);
    in[f] = J->proto[f];
    in[f].data = J->dtext[f];
    in[f].nbytes = tot;
    in[f].on_device = 1;
    free(parts);
    free(lens);
  }
  if (!J->rc) J->rc = bg_load(J->ctx, J->nf, in, &J->set);
  if (!J->rc) J->rc = J->op(J->oparg, J->ctx, J->set, &J->res);
  if (!J->rc) J->rc = bg_result_format(J->ctx, J->res, &J->nbytes);
  if (!J->rc) J->rc = bg_result_text_device(J->res, &J->text, &J->nbytes);
  uint32_t nsc = 0;
  if (!J->rc) J->rc = bg_set_chroms(J->set, &nsc);
  if (!J->rc) {
    uint64_t* o = (uint64_t*)calloc((size_t)nsc + 1, sizeof(uint64_t));
    J->rc = bg_result_chrom_spans(J->ctx, J->res, o, nsc + 1);
    for (uint32_t q = 0; q < nsc && !J->rc; ++q) {
      const int g = sh_gindex(J->gnames, J->ngc, bg_set_chrom_name(J->set, q));
      if (g < 0) { J->rc = BG_E_ARG; break; }
      J->off[g] = o[q];
      J->len[g] = o[q + 1] - o[q];
    }
    free(o);
  }
  bg_sync(J->ctx); /* the copies out of the mapped files have completed */
  free(in);
  return NULL;
}

/* one device's chromosome spans, each at its offset in the output file */
typedef struct {
  shard_job_t* J;
  const int* owner;
  const uint64_t* pos; /* output offset of each global chromosome (relative to off0) */
  int ngc;
  off_t off0;
  int rc;
} sh_write_job_t;
static void* shard_writer(void* p) {
  sh_write_job_t* W = (sh_write_job_t*)p;
  shard_job_t* J = W->J;
  W->rc = bg_bind(J->ctx);
  /* chromosomes adjacent both in this device's text and in the output go out as one range
   * (one ring pass instead of one per contig: assemblies with thousands of scaffolds) */
  uint64_t rt = 0, ro = 0, rl = 0;
  for (int g = 0; g < W->ngc && !W->rc; ++g) {
    if (W->owner[g] != J->dev || !J->len[g]) continue;
    if (rl && J->off[g] == rt + rl && W->pos[g] == ro + rl) {
      rl += J->len[g];
      continue;
    }
    if (rl) W->rc = bg_pwrite_device(J->ctx, J->text + rt, rl, 1, (int64_t)(W->off0 + (off_t)ro));
    rt = J->off[g];
    ro = W->pos[g];
    rl = J->len[g];
  }
  if (rl && !W->rc) W->rc = bg_pwrite_device(J->ctx, J->text + rt, rl, 1, (int64_t)(W->off0 + (off_t)ro));
  return NULL;
}

/* Runs the operation on every device of BEDGPU_DEVICES (>= 2 entries) and writes the
 * reassembled output to fd 1. Returns 0 when done, 1 when the caller should take the
 * one-device path instead (nothing written, no input consumed). */
static int shard_run(const char* prog, int nf, const bg_input* proto, const char* const* paths,
                     shard_op_fn op, void* oparg) {
  int dev[SHARD_MAX_DEV];
  const int nd = env_devices(dev, SHARD_MAX_DEV);
  if (nd < 2) return 1;
  bg_file_image* fm = (bg_file_image*)calloc((size_t)nf, sizeof(bg_file_image));
  int ok = 1;
  for (int f = 0; f < nf && ok; ++f) {
    struct stat st;
    ok = strcmp(paths[f], "-") != 0 && stat(paths[f], &st) == 0 && S_ISREG(st.st_mode) &&
         !file_is_starch(paths[f]) && bg_file_image_open(paths[f], &fm[f]) == 0;
  }
  cruns_t* runs = (cruns_t*)calloc((size_t)nf, sizeof(cruns_t));
  int total_runs = 0;
  for (int f = 0; f < nf && ok; ++f) {
    if (sh_find_runs(fm[f].data, fm[f].n, &runs[f])) ok = 0;
    total_runs += runs[f].n;
  }
  /* the global chromosome list (strcmp order) and bytes per chromosome */
  char(*gn)[BG_CHR_NAME_CAP] = (char(*)[BG_CHR_NAME_CAP])calloc((size_t)total_runs + 1, BG_CHR_NAME_CAP);
  int ngc = 0;
  for (int f = 0; f < nf && ok; ++f)
    for (int k = 0; k < runs[f].n; ++k) strcpy(gn[ngc++], runs[f].r[k].name);
  if (ok && ngc) {
    qsort(gn, (size_t)ngc, BG_CHR_NAME_CAP, (int (*)(const void*, const void*))strcmp);
    int u = 1;
    for (int k = 1; k < ngc; ++k)
      if (strcmp(gn[k], gn[u - 1])) strcpy(gn[u++], gn[k]);
    ngc = u;
  }
  if (!ok || ngc < 2) { /* nothing to split */
    for (int f = 0; f < nf; ++f) {
      free(runs[f].r);
      bg_file_image_close(&fm[f]);
    }
    free(runs);
    free(gn);
    free(fm);
    return 1;
  }
  uint64_t* bytes = (uint64_t*)calloc((size_t)ngc, sizeof(uint64_t));
  for (int f = 0; f < nf; ++f)
    for (int k = 0; k < runs[f].n; ++k)
      bytes[sh_gindex(gn, ngc, runs[f].r[k].name)] += runs[f].r[k].b - runs[f].r[k].a;
  /* longest processing time first */
  int* order = (int*)calloc((size_t)ngc, sizeof(int));
  int* owner = (int*)calloc((size_t)ngc, sizeof(int));
  uint64_t load[SHARD_MAX_DEV] = {0};
  for (int g = 0; g < ngc; ++g) order[g] = g;
  for (int i = 1; i < ngc; ++i) { /* insertion sort by bytes desc, index asc */
    int x = order[i], j = i;
    while (j > 0 && (bytes[order[j - 1]] < bytes[x] ||
                     (bytes[order[j - 1]] == bytes[x] && order[j - 1] > x))) {
      order[j] = order[j - 1];
      --j;
    }
    order[j] = x;
  }
  for (int i = 0; i < ngc; ++i) {
    int best = 0;
    for (int d = 1; d < nd; ++d)
      if (load[d] < load[best]) best = d;
    owner[order[i]] = best;
    load[best] += bytes[order[i]];
  }
  bg_group* grp = NULL;
  int rc = bg_group_open(&grp, dev, nd);
  if (rc) { /* fewer GPUs than listed, RCCL unavailable, ...: one device instead */
    const char* st = getenv("BEDGPU_STATS");
    if (st && *st && strcmp(st, "0") != 0)
      fprintf(stderr, "bedgpu: BEDGPU_DEVICES group not available (%d); one device\n", rc);
    for (int f = 0; f < nf; ++f) {
      free(runs[f].r);
      bg_file_image_close(&fm[f]);
    }
    free(runs);
    free(gn);
    free(bytes);
    free(order);
    free(owner);
    free(fm);
    return 1;
  }
  cli_mark("open");
  for (int f = 0; f < nf; ++f) (void)bg_file_image_register(&fm[f]); /* DMA source for every device */
  shard_job_t* J = (shard_job_t*)calloc((size_t)nd, sizeof(shard_job_t));
  pthread_t* th = (pthread_t*)calloc((size_t)nd, sizeof(pthread_t));
  for (int d = 0; d < nd; ++d) {
    J[d].ctx = bg_group_ctx(grp, d);
    J[d].nf = nf;
    J[d].proto = proto;
    J[d].fm = fm;
    J[d].runs = runs;
    J[d].owner = owner;
    J[d].gnames = gn;
    J[d].ngc = ngc;
    J[d].dev = d;
    J[d].op = op;
    J[d].oparg = oparg;
    J[d].dtext = (void**)calloc((size_t)nf, sizeof(void*));
    J[d].off = (uint64_t*)calloc((size_t)ngc, sizeof(uint64_t));
    J[d].len = (uint64_t*)calloc((size_t)ngc, sizeof(uint64_t));
    pthread_create(&th[d], NULL, shard_worker, &J[d]);
  }
  int failed = 0;
  for (int d = 0; d < nd; ++d) {
    pthread_join(th[d], NULL);
    failed = failed || J[d].rc;
  }
  cli_mark("shards");
  for (int f = 0; f < nf; ++f) bg_file_image_close(&fm[f]); /* the loads have synchronised */
  int done = 0;
  /* stdout a regular file: every device writes its own chromosomes' spans at their offsets
   * in the output (D2H over its own link, pwrite), no gather; anything else (pipes,
   * terminals, appends; BEDGPU_SHARD_GATHER=1): the RCCL gather to device 0 below */
  struct stat ost;
  const int ofl = fcntl(1, F_GETFL);
  const off_t off0 = lseek(1, 0, SEEK_CUR);
  const int direct = !failed && fstat(1, &ost) == 0 && S_ISREG(ost.st_mode) && ofl >= 0 && !(ofl & O_APPEND) &&
                     off0 >= 0 && !cli_env_on("BEDGPU_SHARD_GATHER");
  if (direct) {
    uint64_t* pos = (uint64_t*)calloc((size_t)ngc + 1, sizeof(uint64_t));
    for (int g = 0; g < ngc; ++g) pos[g + 1] = pos[g] + J[owner[g]].len[g];
    sh_write_job_t* W = (sh_write_job_t*)calloc((size_t)nd, sizeof(sh_write_job_t));
    for (int d = 0; d < nd; ++d) {
      W[d].J = &J[d];
      W[d].owner = owner;
      W[d].pos = pos;
      W[d].ngc = ngc;
      W[d].off0 = off0;
      pthread_create(&th[d], NULL, shard_writer, &W[d]);
    }
    int wrc = 0, wd = 0;
    for (int d = 0; d < nd; ++d) {
      pthread_join(th[d], NULL);
      if (W[d].rc && !wrc) { wrc = W[d].rc; wd = d; }
    }
    cli_mark("write");
    if (wrc) die_ctx(prog, J[wd].ctx, wrc);
    if (lseek(1, off0 + (off_t)pos[ngc], SEEK_SET) < 0) die_msg(prog, "seek failed on the output file");
    free(pos);
    free(W);
    maybe_stats(bg_group_ctx(grp, 0));
    fast_exit();
    done = 1;
  } else if (!failed) {
    const char** texts = (const char**)calloc((size_t)nd, sizeof(char*));
    const uint64_t** offs = (const uint64_t**)calloc((size_t)nd, sizeof(uint64_t*));
    const uint64_t** lens = (const uint64_t**)calloc((size_t)nd, sizeof(uint64_t*));
    for (int d = 0; d < nd; ++d) {
      texts[d] = J[d].text;
      offs[d] = J[d].off;
      lens[d] = J[d].len;
    }
    char* out = NULL;
    uint64_t n = 0;
    bg_ctx* c0 = bg_group_ctx(grp, 0);
    rc = bg_group_gather(grp, ngc, texts, offs, lens, &out, &n);
    if (rc) die_ctx(prog, c0, rc);
    if ((rc = bg_write_device(c0, out, n, 1))) die_ctx(prog, c0, rc);
    maybe_stats(c0);
    fast_exit();
    bg_device_free(c0, out);
    free(texts);
    free(offs);
    free(lens);
    done = 1;
  }
  for (int d = 0; d < nd; ++d) {
    bg_bind(J[d].ctx);
    bg_result_free(J[d].res);
    bg_set_free(J[d].set);
    for (int f = 0; f < nf; ++f) bg_device_free(J[d].ctx, J[d].dtext[f]);
    free(J[d].dtext);
    free(J[d].off);
    free(J[d].len);
  }
  bg_group_close(grp);
  for (int f = 0; f < nf; ++f) free(runs[f].r);
  free(runs);
  free(gn);
  free(bytes);
  free(order);
  free(owner);
  free(J);
  free(th);
  free(fm);
  return done ? 0 : 1;
}

#endif
