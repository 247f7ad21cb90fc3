/*
 * cli_stream.h — one GPU, chromosome groups in a pipeline (the front-ends' default for
 * large regular-file inputs of chromosome-local operations).
 *
 * The reference streams: it reads a few rows, prints, reads on (Bedops.cpp:148-152
 * record/Println; performance.rst:29 "O(window) memory"). The whole-file GPU path instead
 * runs read-all -> compute -> write-all, so the page-cache -> HBM copies and the output
 * write(2) (each ~0.1 s for the 100M x 100M benchmark) add up. Here the inputs are cut at
 * chromosome boundaries into G groups of consecutive chromosomes (strcmp order; a group
 * is ONE contiguous byte range of every sorted input), and
 *   main thread : group g's byte ranges -> HBM (pinned ring, ctx's stream) -> bg_load ->
 *                 operation -> format (text stays in HBM) -> pushed to the output queue
 *   bg_writer   : group g-1's text D2H on its own stream -> write(2) to fd 1
 * so the output of a group goes out (device->host direction of the link, one CPU thread)
 * while the next group comes in. Every covered operation is chromosome-local
 * (BedCompare.hpp:42-43: comparators start with strcmp(chrom); the same reasoning as the
 * multi-GPU shards, cli_shard.h, whose run discovery this reuses), so the concatenated
 * group outputs are the whole-file output byte for byte.
 *
 * Stdout a regular file (seekable, not O_APPEND): if anything fails in any group (a
 * malformed or unsorted line, a refusal such as bedmap's file-wide decimal sums), the output
 * written so far is truncated away and the caller runs the whole-file path, which reports
 * exactly what a whole-file run reports (messages, line numbers). Stdout a pipe
 * (BEDGPU_STREAM_PIPE=0: off): the groups go out in order as they are done; on a failure the
 * whole-file path runs with its first `sent` bytes dropped (bg_set_output_skip): the groups
 * already written are exactly that prefix, so a refusal (decimal sums) still ends in the
 * whole file's bytes; an input error leaves those groups followed by the whole-file path's
 * message and status (where that path alone prints the message without output).
 * BEDGPU_STREAM=0 turns it off; BEDGPU_STREAM_GROUPS (default 8), BEDGPU_STREAM_MIN
 * (bytes of input below which the whole-file path is used, default 256 MiB) and
 * BEDGPU_STREAM_MAX_GB (largest group, default 16: more groups for larger inputs, which
 * then need not fit in HBM at once) size it.
 */
#ifndef BEDOPS_AMD_CLI_STREAM_H
#define BEDOPS_AMD_CLI_STREAM_H

#include <pthread.h>

#include "cli_shard.h"

typedef struct {
  int nf;
  const char* const* paths;
  bg_file_image* fm; /* the inputs' mappings (no page-table population: no lock contention
                        with HIP's initialisation) */
  cruns_t* runs;     /* per file */
  int ng;            /* groups */
  uint64_t* ga;      /* [g * nf + f]: byte range [ga, gb) of file f in group g */
  uint64_t* gb;
  int ok, started;
  int pipe;          /* stdout is a pipe: no truncation, see stream_run */
  pthread_t th;
} stream_plan_t;
static stream_plan_t SP;

static long stream_env(const char* name, long def) {
  const char* s = getenv(name);
  return (s && *s) ? atol(s) : def;
}

static void stream_plan_free(void) {
  for (int f = 0; f < SP.nf && SP.fm; ++f) bg_file_image_close(&SP.fm[f]);
  for (int f = 0; f < SP.nf && SP.runs; ++f) free(SP.runs[f].r);
  free(SP.fm);
  free(SP.runs);
  free(SP.ga);
  free(SP.gb);
  SP.fm = NULL;
  SP.runs = NULL;
  SP.ga = SP.gb = NULL;
  SP.ok = 0;
}

/* mappings, chromosome runs by bisection, groups: host work only, on a thread of its own
 * while bg_open initialises HIP */
static void* stream_plan_run(void* unused) {
  (void)unused;
  const int nf = SP.nf;
  SP.fm = (bg_file_image*)calloc((size_t)nf, sizeof(bg_file_image));
  SP.runs = (cruns_t*)calloc((size_t)nf, sizeof(cruns_t));
  uint64_t total = 0;
  int nruns = 0;
  for (int f = 0; f < nf; ++f) {
    struct stat st;
    if (strcmp(SP.paths[f], "-") == 0 || stat(SP.paths[f], &st) != 0 || !S_ISREG(st.st_mode) ||
        file_is_starch(SP.paths[f]) || bg_file_image_open(SP.paths[f], &SP.fm[f]) != 0)
      return NULL;
    if (sh_find_runs(SP.fm[f].data, SP.fm[f].n, &SP.runs[f])) return NULL;
    total += SP.fm[f].n;
    nruns += SP.runs[f].n;
  }
  long G = stream_env("BEDGPU_STREAM_GROUPS", 8);
  if (G < 2 || total < (uint64_t)stream_env("BEDGPU_STREAM_MIN", 256L << 20) || nruns < 2) return NULL;
  /* out of core: no group above BEDGPU_STREAM_MAX_GB (default 16) of text, so inputs larger
   * than the GPU's memory stream through it (a group is whole chromosomes: one chromosome
   * of every input must fit) */
  const uint64_t gmax = (uint64_t)stream_env("BEDGPU_STREAM_MAX_GB", 16) << 30;
  if (gmax && total / (uint64_t)G > gmax) G = (long)((total + gmax - 1) / gmax);
  /* the global chromosome list in strcmp order, bytes per chromosome over all inputs */
  char(*gn)[BG_CHR_NAME_CAP] = (char(*)[BG_CHR_NAME_CAP])calloc((size_t)nruns, BG_CHR_NAME_CAP);
  int ngc = 0;
  for (int f = 0; f < nf; ++f)
    for (int k = 0; k < SP.runs[f].n; ++k) strcpy(gn[ngc++], SP.runs[f].r[k].name);
  qsort(gn, (size_t)ngc, BG_CHR_NAME_CAP, (int (*)(const void*, const void*))strcmp);
  int u = 1;
  for (int k = 1; k < ngc; ++k)
    if (strcmp(gn[k], gn[u - 1])) strcpy(gn[u++], gn[k]);
  ngc = u;
  uint64_t* bytes = (uint64_t*)calloc((size_t)ngc, sizeof(uint64_t));
  for (int f = 0; f < nf; ++f)
    for (int k = 0; k < SP.runs[f].n; ++k)
      bytes[sh_gindex(gn, ngc, SP.runs[f].r[k].name)] += SP.runs[f].r[k].b - SP.runs[f].r[k].a;
  /* consecutive chromosomes, a group closed once it holds total / G bytes; the first group
   * only total / (G * BEDGPU_STREAM_FIRST) (default 4), so the output queue starts early
   * and the fixed costs of the first copies are paid on little data */
  /* and the last group likewise at most total / (G * BEDGPU_STREAM_LAST) (default 4) when the
   * chromosomes allow it: the output queue's tail after the last group is that group's text */
  int* first = (int*)calloc((size_t)ngc + 1, sizeof(int)); /* group -> first chromosome */
  int ng = 0;
  uint64_t acc = 0, left = total;
  const uint64_t target = total / (uint64_t)G;
  const long F = stream_env("BEDGPU_STREAM_FIRST", 4), LF = stream_env("BEDGPU_STREAM_LAST", 4);
  const uint64_t target0 = target / (uint64_t)(F < 1 ? 1 : F);
  const uint64_t target_last = LF > 0 ? target / (uint64_t)LF : 0;
  int tail = 0;
  for (int g = 0; g < ngc; ++g) {
    if (!tail && acc && left <= target_last) { /* the rest is small: one group of its own */
      acc = 0;
      tail = 1;
    }
    if (acc == 0) first[ng++] = g;
    acc += bytes[g];
    left -= bytes[g];
    if (!tail && acc >= (ng == 1 ? target0 : target)) acc = 0;
  }
  first[ng] = ngc;
  if (ng >= 2) {
    SP.ga = (uint64_t*)calloc((size_t)ng * nf, sizeof(uint64_t));
    SP.gb = (uint64_t*)calloc((size_t)ng * nf, sizeof(uint64_t));
    for (int f = 0; f < nf; ++f) {
      const cruns_t* R = &SP.runs[f];
      int k = 0;
      for (int q = 0; q < ng; ++q) { /* runs of f whose chromosome is in [first[q], first[q+1]) */
        const uint64_t a = k < R->n ? R->r[k].a : SP.fm[f].n;
        while (k < R->n && sh_gindex(gn, ngc, R->r[k].name) < first[q + 1]) ++k;
        SP.ga[(size_t)q * nf + f] = a;
        SP.gb[(size_t)q * nf + f] = k < R->n ? R->r[k].a : SP.fm[f].n;
      }
    }
    SP.ng = ng;
    SP.ok = 1;
  }
  free(first);
  free(bytes);
  free(gn);
  return NULL;
}

/* starts the plan (call before bg_open); 0 if streaming is off for this run */
static int stream_prepare(int nf, const char* const* paths) {
  memset(&SP, 0, sizeof(SP));
  if (stream_env("BEDGPU_STREAM", 1) == 0) return 0;
  struct stat st;
  const int fl = fcntl(1, F_GETFL);
  if (fstat(1, &st) != 0 || fl < 0) return 0;
  const int is_pipe = S_ISFIFO(st.st_mode) && stream_env("BEDGPU_STREAM_PIPE", 1) != 0;
  if (!is_pipe && (!S_ISREG(st.st_mode) || (fl & O_APPEND))) return 0;
  {  /* the size test of the plan, up front: small inputs keep the whole-file path and its
        prefetch of the mappings during HIP initialisation */
    uint64_t total = 0;
    for (int f = 0; f < nf; ++f) {
      struct stat si;
      if (strcmp(paths[f], "-") == 0 || stat(paths[f], &si) != 0 || !S_ISREG(si.st_mode)) return 0;
      total += (uint64_t)si.st_size;
    }
    if (total < (uint64_t)stream_env("BEDGPU_STREAM_MIN", 256L << 20)) return 0;
  }
  SP.nf = nf;
  SP.paths = paths;
  SP.pipe = is_pipe;
  if (pthread_create(&SP.th, NULL, stream_plan_run, NULL) != 0) return 0;
  SP.started = 1;
  return 1;
}

/* Read-ahead (BEDGPU_STREAM_AHEAD groups, default 0 = copies in line; off by default: on the
 * 16-CPU box it saved ~30 ms of copies and cost as much in kernel and writer time): a copier thread
 * issues group g's page-cache -> HBM copies (bg_file_image_copy, the context's prefetch
 * stream) while the main thread loads, runs and formats earlier groups on ctx's stream, so
 * the DMA engine never waits for a group's host round trips. The main thread allocates every
 * group's buffers (the allocator is the main thread's) at most AHEAD groups ahead and fences
 * ctx's stream on a group's copies (bg_copy_fence) before loading it. */
typedef struct {
  bg_ctx* ctx;
  int nf, ng;
  void** d;          /* [g * nf + f] device buffers, allocated by the main thread */
  pthread_mutex_t mu;
  pthread_cond_t cv;
  int alloc_upto;    /* groups [0, alloc_upto) have buffers */
  int issued;        /* groups [0, issued) have their copies issued and fenced slots recorded */
  int stop;          /* main thread: stop issuing */
  int rc;            /* copier's first error */
  pthread_t th;
} stream_ahead_t;

static void* stream_copier(void* arg) {
  stream_ahead_t* A = (stream_ahead_t*)arg;
  for (int g = 0; g < A->ng; ++g) {
    pthread_mutex_lock(&A->mu);
    while (!A->stop && A->alloc_upto <= g) pthread_cond_wait(&A->cv, &A->mu);
    const int stop = A->stop;
    pthread_mutex_unlock(&A->mu);
    if (stop) break;
    int rc = 0;
    for (int f = 0; f < A->nf && !rc; ++f) {
      const uint64_t a = SP.ga[(size_t)g * A->nf + f], b = SP.gb[(size_t)g * A->nf + f];
      rc = bg_file_image_copy(A->ctx, &SP.fm[f], a, b - a, A->d[(size_t)g * A->nf + f], g);
    }
    pthread_mutex_lock(&A->mu);
    if (rc) {
      A->rc = rc;
      A->issued = A->ng;  /* wake the main thread: it stops at this group */
    } else {
      A->issued = g + 1;
    }
    pthread_cond_broadcast(&A->cv);
    pthread_mutex_unlock(&A->mu);
    if (rc) break;
  }
  return NULL;
}

/* Runs the operation group by group on ctx and writes the output to fd 1. Returns 0 when
 * done, 1 when the caller should take the whole-file path (nothing left on fd 1). */
static int stream_run(bg_ctx* ctx, const bg_input* proto, shard_op_fn op, void* oparg) {
  if (!SP.started) return 1;
  pthread_join(SP.th, NULL);
  SP.started = 0;
  const off_t off0 = SP.pipe ? 0 : lseek(1, 0, SEEK_CUR);
  if (!SP.ok || off0 < 0) {
    stream_plan_free();
    return 1;
  }
  const int nf = SP.nf, ng = SP.ng;
  bg_writer* w = NULL;
  if (bg_writer_open(ctx, 1, &w)) {
    stream_plan_free();
    return 1;
  }
  bg_result** res = (bg_result**)calloc((size_t)ng, sizeof(bg_result*));
  bg_input* in = (bg_input*)calloc((size_t)nf, sizeof(bg_input));
  void** d = (void**)calloc((size_t)nf, sizeof(void*));
  uint64_t freed = 0;
  int rc = 0, pushed = 0;
  uint64_t sent = 0;  /* bytes handed to the output queue */
  /* the group's input blocks go back to the cache stream-ordered (the next group's copies
   * are queued after its kernels on ctx's stream); a second copy stream needs the host wait */
  const int ordered = stream_env("BEDGPU_COPY_STREAMS", 1) < 2;
  const long ahead = ordered ? stream_env("BEDGPU_STREAM_AHEAD", 0) : 0;
  stream_ahead_t A;
  memset(&A, 0, sizeof(A));
  int copier = 0;
  if (ahead > 0) {
    A.ctx = ctx;
    A.nf = nf;
    A.ng = ng;
    A.d = (void**)calloc((size_t)ng * nf, sizeof(void*));
    pthread_mutex_init(&A.mu, NULL);
    pthread_cond_init(&A.cv, NULL);
    for (int g = 0; g < ng && g < ahead + 1 && !rc; ++g) {
      for (int f = 0; f < nf && !rc; ++f)
        rc = bg_device_alloc(ctx, SP.gb[(size_t)g * nf + f] - SP.ga[(size_t)g * nf + f] + 64, &A.d[(size_t)g * nf + f]);
      if (!rc) rc = bg_copy_order(ctx, g);  /* (reused blocks: after ctx's earlier work) */
      if (!rc) A.alloc_upto = g + 1;
    }
    if (!rc) {
      if (pthread_create(&A.th, NULL, stream_copier, &A) == 0) copier = 1;
      else rc = -1;
    }
  }
  for (int g = 0; g < ng && !rc; ++g) {
    if (copier) {  /* group g's copies issued by the copier: fence ctx's stream on them */
      pthread_mutex_lock(&A.mu);
      while (A.issued <= g) pthread_cond_wait(&A.cv, &A.mu);
      const int crc = A.rc;
      pthread_mutex_unlock(&A.mu);
      rc = crc ? crc : bg_copy_fence(ctx, g);
    }
    for (int f = 0; f < nf && !rc; ++f) {
      const uint64_t a = SP.ga[(size_t)g * nf + f], b = SP.gb[(size_t)g * nf + f];
      if (copier) {
        d[f] = A.d[(size_t)g * nf + f];
        A.d[(size_t)g * nf + f] = NULL;
      } else {
        rc = bg_file_image_to_device(ctx, &SP.fm[f], a, b - a, &d[f]);
      }
      in[f] = proto[f];
      in[f].data = d[f];
      in[f].nbytes = b - a;
      in[f].on_device = 1;
    }
    bg_set* set = NULL;
    if (!rc) cli_mark("  copies");
    if (!rc) rc = bg_load(ctx, nf, in, &set);
    if (!rc) cli_mark("  load");
    if (!rc) rc = op(oparg, ctx, set, &res[g]);
    uint64_t n = 0;
    const char* t = NULL;
    if (!rc) rc = bg_result_format(ctx, res[g], &n);
    if (!rc) rc = bg_result_text_device(res[g], &t, &n);
    if (!rc) rc = bg_writer_push(w, t, n);
    if (!rc) {
      ++pushed;
      sent += n;
    }
    /* the formatted text is all the group leaves behind (the caching allocator hands the
     * freed blocks to the next group's copies, ordered after this group's kernels) */
    bg_set_free(set);
    for (int f = 0; f < nf; ++f) {
      if (d[f]) {
        if (ordered) bg_device_release(ctx, d[f]);
        else bg_device_free(ctx, d[f]);
      }
      d[f] = NULL;
    }
    if (copier && !rc && g + ahead + 1 < ng) {  /* buffers for the group AHEAD + 1 on */
      const int q = (int)(g + ahead + 1);
      for (int f = 0; f < nf && !rc; ++f)
        rc = bg_device_alloc(ctx, SP.gb[(size_t)q * nf + f] - SP.ga[(size_t)q * nf + f] + 64, &A.d[(size_t)q * nf + f]);
      /* the blocks may be group g's, released just above: the copier's DMA into them waits
       * for everything queued on ctx's stream so far */
      if (!rc) rc = bg_copy_order(ctx, q);
      pthread_mutex_lock(&A.mu);
      if (!rc) A.alloc_upto = q + 1;
      pthread_cond_broadcast(&A.cv);
      pthread_mutex_unlock(&A.mu);
    }
    const uint64_t done = bg_writer_done(w);
    while (freed < done) bg_result_free(res[freed++]);
    if (!rc) {
      char m[32];
      snprintf(m, sizeof(m), "group%d", g);
      cli_mark(m);
    }
  }
  if (copier) {  /* stop the copier, wait for its last copies, free what it did not hand over */
    pthread_mutex_lock(&A.mu);
    A.stop = 1;
    pthread_cond_broadcast(&A.cv);
    pthread_mutex_unlock(&A.mu);
    pthread_join(A.th, NULL);
    for (int g = 0; g < A.issued && g < ng; ++g) (void)bg_copy_fence(ctx, g);
    (void)bg_sync(ctx);
  }
  if (A.d) {
    for (size_t k = 0; k < (size_t)ng * nf; ++k)
      if (A.d[k]) bg_device_release(ctx, A.d[k]);
    free(A.d);
    pthread_mutex_destroy(&A.mu);
    pthread_cond_destroy(&A.cv);
  }
  const int wrc = bg_writer_close(w);
  while (freed < (uint64_t)ng) bg_result_free(res[freed++]);
  free(res);
  free(in);
  free(d);
  stream_plan_free();
  if (rc || wrc) { /* the whole-file path starts over on an empty output */
    const char* s = getenv("BEDGPU_STATS");
    if (s && *s && strcmp(s, "0") != 0)
      fprintf(stderr, "bedgpu: chromosome-group pipeline stopped (%d/%d: %s); whole-file path\n", rc, wrc,
              bg_last_error(ctx));
    if (SP.pipe) {
      if (wrc) die_msg(CLI_PROG, "cannot write the output");  /* (the consumer went away) */
      /* the groups written so far are the whole-file output's first `sent` bytes (every
       * covered operation is chromosome-local): the whole-file path continues after them */
      if (pushed && bg_set_output_skip(ctx, sent) != 0) die_ctx(CLI_PROG, ctx, rc);
      if (pushed) CLI_SKIP_CTX = ctx;  /* fast_exit checks the rerun passed `sent` */
      return 1;
    }
    /* never write the whole-file output after leftover group output */
    if (ftruncate(1, off0) != 0 || lseek(1, off0, SEEK_SET) < 0)
      die_msg(CLI_PROG, "cannot truncate the output file to rerun the whole-file path");
    return 1;
  }
  return 0;
}

#endif
