/*
 * cli_common.h — shared host-side plumbing of the bedops_amd front-ends (C).
 *
 * Input files are read whole into pinned host memory and handed to libbedgpu, which
 * parses them on the GPU. '-' reads stdin (at most one per command line, as in
 * applications/bed/bedops/src/Input.hpp:271-287). Error text and exit codes follow
 * the reference front-ends: "May use <prog> --help for more help.\n\nError: <msg>"
 * on stderr and EXIT_FAILURE (applications/bed/bedops/src/Bedops.cpp:117-126).
 */
#ifndef BEDOPS_AMD_CLI_COMMON_H
#define BEDOPS_AMD_CLI_COMMON_H

#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../include/bedgpu.h"

#define BEDOPS_AMD_VERSION "2.4.26 (bedops_amd MI355X engine)"

typedef struct {
  char* data;     /* pinned host buffer */
  uint64_t n;     /* bytes of BED text */
  int pinned;
  void* ddata;    /* the text on the device instead (read_input), freed by free_input */
} text_buf_t;

/* the running front-end (messages of shared helpers), and whether Starch archives are
 * decoded (sort-bed reads every input as BED text, as the reference's sort-bed does) */
static const char* CLI_PROG = "bedops";
static int CLI_NO_STARCH = 0;

static void die_msg(const char* prog, const char* msg) {
  fprintf(stderr, "May use %s --help for more help.\n\nError: %s\n", prog, msg);
  exit(EXIT_FAILURE);
}

static void die_ctx(const char* prog, bg_ctx* ctx, int rc) {
  char msg[1024];
  snprintf(msg, sizeof(msg), "%s", ctx ? bg_last_error(ctx) : "");
  if (!msg[0]) snprintf(msg, sizeof(msg), "GPU engine failure (code %d)", rc);
  die_msg(prog, msg);
}

/* read a whole file (or stdin for "-") into a pinned buffer */
static int read_text(const char* path, text_buf_t* out) {
  int fd = strcmp(path, "-") == 0 ? 0 : open(path, O_RDONLY);
  if (fd < 0) return -1;
  struct stat st;
  uint64_t cap = 1 << 20;
  if (fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && st.st_size > 0) cap = (uint64_t)st.st_size + 1;
  char* buf = (char*)bg_host_alloc(cap + 16);
  int pinned = 1;
  if (!buf) { buf = (char*)malloc(cap + 16); pinned = 0; }
  if (!buf) return -1;
  uint64_t n = 0;
  for (;;) {
    if (n == cap) { /* grow (pipes / stdin) */
      uint64_t nc = cap * 2;
      char* nb = (char*)malloc(nc + 16);
      if (!nb) return -1;
      memcpy(nb, buf, n);
      if (pinned) bg_host_free(buf); else free(buf);
      buf = nb;
      pinned = 0;
      cap = nc;
    }
    ssize_t r = read(fd, buf + n, (size_t)(cap - n));
    if (r < 0) {
      if (errno == EINTR) continue;
      return -1;
    }
    if (r == 0) break;
    n += (uint64_t)r;
  }
  if (fd != 0) close(fd);
  out->data = buf;
  out->n = n;
  out->pinned = pinned;
  /* a Starch archive from a file becomes the BED text its streams hold (the reference
   * reads Starch only from files, not stdin: AllocateIterator_BED_starch.hpp:62) */
  if (fd != 0 && !CLI_NO_STARCH && bg_starch_is(buf, n)) {
    char* txt = NULL;
    uint64_t tn = 0;
    char err[512];
    int rc = bg_starch_decode(buf, n, NULL, &txt, &tn, err, sizeof(err));
    if (pinned) bg_host_free(buf); else free(buf);
    out->data = NULL;
    if (rc) {
      fprintf(stderr, "May use %s --help for more help.\n\nError: %s: %s\n", CLI_PROG, path, err);
      exit(EXIT_FAILURE);
    }
    out->data = txt;
    out->n = tn;
    out->pinned = 0;
  }
  return 0;
}

/* the first bytes of a regular file mark a Starch archive (v2 magic or v1 JSON head) */
static inline int file_is_starch(const char* path) {
  unsigned char b[512];
  int fd = open(path, O_RDONLY);
  if (fd < 0) return 0;
  const ssize_t r = read(fd, b, sizeof(b));
  close(fd);
  if (r >= 4 && b[0] == 0xca && b[1] == 0x5c && b[2] == 0xad && b[3] == 0xe5) return 1;
  return r > 0 && bg_starch_is(b, (uint64_t)r);
}

/* Input files that go straight to device memory are mapped with their pages faulted in
 * (bg_file_image_open, no GPU call) by one thread each, started before bg_open so this
 * overlaps HIP's initialisation; read_input then copies the image to HBM through the
 * context's pinned ring, and cli_prefetch_release unmaps the images once the loads have
 * copied them. */
#include <pthread.h>
#define CLI_MAX_PF 16
typedef struct {
  const char* path;
  bg_file_image m;
  int ok, started;
  pthread_t th;
} cli_pf_t;
static cli_pf_t CLI_PF[CLI_MAX_PF];
static int CLI_NPF;
static inline void* cli_pf_run(void* a) {
  cli_pf_t* p = (cli_pf_t*)a;
  p->ok = bg_file_image_open(p->path, &p->m) == 0;
  if (p->ok && p->m.n >= 4 && !CLI_NO_STARCH) { /* Starch archives: decoded on the host (read_text) */
    const unsigned char* b = (const unsigned char*)p->m.data;
    if ((b[0] == 0xca && b[1] == 0x5c && b[2] == 0xad && b[3] == 0xe5) ||
        bg_starch_is(p->m.data, p->m.n < 512 ? p->m.n : 512)) {
      bg_file_image_close(&p->m);
      p->ok = 0;
    }
  }
  return NULL;
}
static inline void cli_prefetch(const char* path) {
  struct stat st;
  const char* e = getenv("BEDGPU_PF"); /* BEDGPU_PF=0: no mapping before bg_open */
  if (e && !strcmp(e, "0")) return;
  if (CLI_NPF >= CLI_MAX_PF || !strcmp(path, "-") || stat(path, &st) != 0 || !S_ISREG(st.st_mode)) return;
  cli_pf_t* p = &CLI_PF[CLI_NPF];
  memset(p, 0, sizeof(*p));
  p->path = path;
  if (pthread_create(&p->th, NULL, cli_pf_run, p) == 0) {
    p->started = 1;
    ++CLI_NPF;
  }
}
static inline cli_pf_t* cli_pf_take(const char* path) {
  for (int k = 0; k < CLI_NPF; ++k) {
    cli_pf_t* p = &CLI_PF[k];
    if (p->path != path && strcmp(p->path, path) != 0) continue;
    if (p->started) {
      pthread_join(p->th, NULL);
      p->started = 0;
    }
    if (p->ok) return p;
  }
  return NULL;
}
static inline void cli_prefetch_release(bg_ctx* ctx) {
  if (ctx) bg_sync(ctx); /* every copy from the mappings has completed */
  for (int k = 0; k < CLI_NPF; ++k) {
    cli_pf_t* p = &CLI_PF[k];
    if (p->started) {
      pthread_join(p->th, NULL);
      p->started = 0;
    }
    if (p->ok) bg_file_image_close(&p->m);
    p->ok = 0;
  }
  CLI_NPF = 0;
}

/* one input into `in`: regular files whose bytes no host code needs (no --ec/--header)
 * go straight to device memory (their mapped pages copied to HBM through the pinned ring:
 * cli_prefetch / bg_read_file_device); stdin, pipes and checked inputs are read into host
 * memory.
 * Returns 0 or -1 (unreadable). */
static inline int read_input(bg_ctx* ctx, const char* path, int host_needed, text_buf_t* t, bg_input* in) {
  struct stat st;
  memset(t, 0, sizeof(*t));
  cli_pf_t* pf = host_needed ? NULL : cli_pf_take(path);
  if (pf) {
    void* d = NULL;
    (void)bg_file_image_register(&pf->m);
    if (bg_file_image_to_device(ctx, &pf->m, 0, pf->m.n, &d) == 0) {
      t->ddata = d;
      t->n = pf->m.n;
      in->data = d;
      in->nbytes = pf->m.n;
      in->on_device = 1;
      return 0;
    }
  }
  if (!host_needed && strcmp(path, "-") != 0 && stat(path, &st) == 0 && S_ISREG(st.st_mode) &&
      (CLI_NO_STARCH || !file_is_starch(path))) {
    void* d = NULL;
    uint64_t n = 0;
    const int rc = bg_read_file_device(ctx, path, &d, &n);
    if (rc == 0) {
      t->ddata = d;
      t->n = n;
      in->data = d;
      in->nbytes = n;
      in->on_device = 1;
      return 0;
    }
    const char* s = getenv("BEDGPU_STATS");
    if (s && *s && strcmp(s, "0") != 0)
      fprintf(stderr, "bedgpu: device read of %s failed (%d: %s); reading into host memory\n", path, rc,
              bg_last_error(ctx));
  }
  if (read_text(path, t)) return -1;
  in->data = t->data;
  in->nbytes = t->n;
  in->on_device = 0;
  return 0;
}

/* --chrom on a regular, sorted BED file: only that chromosome's lines are read. The
 * reference seeks to them with find_bed_range and stops at the first row of another
 * chromosome (AllocateIterator_BED_starch.hpp:113-160, operator++ :176-181), so rows of
 * other chromosomes are never parsed (nor checked). Bisection over the mapped file on the
 * first token of each line (strcmp order); -1 when a probed line has no usable token
 * (headers, blank lines: the whole file is read instead). */
static int ck_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }
static uint64_t ck_line_start(const char* t, uint64_t p) {
  while (p > 0 && t[p - 1] != '\n') --p;
  return p;
}
static uint64_t ck_next_line(const char* t, uint64_t n, uint64_t p) {
  const char* q = (const char*)memchr(t + p, '\n', (size_t)(n - p));
  return q ? (uint64_t)(q - t) + 1 : n;
}
/* strcmp(token of the line at p, chrom), or 2 when the line has no token */
static int ck_cmp(const char* t, uint64_t n, uint64_t p, const char* chrom) {
  while (p < n && ck_ws(t[p])) ++p;
  uint64_t q = p;
  while (q < n && t[q] != '\n' && !ck_ws(t[q])) ++q;
  if (q == p) return 2;
  const size_t k = strlen(chrom), m = (size_t)(q - p);
  const int v = memcmp(t + p, chrom, m < k ? m : k);
  if (v) return v < 0 ? -1 : 1;
  return m == k ? 0 : (m < k ? -1 : 1);
}
/* first line start whose token compares > `le ? 0 : -1` with chrom */
static int ck_bound(const char* t, uint64_t n, const char* chrom, int le, uint64_t* out) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t ls = ck_line_start(t, lo + (hi - lo) / 2);
    const int c = ck_cmp(t, n, ls, chrom);
    if (c == 2) return -1;
    if (le ? c <= 0 : c < 0) lo = ck_next_line(t, n, ls);
    else hi = ls;
  }
  *out = lo;
  return 0;
}
static int chrom_byte_range(const char* path, const char* chrom, uint64_t* a, uint64_t* b) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) return -1;
  struct stat st;
  if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode) || st.st_size <= 0) { close(fd); return -1; }
  const uint64_t n = (uint64_t)st.st_size;
  const char* t = (const char*)mmap(NULL, (size_t)n, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (t == MAP_FAILED) return -1;
  int rc = ck_bound(t, n, chrom, 0, a);
  if (!rc) rc = ck_bound(t, n, chrom, 1, b);
  munmap((void*)t, (size_t)n);
  return rc;
}
/* read_input for --chrom: the chromosome's byte range of a regular BED file into host
 * memory (the loader copies it to the device); other inputs as read_input */
static inline int read_input_chrom(bg_ctx* ctx, const char* path, const char* chrom, int host_needed,
                                   text_buf_t* t, bg_input* in) {
  uint64_t a = 0, b = 0;
  struct stat st;
  if (chrom && !host_needed && strcmp(path, "-") != 0 && stat(path, &st) == 0 && S_ISREG(st.st_mode) &&
      !file_is_starch(path) && chrom_byte_range(path, chrom, &a, &b) == 0 && b >= a) {
    memset(t, 0, sizeof(*t));
    char* buf = (char*)malloc((size_t)(b - a) + 16);
    int fd = open(path, O_RDONLY);
    if (!buf || fd < 0) { free(buf); if (fd >= 0) close(fd); return -1; }
    uint64_t got = 0;
    while (got < b - a) {
      const ssize_t r = pread(fd, buf + got, (size_t)(b - a - got), (off_t)(a + got));
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) break;
      got += (uint64_t)r;
    }
    close(fd);
    if (got != b - a) { free(buf); return -1; }
    t->data = buf;
    t->n = got;
    t->pinned = 0;
    in->data = buf;
    in->nbytes = got;
    in->on_device = 0;
    return 0;
  }
  return read_input(ctx, path, host_needed, t, in);
}

static void free_text(text_buf_t* t) {
  if (!t->data) return;
  if (t->pinned) bg_host_free(t->data); else free(t->data);
  t->data = NULL;
}
static inline void free_input(bg_ctx* ctx, text_buf_t* t) {
  free_text(t);
  if (t->ddata) bg_device_free(ctx, t->ddata);
  t->ddata = NULL;
}

/* --header / --ec: drop leading UCSC/VCF/SAM header lines ("browser", "track", '#',
 * '@'; BedCheckIterator.hpp:315-350) and keep an unterminated final line (the error
 * checking reader keeps it, the plain reader drops it). */
static inline void apply_ec_header(text_buf_t* t) {
  uint64_t p = 0;
  for (;;) {
    uint64_t e = p;
    while (e < t->n && t->data[e] != '\n') ++e;
    if (e >= t->n) break;
    const char* l = t->data + p;
    uint64_t len = e - p;
    int hdr = (len > 0 && (l[0] == '#' || l[0] == '@')) ||
              (len >= 5 && strncasecmp(l, "track", 5) == 0 && (len == 5 || l[5] == ' ' || l[5] == '\t')) ||
              (len >= 7 && strncasecmp(l, "browser", 7) == 0 && (len == 7 || l[7] == ' ' || l[7] == '\t'));
    if (!hdr) break;
    p = e + 1;
  }
  if (p) {
    memmove(t->data, t->data + p, t->n - p);
    t->n -= p;
  }
  if (t->n > 0 && t->data[t->n - 1] != '\n') t->data[t->n++] = '\n'; /* capacity has +16 */
}

/* --ec (Bed::bed_check_iterator, BedCheckIterator.hpp): every line of `t` checked on the
 * GPU before anything else reads it; the first failing line ends the program with the
 * reference's "in <file>\n<message>\nSee row: <n>" */
static inline void ec_check(const char* prog, bg_ctx* ctx, const char* fn, const text_buf_t* t, int nfields,
                     int has_rest) {
  bg_input in;
  in.data = t->data;
  in.nbytes = t->n;
  in.on_device = 0;
  in.kind = BG_BED3;
  bg_check_result cr;
  int rc = bg_check(ctx, &in, nfields, has_rest, &cr);
  if (rc) die_ctx(prog, ctx, rc);
  if (!cr.row) return;
  char m[2048], b[4096];
  bg_check_message(t->data + cr.line_off, cr.line_len, cr.code, nfields, has_rest & 1, m, sizeof(m));
  snprintf(b, sizeof(b), "in %s\n%s\nSee row: %llu", fn, m, (unsigned long long)cr.row);
  die_msg(prog, b);
}

static int env_device(void) {
  const char* d = getenv("BEDGPU_DEVICE");
  return d ? atoi(d) : 0;
}

/* BEDGPU_SET=0: load every plain input with its row columns (BG_BED3) instead of
 * straight to its merged set (BG_BED3_SET); same output, for A/B checks */
static inline int env_no_set(void) {
  const char* s = getenv("BEDGPU_SET");
  return s && strcmp(s, "0") == 0;
}

#include <time.h>
/* BEDGPU_STATS=1: host wall-clock marks on stderr (never stdout) */
static inline double cli_now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
static inline void cli_mark(const char* what) {
  static double t0 = 0, last = 0;
  const char* s = getenv("BEDGPU_STATS");
  if (!s || !*s || strcmp(s, "0") == 0) return;
  const double t = cli_now();
  if (t0 == 0) t0 = last = t;
  fprintf(stderr, "bedgpu host  %-12s %10.3f ms (+%.3f)\n", what, 1e3 * (t - t0), 1e3 * (t - last));
  if (!strcmp(what, "start") || !strcmp(what, "exit")) /* CLOCK_MONOTONIC, for the caller's clock */
    fprintf(stderr, "bedgpu mono  %-12s %.6f\n", what, t);
  last = t;
}

static void maybe_stats(bg_ctx* ctx) {
  const char* s = getenv("BEDGPU_STATS");
  if (!s || !*s || strcmp(s, "0") == 0) return;
  char buf[4096];
  if (bg_stats(ctx, buf, sizeof(buf)) == 0) fputs(buf, stderr);
}

/* Detached teardown. Even a process that only initialised HIP spends 60-100 ms in the
 * kernel driver after exit(2) (KFD queues and the GPU VM torn down; measured on the box,
 * tools/gpu_exit_r03b.sh, profiles/r03_exit_teardown.txt) before its parent sees it end. So
 * the front-end forks before touching the GPU: the worker (child) does everything and, once
 * its output is complete (written to fd 1, i.e. in the page cache or the pipe), closes its
 * stdout/stderr and reports its status over a pipe; the front process, which never touched
 * the GPU, exits with that status at once while the worker's teardown finishes detached.
 * A worker that fails (die_msg, a crash) is waited for and its status mirrored.
 * BEDGPU_DETACH=0, or BEDGPU_FULL_EXIT=1 (profilers), keep everything in one process. */
#include <signal.h>
#include <sys/prctl.h>
#include <sys/wait.h>
static int CLI_DETACH_FD = -1;
/* a pipe fallback's ctx (cli_stream.h): its whole-file output must have passed the bytes the
 * chromosome groups already sent (bg_set_output_skip), checked before the exit */
static bg_ctx* CLI_SKIP_CTX = NULL;
static pid_t CLI_WORKER = 0;
/* the front process forwards termination signals to the worker (whose exit it mirrors) */
static void cli_forward_signal(int sig) {
  if (CLI_WORKER > 0) kill(CLI_WORKER, sig);
}
static inline int cli_env_on(const char* name) {
  const char* s = getenv(name);
  return s && *s && strcmp(s, "0") != 0;
}
/* stdout a pipe: a 1 MiB pipe buffer (F_SETPIPE_SZ; 64 KiB by default) lets each write(2)
 * of the output hand over 16x more before it waits for the consumer */
#ifndef F_SETPIPE_SZ
#define F_SETPIPE_SZ 1031
#endif
static inline void cli_pipe_size(void) {
  struct stat st;
  if (fstat(1, &st) != 0 || !S_ISFIFO(st.st_mode)) return;
  if (fcntl(1, F_SETPIPE_SZ, 1 << 20) < 0) (void)fcntl(1, F_SETPIPE_SZ, 256 << 10);
}
static inline void cli_detach(void) {
  cli_pipe_size();
  const char* d = getenv("BEDGPU_DETACH");
  if ((d && !strcmp(d, "0")) || cli_env_on("BEDGPU_FULL_EXIT")) return;
  int p[2];
  if (pipe(p) != 0) return;
  fflush(stdout);
  fflush(stderr);
  const pid_t front = getpid();
  const pid_t pid = fork();
  if (pid < 0) {
    close(p[0]);
    close(p[1]);
    return;
  }
  if (pid == 0) { /* the worker */
    close(p[0]);
    CLI_DETACH_FD = p[1];
    /* a front process killed outright (SIGKILL) takes the worker with it; cleared again in
     * fast_exit once the output is complete */
    prctl(PR_SET_PDEATHSIG, SIGKILL);
    /* the front died before prctl: reparented (to init or to a subreaper, whatever its pid) */
    if (getppid() != front) _exit(EXIT_FAILURE);
    return;
  }
  close(p[1]);
  CLI_WORKER = pid;
  {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = cli_forward_signal;
    sigemptyset(&sa.sa_mask);
    const int sigs[4] = {SIGTERM, SIGINT, SIGHUP, SIGQUIT};
    for (int k = 0; k < 4; ++k) sigaction(sigs[k], &sa, NULL);
  }
  close(0); /* stdin belongs to the worker ('-' inputs) */
  unsigned char st = 0;
  ssize_t r;
  do r = read(p[0], &st, 1); while (r < 0 && errno == EINTR);
  if (r == 1) _exit(st);
  int ws = 0;
  while (waitpid(pid, &ws, 0) < 0)
    if (errno != EINTR) _exit(EXIT_FAILURE);
  if (WIFEXITED(ws)) _exit(WEXITSTATUS(ws));
  if (WIFSIGNALED(ws)) {
    signal(WTERMSIG(ws), SIG_DFL);
    raise(WTERMSIG(ws));
  }
  _exit(EXIT_FAILURE);
}

/* after the output is written: leave without tearing down the device state (freeing
 * every HBM block, the pinned ring and the HIP runtime costs ~0.3 s; the kernel driver
 * reclaims a process's GPU resources at exit). Output went through write(2) only. */
static inline void fast_exit(void) {
  if (CLI_SKIP_CTX) {
    uint64_t left = 0;
    if (bg_output_skip_left(CLI_SKIP_CTX, &left) != 0 || left != 0)
      die_msg("bedgpu", "the whole-file output is shorter than the part already sent down the pipe");
    CLI_SKIP_CTX = NULL;
  }
  fflush(stdout);
  fflush(stderr);
  cli_mark("exit");
  /* BEDGPU_FULL_EXIT=1: tear down normally (profilers write their traces at exit) */
  if (cli_env_on("BEDGPU_FULL_EXIT")) return;
  if (CLI_DETACH_FD >= 0) { /* output complete: release the front process (cli_detach) */
    prctl(PR_SET_PDEATHSIG, 0);  /* the teardown outlives the front process */
    close(1);
    close(2);
    const unsigned char ok = EXIT_SUCCESS;
    ssize_t r;
    do r = write(CLI_DETACH_FD, &ok, 1); while (r < 0 && errno == EINTR);
  }
  _exit(EXIT_SUCCESS);
}

#endif
