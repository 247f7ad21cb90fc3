/*
 * bedops — drop-in front-end for the BEDOPS set-operation CLI, running the sweep on
 * an MI355X through libbedgpu.
 *
 * argv grammar follows applications/bed/bedops/src/Input.hpp:57-298 (process flags,
 * one operation, long->short option map :422-433, minimum file counts :389-420, the
 * -e/-n overlap spec :171-206 and :344-382, '-' for stdin :271-287); output and exit
 * behaviour follow Bedops.cpp:81-127. Every operation runs on the GPU: the hot path
 * (--merge, --intersect, --difference, --element-of, --not-element-of; SURVEY.md
 * §8(a)) and --complement [-L], --chop [bp] [--stagger nt] [-x], --symmdiff,
 * --partition, --everything, with --range L:R|S padding (Input.hpp:86-127, 207-258).
 */
#include <ctype.h>

#include "cli_common.h"
#include "cli_stream.h"

static const char* PROG = "bedops";

static void usage(FILE* f) {
  fprintf(f,
          "bedops\n  version:  %s\n\n"
          "      USAGE: bedops [process-flags] <operation> <File(s)>*\n\n"
          "          Every input file must be sorted per the sort-bed utility.\n"
          "          May use '-' for a file to indicate reading from standard input.\n\n"
          "      Process Flags:\n"
          "          --chrom <chromosome> Process data for given <chromosome> only.\n"
          "          --ec                 Error check input files.\n"
          "          --header             Accept headers (browser/track/#/@) in input files.\n"
          "          --help               Print this message and exit successfully.\n"
          "          --version            Print program information.\n\n"
          "          --range L:R          Add 'L' bp to all start coordinates and 'R' bp to end\n"
          "                                 coordinates. Either value may be + or - to grow or\n"
          "                                 shrink regions.  With the -e/-n operations, the first\n"
          "                                 (reference) file is not padded, unlike all other files.\n"
          "          --range S            Pad or shrink input file(s) coordinates symmetrically by S.\n"
          "                                 This is shorthand for: --range -S:S.\n\n"
          "      Operations: (choose one of)\n"
          "          -c, --complement [-L] File1 [File]*\n"
          "          -d, --difference ReferenceFile File2 [File]*\n"
          "          -e, --element-of [bp | percentage] ReferenceFile File2 [File]*\n"
          "          -i, --intersect File1 File2 [File]*\n"
          "          -m, --merge File1 [File]*\n"
          "          -n, --not-element-of [bp | percentage] ReferenceFile File2 [File]*\n"
          "          -p, --partition File1 [File]*\n"
          "          -s, --symmdiff File1 File2 [File]*\n"
          "          -u, --everything File1 [File]*\n"
          "          -w, --chop [bp] [--stagger <nt>] [-x] File1 [File]*\n",
          BEDOPS_AMD_VERSION);
}

static void bad_input(const char* msg) {
  char buf[1024];
  snprintf(buf, sizeof(buf), "Bad Input\n%s", msg);
  die_msg(PROG, buf);
}

static const char* long_to_short(const char* s) {
  static const char* map[][2] = {{"--complement", "-c"}, {"--difference", "-d"}, {"--element-of", "-e"},
                                 {"--intersect", "-i"},  {"--merge", "-m"},      {"--not-element-of", "-n"},
                                 {"--partition", "-p"},  {"--symmdiff", "-s"},   {"--everything", "-u"},
                                 {"--chop", "-w"}};
  for (size_t k = 0; k < sizeof(map) / sizeof(map[0]); ++k)
    if (strcmp(s, map[k][0]) == 0) return map[k][1];
  return NULL;
}

static int all_chars_in(const char* s, const char* set) {
  for (; *s; ++s)
    if (!strchr(set, *s)) return 0;
  return 1;
}

/* -e/-n overlap spec (Input.hpp:344-382) */
static void set_subset(const char* str, double* thres, int* use_pct) {
  const char* pct = strchr(str, '%');
  if (pct) {
    if (pct[1] != '\0') bad_input("Bad placement of %");
    char val[128];
    size_t n = (size_t)(pct - str);
    if (n >= sizeof(val)) bad_input("Bad % value");
    memcpy(val, str, n);
    val[n] = 0;
    const char* v = val;
    if (!*v) bad_input("Bad % value");
    if (*v == '-') {
      ++v;
      if (!*v) bad_input("Bad % value");
    }
    if (!all_chars_in(v, ".1234567890")) bad_input("Bad: % value");
    double d = strtod(v, NULL) / 100.0;
    if (d > 1) bad_input("Expect percentage less than or equal to 100%");
    *thres = d;
    *use_pct = 1;
    if (d == 0) { *thres = 1; *use_pct = 0; }
  } else if (all_chars_in(str, "1234567890")) {
    *thres = atoi(str);
    *use_pct = 0;
  } else if (str[0] && all_chars_in(str + 1, "1234567890")) {
    *thres = atoi(str + 1);
    *use_pct = 0;
  } else if (all_chars_in(str, ".1234567890")) {
    bad_input("Fractional amounts require a '%' symbol (e.g.; 5.4% not 5.4 base-pair)");
  } else {
    char b[512];
    snprintf(b, sizeof(b), "Unknown arg: %s", str);
    bad_input(b);
  }
}

/* one side of --range (Input.hpp:89-111): digits and at most one '-', read like
 * std::stringstream >> int */
static int range_value(const char* v, const char* what) {
  char b[256];
  if (!*v) {
    snprintf(b, sizeof(b), "integer expected for the '%s' value of --range L:R.", what);
    bad_input(b);
  }
  if (!all_chars_in(v, "-0123456789")) {
    snprintf(b, sizeof(b), "integer expected for the '%s' value of --range L:R.", what);
    bad_input(b);
  }
  if (strchr(v, '-') != strrchr(v, '-')) {
    snprintf(b, sizeof(b), "multiple '-' signs detected for '%s' value of --range option", what);
    bad_input(b);
  }
  return atoi(v);
}

static void parse_range(const char* v, int* lpad, int* rpad) {
  const char* colon = strchr(v, ':');
  if (colon) {
    char left[128];
    size_t n = (size_t)(colon - v);
    if (n >= sizeof(left)) n = sizeof(left) - 1;
    memcpy(left, v, n);
    left[n] = 0;
    *lpad = range_value(left, "L");
    *rpad = range_value(colon + 1, "R");
  } else {
    if (!all_chars_in(v, "-0123456789")) bad_input("integer value expected for --range");
    if (strchr(v, '-') != strrchr(v, '-'))
      bad_input("multiple '-' signs detected in <val> for --range option");
    const int r = atoi(v);
    *lpad = -r;
    *rpad = r;
  }
}

/* how each input is parsed (Bedops.cpp:402-421): --everything keeps all columns of every
 * file, element-of those of the reference file; the other inputs of the set operations
 * are read only as merged sets (getNextFileMergedCoords, Bedops.cpp:792-814), so they are
 * parsed straight to their components unless --chrom/--range need the rows */
static int input_kind(int mode, int i, const char* chrom, int has_range) {
  if (mode == 'u' || ((mode == 'e' || mode == 'n') && i == 0)) return BG_BED3_REST;
  if (strchr("midencws", mode) && !chrom && !has_range && !env_no_set()) return BG_BED3_SET;
  return BG_BED3;
}

typedef struct {
  int mode, full_left;
  double thres;
  int use_pct;
  uint64_t chop_bp, chop_stagger;
  int chop_x;
} op_args_t;

/* selectWork (Bedops.cpp:1524-1577): the operation on every loaded file */
static int run_op(void* arg, bg_ctx* ctx, bg_set* set, bg_result** res) {
  const op_args_t* o = (const op_args_t*)arg;
  int nf = 0;
  while (bg_set_rows(set, nf, &(uint64_t){0}) == 0) ++nf;
  int idx[4096];
  if (nf > 4096) return BG_E_ARG;
  for (int i = 0; i < nf; ++i) idx[i] = i;
  switch (o->mode) {
    case 'm': return bg_merge(ctx, set, idx, nf, res);
    case 'i': return bg_intersect(ctx, set, idx, nf, res);
    case 'd': return bg_difference(ctx, set, 0, idx + 1, nf - 1, res);
    case 'e': return bg_element_of(ctx, set, 0, idx + 1, nf - 1, o->thres, o->use_pct, 0, res);
    case 'n': return bg_element_of(ctx, set, 0, idx + 1, nf - 1, o->thres, o->use_pct, 1, res);
    case 'c': return bg_complement(ctx, set, idx, nf, o->full_left, res);
    case 'w': return bg_chop(ctx, set, idx, nf, o->chop_bp, o->chop_stagger, o->chop_x, res);
    case 's': return bg_symmdiff(ctx, set, idx, nf, res);
    case 'p': return bg_partition(ctx, set, idx, nf, res);
    case 'u': return bg_everything(ctx, set, idx, nf, res);
  }
  return BG_E_ARG;
}

int main(int argc, char** argv) {
  CLI_PROG = PROG;
  if (argc <= 1) {
    usage(stderr);
    return EXIT_FAILURE;
  }
  int ec = 0, check = 0, has_op = 0, has_chrom = 0, has_range = 0, lpad = 0, rpad = 0;
  int full_left = 0, chop_x = 0;
  long chop_bp = 1, chop_stagger = 0;
  char mode = 0;
  const char* chrom = NULL;
  double thres = 1.0;
  int use_pct = 1, minfiles = 1;
  int a = 1;
  while (a < argc) {
    const char* nx = argv[a];
    if (!strcmp(nx, "--ec") || !strcmp(nx, "--header")) {
      ec = 1;
      check = 1; /* --header is --ec: errorCheck_ (bedops/src/Input.hpp:77-80, closestfeats/src/Input.hpp:64-65) */
    } else if (!strcmp(nx, "--chrom")) {
      if (has_chrom) bad_input("--chrom specified multiple times.");
      if (++a >= argc) bad_input("No value for --chrom given.");
      chrom = argv[a];
      has_chrom = strcmp(chrom, "all") != 0;
      if (!has_chrom) chrom = NULL;
    } else if (!strcmp(nx, "--range")) {
      if (has_range) bad_input("--range specified multiple times.");
      if (++a >= argc) bad_input("No value for --range given.");
      parse_range(argv[a], &lpad, &rpad);
      has_range = 1;
    } else if (!strcmp(nx, "--help") || !strncmp(nx, "--help-", 7)) {
      usage(stdout);
      return EXIT_SUCCESS;
    } else if (!strcmp(nx, "--version")) {
      printf("bedops\n  version:  %s\n", BEDOPS_AMD_VERSION);
      return EXIT_SUCCESS;
    } else if (nx[0] != '-') {
      break;
    } else if (strlen(nx) > 1) {
      if (strspn(nx, "-") == strlen(nx)) {
        char b[512];
        snprintf(b, sizeof(b), "Bad option: %s", nx);
        bad_input(b);
      }
      if (has_op) {
        char b[512];
        snprintf(b, sizeof(b), "More than one operation specified: %s", nx);
        bad_input(b);
      }
      has_op = 1;
      const char* op = nx;
      if (!strncmp(nx, "--", 2)) {
        op = long_to_short(nx);
        if (!op) {
          char b[512];
          snprintf(b, sizeof(b), "Unknown operation: %s", nx);
          bad_input(b);
        }
      }
      if (strlen(op) != 2) {
        char b[512];
        snprintf(b, sizeof(b), "Unknown operation: %s", op);
        bad_input(b);
      }
      mode = (char)tolower((unsigned char)op[1]);
      switch (mode) {
        case 'm': case 'c': case 'p': case 'u': case 'w': minfiles = 1; break;
        case 'i': case 'd': case 'e': case 'n': case 's': minfiles = 2; break;
        default: {
          char b[512];
          snprintf(b, sizeof(b), "Unknown operation: -%c", op[1]);
          bad_input(b);
        }
      }
      if (mode == 'e' || mode == 'n') { /* optional overlap spec (Input.hpp:171-206) */
        if (a + 1 < argc) {
          const char* q = argv[a + 1];
          size_t sz = strlen(q);
          if ((q[0] == '-' && sz > 1) || all_chars_in(q, "1234567890") || strchr(q, '%')) {
            if (!strstr(q, "--")) {
              if (access(q, F_OK) != 0) {
                set_subset(q, &thres, &use_pct);
                ++a;
              } else if (all_chars_in(q, "0123456789")) {
                fprintf(stderr,
                        "Warning: interpreting argument '%s' as a file input and not as an overlap spec,\n"
                        "         since the file exists.\n"
                        "You can use the legacy syntax '-%s' if you want to use it as an overlap criterion.\n",
                        q, q);
              }
            }
          }
        }
      } else if (mode == 'c') { /* -L (Input.hpp:207-220) */
        int cnt = 0;
        while (a + 1 < argc && !strcmp(argv[a + 1], "-L")) {
          full_left = 1;
          ++a;
          ++cnt;
        }
        if (cnt > 1) bad_input("-L specified multiple times with --complement");
      } else if (mode == 'w') { /* [bp] [--stagger nt] [-x] (Input.hpp:221-258) */
        int cnt = 0, value_set = 0, aux_set = 0, stagger_set = 0;
        while (a + 1 < argc) {
          const char* q = argv[a + 1];
          if (!strcmp(q, "--stagger")) {
            if (stagger_set) bad_input("chop's --stagger suboption specified multiple times.");
            if (a + 2 >= argc) bad_input("No #nt value found for --stagger suboption in --chop");
            const char* v = argv[a + 2];
            if (!all_chars_in(v, "1234567890"))
              bad_input("Invalid --stagger suboption #nt value in --chop.  Expect a +integer.");
            chop_stagger = atol(v);
            if (chop_stagger <= 0) bad_input("nt setting for chop's --stagger suboption must be > 0");
            stagger_set = aux_set = 1;
            a += 2;
          } else if (!strcmp(q, "-x")) {
            if (chop_x) bad_input("chop's -x suboption specified multiple times.");
            chop_x = aux_set = 1;
            ++a;
          } else if (all_chars_in(q, "1234567890")) {
            if (value_set) bad_input("Stray integer found (invalid argument for --chop?)");
            if (aux_set) bad_input("Stray integer value found: not valid for --chop");
            chop_bp = atol(q);
            if (chop_bp <= 0) bad_input("bp setting for chop must be > 0");
            value_set = 1;
            ++a;
          } else {
            break;
          }
          ++cnt;
        }
        if (cnt > 4) bad_input("Too many arguments for a --chop operation");
      }
    } else {
      break; /* "-" = stdin */
    }
    ++a;
  }
  if (a >= argc) bad_input("No input file given.");
  if (!has_op) bad_input("No operation argument given.");
  int nf = argc - a, stdin_seen = 0;
  for (int i = a; i < argc; ++i) {
    if (!strcmp(argv[i], "-")) {
      if (stdin_seen) bad_input("Too many '-'");
      stdin_seen = 1;
    } else {
      char b[1024];
      if (argv[i][0] == '-') {
        snprintf(b, sizeof(b), "Bad option: %s", argv[i]);
        bad_input(b);
      }
      if (access(argv[i], R_OK) != 0) {
        snprintf(b, sizeof(b), "Cannot find %s", argv[i]);
        bad_input(b);
      }
    }
  }
  if (nf < minfiles) bad_input("Not enough files");

  text_buf_t* tx = (text_buf_t*)calloc((size_t)nf, sizeof(text_buf_t));
  bg_input* in = (bg_input*)calloc((size_t)nf, sizeof(bg_input));
  /* every mode is chromosome-local except --range padding, which looks across the whole
   * file: BEDGPU_DEVICES=0,1,... runs chromosome shards on several GPUs (cli_shard.h), and a
   * single GPU runs chromosome groups in a pipeline (cli_stream.h) */
  cli_detach(); /* the GPU work runs in a worker whose teardown the caller does not wait for */
  const int chrom_local = !check && !ec && !chrom && !has_range;
  op_args_t oa = {mode, full_left, thres, use_pct, (uint64_t)chop_bp, (uint64_t)chop_stagger, chop_x};
  if (chrom_local)
    for (int i = 0; i < nf; ++i) in[i].kind = input_kind(mode, i, chrom, has_range);
  if (chrom_local && getenv("BEDGPU_DEVICES") &&
      shard_run(PROG, nf, in, (const char* const*)(argv + a), run_op, &oa) == 0)
    return EXIT_SUCCESS;
  cli_mark("start");
  const int streamed = chrom_local && stream_prepare(nf, (const char* const*)(argv + a));
  if (!chrom && !check && !ec && !streamed) /* map the inputs while HIP initialises */
    for (int i = 0; i < nf; ++i) cli_prefetch(argv[a + i]);
  bg_ctx* ctx = NULL;
  int rc = bg_open(&ctx, env_device());
  if (rc) die_msg(PROG, "cannot open the GPU device (libbedgpu/HIP)");
  cli_mark("open");
  if (streamed && stream_run(ctx, in, run_op, &oa) == 0) {
    cli_mark("write");
    maybe_stats(ctx);
    fast_exit();
    bg_close(ctx);
    free(in);
    free(tx);
    return EXIT_SUCCESS;
  }
  for (int i = 0; i < nf; ++i) {
    if (read_input_chrom(ctx, argv[a + i], chrom, check || ec, &tx[i], &in[i])) {
      char b[1024];
      snprintf(b, sizeof(b), "Unable to read %s", argv[a + i]);
      die_msg(PROG, b);
    }
    const int keep_rest = (mode == 'u' || ((mode == 'e' || mode == 'n') && i == 0));
    if (check) ec_check(PROG, ctx, argv[a + i], &tx[i], 3, keep_rest);
    if (ec) {
      apply_ec_header(&tx[i]);
      in[i].data = tx[i].data;
      in[i].nbytes = tx[i].n;
    }
    /* --everything keeps all columns of every file, element-of those of the reference
     * file (Bedops.cpp:402-421); the other inputs of the set operations are read only as
     * merged sets (getNextFileMergedCoords, Bedops.cpp:792-814), so they are parsed
     * straight to their components unless --chrom/--range need the rows */
    in[i].kind = input_kind(mode, i, chrom, has_range);
  }
  cli_mark("read");
  bg_set* set = NULL;
  if ((rc = bg_load(ctx, nf, in, &set))) die_ctx(PROG, ctx, rc);
  cli_prefetch_release(ctx);
  cli_mark("load");
  for (int i = 0; i < nf; ++i) free_text(&tx[i]);
  if (chrom && (rc = bg_set_restrict_chrom(ctx, set, chrom))) die_ctx(PROG, ctx, rc);
  /* --range pads every file but the element-of reference (Bedops.cpp:230-236) */
  for (int i = 0; has_range && i < nf; ++i)
    if (!((mode == 'e' || mode == 'n') && i == 0) && (rc = bg_set_pad(ctx, set, i, lpad, rpad)))
      die_ctx(PROG, ctx, rc);
  bg_result* res = NULL;
  if ((rc = run_op(&oa, ctx, set, &res))) die_ctx(PROG, ctx, rc);
  cli_mark("operation");
  if ((rc = bg_result_write(ctx, res, 1))) die_ctx(PROG, ctx, rc);
  cli_mark("write");
  maybe_stats(ctx);
  fast_exit();
  bg_result_free(res);
  bg_set_free(set);
  for (int i = 0; i < nf; ++i) free_input(ctx, &tx[i]);
  bg_close(ctx);
  free(in);
  free(tx);
  return EXIT_SUCCESS;
}
