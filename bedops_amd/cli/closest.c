/*
 * closest-features — drop-in front-end for
 *   closest-features [process-flags] <input-file> <query-file>
 * computing, for every <input-file> row, the nearest <query-file> rows on an MI355X
 * through libbedgpu (bg_closest).
 *
 * argv grammar follows applications/bed/closestfeats/src/Input.hpp:46-103: flags
 * --closest/--shortest (at most one output option), --dist, --no-ref, --no-overlaps,
 * --delim, --chrom, --ec/--header, --help, --version; then exactly two files. Both
 * inputs are read as BED3 + verbatim rest (ClosestFeature.cpp:217-221) and printed as
 * "%s\t%lu\t%lu%s"; errors as "May use closest-features --help for more help.\n\nError:
 * <msg>" (ClosestFeature.cpp:93-95).
 */
#include "cli_common.h"
#include "cli_stream.h"

static const char* PROG = "closest-features";

static void usage(FILE* f) {
  fprintf(f,
          "closest-features\n  version:  %s\n\n"
          "USAGE: closest-features [Process-Flags] <input-file> <query-file>\n"
          "   All input files must be sorted per sort-bed.\n"
          "   May use '-' for a file to indicate reading from standard input.\n\n"
          "   For every element in <input-file>, determine the two elements from <query-file> falling\n"
          "     nearest to its left and right edges. By default, echo the <input-file>\n"
          "     element, followed by those left and right elements found in <query-file>.\n\n"
          "  Process Flags:\n"
          "    --chrom <chromosome>   Jump to and process data for given <chromosome> only.\n"
          "    --closest              Choose the closest element for output only.  Ties go the left element.\n"
          "    --delim <delim>        Change output delimiter from '|' to <delim> between columns.\n"
          "    --dist                 Print the signed distances to the <input-file> element as additional\n"
          "                             columns of output.  An overlapping element has a distance of 0.\n"
          "    --ec / --header        Error check / accept headers.\n"
          "    --help                 Print this message and exit successfully.\n"
          "    --no-overlaps          Overlapping elements from <query-file> will not be reported.\n"
          "    --no-ref               Do not echo elements from <input-file>.\n"
          "    --version              Print program information.\n",
          BEDOPS_AMD_VERSION);
}

static void arg_error(const char* msg) { die_msg(PROG, msg); }

/* one chromosome shard: findDistances never looks across chromosomes (rows of earlier
 * chromosomes are dropped, ClosestFeature.cpp:289-291; a later chromosome ends the scan,
 * :292-298), so the same call on a member's set gives that member's lines */
static int run_closest(void* arg, bg_ctx* ctx, bg_set* set, bg_result** res) {
  return bg_closest(ctx, set, 0, 1, (const bg_closest_opts*)arg, res);
}

int main(int argc, char** argv) {
  CLI_PROG = PROG;
  if (argc <= 1) {
    usage(stderr);
    return EXIT_FAILURE;
  }
  bg_closest_opts o;
  memset(&o, 0, sizeof(o));
  strcpy(o.delim, "|");
  int ec = 0, check = 0, outopt = 0;
  const char* chrom = NULL;
  int a = 1;
  for (; a < argc; ++a) {
    const char* nx = argv[a];
    if (!strcmp(nx, "--help")) { usage(stdout); return EXIT_SUCCESS; }
    if (!strcmp(nx, "--version")) { printf("closest-features\n  version:  %s\n", BEDOPS_AMD_VERSION); return EXIT_SUCCESS; }
    if (!strcmp(nx, "--ec") || !strcmp(nx, "--header")) {
      ec = 1;
      check = 1; /* --header is --ec: errorCheck_ (bedops/src/Input.hpp:77-80, closestfeats/src/Input.hpp:64-65) */
    }
    else if (!strcmp(nx, "--no-overlaps")) o.no_overlaps = 1;
    else if (!strcmp(nx, "--delim")) {
      if (++a >= argc) arg_error("No value given for --delim.");
      if (strlen(argv[a]) >= sizeof(o.delim)) arg_error("--delim value too long for this build");
      strcpy(o.delim, argv[a]);
    } else if (!strcmp(nx, "--chrom")) {
      if (++a >= argc) arg_error("No value given for --chrome.");
      chrom = argv[a];
      if (!strcmp(chrom, "all")) chrom = NULL;
    } else if (!strcmp(nx, "--closest") || !strcmp(nx, "--shortest")) {
      if (outopt) arg_error("Multiple output options not allowed.");
      o.shortest = outopt = 1;
    } else if (!strcmp(nx, "--dist")) o.print_dist = 1;
    else if (!strcmp(nx, "--no-ref")) o.no_ref = 1;
    else {
      if (a + 2 != argc) {
        char b[512];
        snprintf(b, sizeof(b), "Unknown option: %s.", nx);
        arg_error(b);
      }
      break;
    }
  }
  if (a + 2 != argc) arg_error("Not enough input files given.");
  for (int i = a; i < argc; ++i) {
    char b[1024];
    if (!strncmp(argv[i], "--", 2)) {
      snprintf(b, sizeof(b), "Option given where file expected: %s.", argv[i]);
      arg_error(b);
    }
    if (strcmp(argv[i], "-") && access(argv[i], R_OK) != 0) {
      snprintf(b, sizeof(b), "Unable to find file: %s", argv[i]);
      arg_error(b);
    }
  }
  if (!strcmp(argv[a], "-") && !strcmp(argv[a + 1], "-")) arg_error("Cannot have both input files set to '-'");

  /* BEDGPU_DEVICES=0,1,...: chromosome shards on several GPUs (cli_shard.h); one GPU:
   * chromosome groups in a pipeline (cli_stream.h) */
  cli_detach(); /* the GPU work runs in a worker whose teardown the caller does not wait for */
  const int chrom_local = !check && !ec && !chrom && strcmp(argv[a], "-") && strcmp(argv[a + 1], "-");
  bg_input sin[2];
  memset(sin, 0, sizeof(sin));
  for (int k = 0; k < 2; ++k) sin[k].kind = BG_BED3_REST;
  if (chrom_local && getenv("BEDGPU_DEVICES") &&
      shard_run(PROG, 2, sin, (const char* const*)(argv + a), run_closest, &o) == 0)
    return EXIT_SUCCESS;

  cli_mark("start");
  const int streamed = chrom_local && stream_prepare(2, (const char* const*)(argv + a));
  if (!chrom && !check && !ec && !streamed) /* map the inputs while HIP initialises */
    for (int k = 0; k < 2; ++k) cli_prefetch(argv[a + k]);
  bg_ctx* ctx = NULL;
  int rc = bg_open(&ctx, env_device());
  if (rc) die_msg(PROG, "cannot open the GPU device (libbedgpu/HIP)");
  cli_mark("open");
  if (streamed && stream_run(ctx, sin, run_closest, &o) == 0) {
    cli_mark("write");
    maybe_stats(ctx);
    fast_exit();
    bg_close(ctx);
    return EXIT_SUCCESS;
  }
  text_buf_t t[2] = {{0}, {0}};
  bg_input in[2];
  for (int k = 0; k < 2; ++k) {
    if (read_input_chrom(ctx, argv[a + k], chrom, check || ec, &t[k], &in[k])) arg_error("Unable to read an input file");
    if (check) ec_check(PROG, ctx, argv[a + k], &t[k], 3, 1);
    if (ec) {
      apply_ec_header(&t[k]);
      in[k].data = t[k].data;
      in[k].nbytes = t[k].n;
    }
    in[k].kind = BG_BED3_REST;
  }
  bg_set* set = NULL;
  if ((rc = bg_load(ctx, 2, in, &set))) die_ctx(PROG, ctx, rc);
  cli_prefetch_release(ctx);
  cli_mark("load");
  free_text(&t[0]);
  free_text(&t[1]);
  if (chrom && (rc = bg_set_restrict_chrom(ctx, set, chrom))) die_ctx(PROG, ctx, rc);
  bg_result* res = NULL;
  if ((rc = bg_closest(ctx, set, 0, 1, &o, &res))) die_ctx(PROG, ctx, rc);
  if ((rc = bg_result_write(ctx, res, 1))) die_ctx(PROG, ctx, rc);
  maybe_stats(ctx);
  fast_exit();
  bg_result_free(res);
  bg_set_free(set);
  free_input(ctx, &t[0]);
  free_input(ctx, &t[1]);
  bg_close(ctx);
  return EXIT_SUCCESS;
}
