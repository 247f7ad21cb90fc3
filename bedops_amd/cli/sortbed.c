/*
 * sort-bed — drop-in front-end of applications/bed/sort-bed (Sort.cpp:41-234) on the GPU.
 *
 * Same argument grammar and messages: --help / --version, --check-sort (each input read
 * through the --ec grammar: CheckSort.cpp:17-40, here bg_check), --max-mem <val> and
 * --tmpdir <path> (accepted and checked; the sort happens in HBM, so no external merge is
 * needed), at most one '-'. The sort itself is bg_sortbed (bedops_amd/csrc/bg_sortbed.hip):
 * every line checked with sort-bed's grammar, sorted by chromosome (strcmp), start, end and
 * the rest of the line, printed "%s\t%ld\t%ld[\t%s]\n" (SortDetails.cpp:1120-1140).
 */
#include <ctype.h>

#include "cli_common.h"

#define PROG "sort-bed"

static const char* NAME = "sort-bed";
static const char* CITATION =
    "\n  Shane Neph, M. Scott Kuehn, Alex P. Reynolds, et al.\n  BEDOPS: high-performance genomic "
    "feature operations\n  Bioinformatics (2012) 28 (14): 1919-1920\n  "
    "https://doi.org/10.1093/bioinformatics/bts277";
static const char* AUTHORS = "Scott Kuehn";
static const char* USAGE =
    "\nUSAGE: sort-bed [--help] [--version] [--check-sort] [--max-mem <val>] [--tmpdir <path>] "
    "<file1.bed> <file2.bed> <...>\n        Sort BED file(s).\n        May use '-' to indicate "
    "stdin.\n        Results are sent to stdout.\n\n        <val> for --max-mem may be 8G, "
    "8000M, or 8000000000 to specify 8 GB of memory.\n        --tmpdir is useful only with "
    "--max-mem.\n";

static void banner(FILE* f, int with_usage) {
  fprintf(f, "%s\n  citation: %s\n  version:  %s\n  authors:  %s\n", NAME, CITATION,
          BEDOPS_AMD_VERSION, AUTHORS);
  if (with_usage) fprintf(f, "%s\n", USAGE);
}

/* the reference's message for a bad line (SortDetails.cpp:634-780) */
static void line_error(const bg_sortbed_error* e, const char* fn) {
  const unsigned long long ln = (unsigned long long)e->line;
  switch (e->code) {
    case BG_SB_ROW_LONG:
      fprintf(stderr, "BED row length exceeds capacity at line %llu in %s.\n", ln, fn);
      fprintf(stderr, "Check that you have unix newlines (cat -A) or increase TOKENS_MAX_LENGTH in BEDOPS.Constants.hpp and recompile BEDOPS.\n");
      break;
    case BG_SB_LEADING_WS:
      fprintf(stderr, "Row begins with a tab or space at line %llu in %s.\n", ln, fn);
      break;
    case BG_SB_NO_TAB:
      fprintf(stderr, "No tabs/spaces found at line %llu in %s.\n", ln, fn);
      break;
    case BG_SB_CHROM_LONG:
      fprintf(stderr, "Chromosome name too long at line %llu in %s.\n", ln, fn);
      fprintf(stderr, "Check that you have unix newlines (cat -A) or increase TOKEN_CHR_MAX_LENGTH in BEDOPS.Constants.hpp and recompile BEDOPS.\n");
      break;
    case BG_SB_NO_START_SEP:
      fprintf(stderr, "No tabs/spaces found after the start coordinate (or no start coordinate at all) at line %llu in %s.\n", ln, fn);
      break;
    case BG_SB_START_LONG:
      fprintf(stderr, "Start coordinate is too large.  Max decimal digits allowed is %ld in BEDOPS.Constants.hpp.  See line %llu in %s.\n", 12L, ln, fn);
      break;
    case BG_SB_START_EMPTY:
      fprintf(stderr, "Consecutive tabs and/or spaces between chromosome and start coordinate.  See line %llu in %s.\n", ln, fn);
      break;
    case BG_SB_START_NONNUM:
      fprintf(stderr, "Non-numeric start coordinate.  See line %llu in %s.\n(remember that chromosome names should not contain spaces.)\n", ln, fn);
      break;
    case BG_SB_NO_EOL:
      fprintf(stderr, "No end of line found at %llu in %s.\nMay need to increase BED_LINE_LEN and recompile.\nFirst check that you have unix newlines (cat -A).", ln, fn);
      break;
    case BG_SB_END_LONG:
      fprintf(stderr, "End coordinate is too large.  Max decimal digits allowed is %ld in BEDOPS.Constants.hpp.  See line %llu in %s.\n", 12L, ln, fn);
      break;
    case BG_SB_END_EMPTY:
      fprintf(stderr, "Extra tab and/or space found in between start and end coordinates.  See line %llu in %s.\n", ln, fn);
      break;
    case BG_SB_END_NONNUM:
      fprintf(stderr, "Non-numeric end coordinate.  See line %llu in %s.\n", ln, fn);
      break;
    case BG_SB_END_LE_START:
      fprintf(stderr, "Error on line %llu in %s. Genomic end coordinate is less than (or equal to) start coordinate.\n", ln, fn);
      break;
    case BG_SB_ID_LONG:
      fprintf(stderr, "ID field too long at line %llu in %s.\n", ln, fn);
      fprintf(stderr, "Check that you have unix newlines (cat -A) or increase TOKEN_ID_MAX_LENGTH in BEDOPS.Constants.hpp and recompile BEDOPS.\n");
      fprintf(stderr, "You may instead choose to put a dummy id column (like 'id') in as the 4th field to fix this.\n");
      break;
  }
}

int main(int argc, char** argv) {
  CLI_PROG = PROG;
  CLI_NO_STARCH = 1; /* the reference's sort-bed reads Starch archives as BED text */
  if (argc < 2) {
    banner(stderr, 1);
    return EXIT_FAILURE;
  }
  const char* files[4096];
  int nfiles = 0, just_check = 0, stdin_cnt = 0, mem_set = 0, tmp_set = 0;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--help")) {
      banner(stdout, 1);
      return EXIT_SUCCESS;
    } else if (!strcmp(argv[i], "--version")) {
      banner(stdout, 0);
      return EXIT_SUCCESS;
    } else if (!strcmp(argv[i], "--max-mem")) { /* Sort.cpp:82-143 */
      if (mem_set) { fprintf(stderr, "Specify --max-mem at most one time!\n"); return EXIT_FAILURE; }
      if (i + 1 >= argc) { fprintf(stderr, "No value given for --max-mem.\n"); return EXIT_FAILURE; }
      const char* v = argv[++i];
      size_t k = 0;
      while (v[k] && isdigit((unsigned char)v[k])) ++k;
      if (k == 0) {
        fprintf(stderr, "Bad number for --max-mem.  Expect value to be like 10G (for 10 gigabytes) or 1000M (for 1000 megabytes) or just 1000000000 (for 1 gigabyte).\n");
        return EXIT_FAILURE;
      }
      if (v[k] && !(v[k + 1] == 0 && strchr("GgMmKk", v[k]))) {
        fprintf(stderr, "Unrecognized units for --max-mem.  Expect value to be like 10G (for 10 gigabytes) or 1000M (for 1000 megabytes) or just 1000000000 (for 1 gigabyte).\n");
        return EXIT_FAILURE;
      }
      mem_set = 1; /* the sort runs in HBM: no external merge is needed */
    } else if (!strcmp(argv[i], "--tmpdir")) {
      if (tmp_set) { fprintf(stderr, "Specify --tmpdir at most one time!\n"); return EXIT_FAILURE; }
      if (i + 1 >= argc) { fprintf(stderr, "No value given for --tmpdir.\n"); return EXIT_FAILURE; }
      ++i;
      tmp_set = 1;
    } else if (!strcmp(argv[i], "--check-sort")) {
      just_check = 1;
    } else {
      if (!strcmp(argv[i], "-")) ++stdin_cnt;
      if (nfiles < 4096) files[nfiles++] = argv[i];
    }
  }
  if (stdin_cnt > 1) {
    fprintf(stderr, "Cannot specify '-' more than once\n");
    return EXIT_FAILURE;
  }
  if (nfiles < 1) {
    banner(stderr, 1);
    fprintf(stderr, "No file given.\n");
    return EXIT_FAILURE;
  }
  for (int i = 0; i < nfiles; ++i) /* checkfiles, SortDetails.cpp:360-386 */
    if (strcmp(files[i], "-") && access(files[i], R_OK) != 0) {
      fprintf(stderr, "Unable to access %s\n", files[i]);
      return EXIT_FAILURE;
    }
  bg_ctx* ctx = NULL;
  cli_detach(); /* the GPU work runs in a worker whose teardown the caller does not wait for */
  if (bg_open(&ctx, env_device())) {
    fprintf(stderr, "cannot open the GPU device (libbedgpu/HIP)\n");
    return EXIT_FAILURE;
  }
  text_buf_t* tx = (text_buf_t*)calloc((size_t)nfiles, sizeof(text_buf_t));
  bg_input* in = (bg_input*)calloc((size_t)nfiles, sizeof(bg_input));
  for (int i = 0; i < nfiles; ++i) {
    if (read_input(ctx, files[i], just_check, &tx[i], &in[i])) {
      fprintf(stderr, "Unable to access %s\n", files[i]);
      return EXIT_FAILURE;
    }
    in[i].kind = BG_BED3_REST;
  }
  if (just_check) { /* Bed::bed_check_iterator<B3Rest*> over each input (CheckSort.cpp:17-40) */
    for (int i = 0; i < nfiles; ++i) {
      bg_check_result cr;
      int rc = bg_check(ctx, &in[i], 3, 1, &cr);
      if (rc) {
        fprintf(stderr, "%s\n", bg_last_error(ctx));
        return EXIT_FAILURE;
      }
      if (cr.row) {
        char m[2048];
        bg_check_message(tx[i].data + cr.line_off, cr.line_len, cr.code, 3, 1, m, sizeof(m));
        fprintf(stderr, "in %s\n%s\nSee row: %llu\n", files[i], m, (unsigned long long)cr.row);
        return EXIT_FAILURE;
      }
    }
    return EXIT_SUCCESS;
  }
  bg_result* res = NULL;
  bg_sortbed_error se;
  int rc = bg_sortbed(ctx, nfiles, in, &res, &se);
  if (rc == BG_E_PARSE) {
    line_error(&se, files[se.input]);
    return EXIT_FAILURE;
  }
  if (rc) {
    fprintf(stderr, "Error: %s\n", bg_last_error(ctx));
    return EXIT_FAILURE;
  }
  if ((rc = bg_result_write(ctx, res, 1))) {
    fprintf(stderr, "Error: %s\n", bg_last_error(ctx));
    return EXIT_FAILURE;
  }
  maybe_stats(ctx);
  fast_exit();
  return EXIT_SUCCESS;
}
