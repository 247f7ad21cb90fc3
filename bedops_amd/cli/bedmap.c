/*
 * bedmap — drop-in front-end for `bedmap [options] <ops> <ref-file> [map-file]`,
 * computing the per-reference overlap aggregates on an MI355X through libbedgpu.
 *
 * argv grammar follows applications/bed/bedmap/src/Input.hpp:75-367 (options start
 * with "--", the last one or two arguments are files, --delim/--prec/--sci/
 * --skip-unmapped/--bp-ovr/--chrom/--ec/--header/--faster/--sweep-all); output per
 * reference row is the operations' values in command-line order joined by --delim
 * (MultiVisitor.hpp:83-98). GPU path: --count --mean --sum --min --max --indicator
 * --bases --bases-uniq --bases-uniq-f --echo --echo-ref-size --echo-ref-name under any
 * overlap option (--bp-ovr --range --fraction-{ref,map,either,both} --exact; checks and
 * messages of Input.hpp:143-215,330-345); other operations are reported as not
 * available in this build.
 */
#include "cli_common.h"
#include "cli_stream.h"

static const char* PROG = "bedmap";

static void usage(FILE* f) {
  fprintf(f,
          "bedmap\n  version:  %s\n\n"
          " USAGE: bedmap [process-flags] [overlap-option] <operation(s)...> <ref-file> [map-file]\n"
          "     Any input file must be sorted per the sort-bed utility.\n\n"
          "    Process Flags:\n"
          "      --chrom <chromosome>  Jump to and process data only for <chromosome>.\n"
          "      --delim <delim>       Change output delimiter from '|' to <delim> between columns.\n"
          "      --multidelim <delim>  Change delimiter of multi-value output columns from ';' to <delim>.\n"
          "      --ec / --header       Error check / accept header lines.\n"
          "      --prec <int>          Change the post-decimal precision of scores to <int>.\n"
          "      --skip-unmapped       Print no output for a row with no mapped elements.\n\n"
          "    Overlap Options (At most, one may be selected.  By default, --bp-ovr 1 is used):\n"
          "      --bp-ovr <int>           Require <int> bp overlap between elements of input files.\n"
          "      --exact                  First 3 fields from <map-file> must be identical to <ref-file>'s.\n"
          "      --fraction-both <val>    Both --fraction-ref <val> and --fraction-map <val> must be true.\n"
          "      --fraction-either <val>  Either --fraction-ref <val> or --fraction-map <val> must be true.\n"
          "      --fraction-map <val>     The fraction of the element's size from <map-file> that must overlap.\n"
          "      --fraction-ref <val>     The fraction of the element's size from <ref-file> that must overlap.\n"
          "      --range <int>            Grab <map-file> elements within <int> bp of <ref-file>'s element.\n\n"
          "    Operations (GPU path):\n"
          "      --bases --bases-uniq --bases-uniq-f --count --echo --echo-ref-name --echo-ref-size\n"
          "      --echo-map --echo-map-id --echo-map-range --echo-map-score --echo-map-size\n"
          "      --echo-overlap-size --indicator --max --mean --min --sum\n"
          "      --cv --kth <val> --mad [mult] --median --stdev --variance --echo-map-id-uniq\n"
          "      --echo-ref-row-id --min-element --max-element --min-element-rand\n"
          "      --max-element-rand --tmean <low> <hi> --wmean\n",
          BEDOPS_AMD_VERSION);
}

static void arg_error(const char* msg) { die_msg(PROG, msg); }

typedef struct {
  bg_map_opts o;
  int single;
} map_args_t;
/* one chromosome shard: the same bg_map call on the member's set */
static int run_map(void* arg, bg_ctx* ctx, bg_set* set, bg_result** res) {
  const map_args_t* m = (const map_args_t*)arg;
  return bg_map(ctx, set, 0, m->single ? 0 : 1, &m->o, res);
}

int main(int argc, char** argv) {
  CLI_PROG = PROG;
  if (argc <= 1) {
    usage(stderr);
    return EXIT_FAILURE;
  }
  bg_map_opts o;
  memset(&o, 0, sizeof(o));
  o.overlap_bp = 1;
  o.precision = 6;
  strcpy(o.delim, "|");
  strcpy(o.multidelim, ";");
  int ec = 0, check = 0, need4 = 0, need5 = 0, need_rest = 0, map_rest = 0, addr_ops = 0, set_prec = 0, set_delim = 0;
  int is_bp = 0, is_range = 0, range_alias = 0, is_exact = 0, is_frac[4] = {0, 0, 0, 0};
  static const struct { const char* name; int op; } OPS[] = {
      {"count", BG_MAP_COUNT}, {"mean", BG_MAP_MEAN}, {"sum", BG_MAP_SUM}, {"min", BG_MAP_MIN},
      {"max", BG_MAP_MAX}, {"indicator", BG_MAP_INDICATOR}, {"bases", BG_MAP_BASES},
      {"bases-uniq", BG_MAP_BASES_UNIQ}, {"bases-uniq-f", BG_MAP_BASES_UNIQ_F}, {"echo", BG_MAP_ECHO},
      {"echo-ref-size", BG_MAP_ECHO_SIZE}, {"echo-ref-name", BG_MAP_ECHO_NAME},
      {"echo-map", BG_MAP_ECHO_MAP}, {"echo-map-id", BG_MAP_ECHO_MAP_ID},
      {"echo-map-score", BG_MAP_ECHO_MAP_SCORE}, {"echo-map-size", BG_MAP_ECHO_MAP_SIZE},
      {"echo-overlap-size", BG_MAP_ECHO_OVERLAP_SIZE}, {"echo-map-range", BG_MAP_ECHO_MAP_RANGE},
      {"median", BG_MAP_MEDIAN}, {"variance", BG_MAP_VARIANCE}, {"stdev", BG_MAP_STDEV}, {"cv", BG_MAP_CV},
      {"echo-map-id-uniq", BG_MAP_ECHO_MAP_ID_UNIQ}, {"echo-ref-row-id", BG_MAP_ECHO_REF_ROW_ID},
      {"min-element", BG_MAP_MIN_ELEMENT}, {"max-element", BG_MAP_MAX_ELEMENT},
      {"min-element-rand", BG_MAP_MIN_ELEMENT_RAND}, {"max-element-rand", BG_MAP_MAX_ELEMENT_RAND},
      {"wmean", BG_MAP_WMEAN}};
  const char* chrom = NULL;
  int a = 1;
  while (a < argc) {
    const char* nx = argv[a++];
    if (strncmp(nx, "--", 2) != 0 && argc - a < 2) { --a; break; }
    if (strncmp(nx, "--", 2) != 0) {
      char b[512];
      snprintf(b, sizeof(b), "Option %s does not start with '--'", nx);
      arg_error(b);
    }
    const char* k = nx + 2;
    if (!strcmp(k, "help")) { usage(stdout); return EXIT_SUCCESS; }
    else if (!strcmp(k, "version")) { printf("bedmap\n  version:  %s\n", BEDOPS_AMD_VERSION); return EXIT_SUCCESS; }
    else if (!strcmp(k, "ec") || !strcmp(k, "header")) {
      ec = 1;
      check = 1; /* --header is --ec: errorCheck_ (bedmap/src/Input.hpp:104-106) */
    }
    else if (!strcmp(k, "faster")) o.faster = 1;
    else if (!strcmp(k, "sweep-all")) {}  /* reads the rest of the map file; no output effect */
    else if (!strcmp(k, "delim")) {
      if (set_delim) arg_error("--delim specified multiple times");
      if (a >= argc) arg_error("No output delimiter given");
      if (strlen(argv[a]) >= sizeof(o.delim)) arg_error("--delim value too long for this build");
      strcpy(o.delim, argv[a++]);
      set_delim = 1;
    } else if (!strcmp(k, "multidelim")) {
      if (strcmp(o.multidelim, ";")) arg_error("--multidelim specified multiple times");
      if (a >= argc) arg_error("No multi-value column delimmiter given");
      if (strlen(argv[a]) >= sizeof(o.multidelim)) arg_error("--multidelim value too long for this build");
      strcpy(o.multidelim, argv[a++]);
    } else if (!strcmp(k, "chrom")) {
      if (a >= argc) arg_error("No chromosome name given");
      chrom = argv[a++];
      if (!strcmp(chrom, "all")) chrom = NULL;
    } else if (!strcmp(k, "skip-unmapped")) o.skip_unmapped = 1;
    else if (!strcmp(k, "sci")) o.scientific = 1;
    else if (!strcmp(k, "prec")) {
      if (a >= argc) arg_error("No precision value given");
      if (set_prec) arg_error("--prec specified multiple times.");
      const char* v = argv[a++];
      if (strspn(v, "0123456789") != strlen(v)) {
        char b[512];
        snprintf(b, sizeof(b), "Non-positive-integer argument: %s for --prec", v);
        arg_error(b);
      }
      o.precision = atoi(v);
      set_prec = 1;
    } else if (!strcmp(k, "bp-ovr")) {
      if (range_alias) arg_error("--range and --bp-ovr detected.  Choose one.");
      if (is_bp) arg_error("multiple --bp-ovr's detected");
      if (a >= argc) arg_error("No arg for --bp-ovr");
      const char* v = argv[a++];
      if (strspn(v, "0123456789") != strlen(v)) {
        char b[512];
        snprintf(b, sizeof(b), "Non-positive-integer argument: %s for --bp-ovr", v);
        arg_error(b);
      }
      o.overlap_bp = strtoull(v, NULL, 10);
      if (o.overlap_bp == 0) arg_error("--bp-ovr value must be > 0");
      is_bp = 1;
    } else if (!strcmp(k, "range")) {
      if (is_range || range_alias) arg_error("multiple --range's detected");
      if (a >= argc) arg_error("No arg for --range");
      const char* v = argv[a++];
      if (strspn(v, "0123456789") != strlen(v)) {
        char b[512];
        snprintf(b, sizeof(b), "Non-positive-integer argument: %s for --range", v);
        arg_error(b);
      }
      o.range_bp = strtoull(v, NULL, 10);
      is_range = 1;
      if (o.range_bp == 0) {  /* alias for --bp-ovr 1 (Input.hpp:165-171) */
        if (is_bp) arg_error("--bp-ovr and --range detected.  Choose one.");
        is_range = 0;
        is_bp = 1;
        range_alias = 1;
        o.overlap_bp = 1;
      }
    } else if (!strncmp(k, "fraction-", 9) &&
               (!strcmp(k + 9, "ref") || !strcmp(k + 9, "map") || !strcmp(k + 9, "either") || !strcmp(k + 9, "both"))) {
      const int which = !strcmp(k + 9, "ref") ? 0 : !strcmp(k + 9, "map") ? 1 : !strcmp(k + 9, "either") ? 2 : 3;
      char b[512];
      if (is_frac[which]) { snprintf(b, sizeof(b), "multiple --%s's detected", k); arg_error(b); }
      if (a >= argc) { snprintf(b, sizeof(b), "No arg for --%s", k); arg_error(b); }
      const char* v = argv[a++];
      if (strspn(v, ".-0123456789") != strlen(v)) {
        snprintf(b, sizeof(b), "Non-numeric argument: %s for --%s", v, k);
        arg_error(b);
      }
      o.fraction = strtod(v, NULL);
      if (!(o.fraction > 0 && o.fraction <= 1)) { snprintf(b, sizeof(b), "--%s value must be: >0-1.0", k); arg_error(b); }
      is_frac[which] = 1;
      static const int crit[4] = {BG_OVR_FRAC_REF, BG_OVR_FRAC_MAP, BG_OVR_FRAC_EITHER, BG_OVR_FRAC_BOTH};
      o.criterion = crit[which];
    } else if (!strcmp(k, "mad")) {  /* optional multiplier (Input.hpp:275-288) */
      double mult = 0;
      if (a < argc && strspn(argv[a], ".-0123456789") == strlen(argv[a])) {
        const char* v = argv[a++];
        mult = strtod(v, NULL);
        if (!(mult > 0)) arg_error("--mad Expect 0 < val");
      }
      if (o.n_ops >= 16) arg_error("too many operations for this build");
      o.op_arg[o.n_ops] = mult;
      o.ops[o.n_ops++] = BG_MAP_MAD;
      need5 = 1;
    } else if (!strcmp(k, "kth")) {  /* Input.hpp:290-302; 0 / 1 are Min / Max (Bedmap.cpp:490-501) */
      char b[512];
      if (a >= argc) arg_error("No arg for --kth");
      const char* v = argv[a++];
      if (strspn(v, ".-0123456789") != strlen(v)) {
        snprintf(b, sizeof(b), "Non-numeric argument: %s for --kth", v);
        arg_error(b);
      }
      const double kv = strtod(v, NULL);
      if (!(kv >= 0 && kv <= 1)) arg_error("--kth Expect 0 <= val <= 1");
      if (o.n_ops >= 16) arg_error("too many operations for this build");
      o.op_arg[o.n_ops] = kv;
      o.ops[o.n_ops++] = kv == 0 ? BG_MAP_MIN : (kv == 1 ? BG_MAP_MAX : BG_MAP_KTH);
      need5 = 1;
    } else if (!strcmp(k, "tmean")) {  /* Input.hpp:303-325 */
      char b[512];
      if (a >= argc) arg_error("No <low> arg given for --tmean");
      const char* lo = argv[a++];
      if (strspn(lo, ".-0123456789") != strlen(lo)) {
        snprintf(b, sizeof(b), "Non-numeric argument: %s for --tmean", lo);
        arg_error(b);
      }
      if (a >= argc) arg_error("No <hi> arg given for --tmean");
      const char* hi = argv[a++];
      if (strspn(hi, ".-0123456789") != strlen(hi)) {
        snprintf(b, sizeof(b), "Non-numeric argument: %s for --tmean", hi);
        arg_error(b);
      }
      const double vl = strtod(lo, NULL), vh = strtod(hi, NULL);
      if (!(vl >= 0 && vl <= 1) || !(vh >= 0 && vh <= 1)) arg_error("--tmean Expect 0 <= low < hi <= 1");
      if (!(vl + vh <= 1)) arg_error("--tmean Expect (low + hi) <= 1.");
      if (o.n_ops >= 16) arg_error("too many operations for this build");
      o.op_arg[o.n_ops] = vl;
      o.op_arg2[o.n_ops] = vh;
      o.ops[o.n_ops++] = BG_MAP_TMEAN;
      need5 = 1;
      map_rest = 1;  /* equal scores are ordered by row (set order) in its replay */
    } else if (!strcmp(k, "exact")) {
      if (is_exact) arg_error("multiple --exact's detected - use one");
      is_exact = 1;
    } else {
      int op = 0;
      for (size_t q = 0; q < sizeof(OPS) / sizeof(OPS[0]); ++q)
        if (!strcmp(k, OPS[q].name)) op = OPS[q].op;
      if (!op) {
        char b[512];
        snprintf(b, sizeof(b), "--%s is not available in this build (GPU path: see --help)", k);
        arg_error(b);
      }
      if (o.n_ops >= 16) arg_error("too many operations for this build");
      o.ops[o.n_ops++] = op;
      if (op == BG_MAP_MEAN || op == BG_MAP_SUM || op == BG_MAP_MIN || op == BG_MAP_MAX ||
          op == BG_MAP_ECHO_MAP_SCORE || (op >= BG_MAP_MEDIAN && op <= BG_MAP_CV) ||
          (op >= BG_MAP_MIN_ELEMENT && op <= BG_MAP_WMEAN))
        need5 = 1;
      /* element operations print the whole map row and break ties by its remainder */
      if (op >= BG_MAP_MIN_ELEMENT && op <= BG_MAP_MAX_ELEMENT_RAND) map_rest = 1;
      if (op == BG_MAP_ECHO) need_rest = 1;
      if (op == BG_MAP_ECHO_MAP || op == BG_MAP_ECHO_MAP_ID || op == BG_MAP_ECHO_MAP_ID_UNIQ) map_rest = 1;
      // running-double operations order equal rows by their id and remainder
      // (CoordRestAddressCompare, BedCompare.hpp:143-194) when the scores are decimals
      if (op == BG_MAP_MEAN || op == BG_MAP_SUM || op == BG_MAP_VARIANCE || op == BG_MAP_STDEV ||
          op == BG_MAP_CV)
        map_rest = 1;
      if (op == BG_MAP_ECHO_MAP_ID || op == BG_MAP_ECHO_MAP_ID_UNIQ) need4 = 1;
      /* operations that can see the reference's heap-address order of equal rows: the
       * replay (bg_heap.hip) sizes each row's strings from both files' remainders */
      if (op == BG_MAP_WMEAN || op == BG_MAP_TMEAN || op == BG_MAP_ECHO_MAP || op == BG_MAP_ECHO_MAP_ID ||
          op == BG_MAP_ECHO_MAP_SCORE || op == BG_MAP_ECHO_MAP_SIZE || op == BG_MAP_ECHO_OVERLAP_SIZE ||
          (op >= BG_MAP_MIN_ELEMENT && op <= BG_MAP_MAX_ELEMENT_RAND))
        map_rest = addr_ops = 1;
    }
  }
  {  /* one overlap specification (Input.hpp:330-343) */
    const int count = is_frac[0] + is_frac[1] + is_frac[2] + is_frac[3] + is_range + is_bp + is_exact;
    if (count > 1) arg_error("More than one overlap specification used.");
    if (is_range) o.criterion = BG_OVR_RANGE;
    else if (is_exact) o.criterion = BG_OVR_EXACT;
    else if (is_bp || count == 0) o.criterion = BG_OVR_BP;
  }
  if (o.n_ops == 0) arg_error("No processing option specified (ie; --max).");
  if (o.faster && !(o.criterion == BG_OVR_BP || o.criterion == BG_OVR_RANGE || o.criterion == BG_OVR_FRAC_BOTH ||
                    o.criterion == BG_OVR_EXACT))  /* Input.hpp:349 */
    arg_error("--faster compatible with --range, --bp-ovr, --fraction-both, and --exact only");
  int nf = argc - a;
  if (nf < 1 || nf > 2) arg_error("Need one or two input files");
  for (int i = a; i < argc; ++i) {
    if (strcmp(argv[i], "-") && access(argv[i], R_OK) != 0) {
      char b[1024];
      snprintf(b, sizeof(b), "Unable to find file: %s", argv[i]);
      arg_error(b);
    }
  }
  if (nf == 2 && !strcmp(argv[a], "-") && !strcmp(argv[a + 1], "-")) arg_error("Cannot have both input files set to '-'");

  /* input kinds: the reference file B3Rest (--echo), the map file by the operations'
   * MapFields (Input.hpp:401-418); single-file mode reads the one file as the map type */
  const int mkind = need5 ? (map_rest ? BG_BED5_REST : BG_BED5) : (map_rest ? BG_BED3_REST : BG_BED3);
  const int rkind = (need_rest || addr_ops) ? BG_BED3_REST : BG_BED3;
  const int skind = need5 ? ((map_rest || need_rest) ? BG_BED5_REST : BG_BED5)
                          : ((map_rest || need_rest || (need4 && !need5)) ? BG_BED3_REST : BG_BED3);
  /* BEDGPU_DEVICES=0,1,...: chromosome shards on several GPUs (cli_shard.h). Overlaps and
   * visitors are chromosome-local except --echo-ref-row-id (one line counter for the file),
   * an element operation's stop at the file's first unmapped row, and decimal running sums
   * (one double across the file: bg_map refuses them on a shard and the run falls back to
   * one device, as on any shard error) */
  cli_detach(); /* the GPU work runs in a worker whose teardown the caller does not wait for */
  int shardable = !check && !ec && !chrom;
  for (int k = 0; k < o.n_ops; ++k) {
    if (o.ops[k] == BG_MAP_ECHO_REF_ROW_ID) shardable = 0;
    if (o.ops[k] >= BG_MAP_MIN_ELEMENT && o.ops[k] <= BG_MAP_MAX_ELEMENT_RAND && !o.skip_unmapped) shardable = 0;
  }
  for (int i = a; i < argc; ++i)
    if (!strcmp(argv[i], "-")) shardable = 0;
  bg_input sin[2];
  memset(sin, 0, sizeof(sin));
  sin[0].kind = nf == 1 ? skind : rkind;
  sin[1].kind = mkind;
  map_args_t ma;
  ma.o = o;
  ma.o.shard = 1;
  ma.single = nf == 1;
  if (shardable && getenv("BEDGPU_DEVICES") &&
      shard_run(PROG, nf, sin, (const char* const*)(argv + a), run_map, &ma) == 0)
    return EXIT_SUCCESS;

  cli_mark("start");
  /* one GPU: chromosome groups in a pipeline (cli_stream.h), same conditions as the shards */
  const int streamed = shardable && stream_prepare(nf, (const char* const*)(argv + a));
  if (!chrom && !check && !ec && !streamed) /* map the inputs while HIP initialises */
    for (int i = 0; i < nf; ++i) cli_prefetch(argv[a + i]);
  bg_ctx* ctx = NULL;
  int rc = bg_open(&ctx, env_device());
  if (rc) die_msg(PROG, "cannot open the GPU device (libbedgpu/HIP)");
  cli_mark("open");
  if (streamed && stream_run(ctx, sin, run_map, &ma) == 0) {
    cli_mark("write");
    maybe_stats(ctx);
    fast_exit();
    bg_close(ctx);
    return EXIT_SUCCESS;
  }
  text_buf_t tr = {0}, tm = {0};
  bg_input in[2];
  memset(in, 0, sizeof(in));
  if (read_input_chrom(ctx, argv[a], chrom, check || ec, &tr, &in[0])) arg_error("Unable to read the reference file");
  /* --ec: the reference file is B3Rest, the map file B3Rest/B4Rest/B5Rest by the
   * operations' MapFields (Input.hpp:401-418, Bedmap.cpp:601-655) */
  const int mapfields = need5 ? 5 : (need4 ? 4 : 3);
  /* --faster checks for nested rows too (nestCheck = ProcessMode, Bedmap.cpp:622, 670) */
  const int nest = o.faster ? BG_CHECK_NEST : 0;
  if (check) ec_check(PROG, ctx, argv[a], &tr, nf == 1 ? mapfields : 3, 1 | nest);
  if (ec) {
    apply_ec_header(&tr);
    in[0].data = tr.data;
    in[0].nbytes = tr.n;
  }
  in[0].kind = rkind;
  if (nf == 1) {
    /* single-file mode (Bedmap.cpp:196-246, sweep overload 1): every row is a reference row
     * and a map row, read as the map type (Bedmap.cpp:660-700) */
    in[0].kind = skind;
    bg_set* set = NULL;
    if ((rc = bg_load(ctx, 1, in, &set))) die_ctx(PROG, ctx, rc);
    cli_prefetch_release(ctx);
    free_text(&tr);
    if (chrom && (rc = bg_set_restrict_chrom(ctx, set, chrom))) die_ctx(PROG, ctx, rc);
    bg_result* res = NULL;
    if ((rc = bg_map(ctx, set, 0, 0, &o, &res))) die_ctx(PROG, ctx, rc);
    if ((rc = bg_result_write(ctx, res, 1))) die_ctx(PROG, ctx, rc);
    maybe_stats(ctx);
    fast_exit();
    bg_result_free(res);
    bg_set_free(set);
    free_input(ctx, &tr);
    bg_close(ctx);
    return EXIT_SUCCESS;
  }
  {
    if (read_input_chrom(ctx, argv[a + 1], chrom, check || ec, &tm, &in[1])) arg_error("Unable to read the map file");
    if (check) ec_check(PROG, ctx, argv[a + 1], &tm, mapfields, 1 | nest);
    if (ec) {
      apply_ec_header(&tm);
      in[1].data = tm.data;
      in[1].nbytes = tm.n;
    }
  }
  in[1].kind = mkind;
  bg_set* set = NULL;
  if ((rc = bg_load(ctx, 2, in, &set))) die_ctx(PROG, ctx, rc);
  cli_prefetch_release(ctx);
  cli_mark("load");
  free_text(&tr);
  free_text(&tm);
  if (chrom && (rc = bg_set_restrict_chrom(ctx, set, chrom))) die_ctx(PROG, ctx, rc);
  bg_result* res = NULL;
  if ((rc = bg_map(ctx, set, 0, 1, &o, &res))) die_ctx(PROG, ctx, rc);
  if ((rc = bg_result_write(ctx, res, 1))) die_ctx(PROG, ctx, rc);
  maybe_stats(ctx);
  fast_exit();
  bg_result_free(res);
  bg_set_free(set);
  free_input(ctx, &tr);
  free_input(ctx, &tm);
  bg_close(ctx);
  return EXIT_SUCCESS;
}
