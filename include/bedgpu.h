/*
 * bedgpu.h — C ABI of libbedgpu, the MI355X (gfx950) engine behind the drop-in
 * `bedops` / `bedmap` / `closest-features` front-ends of bedops_amd.
 *
 * BEDOPS has no library API: its only boundary is the process (argv, BED text on
 * stdin/files, BED text on stdout). This ABI is the seam that
 * replaces the reference's internal sweep entry points. Each entry point below
 * names the reference function it replaces:
 *
 *   bg_load .............. Bed readers + per-line parse
 *                          (interfaces/general-headers/data/bed/AllocateIterator_BED_starch.hpp:47-230,
 *                           Bed.hpp:244-255 BED3, :277-383 BED3+rest, :829-860 BED5)
 *   bg_merge ............. doMerge / nextMergeAllLines  (applications/bed/bedops/src/Bedops.cpp:593-606, :1186-1243)
 *   bg_intersect ......... doIntersection / nextIntersectLine (Bedops.cpp:575-587, :1105-1181)
 *   bg_difference ........ doDifference / nextDifferenceLine (Bedops.cpp:500-524, :950-1018)
 *   bg_element_of ........ doElementOf / nextElementOfLine (Bedops.cpp:538-566, :1023-1100)
 *   bg_complement ........ doComplement / nextComplementLine (Bedops.cpp:475-489, :891-945)
 *   bg_chop .............. doChop (Bedops.cpp:437-467)
 *   bg_partition ......... doPartitions / nextPartitionGroup (Bedops.cpp:614-686, :1249-1337)
 *   bg_symmdiff .......... doSymmetricDifference / nextSymmetricDiffLine (Bedops.cpp:697-747, :1343-1467)
 *   bg_everything ........ doUnionAll / nextUnionAllLine (Bedops.cpp:752-786, :1472-1518)
 *   bg_set_pad ........... BedPadReader --range padding (applications/bed/bedops/src/BedPadReader.hpp:71-284)
 *   bg_map ............... WindowSweep::sweep overload 2 + MultiVisitor{Count,Average}
 *                          (interfaces/src/algorithm/sweep/WindowSweepImpl.cpp:168-256,
 *                           algorithm/visitors/other/MultiVisitor.hpp:45-129)
 *   bg_closest ........... FeatDist::findDistances + PrintAll / PrintShortest
 *                          (applications/bed/closestfeats/src/ClosestFeature.cpp:260-413,
 *                           Printers.hpp:46-205; options closestfeats/src/Input.hpp:46-103)
 *   bg_result_format /
 *   bg_result_write ...... record() -> printf("%s\t%lu\t%lu\n") (Bedops.cpp:148-152, Bed.hpp:228-232,321-325),
 *                          visitor printing ("%d", "%.6lf", "NAN": Formats.hpp:31-50, NaN.cpp:26)
 *
 * Conventions: plain pointers and sizes only. Every call returns 0 on success or a
 * negative BG_E* code, never aborts; bg_last_error() gives the message. One context
 * per device, not thread-safe; all device work is ordered on the context's stream.
 * Handles are owned by the caller and released with the matching bg_*_free().
 */
#ifndef BEDGPU_H
#define BEDGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BG_OK 0
#define BG_E_HIP (-1)         /* HIP runtime failure */
#define BG_E_PARSE (-2)       /* malformed BED line */
#define BG_E_UNSORTED (-3)    /* input not sorted per sort-bed (strcmp chrom, start) */
#define BG_E_RANGE (-4)       /* coordinate > 999999999999 or end < start */
#define BG_E_BLANK (-5)       /* blank line inside the data */
#define BG_E_ARG (-6)         /* bad argument */
#define BG_E_NOMEM (-7)       /* device or host allocation failed */
#define BG_E_UNSUPPORTED (-8) /* input/option outside the GPU path (message says which) */
#define BG_E_CHROM (-9)       /* chromosome name longer than 127 bytes */
#define BG_E_IO (-10)         /* read/write failure */
#define BG_E_INTERNAL (-11)   /* a kernel-side consistency check failed (a bug: please report) */
#define BG_E_VISITOR (-12)    /* the reference stops mid-output here (a visitor throws): the
                                 formatted text up to that point is valid and is written /
                                 copied; bg_last_error() has the reference's message */

/* kinds of input, decided by the operation (Bedops.cpp:402-429, Bedmap.cpp:643-654) */
#define BG_BED3 0      /* chrom start end; remainder ignored            (Bed::B3NoRest) */
#define BG_BED3_REST 1 /* remainder after `end` kept verbatim for output (Bed::B3Rest)  */
#define BG_BED5 2      /* chrom start end id score; score parsed         (Bed::B5Rest)  */
/* BED3 parsed straight to the file's merged set (getNextFileMergedCoords,
 * Bedops.cpp:792-814): no per-row columns are kept. Valid for the inputs of
 * merge/intersect/difference/complement/chop/symmdiff and element-of's non-reference
 * files; operations that need rows (element-of's reference, partition, everything,
 * bedmap, closest-features, --chrom, --range) refuse such a table with BG_E_ARG. */
#define BG_BED3_SET 3
/* BED5 with the remainder after `end` kept too (bedmap map files under --echo-map*: the
 * id and the verbatim row are printed, Bed::B5Rest)                                    */
#define BG_BED5_REST 4

typedef struct bg_ctx bg_ctx;
typedef struct bg_set bg_set;       /* N parsed inputs sharing one chromosome dictionary */
typedef struct bg_result bg_result; /* an operation's output, resident on the device   */

typedef struct bg_input {
  const void* data;   /* BED text */
  uint64_t nbytes;
  int on_device;      /* 0: host memory (copied to HBM); 1: device pointer (16-B aligned) */
  int kind;           /* BG_BED3 / BG_BED3_REST / BG_BED5 / BG_BED3_SET */
} bg_input;

typedef struct bg_map_opts {
  uint64_t overlap_bp; /* --bp-ovr (default 1)                                  */
  int n_ops;           /* number of entries in ops[]                            */
  int ops[16];         /* BG_MAP_COUNT / BG_MAP_MEAN, in command-line order     */
  int precision;       /* --prec (default 6)                                    */
  int scientific;      /* --sci                                                 */
  int skip_unmapped;   /* --skip-unmapped                                       */
  char delim[16];      /* --delim (default "|")                                 */
  int criterion;       /* overlap option: BG_OVR_* (0 = --bp-ovr, the default)    */
  uint64_t range_bp;   /* --range <int> (> 0; --range 0 is --bp-ovr 1)          */
  double fraction;     /* --fraction-{ref,map,either,both} <val>, as given       */
  char multidelim[16]; /* --multidelim between --echo-map* items ("" = the default ";") */
  double op_arg[16];   /* argument of ops[k] (--kth <val>; --tmean <low>)           */
  double op_arg2[16];  /* second argument of ops[k] (--tmean <hi>)                  */
  int shard;           /* 1: the set holds some chromosomes of the inputs (multi-GPU shard):
                          results that depend on other chromosomes (decimal-score running
                          sums, one double across the file) are refused, BG_E_UNSUPPORTED */
  int faster;          /* --faster: the sweep runs with the criterion itself and no window
                          re-test (Bedmap.cpp:287-290, 728-745); criterion BG_OVR_BP / RANGE /
                          FRAC_BOTH / EXACT only (bedmap/src/Input.hpp:349), else BG_E_ARG */
} bg_map_opts;
/* operations (applications/bed/bedmap/src/TDefs.hpp:70-103; option names
 * interfaces/general-headers/algorithm/visitors/helpers/NamedVisitors.hpp:52-178) */
#define BG_MAP_COUNT 1         /* --count          Count<PrintScore>          "%d"     */
#define BG_MAP_MEAN 2          /* --mean           Average<PrintScorePrecision>         */
#define BG_MAP_SUM 3           /* --sum            Sum<PrintScorePrecision>             */
#define BG_MAP_MIN 4           /* --min            Extreme<.., CompValueThenAddressLesser>  */
#define BG_MAP_MAX 5           /* --max            Extreme<.., CompValueThenAddressGreater> */
#define BG_MAP_INDICATOR 6     /* --indicator      Indicator<PrintScore>      "%d"     */
#define BG_MAP_BASES 7         /* --bases          OvrAggregate               "%lu"    */
#define BG_MAP_BASES_UNIQ 8    /* --bases-uniq     OvrUnique                  "%u"     */
#define BG_MAP_BASES_UNIQ_F 9  /* --bases-uniq-f   OvrUniqueFract                      */
#define BG_MAP_ECHO 10         /* --echo           Echo<Print> (ref row, BG_BED3_REST)  */
#define BG_MAP_ECHO_SIZE 11    /* --echo-ref-size  Echo<PrintLength>          "%lu"    */
#define BG_MAP_ECHO_NAME 12    /* --echo-ref-name  Echo<PrintSpanName>  chrom:start-end */
/* per map row of the window, in genomic order, joined by multidelim (EchoMapBed,
 * algorithm/visitors/bed/EchoMapBedVisitor.hpp:38-64 + PrintRangeDelim) */
#define BG_MAP_ECHO_MAP 13           /* --echo-map          the map row verbatim     */
#define BG_MAP_ECHO_MAP_ID 14        /* --echo-map-id       its 4th column (id)      */
#define BG_MAP_ECHO_MAP_SCORE 15     /* --echo-map-score    its score, "%.{p}lf"     */
#define BG_MAP_ECHO_MAP_SIZE 16      /* --echo-map-size     its length               */
#define BG_MAP_ECHO_OVERLAP_SIZE 17  /* --echo-overlap-size |ref ∩ map row| (EchoMapIntersectLength) */
#define BG_MAP_ECHO_MAP_RANGE 18     /* --echo-map-range    chrom\tmin start\tmax end (PrintGenomicRange) */
/* order statistics and moments of the window scores (algorithm/visitors/numerical) */
#define BG_MAP_MEDIAN 19       /* --median         Median = RollingKthAverage(0.5)     */
#define BG_MAP_KTH 20          /* --kth <val>      RollingKthAverage(val), 0 < val < 1 */
#define BG_MAP_VARIANCE 21     /* --variance       Variance (running double sums)      */
#define BG_MAP_STDEV 22        /* --stdev          StdDev                              */
#define BG_MAP_CV 23           /* --cv             CoeffVariation                      */
#define BG_MAP_MAD 24          /* --mad [mult]     MedianAbsoluteDeviation (op_arg = mult, 0 = 1) */
#define BG_MAP_ECHO_MAP_ID_UNIQ 25  /* --echo-map-id-uniq  the window's ids, sorted (strcmp) and unique */
#define BG_MAP_ECHO_REF_ROW_ID 26   /* --echo-ref-row-id   "id-<n>", n = printed-line counter (PrintRowID) */
/* one map row of the window, printed whole with its score at --prec
 * (Extreme<PrintAllScorePrecision>, ExtremeVisitor.hpp:84-135; ProcessBedVisitorRow.hpp:181-207).
 * A reference row with no mapped element makes the reference throw ("Unable to process a
 * 'NAN' with PrintAllScorePrecision.") after the text before it: BG_E_VISITOR. */
#define BG_MAP_MIN_ELEMENT 27       /* --min-element       lowest score, ties: lowest (start,end), then first added */
#define BG_MAP_MAX_ELEMENT 28       /* --max-element       highest score, ties: highest (start,end), then first added */
#define BG_MAP_MIN_ELEMENT_RAND 29  /* --min-element-rand  lowest score (the reference picks among ties at random; here the first row) */
#define BG_MAP_MAX_ELEMENT_RAND 30  /* --max-element-rand  highest score (ties: here the last row) */
#define BG_MAP_TMEAN 31             /* --tmean <low> <hi>  TrimmedMean (TrimmedMeanVisitor.hpp), its running sums replayed */
#define BG_MAP_WMEAN 32             /* --wmean             WeightedAverage (bed/WeightedAverageVisitor.hpp) */
/* overlap criteria (Bedmap.cpp:95-155 -> data/bed/BedDistances.hpp) */
#define BG_OVR_BP 0            /* --bp-ovr N       Overlapping(N)            :80-118   */
#define BG_OVR_RANGE 1         /* --range R        RangedDist(R)             :41-67    */
#define BG_OVR_FRAC_REF 2      /* --fraction-ref   PercentOverlapReference   :196-218  */
#define BG_OVR_FRAC_MAP 3      /* --fraction-map   PercentOverlapMapping     :123-190  */
#define BG_OVR_FRAC_EITHER 4   /* --fraction-either PercentOverlapEither     :223-253  */
#define BG_OVR_FRAC_BOTH 5     /* --fraction-both  PercentOverlapBoth        :258-288  */
#define BG_OVR_EXACT 6         /* --exact          Exact                     :293-317  */

typedef struct bg_closest_opts {
  int shortest;       /* --closest / --shortest: one element per row, ties to the left */
  int print_dist;     /* --dist: signed distance columns                              */
  int no_ref;         /* --no-ref: do not echo the <input-file> row                   */
  int no_overlaps;    /* --no-overlaps                                                */
  char delim[16];     /* --delim (default "|")                                        */
} bg_closest_opts;

/* context */
int bg_open(bg_ctx** ctx, int device);
void bg_close(bg_ctx* ctx);
const char* bg_last_error(const bg_ctx* ctx);
int bg_sync(bg_ctx* ctx);
void* bg_stream(bg_ctx* ctx); /* the hipStream_t all work of this context runs on */
/* content hash of the sources, Makefile and flags this library was built from
   (tools/src_hash.py); the test harness refuses a library whose hash differs from the tree */
const char* bg_build_hash(void);

/* loading: parse N BED texts into device-resident keyed SoA columns */
int bg_load(bg_ctx* ctx, int n, const bg_input* inputs, bg_set** out);
int bg_set_rows(const bg_set* set, int i, uint64_t* rows);
int bg_set_restrict_chrom(bg_ctx* ctx, bg_set* set, const char* chrom); /* --chrom */
void bg_set_free(bg_set* set);

/* operations (file indices refer to the set) */
int bg_merge(bg_ctx* ctx, bg_set* set, const int* files, int nfiles, bg_result** out);
int bg_intersect(bg_ctx* ctx, bg_set* set, const int* files, int nfiles, bg_result** out);
int bg_difference(bg_ctx* ctx, bg_set* set, int ref, const int* others, int nothers,
                  bg_result** out);
int bg_element_of(bg_ctx* ctx, bg_set* set, int ref, const int* others, int nothers,
                  double threshold, int use_percent, int invert, bg_result** out);
/* --complement [-L]: gaps between the union's components (full_left: also from base 0) */
int bg_complement(bg_ctx* ctx, bg_set* set, const int* files, int nfiles, int full_left,
                  bg_result** out);
/* --chop chunk [--stagger n] [-x]: pieces of the union's components (stagger 0 = chunk) */
int bg_chop(bg_ctx* ctx, bg_set* set, const int* files, int nfiles, uint64_t chunk,
            uint64_t stagger, int exclude_short, bg_result** out);
int bg_partition(bg_ctx* ctx, bg_set* set, const int* files, int nfiles, bg_result** out);
int bg_symmdiff(bg_ctx* ctx, bg_set* set, const int* files, int nfiles, bg_result** out);
/* --everything: every row of every file (all loaded as BG_BED3_REST), merged in order */
int bg_everything(bg_ctx* ctx, bg_set* set, const int* files, int nfiles, bg_result** out);
/* --range L:R applied to one loaded file (in place; before the operation) */
int bg_set_pad(bg_ctx* ctx, bg_set* set, int file, int lpad, int rpad);
/* --ec validation (replaces Bed::bed_check_iterator::check and its order checks,
 * interfaces/general-headers/data/bed/BedCheckIterator.hpp:215-634): every line of one
 * input checked on the GPU; row = 0 when the file passes, else the first failing line
 * (1-based, headers counted), its code and byte range (and the line before it).
 * nfields: 3 (BED3 types), 5 (bedmap's map file under score operations); has_rest: the
 * reader keeps the remainder (B3Rest), or'ed with BG_CHECK_NEST for bedmap --faster's
 * nested-row check (bed_check_iterator nestCheck, BedCheckIterator.hpp:612-615). */
#define BG_CHECK_NEST 2
typedef struct bg_check_result {
  uint64_t row;
  int code;
  uint64_t line_off, line_len, prev_off, prev_len;
} bg_check_result;
int bg_check(bg_ctx* ctx, const bg_input* in, int nfields, int has_rest, bg_check_result* out);
/* the reference's message for `code` on `line` (host): the text after "in <file>\n" */
int bg_check_message(const char* line, uint64_t len, int code, int nfields, int has_rest,
                     char* buf, uint64_t cap);
/* ref == map: single-file mode (Bedmap.cpp:196-246, sweep overload 1): every row is a
 * reference row and a map row, printed by --echo as the map type prints it */
int bg_map(bg_ctx* ctx, bg_set* set, int ref, int map, const bg_map_opts* opts,
           bg_result** out);
/* closest-features <input-file> <query-file>: `ref` = the <input-file> table, `query` =
 * the <query-file> table, both loaded as BG_BED3_REST; one output line per ref row */
int bg_closest(bg_ctx* ctx, bg_set* set, int ref, int query, const bg_closest_opts* opts,
               bg_result** out);

/* results */
int bg_result_rows(const bg_result* res, uint64_t* rows);
int bg_result_format(bg_ctx* ctx, bg_result* res, uint64_t* nbytes); /* text in HBM */
int bg_result_text_device(const bg_result* res, const char** dptr, uint64_t* nbytes);
int bg_result_copy_text(bg_ctx* ctx, bg_result* res, char* host, uint64_t cap);
int bg_result_write(bg_ctx* ctx, bg_result* res, int fd); /* format + stream to fd */
int bg_result_copy_text_device(bg_ctx* ctx, bg_result* res, void* dst, uint64_t cap);
/* offsets[g] = byte offset of chromosome g's first output line (g in the set's strcmp-
 * ordered dictionary), offsets[nchroms] = total bytes; used to reassemble per-GPU
 * chromosome shards in sorted order */
int bg_result_chrom_spans(bg_ctx* ctx, bg_result* res, uint64_t* offsets, uint32_t cap);
int bg_set_chroms(const bg_set* set, uint32_t* n);
const char* bg_set_chrom_name(const bg_set* set, uint32_t g);
void bg_result_free(bg_result* res);

/* stream n bytes of device memory (on ctx's device) to fd: a regular file by parallel
 * pwrite(2) of DMA'd chunks (BEDGPU_WRITE_PAR=0: not), anything else by double-buffered D2H
 * + write(2) */
int bg_write_device(bg_ctx* ctx, const void* dptr, uint64_t n, int fd);
/* n bytes of device memory to the regular file fd at byte offset `at` (pwrite; the file
 * position is neither used nor moved): the multi-GPU drop-in's per-device output parts */
int bg_pwrite_device(bg_ctx* ctx, const void* dptr, uint64_t n, int fd, int64_t at);
/* the next n bytes ctx's bg_write_device / bg_result_write would write are dropped (counted
 * across calls): a run whose first part already went down a pipe (the drop-ins' chromosome
 * groups, cli_stream.h) redoes the whole file and continues the output after that part */
int bg_set_output_skip(bg_ctx* ctx, uint64_t n);
/* the part of a bg_set_output_skip not yet dropped (0 once the output has passed it) */
int bg_output_skip_left(const bg_ctx* ctx, uint64_t* n);
/* read a regular file into a new device buffer of ctx's device (its host image DMA'd to HBM,
 * see bg_file_image below); load it with bg_input.on_device = 1, free with bg_device_free.
 * Replaces the reader side of allocate_iterator_starch_bed for plain BED files
 * (AllocateIterator_BED_starch.hpp:205-215). */
int bg_read_file_device(bg_ctx* ctx, const char* path, void** dptr, uint64_t* nbytes);
/* File images (inputs as the host reads them, copied to HBM through a pinned ring):
 *   bg_file_image_open      map a regular file read-only with its pages faulted in; no GPU
 *                           call, so it may run on any thread while bg_open initialises
 *   bg_file_image_register  optional (BEDGPU_IMG_COPY=reg: DMA straight from the mapping)
 *   bg_file_image_to_device copy bytes [off, off + len) into a new device buffer of ctx, on
 *                           ctx's stream (free with bg_device_free)
 *   bg_file_image_close     unmap, once every copy from it has completed (bg_sync) */
typedef struct {
  const char* data; /* the file's bytes (NULL when empty) */
  uint64_t n;       /* its size */
  int registered;
} bg_file_image;
int bg_file_image_open(const char* path, bg_file_image* m);
int bg_file_image_register(bg_file_image* m);
int bg_file_image_to_device(bg_ctx* ctx, const bg_file_image* m, uint64_t off, uint64_t len, void** dptr);
void bg_file_image_close(bg_file_image* m);
/* Prefetch (the chromosome-group pipeline's read-ahead): a host thread of the caller's copies
 * the next groups while ctx's stream runs the current one.
 *   bg_device_alloc     a device buffer of ctx (free with bg_device_release / bg_device_free);
 *                       from the thread that launches ctx's work
 *   bg_file_image_copy  bytes [off, off + len) of an image into dst on ctx's prefetch stream,
 *                       then records slot's event (0 <= slot < 65536); any one thread
 *   bg_copy_order       records ctx's stream position: slot's later copies start after it
 *                       (call it once slot's buffers are allocated: a buffer may be a block
 *                       ctx's earlier work used, handed back by the caching allocator)
 *   bg_copy_fence       ctx's stream waits for slot's last recorded copy (call it after the
 *                       bg_file_image_copy for that slot returned) */
int bg_device_alloc(bg_ctx* ctx, uint64_t n, void** dptr);
int bg_file_image_copy(bg_ctx* ctx, const bg_file_image* m, uint64_t off, uint64_t len, void* dst, int slot);
int bg_copy_order(bg_ctx* ctx, int slot);
int bg_copy_fence(bg_ctx* ctx, int slot);
/* Output queue: texts (device pointers of ctx, e.g. bg_result_text_device) written to fd in
 * the order they are pushed, by a host thread of the queue's own (D2H on its own stream into
 * pinned slots, then write(2)), so output can go out while the caller reads and computes the
 * next chromosome group. A pushed text must stay allocated until bg_writer_done() counts it.
 * Replaces the reference's record/Println streaming to stdout (Bedops.cpp:148-152) for the
 * chromosome-group pipeline of the front-ends (bedops_amd/cli/cli_stream.h). */
typedef struct bg_writer bg_writer;
int bg_writer_open(bg_ctx* ctx, int fd, bg_writer** w);
int bg_writer_push(bg_writer* w, const void* dptr, uint64_t n); /* after ctx's queued work */
uint64_t bg_writer_done(bg_writer* w);                         /* pushes fully written */
int bg_writer_close(bg_writer* w); /* waits for every push; first error (message on ctx) */
/* make ctx's device current on the calling thread (a host thread per device in a group) */
int bg_bind(bg_ctx* ctx);

/* ---- Starch input (replaces the Starch branch of Bed::allocate_iterator_starch_bed,
 * interfaces/general-headers/data/bed/AllocateIterator_BED_starch.hpp:62,100-112, and
 * starch::Starch::extractLine, data/starch/starchApi.hpp:1490-1760) ------------------------
 * bg_starch_is: the bytes start a Starch v2 archive (magic ca 5c ad e5, starchApi.hpp:645-676).
 * bg_starch_decode: every stream (or only `chrom`; NULL = all) decompressed on the host
 * (bzip2 / gzip) and reverse-transformed into the BED text the reference's reader yields
 * (unstarchHelpers.c:884-1160); *out is malloc'd (free()), err gets a message. */
int bg_starch_is(const void* data, uint64_t nbytes);
int bg_starch_decode(const void* data, uint64_t nbytes, const char* chrom, char** out, uint64_t* outlen,
                     char* err, uint64_t errcap);

/* ---- multi-GPU: chromosome shards reassembled over RCCL ------------
 * Replaces the reference's per-chromosome process fan-out (`--chrom` per process,
 * docs/content/reference/set-operations/bedops.rst:721-726; comparators start with
 * strcmp(chrom), BedCompare.hpp:42-43): each member of a group processes whole
 * chromosomes on its own GPU; bg_group_gather puts their formatted texts on member 0 in
 * strcmp chromosome order with grouped ncclSend/ncclRecv over xGMI. */
typedef struct bg_group bg_group;
#define BG_UID_BYTES 128
int bg_group_uid(void* uid); /* ncclGetUniqueId: rank 0 of a multi-process group */
/* one process driving n devices (ncclCommInitAll); a device listed twice gets no
 * communicator (transfers become device copies: tests on one GPU) */
int bg_group_open(bg_group** g, const int* devices, int n);
/* one rank of a multi-process group (one process per GPU; uid from rank 0) */
int bg_group_open_rank(bg_group** g, int device, const void* uid, int nranks, int rank);
int bg_group_size(const bg_group* g, int* nlocal, int* nranks, int* rank0);
bg_ctx* bg_group_ctx(bg_group* g, int local);
void bg_group_close(bg_group* g);
/* nchrom: the GLOBAL chromosome list (identical on every rank, strcmp order). For each
 * local member k: text[k] its formatted text (device), off[k][q] / len[k][q] the bytes of
 * global chromosome q in it (len 0: none). Rank 0 gets *out = a device buffer on member
 * 0's device with every chromosome's text in order (free with bg_device_free). */
int bg_group_gather(bg_group* g, int nchrom, const char* const* text, const uint64_t* const* off,
                    const uint64_t* const* len, char** out, uint64_t* out_len);
void bg_device_free(bg_ctx* ctx, void* dptr);
/* bg_device_free without the host wait: the block is reused only by work queued later on
 * ctx's stream (so not with a second copy stream, BEDGPU_COPY_STREAMS=2) */
void bg_device_release(bg_ctx* ctx, void* dptr);
/* host byte ranges copied back to back into one new device buffer of ctx's device (a
 * file's chromosome shard, then loaded with bg_input.on_device = 1) */
int bg_device_gather_host(bg_ctx* ctx, int n, const void* const* parts, const uint64_t* lens,
                          void** out, uint64_t* total);

/* ---- sort-bed (applications/bed/sort-bed/src: Sort.cpp:41-234, SortDetails.cpp:536-1140) ----
 * every line of the inputs checked with sort-bed's own grammar, sorted by chromosome
 * (strcmp), start, end and the rest of the line (strcmp, none first), printed
 * "%s\t%ld\t%ld[\t<rest>]\n" by the bg_result_* calls. On a bad line the call fails with
 * BG_E_PARSE and *err names it (input index, 1-based line, BG_SB_* code). */
typedef struct bg_sortbed_error {
  int input;
  uint64_t line;
  int code;
} bg_sortbed_error;
#define BG_SB_LEADING_WS 1
#define BG_SB_NO_TAB 2
#define BG_SB_CHROM_LONG 3
#define BG_SB_NO_START_SEP 4
#define BG_SB_START_LONG 5
#define BG_SB_START_EMPTY 6
#define BG_SB_START_NONNUM 7
#define BG_SB_NO_EOL 8
#define BG_SB_END_LONG 9
#define BG_SB_END_EMPTY 10
#define BG_SB_END_NONNUM 11
#define BG_SB_END_LE_START 12
#define BG_SB_ID_LONG 13
#define BG_SB_ROW_LONG 14
int bg_sortbed(bg_ctx* ctx, int n, const bg_input* inputs, bg_result** out, bg_sortbed_error* err);

/* per-stage device timings of the last call sequence (ms), for BEDGPU_STATS */
int bg_stats(const bg_ctx* ctx, char* buf, uint64_t cap);

/* kernel timing with HIP events on the context stream: filter NULL/"" = off, "*" = all
 * kernels, else one kernel name (e.g. "k_parse"); bg_prof_read returns lines
 * "<kernel> <launches> <total_ms>" accumulated since bg_prof_enable */
int bg_prof_enable(bg_ctx* ctx, const char* filter);
int bg_prof_read(bg_ctx* ctx, char* buf, uint64_t cap);

/* pinned host buffers for input text (faster H2D); NULL on failure */
void* bg_host_alloc(uint64_t bytes);
void bg_host_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
