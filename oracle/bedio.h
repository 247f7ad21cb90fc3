/*
 * oracle/bedio.h — TEST INFRASTRUCTURE ONLY (the CPU oracle; never linked into the
 * product library or CLIs, never measured as the product).
 *
 * BED record input/output restated from the reference's libc-level behaviour:
 *   - BED3 "NoRest" rows are read with fscanf("%s\t%lu\t%lu%*[^\n]s\n") + fgetc
 *     (interfaces/general-headers/data/bed/Bed.hpp:244-255, format :270-272);
 *   - BED3 "Rest" rows keep the remainder via "%[^\n]" (Bed.hpp:277-383, :380-382);
 *   - a row is kept only if the stream is not at EOF after reading it
 *     (data/bed/AllocateIterator_BED_starch.hpp:161-176), so a final line without
 *     '\n' is dropped;
 *   - output rows are printf("%s\t%lu\t%lu\n") (Bed.hpp:228-232,266-268) and
 *     printf("%s\t%lu\t%lu%s\n") with the rest (Bed.hpp:321-325).
 * Chrom names are interned; comparisons stay strcmp() on the names, as every
 * reference comparator does (data/bed/BedCompare.hpp:42-43).
 */
#ifndef ORACLE_BEDIO_H
#define ORACLE_BEDIO_H
#include <inttypes.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  char** names;
  int n, cap;
  int last;
} chrom_pool_t;

static inline int pool_intern(chrom_pool_t* p, const char* s) {
  if (p->n && p->last >= 0 && strcmp(p->names[p->last], s) == 0) return p->last;
  for (int i = p->n - 1; i >= 0; --i)
    if (strcmp(p->names[i], s) == 0) return p->last = i;
  if (p->n == p->cap) {
    p->cap = p->cap ? 2 * p->cap : 64;
    p->names = (char**)realloc(p->names, (size_t)p->cap * sizeof(char*));
  }
  p->names[p->n] = strdup(s);
  return p->last = p->n++;
}

typedef struct {
  int* chrom;
  uint64_t* start;
  uint64_t* end;
  char** rest;      /* NULL unless read with keep_rest (BED5 / BED4: after score / id) */
  char** id;        /* NULL unless read as BED4 / BED5 */
  double* score;    /* NULL unless read as BED5 */
  int64_t n, cap;
} bedfile_t;

static void bf_push(bedfile_t* f, int c, uint64_t s, uint64_t e, const char* rest, int keep_rest,
                    double score, int keep_score) {
  if (f->n == f->cap) {
    f->cap = f->cap ? 2 * f->cap : 1024;
    f->chrom = (int*)realloc(f->chrom, (size_t)f->cap * sizeof(int));
    f->start = (uint64_t*)realloc(f->start, (size_t)f->cap * sizeof(uint64_t));
    f->end = (uint64_t*)realloc(f->end, (size_t)f->cap * sizeof(uint64_t));
    if (keep_rest) f->rest = (char**)realloc(f->rest, (size_t)f->cap * sizeof(char*));
    if (keep_score) f->score = (double*)realloc(f->score, (size_t)f->cap * sizeof(double));
  }
  f->chrom[f->n] = c;
  f->start[f->n] = s;
  f->end[f->n] = e;
  if (keep_rest) f->rest[f->n] = strdup(rest ? rest : "");
  if (keep_score) f->score[f->n] = score;
  f->n++;
}
static void bf_set_id(bedfile_t* f, const char* id) {
  f->id = (char**)realloc(f->id, (size_t)f->cap * sizeof(char*));
  f->id[f->n - 1] = strdup(id);
}

#define ORACLE_CHR_MAX 127
#define ORACLE_REST_MAX (8 * 131072)

/* Read a BED3 file. keep_rest: remainder of each line is kept (B3Rest). */
static int read_bed3(FILE* fp, chrom_pool_t* pool, bedfile_t* f, int keep_rest) {
  static char chr[ORACLE_CHR_MAX + 1];
  static char rest[ORACLE_REST_MAX + 1];
  memset(f, 0, sizeof(*f));
  for (;;) {
    uint64_t s = 0, e = 0;
    chr[0] = '\0';
    rest[0] = '\0';
    if (keep_rest)
      (void)fscanf(fp, "%127s\t%" SCNu64 "\t%" SCNu64 "%1048576[^\n]s\n", chr, &s, &e, rest);
    else
      (void)fscanf(fp, "%127s\t%" SCNu64 "\t%" SCNu64 "%*[^\n]s\n", chr, &s, &e);
    (void)fgetc(fp);
    if (feof(fp)) break; /* row read while hitting EOF is not kept */
    bf_push(f, pool_intern(pool, chr), s, e, rest, keep_rest, 0.0, 0);
  }
  return 0;
}

/* Read a BED5 map file: chrom start end id score [rest]
 * (Bed::Bed5 readline, Bed.hpp:829-860: "%s\t%lu\t%lu\t%s\t%lf%[^\n]s\n"). */
static int read_bed5(FILE* fp, chrom_pool_t* pool, bedfile_t* f) {
  static char chr[ORACLE_CHR_MAX + 1];
  static char id[16384];
  static char rest[ORACLE_REST_MAX + 1];
  memset(f, 0, sizeof(*f));
  for (;;) {
    uint64_t s = 0, e = 0;
    double sc = 0;
    chr[0] = id[0] = rest[0] = '\0';
    (void)fscanf(fp, "%127s\t%" SCNu64 "\t%" SCNu64 "\t%16383s\t%lf%1048576[^\n]s\n", chr, &s, &e,
                 id, &sc, rest);
    (void)fgetc(fp);
    if (feof(fp)) break;
    bf_push(f, pool_intern(pool, chr), s, e, rest, 1, sc, 1);
    bf_set_id(f, id);
  }
  return 0;
}

/* Read a BED4 file: chrom start end id [rest] (Bed::Bed4 with rest, Bed.hpp:
 * "%s\t%lu\t%lu\t%s%[^\n]s\n"); rest keeps what follows the id. */
static int read_bed4(FILE* fp, chrom_pool_t* pool, bedfile_t* f) {
  static char chr[ORACLE_CHR_MAX + 1];
  static char id[16384];
  static char rest[ORACLE_REST_MAX + 1];
  memset(f, 0, sizeof(*f));
  for (;;) {
    uint64_t s = 0, e = 0;
    chr[0] = id[0] = rest[0] = '\0';
    (void)fscanf(fp, "%127s\t%" SCNu64 "\t%" SCNu64 "\t%16383s%1048576[^\n]s\n", chr, &s, &e, id, rest);
    (void)fgetc(fp);
    if (feof(fp)) break;
    bf_push(f, pool_intern(pool, chr), s, e, rest, 1, 0.0, 0);
    bf_set_id(f, id);
  }
  return 0;
}

static FILE* open_input(const char* path) {
  if (strcmp(path, "-") == 0) return stdin;
  return fopen(path, "r");
}

#endif
