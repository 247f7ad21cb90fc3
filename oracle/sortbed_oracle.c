/*
 * oracle/sortbed_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C) of `sort-bed file...` (applications/bed/sort-bed/src):
 *   per-line grammar and messages ...... SortDetails.cpp:625-781 (fgets lines; blank lines
 *                                        skipped; "browser"/"track"/"#"/"@" headers only
 *                                        before a file's first data line; tab or space
 *                                        separators; digits only, <= 12 of them; end > start;
 *                                        the rest after "\t%[^\n]"; id length check :832-853)
 *   chromosome order ................... lexCompareBedData, strcmp (:1202-1208)
 *   row order .......................... bcd_cmp: start, end, rest strcmp, no rest first
 *                                        (Structures.hpp:50-81)
 *   output ............................. printBed "%s\t%ld\t%ld" + "\t%s\n" | "\n" (:1120-1140)
 * Used only by tests/ as the parity checker of bg_sortbed; never linked into the product.
 *
 * usage: sortbed_oracle file1 [file2 ...]   ('-' = stdin)
 */
#include <ctype.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  char* chrom;
  int64_t s, e;
  char* data; /* NULL: no rest */
} row_t;

static int cmp_row(const void* a, const void* b) {
  const row_t *x = (const row_t*)a, *y = (const row_t*)b;
  int v = strcmp(x->chrom, y->chrom);
  if (v) return v;
  if (x->s != y->s) return x->s < y->s ? -1 : 1;
  if (x->e != y->e) return x->e < y->e ? -1 : 1;
  if (x->data) return y->data ? strcmp(x->data, y->data) : 1;
  return y->data ? -1 : 0;
}

static int isdig(const char* p, size_t n) {
  for (size_t k = 0; k < n; ++k)
    if (!isdigit((unsigned char)p[k])) return 0;
  return 1;
}

int main(int argc, char** argv) {
  row_t* rows = NULL;
  size_t n = 0, cap = 0;
  for (int f = 1; f < argc; ++f) {
    const char* fn = argv[f];
    FILE* fp = strcmp(fn, "-") ? fopen(fn, "r") : stdin;
    if (!fp) { fprintf(stderr, "Unable to access %s\n", fn); return 1; }
    char* line = NULL;
    size_t lcap = 0;
    ssize_t got;
    uint64_t lines = 1;
    int head = 1;
    while ((got = getline(&line, &lcap, fp)) > 0) {
      if (line[0] == '\n') { lines++; continue; }
      if (line[0] == ' ' || line[0] == '\t') {
        fprintf(stderr, "Row begins with a tab or space at line %" PRIu64 " in %s.\n", lines, fn);
        return 1;
      }
      if (head && (!strncmp(line, "browser", 7) || !strncmp(line, "track", 5) || line[0] == '#' ||
                   line[0] == '@')) {
        lines++;
        continue;
      }
      char* c = strpbrk(line, "\t ");
      if (!c) { fprintf(stderr, "No tabs/spaces found at line %" PRIu64 " in %s.\n", lines, fn); return 1; }
      if ((size_t)(c - line) > 127) {
        fprintf(stderr, "Chromosome name too long at line %" PRIu64 " in %s.\n", lines, fn);
        fprintf(stderr, "Check that you have unix newlines (cat -A) or increase TOKEN_CHR_MAX_LENGTH in BEDOPS.Constants.hpp and recompile BEDOPS.\n");
        return 1;
      }
      char* chrom = strndup(line, (size_t)(c - line));
      char* d = strpbrk(++c, "\t ");
      if (!d) {
        fprintf(stderr, "No tabs/spaces found after the start coordinate (or no start coordinate at all) at line %" PRIu64 " in %s.\n", lines, fn);
        return 1;
      }
      if (d - c > 12) {
        fprintf(stderr, "Start coordinate is too large.  Max decimal digits allowed is %ld in BEDOPS.Constants.hpp.  See line %" PRIu64 " in %s.\n", 12L, lines, fn);
        return 1;
      }
      if (d == c) {
        fprintf(stderr, "Consecutive tabs and/or spaces between chromosome and start coordinate.  See line %" PRIu64 " in %s.\n", lines, fn);
        return 1;
      }
      if (!isdig(c, (size_t)(d - c))) {
        fprintf(stderr, "Non-numeric start coordinate.  See line %" PRIu64 " in %s.\n(remember that chromosome names should not contain spaces.)\n", lines, fn);
        return 1;
      }
      int64_t s = strtoll(c, NULL, 10);
      c = strpbrk(++d, "\t ");
      if (!c) {
        c = strchr(d, '\n');
        if (!c) {
          fprintf(stderr, "No end of line found at %" PRIu64 " in %s.\nMay need to increase BED_LINE_LEN and recompile.\nFirst check that you have unix newlines (cat -A).", lines, fn);
          return 1;
        }
      }
      if (c - d > 12) {
        fprintf(stderr, "End coordinate is too large.  Max decimal digits allowed is %ld in BEDOPS.Constants.hpp.  See line %" PRIu64 " in %s.\n", 12L, lines, fn);
        return 1;
      }
      if (c == d) {
        fprintf(stderr, "Extra tab and/or space found in between start and end coordinates.  See line %" PRIu64 " in %s.\n", lines, fn);
        return 1;
      }
      if (!isdig(d, (size_t)(c - d))) {
        fprintf(stderr, "Non-numeric end coordinate.  See line %" PRIu64 " in %s.\n", lines, fn);
        return 1;
      }
      int64_t e = strtoll(d, NULL, 10);
      static char rest[1 << 21];
      rest[0] = 0;
      const int val = sscanf(c, "\t%[^\n]s\n", rest);
      head = 0;
      if (e <= s) {
        fprintf(stderr, "Error on line %" PRIu64 " in %s. Genomic end coordinate is less than (or equal to) start coordinate.\n", lines, fn);
        return 1;
      }
      char* data = NULL;
      if (val == 1) {
        char* q = strpbrk(rest, "\t ");
        size_t idl = q ? (size_t)(q - rest) : strlen(rest);
        if (idl > 16383) {
          fprintf(stderr, "ID field too long at line %" PRIu64 " in %s.\n", lines, fn);
          fprintf(stderr, "Check that you have unix newlines (cat -A) or increase TOKEN_ID_MAX_LENGTH in BEDOPS.Constants.hpp and recompile BEDOPS.\n");
          fprintf(stderr, "You may instead choose to put a dummy id column (like 'id') in as the 4th field to fix this.\n");
          return 1;
        }
        data = strdup(rest);
      }
      if (n == cap) { cap = cap ? 2 * cap : 1024; rows = (row_t*)realloc(rows, cap * sizeof(row_t)); }
      rows[n].chrom = chrom;
      rows[n].s = s;
      rows[n].e = e;
      rows[n].data = data;
      ++n;
      lines++;
    }
    free(line);
    if (fp != stdin) fclose(fp);
  }
  qsort(rows, n, sizeof(row_t), cmp_row);
  static char obuf[1 << 20];
  setvbuf(stdout, obuf, _IOFBF, sizeof(obuf));
  for (size_t k = 0; k < n; ++k) {
    printf("%s\t%" PRId64 "\t%" PRId64, rows[k].chrom, rows[k].s, rows[k].e);
    if (rows[k].data) printf("\t%s\n", rows[k].data);
    else printf("\n");
  }
  return 0;
}
