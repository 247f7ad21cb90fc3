/*
 * oracle/ec_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's `--ec` input check, Bed::bed_check_iterator
 * (interfaces/general-headers/data/bed/BedCheckIterator.hpp): lines read with getline
 * (Ext::ByLine, utility/ByLine.hpp), header lines skipped at the top (:215-228) and rejected
 * later (:238-246), check() (:326-593) field by field with the same marker loop, then the
 * order checks against the previous row and end > start (:594-624). Prints the exception
 * text "in <file>\n<message>\nSee row: <n>" of the first failing line (nothing if the file
 * passes) and exits 1 / 0.
 * usage: ec_oracle <nfields> <has_rest 0|1> <file>
 * Only used by tests/; never linked into the product.
 */
#include <ctype.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int NF, REST;
static char MSG[4096];

static int ucsc(const char* s, size_t n) {
  char t[8];
  if (n != 5 && n != 7) return 0;
  for (size_t i = 0; i < n; ++i) t[i] = (char)tolower((unsigned char)s[i]);
  return (n == 7 && !memcmp(t, "browser", 7)) || (n == 5 && !memcmp(t, "track", 5));
}

typedef struct { size_t chrom_len; unsigned long start, end; size_t rest_at; } row_t;

/* returns 1 = row, 0 = header, -1 = error (MSG set) */
static int check(const char* bl, size_t sz, row_t* R) {
  MSG[0] = 0;
  if (sz == 0) { strcpy(MSG, "Empty line found."); return -1; }
  if (ucsc(bl, sz)) return 0;
  size_t marker = 0;
  while (!MSG[0] && marker < sz) {
    if (bl[marker] == ' ') {
      if (ucsc(bl, marker)) return 0;
      strcpy(MSG, "First column should not have spaces.  Consider 'chr1' vs. 'chr1 '.  These are different names.\nsort-bed can correct this for you.");
    } else if (marker == 0 && bl[marker] == '@') {
      return 0;
    } else if (marker == 0 && bl[marker] == '#') {
      return 0;
    } else if (bl[marker] == '\t') {
      if (marker == 0) strcpy(MSG, "First column name should not start with a tab.");
      else {
        if (ucsc(bl, marker)) return 0;
        break;
      }
    }
    ++marker;
  }
  if (!MSG[0]) {
    if (sz <= marker) strcpy(MSG, "No tabs found in BED row.");
    else if (marker > 127)
      sprintf(MSG, "Chromosome name does not fit in MAXCHROMSIZE chars.\nIncrease TOKEN_CHR_MAX_LENGTH in BEDOPS.Constants.hpp and recompile BEDOPS.\nMAXCHROMSIZE = 127; Size given = %zu", marker);
    else ++marker;
  }
  R->chrom_len = marker ? marker - 1 : 0;
  for (int which = 0; which < 2; ++which) { /* start, end */
    const char* nm = which ? "End" : "Start";
    size_t pos = marker;
    if (which) R->rest_at = marker;
    while (!MSG[0] && marker < sz) {
      const char c = bl[marker];
      if (!isdigit((unsigned char)c)) {
        if (c == '\t' && pos != marker) break;
        else if (c == '\t') sprintf(MSG, "Two or more consecutive tabs.  No %s coordinate.", which ? "end" : "start");
        else if (c == '-' && marker == pos) sprintf(MSG, "%s coordinate cannot be < 0: ", nm);
        else if (c == ' ') sprintf(MSG, "%s coordinate may not contain a space: ", nm);
        else sprintf(MSG, "%s coordinate contains non-numeric character: %c", nm, c);
      }
      ++marker;
    }
    if (!MSG[0]) {
      if (sz <= marker && !which) strcpy(MSG, "No tabs after start coordinate.");
      else if (sz <= marker && which && NF > 3) sprintf(MSG, "Only 3 columns given.  Require at least %d", NF);
      else {
        char num[64] = {0};
        size_t n = marker - pos;
        if (n > 12) strcpy(MSG, "Sanity check failure - start coordinate has too many digits as defined by MAX_DEC_INTEGERS in BEDOPS.Constants.hpp");
        else {
          memcpy(num, bl + pos, n < 63 ? n : 63);
          if (atof(num) > 999999999999.0) strcpy(MSG, "Sanity check failure - start coordinate is more than allowed by MAX_COORD_VALUE in BEDOPS.Constants.hpp");
          else {
            unsigned long v = strtoul(num, NULL, 10);
            if (which) R->end = v; else R->start = v;
            ++marker;
          }
        }
      }
    }
  }
  if (NF > 3) {
    size_t pos = marker;
    while (!MSG[0] && marker < sz) {
      if (bl[marker] == '\t' && pos != marker) break;
      else if (bl[marker] == '\t') strcpy(MSG, "Two or more consecutive tabs.  No ID field.");
      else if (bl[marker] == ' ') strcpy(MSG, "ID field may not contain a space.");
      ++marker;
    }
    if (!MSG[0]) {
      if (sz <= marker && NF > 4) sprintf(MSG, "Only 4 columns given.  Require at least %d", NF);
      else if (pos == marker) strcpy(MSG, "Fourth (id) column is empty.");
      else if (marker - pos > 16383)
        sprintf(MSG, "ID field does not fit in MAXCHROMSIZE chars.\nIncrease TOKEN_ID_MAX_LENGTH in BEDOPS.Constants.hpp and recompile BEDOPS.\nMAXIDSIZE = 16383; Size given = %zu", marker - pos);
      else ++marker;
    }
    if (NF > 4) {
      pos = marker;
      int dec = 0, exps = 0, minus = 0;
      size_t exp_pos = 0, minus_pos = 0;
      while (!MSG[0] && marker < sz) {
        const char c = bl[marker];
        if (!isdigit((unsigned char)c)) {
          if (c == '\t' && pos != marker) break;
          else if (c == '\t') strcpy(MSG, "Two or more consecutive tabs.  No measurement given.");
          else if (c == '.') {
            if (++dec > 1) strcpy(MSG, "More than one decimal point in measurement field.");
            else if (exps > 0) strcpy(MSG, "Bad decimal point - part of exponent.");
          } else if (c == 'e' || c == 'E') {
            if (++exps > 1) strcpy(MSG, "Measurement value contains non-numeric character (multiple 'E' or 'e' characters detected).");
            exp_pos = marker;
          } else if (c == ' ') strcpy(MSG, "Measurement value may not contain a space.");
          else if (c == '-' || c == '+') {
            if (marker != pos && exps < 1) strcpy(MSG, "Measurement value has '-' or '+' in wrong place.");
            if (!MSG[0] && marker != pos) {
              if (++minus > 1) strcpy(MSG, "Measurement value has multiple '-' and/or '+' characters.");
              else if (exp_pos + 1 != marker) strcpy(MSG, "Measurement value has bad '-' in the exponent.");
              minus_pos = marker;
            }
          } else sprintf(MSG, "Measurement value contains non-numeric character: %c", c);
        }
        ++marker;
      }
      if (!MSG[0]) {
        if (sz <= marker && NF > 5) sprintf(MSG, "Only 5 columns given.  Require at least %d", NF);
        else if (pos == marker) strcpy(MSG, "Fifth (measure) column is empty.");
        else if (minus_pos > 0 && minus_pos + 1 == marker) strcpy(MSG, "Measurement value ends with a '-'.");
        else ++marker;
      }
      if (NF > 5) {
        pos = marker;
        while (!MSG[0] && marker < sz) {
          const char c = bl[marker];
          if (c != '+' && c != '-') {
            if (c == '\t' && pos != marker) break;
            else if (c == '\t') strcpy(MSG, "Two or more consecutive tabs.  No strand information given.");
            else sprintf(MSG, "Strand (6th) column must be '+' or '-' (with no spaces).  Received: %c\nsort-bed can correct this for you.", c);
          } else if (marker != pos) strcpy(MSG, "Two or more consecutive '+' or '-'s detected.");
          ++marker;
        }
      }
      if (!MSG[0]) {
        if (pos == marker) strcpy(MSG, "Sixth (strand) column is empty.");
        else ++marker;
      }
    }
  }
  if (!MSG[0] && REST && marker < sz && sz - marker > 8 * 131072)
    sprintf(MSG, "The 'rest' of the input row (everything beyond the first %d fields) cannot fit into MAXRESTSIZE chars.\nIncrease TOKEN_REST_MAX_LENGTH in BEDOPS.Constants.hpp and recompile BEDOPS.\nMAXRESTSIZE = %u; Size given = %zu", NF, 8u * 131072u, sz - marker);
  return MSG[0] ? -1 : 1;
}

int main(int argc, char** argv) {
  if (argc != 4) return 2;
  NF = atoi(argv[1]);
  REST = atoi(argv[2]);
  FILE* f = strcmp(argv[3], "-") ? fopen(argv[3], "rb") : stdin;
  if (!f) return 2;
  char* line = NULL;
  size_t cap = 0;
  ssize_t n;
  unsigned long cnt = 0;
  int seen_row = 0;
  char* last = NULL;
  size_t last_n = 0;
  row_t L = {0}, R = {0};
  while ((n = getline(&line, &cap, f)) >= 0) {
    size_t sz = (size_t)n;
    if (sz && line[sz - 1] == '\n') --sz;
    ++cnt;
    memset(&R, 0, sizeof(R));
    int k = check(line, sz, &R);
    if (k == 0) {
      if (!seen_row) continue;
      strcpy(MSG, "Header found but should be at top of file.");
    } else if (k > 0) {
      if (seen_row) {
        int cmp = 0;
        size_t m = R.chrom_len < L.chrom_len ? R.chrom_len : L.chrom_len;
        cmp = memcmp(line, last, m);
        if (!cmp && R.chrom_len != L.chrom_len) cmp = R.chrom_len < L.chrom_len ? -1 : 1;
        if (cmp < 0) strcpy(MSG, "Bed file not properly sorted by first column.");
        else if (cmp == 0) {
          if (R.start < L.start) strcpy(MSG, "Bed file not properly sorted by start coordinates.");
          else if (R.start == L.start) {
            if (R.end < L.end) strcpy(MSG, "Bed file not properly sorted by end coordinates when start coordinates are identical.");
            else if (REST && R.end == L.end) {
              const char* a = line + R.rest_at;
              const char* b = last + L.rest_at;
              size_t la = sz - R.rest_at, lb = last_n - L.rest_at, mm = la < lb ? la : lb;
              int c2 = memcmp(a, b, mm);
              if (!c2 && la < lb) c2 = -1;
              if (c2 < 0) strcpy(MSG, "Bed file not sorted by information following the 3rd column (columns 1-3 equal to previous row).");
            }
          }
        }
      }
      if (!MSG[0] && R.end <= R.start) strcpy(MSG, "End coordinates must be greater than start coordinates.");
    }
    if (MSG[0]) {
      printf("in %s\n%s\nSee row: %lu", argv[3], MSG, cnt);
      return 1;
    }
    if (k > 0) {
      seen_row = 1;
      free(last);
      last = (char*)malloc(sz + 1);
      memcpy(last, line, sz);
      last_n = sz;
      L = R;
    }
  }
  return 0;
}
