/* input.c -- SNP-frequency file reader (snp-input.c:19-145) and an ms reader
 * with defined semantics (the reference's ms path is non-functional). */
#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "fscl_host.h"

typedef struct { snp_t s; long seq; } rec_t;

static int rec_cmp(const void *va, const void *vb) {
  /* (chr index, pos) as snp-input.c:11-17; input order breaks ties, which is
     what glibc's merge-sort qsort does for equal keys */
  const rec_t *a = va, *b = vb;
  if (a->s.chr != b->s.chr) return a->s.chr < b->s.chr ? -1 : 1;
  if (a->s.pos != b->s.pos) return a->s.pos < b->s.pos ? -1 : 1;
  return (a->seq > b->seq) - (a->seq < b->seq);
}

typedef struct {
  char **names;
  int n, cap, cur;
} names_t;

static int name_index(names_t *t, const char *name) {
  int i;
  if (t->cur >= 0 && strcmp(t->names[t->cur], name) == 0) return t->cur;
  for (i = 0; i < t->n; i++)
    if (strcmp(t->names[i], name) == 0) return t->cur = i;
  if (t->n == t->cap) {
    t->cap = t->cap ? 2 * t->cap : 32;
    t->names = fh_realloc(t->names, sizeof(char *) * t->cap, "chromosome names");
  }
  t->names[t->n] = strdup(name);
  return t->cur = t->n++;
}

static int depth_index(scan_t *s, int depth) {
  int j;
  for (j = 0; j < s->n_depths; j++)
    if (s->sample_depths[j] == depth) return j;
  if (s->n_depths % 32 == 0)
    s->sample_depths = fh_realloc(s->sample_depths, sizeof(int) * (s->n_depths + 32), "sample depths");
  s->sample_depths[s->n_depths] = depth;
  return s->n_depths++;
}

/* sort, then build chr_limits (snp-input.c:123-141) */
static void finish_scan(scan_t *s, rec_t *r, long n, names_t *nm) {
  long i;
  qsort(r, n, sizeof(rec_t), rec_cmp);
  s->n_snps = (int)n;
  s->snps = fh_malloc(sizeof(snp_t) * n, "snps");
  for (i = 0; i < n; i++) s->snps[i] = r[i].s;
  s->n_chromosomes = nm->n;
  s->chr_limits = fh_calloc(nm->n, sizeof(chr_limits_t), "chr_limits");
  for (i = 0; i < n;) {
    long j = i;
    int c = s->snps[i].chr;
    while (j < n && s->snps[j].chr == c) j++;
    s->chr_limits[c].chr = c;
    s->chr_limits[c].start_index = (int)i;
    s->chr_limits[c].n_snps = (int)(j - i);
    s->chr_limits[c].start_pos = s->snps[i].pos;
    s->chr_limits[c].bp_length = s->snps[j - 1].pos; /* last SNP position, not a length */
    s->chr_limits[c].name = nm->names[c];
    i = j;
  }
  free(nm->names);
}

scan_t *load_snp_input(char *snp_fname, int include_invariant, int minimum_obs_depth) {
  FILE *f = fopen(snp_fname, "r");
  char line[8192], name[8192];
  names_t nm = {NULL, 0, 0, -1};
  rec_t *r = NULL;
  long n = 0, cap = 0;
  int line_no = 0;
  scan_t *s;
  if (!f) {
    fprintf(stderr, "Can't open snp file \"%s\"\n", snp_fname);
    exit(-1);
  }
  s = fh_calloc(1, sizeof(scan_t), "scan_t");
  while (fgets(line, sizeof line, f)) {
    int pos, obs, ss, folded, l;
    line_no++;
    for (l = (int)strlen(line) - 1; l >= 0 && (line[l] == '\n' || line[l] == '\r'); l--) line[l] = 0;
    if (line[0] == 0 || line[0] == '#') continue;
    if (sscanf(line, "%s %d %d %d %d", name, &pos, &obs, &ss, &folded) != 5) {
      if (strcmp(line, "chromosome") != 0)
        fprintf(stderr, "Can't parse SNP input at line %d: \"%s\"\n", line_no, line);
      continue;
    }
    if (ss < minimum_obs_depth) continue;
    if (!include_invariant && (obs < 1 || obs > ss - 1)) continue;
    if (n == cap) {
      cap = cap ? 2 * cap : 1 << 16;
      r = fh_realloc(r, sizeof(rec_t) * cap, "snp records");
    }
    r[n].s.chr = name_index(&nm, name);
    r[n].s.pos = pos;
    r[n].s.obs_freq = (folded && obs > ss - obs) ? ss - obs : obs;
    r[n].s.folded = folded;
    r[n].s.depth_p = depth_index(s, ss);
    r[n].s.null_logl = 0.0;
    r[n].seq = n;
    n++;
  }
  fclose(f);
  fprintf(stderr, "Loading SNPs and allele frequencies.... %11ld SNPs - complete.\n", n);
  if (n == 0) {
    fprintf(stderr, "No usable snps found in file \"%s\"\n", snp_fname);
    exit(1);
  }
  finish_scan(s, r, n, &nm);
  free(r);
  return s;
}

/* ---- ms (Hudson) output ----------------------------------------------------
 * Defined semantics, fixing what ms-input.c:93-151 leaves
 * undefined: every "//" block is one chromosome named by its 1-based block
 * number; a site's position is (int)(x * segment_length) (ms-input.c:127);
 * the sample is haplotypes [first, first+size) (size 0 = all from first);
 * sites monomorphic in the sample are dropped (:134); with ms_folded the
 * minor count is kept and folded=1 (the evident intent of :137-140). */
scan_t *fh_load_ms(const char *fname, int segment_length, int folded, int sample_first, int sample_size) {
  FILE *f = fopen(fname, "r");
  names_t nm = {NULL, 0, 0, -1};
  rec_t *r = NULL;
  long n = 0, cap = 0;
  char *line = NULL;
  size_t lcap = 0;
  ssize_t len;
  int block = 0;
  scan_t *s;
  if (!f) logmsg(MSG_FATAL, "Can't open ms input file \"%s\"", fname);
  if (segment_length <= 0) logmsg(MSG_FATAL, "ms input needs --ms-segment-length=<bp> > 0");
  s = fh_calloc(1, sizeof(scan_t), "scan_t");
  while ((len = getline(&line, &lcap, f)) >= 0) {
    int segsites = -1, i, nh = 0, hcap = 0, depth, c, dp;
    double *x = NULL;
    char **hap = NULL;
    char bname[32];
    if (strncmp(line, "//", 2) != 0) continue;
    /* segsites, optional prob, positions */
    while ((len = getline(&line, &lcap, f)) >= 0) {
      if (sscanf(line, "segsites: %d", &segsites) == 1) {
        if (segsites == 0) break;
        continue;
      }
      if (strncmp(line, "positions:", 10) == 0) {
        char *p = line + 10, *e;
        x = fh_malloc(sizeof(double) * (segsites > 0 ? segsites : 1), "ms positions");
        for (i = 0; i < segsites; i++) {
          x[i] = strtod(p, &e);
          if (e == p) logmsg(MSG_FATAL, "ms input: short positions line in block %d", block + 1);
          p = e;
        }
        break;
      }
    }
    block++;
    if (segsites <= 0 || !x) { free(x); continue; }
    /* haplotype lines until a blank line, "//" or EOF */
    for (;;) {
      long pos0 = ftell(f);
      if ((len = getline(&line, &lcap, f)) < 0) break;
      while (len > 0 && (line[len - 1] == '\n' || line[len - 1] == '\r')) line[--len] = 0;
      if (len == 0) break;
      if (strncmp(line, "//", 2) == 0) { fseek(f, pos0, SEEK_SET); break; }
      if (len < segsites) logmsg(MSG_FATAL, "ms input: haplotype shorter than segsites in block %d", block);
      if (nh == hcap) { hcap = hcap ? 2 * hcap : 64; hap = fh_realloc(hap, sizeof(char *) * hcap, "ms haplotypes"); }
      hap[nh++] = strdup(line);
    }
    depth = sample_size > 0 ? sample_size : nh - sample_first;
    if (sample_first < 0 || depth <= 0 || sample_first + depth > nh)
      logmsg(MSG_FATAL, "ms input: sample [%d, %d) outside the %d haplotypes of block %d", sample_first,
             sample_first + depth, nh, block);
    snprintf(bname, sizeof bname, "%d", block);
    c = name_index(&nm, bname);
    dp = depth_index(s, depth);
    for (i = 0; i < segsites; i++) {
      int d = 0, h;
      for (h = sample_first; h < sample_first + depth; h++) d += hap[h][i] == '1';
      if (d == 0 || d == depth) continue;
      if (n == cap) { cap = cap ? 2 * cap : 1 << 16; r = fh_realloc(r, sizeof(rec_t) * cap, "snp records"); }
      r[n].s.chr = c;
      r[n].s.pos = (int)(x[i] * segment_length);
      r[n].s.obs_freq = folded ? (d > depth - d ? depth - d : d) : d;
      r[n].s.folded = folded ? 1 : 0;
      r[n].s.depth_p = dp;
      r[n].s.null_logl = 0.0;
      r[n].seq = n;
      n++;
    }
    for (i = 0; i < nh; i++) free(hap[i]);
    free(hap);
    free(x);
  }
  free(line);
  fclose(f);
  if (n == 0) logmsg(MSG_FATAL, "No usable snps found in ms file \"%s\"", fname);
  finish_scan(s, r, n, &nm);
  free(r);
  return s;
}

scan_t *fscl_amd_load_ms_input(const char *ms_fname, int segment_length, int ms_folded, int sample_first,
                               int sample_size) {
  return fh_load_ms(ms_fname, segment_length, ms_folded, sample_first, sample_size);
}
