/* input.c -- SNP-frequency file reader (snp-input.c:19-145) and an ms reader
 * with defined semantics (the reference's ms path is non-functional). */
#include <ctype.h>
#include <errno.h>
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
  for (i = 0; i < nm->n; i++) {
    s->chr_limits[i].chr = (int)i;
    s->chr_limits[i].name = nm->names[i];
  }
  for (i = 0; i < n;) {
    long j = i;
    int c = s->snps[i].chr;
    while (j < n && s->snps[j].chr == c) j++;
    s->chr_limits[c].start_index = (int)i;
    s->chr_limits[c].n_snps = (int)(j - i);
    s->chr_limits[c].start_pos = s->snps[i].pos;
    s->chr_limits[c].bp_length = s->snps[j - 1].pos; /* last SNP position, not a length */
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
typedef struct {
  FILE *f;
  char *line;
  size_t lcap;
  int block; /* blocks read so far */
} msf_t;

typedef struct {
  rec_t *r;
  long n, cap;
} recs_t;

/* Read the next "//" block of M->f.  Returns 0 at end of file; otherwise 1,
   with the block's polymorphic sites appended to R as the chromosome named by
   the block number (a block without segregating sites adds no chromosome). */
static int ms_read_block(msf_t *M, int segment_length, int folded, int sample_first, int sample_size,
                         names_t *nm, scan_t *s, recs_t *R) {
  int segsites = -1, i, nh = 0, hcap = 0, depth, c, dp, found = 0;
  double *x = NULL;
  char **hap = NULL;
  char bname[32];
  ssize_t len;
  while ((len = getline(&M->line, &M->lcap, M->f)) >= 0)
    if (strncmp(M->line, "//", 2) == 0) { found = 1; break; }
  if (!found) return 0;
  /* segsites, optional prob, positions */
  while ((len = getline(&M->line, &M->lcap, M->f)) >= 0) {
    if (sscanf(M->line, "segsites: %d", &segsites) == 1) {
      if (segsites == 0) break;
      continue;
    }
    if (strncmp(M->line, "positions:", 10) == 0) {
      char *p = M->line + 10, *e;
      x = fh_malloc(sizeof(double) * (segsites > 0 ? segsites : 1), "ms positions");
      for (i = 0; i < segsites; i++) {
        x[i] = strtod(p, &e);
        if (e == p) logmsg(MSG_FATAL, "ms input: short positions line in block %d", M->block + 1);
        p = e;
      }
      break;
    }
  }
  M->block++;
  if (segsites <= 0 || !x) { free(x); return 1; }
  /* haplotype lines until a blank line, "//" or EOF */
  for (;;) {
    long pos0 = ftell(M->f);
    if ((len = getline(&M->line, &M->lcap, M->f)) < 0) break;
    while (len > 0 && (M->line[len - 1] == '\n' || M->line[len - 1] == '\r')) M->line[--len] = 0;
    if (len == 0) break;
    if (strncmp(M->line, "//", 2) == 0) { fseek(M->f, pos0, SEEK_SET); break; }
    if (len < segsites) logmsg(MSG_FATAL, "ms input: haplotype shorter than segsites in block %d", M->block);
    if (nh == hcap) { hcap = hcap ? 2 * hcap : 64; hap = fh_realloc(hap, sizeof(char *) * hcap, "ms haplotypes"); }
    hap[nh++] = strdup(M->line);
  }
  depth = sample_size > 0 ? sample_size : nh - sample_first;
  if (sample_first < 0 || depth <= 0 || sample_first + depth > nh)
    logmsg(MSG_FATAL, "ms input: sample [%d, %d) outside the %d haplotypes of block %d", sample_first,
           sample_first + depth, nh, M->block);
  snprintf(bname, sizeof bname, "%d", M->block);
  c = name_index(nm, bname);
  dp = depth_index(s, depth);
  for (i = 0; i < segsites; i++) {
    int d = 0, h;
    rec_t *q;
    for (h = sample_first; h < sample_first + depth; h++) d += hap[h][i] == '1';
    if (d == 0 || d == depth) continue;
    if (R->n == R->cap) {
      R->cap = R->cap ? 2 * R->cap : 1 << 16;
      R->r = fh_realloc(R->r, sizeof(rec_t) * R->cap, "snp records");
    }
    q = &R->r[R->n];
    q->s.chr = c;
    q->s.pos = (int)(x[i] * segment_length);
    q->s.obs_freq = folded ? (d > depth - d ? depth - d : d) : d;
    q->s.folded = folded ? 1 : 0;
    q->s.depth_p = dp;
    q->s.null_logl = 0.0;
    q->seq = R->n++;
  }
  for (i = 0; i < nh; i++) free(hap[i]);
  free(hap);
  free(x);
  return 1;
}

static FILE *ms_open(const char *fname, int segment_length) {
  FILE *f = fopen(fname, "r");
  if (!f) logmsg(MSG_FATAL, "Can't open ms input file \"%s\" (%s)", fname, strerror(errno));
  if (segment_length <= 0) logmsg(MSG_FATAL, "ms input needs --ms-segment-length=<bp> > 0");
  return f;
}

/* every block of the file in one scan_t (one chromosome per block) */
scan_t *fh_load_ms(const char *fname, int segment_length, int folded, int sample_first, int sample_size) {
  msf_t M = {ms_open(fname, segment_length), NULL, 0, 0};
  names_t nm = {NULL, 0, 0, -1};
  recs_t R = {NULL, 0, 0};
  scan_t *s = fh_calloc(1, sizeof(scan_t), "scan_t");
  while (ms_read_block(&M, segment_length, folded, sample_first, sample_size, &nm, s, &R)) {}
  free(M.line);
  fclose(M.f);
  if (R.n == 0) logmsg(MSG_FATAL, "No usable snps found in ms file \"%s\"", fname);
  finish_scan(s, R.r, R.n, &nm);
  free(R.r);
  return s;
}

scan_t *fscl_amd_load_ms_input(const char *ms_fname, int segment_length, int ms_folded, int sample_first,
                               int sample_size) {
  return fh_load_ms(ms_fname, segment_length, ms_folded, sample_first, sample_size);
}

/* ---- the reference's block-at-a-time ms interface (fscl.h:118-123) -----------
 * fscl.c:281-313 computes the spectrum from ms_background's scan_t, frees it,
 * then calls ms_openfile and scans each ms_next_block scan_t in turn.  Same
 * semantics as fh_load_ms: ms_background is the whole file, ms_next_block is
 * one block (its one chromosome named by the block's 1-based number in the
 * file; n_snps 0 for a block without polymorphic sites), NULL at the end. */
static msf_t g_ms = {NULL, NULL, 0, 0};

void ms_openfile(char *ms_fname) {
  if (g_ms.f) fclose(g_ms.f);
  g_ms.f = fopen(ms_fname, "r");
  if (!g_ms.f) logmsg(MSG_FATAL, "Can't open ms input file \"%s\" (%s)", ms_fname, strerror(errno));
  g_ms.block = 0;
}

scan_t *ms_background(char *ms_fname, int ms_segment_length, int ms_folded, int ms_sample_first,
                      int ms_sample_size) {
  return fh_load_ms(ms_fname, ms_segment_length, ms_folded, ms_sample_first, ms_sample_size);
}

scan_t *ms_next_block(int ms_segment_length, int ms_folded, int ms_sample_first, int ms_sample_size) {
  names_t nm = {NULL, 0, 0, -1};
  recs_t R = {NULL, 0, 0};
  scan_t *s;
  if (!g_ms.f) return NULL;
  if (ms_segment_length <= 0) logmsg(MSG_FATAL, "ms input needs --ms-segment-length=<bp> > 0");
  s = fh_calloc(1, sizeof(scan_t), "scan_t");
  if (!ms_read_block(&g_ms, ms_segment_length, ms_folded, ms_sample_first, ms_sample_size, &nm, s, &R)) {
    free(s);
    fclose(g_ms.f);
    free(g_ms.line);
    g_ms = (msf_t){NULL, NULL, 0, 0};
    return NULL;
  }
  finish_scan(s, R.r, R.n, &nm);
  free(R.r);
  return s;
}
