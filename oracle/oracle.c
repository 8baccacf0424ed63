/*
 * oracle.c -- CPU restatement of slowkoni/fscl's CLR sweep scan and
 * block-permutation test.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Build with -O2 -ffp-contract=off (no -march, no fast-math): the reference's
 * canonical arithmetic.  Each function names the
 * reference lines it restates; the floating-point expression order is kept
 * operation for operation, the control flow is written fresh.
 */
#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "oracle.h"

#define LOG_AD_MIN (-20.0) /* fscl.h:79 */
#define LOG_AD_MAX (4.0)   /* fscl.h:80 */
#define CLR_NULL_DIST_SAVE 10000 /* scan-chromosome.c:227 */

static void *xmalloc(size_t n) {
  void *p = malloc(n ? n : 1);
  if (!p) { fprintf(stderr, "oracle: out of memory (%zu bytes)\n", n); abort(); }
  return p;
}
static void *xcalloc(size_t n, size_t m) {
  void *p = calloc(n ? n : 1, m ? m : 1);
  if (!p) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
  return p;
}

/* ---------------------------------------------------------------- rand() */
/* glibc __srandom_r / __random_r, TYPE_3 (degree 31, separation 3). */
void orc_srand(orc_rand_t *g, unsigned seed) {
  int32_t word;
  int i;
  if (seed == 0) seed = 1;
  g->r[0] = (int32_t)seed;
  word = (int32_t)seed;
  for (i = 1; i < 31; i++) {
    long hi = word / 127773, lo = word % 127773;
    word = (int32_t)(16807 * lo - 2836 * hi);
    if (word < 0) word += 2147483647;
    g->r[i] = word;
  }
  g->f = 3;
  g->b = 0;
  for (i = 0; i < 310; i++) (void)orc_rand(g);
}

int orc_rand(orc_rand_t *g) {
  uint32_t v = (uint32_t)g->r[g->f] + (uint32_t)g->r[g->b];
  g->r[g->f] = (int32_t)v;
  g->f = (g->f + 1) % 31;
  g->b = (g->b + 1) % 31;
  return (int)(v >> 1);
}

/* ------------------------------------------------------ logs and tables */
static double *g_log_table = NULL;
static int g_spline_pts = 200;
static double g_log_ad_step = 24.0 / 201.0;

/* sm-search.c:14-26 */
void orc_init_log_table(void) {
  int i;
  if (g_log_table) return;
  g_log_table = xmalloc(sizeof(double) * 0x10000);
  for (i = 1; i <= 0xFFFF; i++) g_log_table[i] = log(i);
  g_log_table[0] = 0.;
}
const double *orc_log_table(void) { orc_init_log_table(); return g_log_table; }

/* sm-search.c:40-46 */
double orc_logt(int d) {
  if (d < 0) d = -d;
  if (d > 0xFFFFFF) return 11.783502069519070 + g_log_table[d >> 16];
  if (d > 0xFFFF) return 5.545177444479562 + g_log_table[d >> 8];
  return g_log_table[d];
}

/* sm-spline.c:325 */
void orc_set_spline_pts(int spline_pts) {
  g_spline_pts = spline_pts;
  g_log_ad_step = (LOG_AD_MAX - LOG_AD_MIN) / (spline_pts + 1.);
}
double orc_log_ad_step(void) { return g_log_ad_step; }

/* sm-spline.c:18-39: lf[i] = lf[i-1] + log(i), accumulated from lf[0] = 0 */
static double *g_lf = NULL;
static int g_lf_max = 0;
double orc_log_fact(int n) {
  if (n < 0) return -DBL_MAX;
  if (n == 0 || n == 1) return 0.;
  if (n > g_lf_max) {
    int i, from;
    double *t = realloc(g_lf, sizeof(double) * (n + 1));
    if (!t) abort();
    g_lf = t;
    if (g_lf_max == 0) { g_lf[0] = 0; g_lf_max = 1; }
    from = g_lf_max;
    for (i = from; i <= n; i++) g_lf[i] = g_lf[i - 1] + log(i);
    g_lf_max = n;
  }
  return g_lf[n];
}

/* sm-spline.c:41-46 */
double orc_lchoose(int n, int k) {
  if (n == 0 && k == 0) return 0.;
  if (k > n || n == 0) return -DBL_MAX;
  return orc_log_fact(n) - orc_log_fact(k) - orc_log_fact(n - k);
}

/* ------------------------------------------------------------- input */
typedef struct { orc_snp_t s; long seq; } keyed_snp_t;

static int snp_cmp(const keyed_snp_t *a, const keyed_snp_t *b) {
  /* snp-input.c:11-17, made explicitly stable (glibc qsort is a merge sort) */
  if (a->s.chr != b->s.chr) return a->s.chr < b->s.chr ? -1 : 1;
  if (a->s.pos != b->s.pos) return a->s.pos < b->s.pos ? -1 : 1;
  return a->seq < b->seq ? -1 : (a->seq > b->seq);
}
static int snp_cmp_v(const void *a, const void *b) { return snp_cmp(a, b); }

/* snp-input.c:19-145 */
orc_scan_t *orc_load_snp_input(const char *fname, int include_invariant, int minimum_depth) {
  FILE *f = fopen(fname, "r");
  char line[8192], name[8192];
  char **names = NULL;
  int n_names = 0, cur = -1, line_no = 0;
  keyed_snp_t *tmp = NULL;
  long n = 0, cap = 0;
  orc_scan_t *s;
  long i;
  if (!f) { fprintf(stderr, "Can't open snp file \"%s\"\n", fname); return NULL; }
  s = xcalloc(1, sizeof(*s));
  while (fgets(line, sizeof line, f)) {
    int pos, obs, ss, folded, j, l;
    line_no++;
    l = (int)strlen(line) - 1;
    while (l >= 0 && (line[l] == '\n' || line[l] == '\r')) line[l--] = 0;
    if (line[0] == 0 || line[0] == '#') continue;
    if (sscanf(line, "%s %d %d %d %d", name, &pos, &obs, &ss, &folded) != 5) {
      if (strcmp(line, "chromosome") != 0)
        fprintf(stderr, "Can't parse SNP input at line %d: \"%s\"\n", line_no, line);
      continue;
    }
    if (ss < minimum_depth) continue;
    if (!include_invariant && (obs < 1 || obs > ss - 1)) continue;
    if (cur == -1 || strcmp(name, names[cur]) != 0) {
      for (cur = 0; cur < n_names && strcmp(names[cur], name) != 0; cur++) {}
      if (cur == n_names) {
        names = realloc(names, sizeof(char *) * (n_names + 1));
        names[n_names++] = strdup(name);
      }
    }
    if (folded && obs > ss - obs) obs = ss - obs;
    for (j = 0; j < s->n_depths && s->sample_depths[j] != ss; j++) {}
    if (j == s->n_depths) {
      s->sample_depths = realloc(s->sample_depths, sizeof(int) * (s->n_depths + 1));
      s->sample_depths[s->n_depths++] = ss;
    }
    if (n == cap) { cap = cap ? 2 * cap : 4096; tmp = realloc(tmp, sizeof(*tmp) * cap); }
    tmp[n].s.chr = cur; tmp[n].s.pos = pos; tmp[n].s.obs_freq = obs;
    tmp[n].s.folded = folded; tmp[n].s.depth_p = j; tmp[n].s.null_logl = 0.;
    tmp[n].seq = n;
    n++;
  }
  fclose(f);
  if (n == 0) { fprintf(stderr, "No usable snps found in file \"%s\"\n", fname); free(s); return NULL; }
  qsort(tmp, n, sizeof(*tmp), snp_cmp_v);
  s->n_snps = (int)n;
  s->snps = xmalloc(sizeof(orc_snp_t) * n);
  for (i = 0; i < n; i++) s->snps[i] = tmp[i].s;
  free(tmp);
  s->n_chr = n_names;
  s->chr = xcalloc(n_names, sizeof(orc_chr_t));
  for (i = 0; i < n;) {
    long j = i;
    int c = s->snps[i].chr;
    while (j < n && s->snps[j].chr == c) j++;
    s->chr[c].chr = c;
    s->chr[c].start_index = (int)i;
    s->chr[c].n_snps = (int)(j - i);
    s->chr[c].start_pos = s->snps[i].pos;
    s->chr[c].bp_length = s->snps[j - 1].pos;
    s->chr[c].name = names[c];
    i = j;
  }
  free(names);
  return s;
}

/* ------------------------------------------------- background spectrum */
/* background-fsp.c:19-51 */
static double **neutral_spectra(orc_scan_t *s) {
  int n_inv = 0, n_fix = 0, i, k, m, n_seg;
  double seg_sum, **fsp = xmalloc(sizeof(double *) * s->n_depths);
  for (i = 0; i < s->n_snps; i++) {
    if (s->snps[i].obs_freq == 0) n_inv++;
    if (s->snps[i].obs_freq == s->sample_depths[s->snps[i].depth_p]) n_fix++;
  }
  for (i = 0; i < s->n_depths; i++) {
    m = s->sample_depths[i];
    fsp[i] = xmalloc(sizeof(double) * (m + 1));
    fsp[i][0] = n_inv;
    fsp[i][m] = n_fix;
    seg_sum = 0.;
    for (k = 1; k < m; k++) seg_sum += 1 / (double)k;
    n_seg = s->n_snps - n_fix - n_inv;
    for (k = 1; k < m; k++) fsp[i][k] = (1. / (double)k) / seg_sum * n_seg;
    for (k = 0; k <= m; k++) fsp[i][k] /= (double)s->n_snps;
  }
  return fsp;
}

/* background-fsp.c:72-88 (n = target depth, N = source depth) */
static void hyper_downsample(double *d_fsp, const double *fsp, int n, int N, int include_invariant) {
  int m, k;
  if (include_invariant) {
    for (m = 0; m <= N; m++)
      for (k = 0; k <= m && k <= n; k++)
        d_fsp[k] += exp(orc_lchoose(m, k) + orc_lchoose(N - m, n - k) - orc_lchoose(N, n)) * fsp[m];
  } else {
    for (m = 1; m <= N; m++)
      for (k = 1; k <= m && k < n; k++)
        d_fsp[k] += exp(orc_lchoose(m, k) + orc_lchoose(N - m, n - k) - orc_lchoose(N, n)) * fsp[m];
  }
}

/* background-fsp.c:182-316 (the -b loader at :127-180 is out of scope) */
double **orc_background_fsp(orc_scan_t *s, int force_neutral, int include_invariant) {
  int m, k, i, depth, max_depth = -1000;
  double sum, **fsp, *tmp, wa, wd;
  if (force_neutral) return neutral_spectra(s);
  fsp = xmalloc(sizeof(double *) * s->n_depths);
  for (m = 0; m < s->n_depths; m++) {
    fsp[m] = xcalloc(s->sample_depths[m] + 1, sizeof(double));
    if (s->sample_depths[m] > max_depth) max_depth = s->sample_depths[m];
  }
  orc_log_fact(max_depth + 1);
  tmp = xcalloc(max_depth + 1, sizeof(double));
  for (i = 0; i < s->n_snps; i++) {
    const orc_snp_t *p = s->snps + i;
    depth = s->sample_depths[p->depth_p];
    if (p->folded) {
      if (p->obs_freq == 0) { wa = 1; wd = 0; }
      else if (p->obs_freq == depth) { wa = 0; wd = 1; }
      else { wa = 1. / (p->obs_freq); wd = 1. / (depth - p->obs_freq); }
    } else { wd = 1.; wa = 0.; }
    if (depth == max_depth) {
      tmp[p->obs_freq] += wa / (wa + wd);
      tmp[depth - p->obs_freq] += wd / (wa + wd); /* Q1: mirrored polarity */
    }
  }
  sum = 0.;
  for (k = 0; k <= max_depth; k++) sum += tmp[k];
  for (k = 0; k <= max_depth; k++) tmp[k] /= sum;
  for (m = 0; m < s->n_depths; m++) {
    depth = s->sample_depths[m];
    hyper_downsample(fsp[m], tmp, depth, max_depth, include_invariant);
    sum = 0.;
    for (k = 0; k <= depth; k++) sum += fsp[m][k];
    for (k = 0; k <= depth; k++) fsp[m][k] /= sum;
  }
  free(tmp);
  return fsp;
}

/* ---------------------------------------------------------- asc-bias */
/* asc-bias.c:12-25 */
static double ascprob_subsample(int k, int d, int min_obs, int n) {
  int i;
  double no_asc = 0.;
  for (i = 0; i < min_obs; i++)
    no_asc += exp(orc_lchoose(k, d - i) + orc_lchoose(n - k, i)) +
              exp(orc_lchoose(n - k, d - i) + orc_lchoose(k, i));
  no_asc /= exp(orc_lchoose(n, d));
  return 1.0 - no_asc;
}

/* asc-bias.c:27-95 */
double *orc_ascbias_adjust_background(const double *bsf, int n, int asc_depth, int min_obs) {
  double *asc = xmalloc(sizeof(double) * (n + 1)), *adj = xmalloc(sizeof(double) * (n + 1));
  double asc_sum = 0., adj_sum = 0.;
  int i;
  asc[0] = asc[n] = 0.;
  for (i = 1; i < n; i++) { asc[i] = ascprob_subsample(i, asc_depth, min_obs, n); asc_sum += asc[i]; }
  for (i = 1; i < n; i++) asc[i] /= asc_sum;
  adj[0] = adj[n] = 0.;
  for (i = 1; i < n; i++) { adj[i] = bsf[i] / asc[i]; adj_sum += adj[i]; }
  for (i = 1; i < n; i++) adj[i] /= adj_sum;
  free(asc);
  return adj;
}

/* asc-bias.c:97-109 */
void orc_ascbias_adjust_expect(double *fsp, int n, int min_obs, int d) {
  int i;
  double asc_sum = 0;
  for (i = 0; i <= n; i++) asc_sum += fsp[i] * ascprob_subsample(i, d, min_obs, n);
  for (i = 0; i <= n; i++) fsp[i] = fsp[i] * ascprob_subsample(i, d, min_obs, n) / asc_sum;
}

/* ------------------------------------------------------- spline tables */
/* sm-spline.c:63-118: banded Gauss elimination on a dense matrix, as written */
static void solve_linear_system(double *b, double **m, double *v, int n) {
  int i, j, k;
  double f;
  for (i = 0; i < n; i++) {
    if (fabs(m[i][i]) < 1e-20) {
      int mx = i;
      for (j = i + 1; j < n; j++)
        if (fabs(m[j][i]) > 0 && (mx == i || fabs(fabs(m[j][i]) - 1) < fabs(fabs(m[mx][i]) - 1))) mx = j;
      if (mx == i) {
        fprintf(stderr, "Ill conditioned matrix while trying to estimate spline functions to "
                        "approximate sweep model likelihoods.\n");
        exit(1);
      }
      for (k = 0; k < n; k++) m[i][k] += m[mx][k];
      v[i] += v[mx];
    }
    f = m[i][i];
    for (k = i; k < i + 8 && k < n; k++) m[i][k] /= f;
    v[i] /= f;
    for (j = i + 1; j < i + 8 && j < n; j++) {
      f = m[j][i];
      for (k = i; k < i + 8 && k < n; k++) m[j][k] = m[j][k] - m[i][k] * f;
      v[j] = v[j] - v[i] * f;
    }
  }
  for (i = n - 1; i >= 0;) {
    if (fabs(m[i][i]) < 1e-10) {
      fprintf(stderr, "Warning: setting a spline coefficient %d to zero\n", i);
      b[i--] = 0;
      continue;
    }
    b[i] = v[i];
    for (k = i + 1; k < i + 8 && k < n; k++) b[i] -= m[i][k] * b[k];
    i--;
  }
}

/* sm-spline.c:120-220: natural cubic spline through (x[0..n], y[0..n]) */
static void estimate_spline(orc_spline_t *out, const double *x, const double *y, int n) {
  int dim = 4 * (n + 1), i, j, k;
  double **m = xmalloc(sizeof(double *) * dim);
  double *v = xcalloc(dim, sizeof(double)), *b = xcalloc(dim, sizeof(double));
  double *store = xcalloc((size_t)dim * dim, sizeof(double));
  for (i = 0; i < dim; i++) m[i] = store + (size_t)i * dim;

  m[0][0] = 6 * x[0];
  m[0][1] = 2;
  for (i = 1, j = 0, k = 0; k < n - 1; i += 4, j += 4, k++) {
    m[i][j] = x[k] * x[k] * x[k];
    m[i][j + 1] = x[k] * x[k];
    m[i][j + 2] = x[k];
    m[i][j + 3] = 1.;
    v[i] = y[k];
    m[i + 1][j] = x[k + 1] * x[k + 1] * x[k + 1];
    m[i + 1][j + 1] = x[k + 1] * x[k + 1];
    m[i + 1][j + 2] = x[k + 1];
    m[i + 1][j + 3] = 1;
    v[i + 1] = y[k + 1];
    m[i + 2][j] = 3 * x[k + 1] * x[k + 1];
    m[i + 2][j + 1] = 2 * x[k + 1];
    m[i + 2][j + 2] = 1;
    m[i + 2][j + 4] = -3 * x[k + 1] * x[k + 1];
    m[i + 2][j + 5] = -2 * x[k + 1];
    m[i + 2][j + 6] = -1;
    m[i + 3][j] = 6 * x[k + 1];
    m[i + 3][j + 1] = 2;
    m[i + 3][j + 4] = -6 * x[k + 1];
    m[i + 3][j + 5] = -2;
  }
  m[i][j] = x[k] * x[k] * x[k];
  m[i][j + 1] = x[k] * x[k];
  m[i][j + 2] = x[k];
  m[i][j + 3] = 1;
  v[i] = y[k];
  m[i + 1][j] = x[n] * x[n] * x[n];
  m[i + 1][j + 1] = x[n] * x[n];
  m[i + 1][j + 2] = x[n];
  m[i + 1][j + 3] = 1;
  v[i + 1] = y[n];
  m[i + 2][j] = 6 * x[n];
  m[i + 2][j + 1] = 2;

  solve_linear_system(b, m, v, 4 * n);

  out->n = n;
  out->knots = xmalloc(sizeof(double) * (n + 1));
  out->coef = xmalloc(sizeof(double) * 4 * n);
  for (i = 0; i <= n; i++) out->knots[i] = x[i];
  for (i = 0; i < 4 * n; i++) out->coef[i] = b[i];
  free(store); free(m); free(v); free(b);
}

/* sm-spline.c:48-60 */
double orc_spline_interpolate(const orc_spline_t *sp, double x) {
  int i = (x - LOG_AD_MIN) / g_log_ad_step;
  const double *c;
  if (i >= sp->n) i = sp->n - 1;
  if (i < 0) i = 0;
  c = sp->coef + 4 * i;
  return x * (c[0] * x * x + c[1] * x + c[2]) + c[3];
}

/* sm-spline.c:236-240 */
static double p_kescape(int k, int n, double ad) {
  if (k == 0) return exp(-n * ad);
  return exp(orc_lchoose(n, k) + k * log(1.0 - exp(-ad)) - (n - k) * ad);
}

/* sm-spline.c:316-484 for one sample depth */
static void sweep_model_fsp(orc_table_t *t, const double *fsp, int n, const orc_opts_t *o) {
  int b, h, i, j, k, q, f, np = o->spline_pts;
  double *pjh = xmalloc(sizeof(double) * (n + 1) * (n + 1));
  double *pbk = xmalloc(sizeof(double) * (n + 1) * (n + 1));
  double *x = xmalloc(sizeof(double) * (np + 1)), *p = xmalloc(sizeof(double) * (n + 1));
  double *y = xmalloc(sizeof(double) * (n + 1) * (np + 1));
  double *fy = xmalloc(sizeof(double) * (n / 2 + 1) * (np + 1));
  double p_sum;

  for (j = 0; j <= n; j++)
    for (h = 0; h <= n; h++) {
      double acc = 0.;
      for (i = j; i <= n; i++)
        acc += fsp[i] * exp(orc_lchoose(i, j) + orc_lchoose(n - i, h - j) - orc_lchoose(n, h));
      pjh[j * (n + 1) + h] = acc;
    }
  for (b = 0; b <= n; b++)
    for (k = 0; k < n; k++) {
      double acc = 0.;
      q = b - (n - k) + 1;
      if (q > 0) acc += pjh[q * (n + 1) + k + 1] * (q / (double)(k + 1));
      if (b < k + 1) acc += pjh[b * (n + 1) + k + 1] * ((k + 1 - b) / (double)(k + 1));
      pbk[b * (n + 1) + k] = acc;
    }
  for (i = 0; i <= np; i++) {
    double log_ad = LOG_AD_MIN + i * g_log_ad_step, ad = exp(log_ad);
    p_sum = 0.;
    for (f = 0; f <= n; f++) {
      p[f] = p_kescape(n, n, ad) * fsp[f];
      for (k = 0; k < n; k++) p[f] += p_kescape(k, n, ad) * pbk[f * (n + 1) + k];
      p_sum += p[f];
    }
    if (!o->include_invariant) {
      p_sum -= p[0] + p[n];
      p[0] = p[n] = 0.;
    }
    for (f = 0; f <= n; f++) p[f] /= p_sum;
    if (o->asc_depth > 0 && o->ascbias_background_only == 0)
      orc_ascbias_adjust_expect(p, n, o->asc_min_freq, o->asc_depth);
    for (f = 0; f <= n; f++) y[f * (np + 1) + i] = p[f] == 0. ? log(DBL_MIN) : log(p[f]);
    for (f = 0; f < n - f; f++)
      fy[f * (np + 1) + i] = p[f] + p[n - f] == 0. ? log(DBL_MIN) : log(p[f] + p[n - f]);
    if (f == n - f) fy[f * (np + 1) + i] = p[f] == 0. ? log(DBL_MIN) : log(p[f]);
    x[i] = log_ad;
  }
  t->sample_size = n;
  t->spline = xmalloc(sizeof(orc_spline_t) * (n + 1));
  t->fspline = xmalloc(sizeof(orc_spline_t) * (n / 2 + 1));
  for (f = 0; f <= n; f++) estimate_spline(t->spline + f, x, y + f * (np + 1), np);
  for (f = 0; f <= n - f; f++) estimate_spline(t->fspline + f, x, fy + f * (np + 1), np);
  free(pjh); free(pbk); free(x); free(p); free(y); free(fy);
}

/* sm-spline.c:486-520 (with the per-depth asc variable of Q14 fixed) */
orc_table_t *orc_compute_tables(orc_scan_t *s, double **fsp, const orc_opts_t *o) {
  int i, maxd = 0;
  orc_table_t *t = xcalloc(s->n_depths, sizeof(orc_table_t));
  orc_set_spline_pts(o->spline_pts);
  for (i = 0; i < s->n_depths; i++) if (s->sample_depths[i] > maxd) maxd = s->sample_depths[i];
  orc_log_fact(maxd + 2); /* pre-grow: values are order-independent, avoids realloc under threads */
#pragma omp parallel for schedule(dynamic, 1) num_threads(o->n_threads > 0 ? o->n_threads : 1)
  for (i = 0; i < s->n_depths; i++) {
    int n = s->sample_depths[i];
    if (o->asc_depth > 0) {
      double *asc = orc_ascbias_adjust_background(fsp[i], n, o->asc_depth, o->asc_min_freq);
      sweep_model_fsp(t + i, asc, n, o);
      free(asc);
    } else {
      sweep_model_fsp(t + i, fsp[i], n, o);
    }
  }
  return t;
}

/* scan-chromosome.c:23-37 */
void orc_null_model(orc_scan_t *s, double **fsp) {
  int i;
  for (i = 0; i < s->n_snps; i++) {
    orc_snp_t *p = s->snps + i;
    int depth = s->sample_depths[p->depth_p];
    if (p->folded && p->obs_freq != depth - p->obs_freq)
      p->null_logl = log(fsp[p->depth_p][p->obs_freq] + fsp[p->depth_p][depth - p->obs_freq]);
    else
      p->null_logl = log(fsp[p->depth_p][p->obs_freq]);
  }
}

/* ---------------------------------------------------------- hot path */
/* sm-search.c:85-103 */
static double snp_likelihood(const orc_snp_t *p, double log_ad, const orc_table_t *tab) {
  const orc_table_t *t = tab + p->depth_p;
  double logl = p->folded ? orc_spline_interpolate(t->fspline + p->obs_freq, log_ad)
                          : orc_spline_interpolate(t->spline + p->obs_freq, log_ad);
  return logl - p->null_logl;
}

/* sm-search.c:105-150: nearest, then left descending, then right ascending */
static void sm_likelihood(orc_pt_t *r, const orc_snp_t *snps, const orc_table_t *tab, orc_stats_t *st) {
  double log_ad, acc;
  long long nt = 0;
  int i;
  acc = r->null_logl;
  log_ad = orc_logt(abs(r->sweep_pos - snps[r->nearest_snp].pos)) + r->lalpha;
  if (st) st->n_walks++;
  if (log_ad > LOG_AD_MAX) { r->sm_logl = acc; return; }
  acc += snp_likelihood(snps + r->nearest_snp, log_ad, tab);
  nt++;
  for (i = r->nearest_snp - 1; i >= r->window_start; i--) {
    log_ad = orc_logt(r->sweep_pos - snps[i].pos) + r->lalpha;
    if (log_ad > LOG_AD_MAX) break;
    acc += snp_likelihood(snps + i, log_ad, tab);
    nt++;
  }
  for (i = r->nearest_snp + 1; i <= r->window_end; i++) {
    log_ad = orc_logt(abs(snps[i].pos - r->sweep_pos)) + r->lalpha;
    if (log_ad > LOG_AD_MAX) break;
    acc += snp_likelihood(snps + i, log_ad, tab);
    nt++;
  }
  r->sm_logl = acc;
  if (st) st->n_terms += nt;
}

/* sm-search.c:269-300 */
void orc_search_maxalpha(orc_pt_t *r, const orc_snp_t *snps, const orc_table_t *tab, orc_stats_t *st) {
  double la, step, le, re;
  orc_pt_t tmp = *r, best = *r;
  best.sm_logl = -DBL_MAX;
  step = (LOG_AD_MAX - LOG_AD_MIN) / 10.0;
  for (la = LOG_AD_MIN; la <= LOG_AD_MAX; la += step) {
    tmp.lalpha = la;
    sm_likelihood(&tmp, snps, tab, st);
    if (tmp.sm_logl > best.sm_logl) best = tmp;
  }
  le = best.lalpha - step;
  if (le < LOG_AD_MIN) le = LOG_AD_MIN;
  re = best.lalpha + step;
  if (re > LOG_AD_MAX) re = LOG_AD_MAX;
  step = (re - le) / 15.;
  for (la = le + step; la < re; la += step) {
    tmp.lalpha = la;
    sm_likelihood(&tmp, snps, tab, st);
    if (tmp.sm_logl > best.sm_logl) best = tmp;
  }
  best.clr = 2.0 * (best.sm_logl - best.null_logl);
  *r = best;
  if (st) st->n_maxalpha++;
}

static orc_maxalpha_hook_t g_hook = NULL;
static void *g_hook_ctx = NULL;
void orc_set_maxalpha_hook(orc_maxalpha_hook_t hook, void *ctx) { g_hook = hook; g_hook_ctx = ctx; }

static void maxalpha(orc_pt_t *r, const orc_snp_t *snps, const orc_table_t *tab, orc_stats_t *st) {
  if (g_hook) { g_hook(r, snps, g_hook_ctx); if (st) st->n_maxalpha++; }
  else orc_search_maxalpha(r, snps, tab, st);
}

/* scan-chromosome.c:39-56 */
static int search_snppos(const orc_snp_t *snps, int n, double sweep_pos) {
  int i = 0, j = n, m;
  while (j - i > 1) {
    m = (i + j) / 2;
    if (snps[m].pos < sweep_pos) i = m; else j = m;
  }
  if (j == n) return n - 1;
  if ((sweep_pos - snps[i].pos) < (snps[j].pos - sweep_pos)) return i;
  return j;
}

/* scan-chromosome.c:58-101 */
void orc_init_scan_result(orc_pt_t *pt, int chr, const orc_snp_t *snps, const orc_chr_t *lim,
                          int eval_range, int pos, orc_stats_t *st) {
  int i, a, z;
  double acc;
  pt->chr = chr;
  pt->nearest_snp = lim->start_index + search_snppos(snps + lim->start_index, lim->n_snps, pos);
  /* Q3: global index compared with the per-chromosome count */
  for (i = pt->nearest_snp; i < lim->n_snps && snps[i].pos == pos; i++) pos++;
  pt->sweep_pos = pos;
  a = lim->start_index;
  z = lim->start_index + lim->n_snps - 1;
  if (pt->nearest_snp - eval_range < a) {
    pt->window_start = a;
    pt->window_end = a + eval_range * 2;
    if (pt->window_end > z) pt->window_end = z;
  } else if (pt->nearest_snp + eval_range > z) {
    pt->window_end = z;
    pt->window_start = z - eval_range * 2;
    if (pt->window_start < a) pt->window_start = a;
  } else {
    pt->window_start = pt->nearest_snp - eval_range;
    pt->window_end = pt->nearest_snp + eval_range;
  }
  pt->n_snps = pt->window_end - pt->window_start + 1;
  acc = 0.;
  for (i = pt->window_start; i <= pt->window_end; i++) acc += snps[i].null_logl;
  pt->null_logl = acc;
  if (st) st->n_null += pt->n_snps;
  pt->sm_logl = -DBL_MAX;
  pt->lalpha = LOG_AD_MAX;
  pt->permute_n = pt->permute_p = pt->permute_finished = 0;
  pt->scan_running = 0;
  pt->permute_clr = NULL;
  pt->clr = 0.;
}

/* scan-chromosome.c:103-139, recursion unrolled */
orc_pt_t orc_search_maxpos(int chr, int start_pos, int end_pos, const orc_snp_t *snps,
                           const orc_chr_t *lim, int eval_range, int bp_resl,
                           const orc_table_t *tab, orc_stats_t *st) {
  orc_pt_t s, e, m;
  int iter = 0;
  orc_init_scan_result(&s, chr, snps, lim, eval_range, start_pos, st);
  maxalpha(&s, snps, tab, st);
  orc_init_scan_result(&e, chr, snps, lim, eval_range, end_pos, st);
  maxalpha(&e, snps, tab, st);
  while (e.sweep_pos - s.sweep_pos > bp_resl) {
    if (++iter > 64) { fprintf(stderr, "oracle: position bisection did not converge\n"); abort(); }
    orc_init_scan_result(&m, chr, snps, lim, eval_range, (s.sweep_pos + e.sweep_pos) / 2, st);
    maxalpha(&m, snps, tab, st);
    if ((s.clr + m.clr) >= (e.clr + m.clr)) e = m; else s = m;
  }
  if (st) st->n_gp++;
  return s.clr > e.clr ? s : e;
}

typedef struct { int chr, start, end; } cell_t;

/* scan-chromosome.c:162-216: the cell sequence one scan thread walks */
static cell_t *scan_cells(const orc_scan_t *s, int G, int *n_out) {
  int chm = 0, pos, n = 0, cap = 64;
  cell_t *c = xmalloc(sizeof(cell_t) * cap);
  if (s->n_chr == 0) { *n_out = 0; return c; }
  pos = s->chr[0].start_pos;
  for (;;) {
    if (pos >= s->chr[chm].bp_length) {
      chm++;
      if (chm == s->n_chr) break;
      pos = s->chr[chm].start_pos;
    }
    if (n == cap) { cap *= 2; c = realloc(c, sizeof(cell_t) * cap); }
    c[n].chr = chm;
    c[n].start = pos;
    c[n].end = pos + G > s->chr[chm].bp_length ? s->chr[chm].bp_length : pos + G;
    n++;
    pos += G;
  }
  *n_out = n;
  return c;
}

typedef struct { orc_pt_t p; int seq; } keyed_pt_t;
static int pt_cmp(const void *va, const void *vb) {
  const keyed_pt_t *a = va, *b = vb;
  if (a->p.chr != b->p.chr) return a->p.chr < b->p.chr ? -1 : 1;
  if (a->p.sweep_pos != b->p.sweep_pos) return a->p.sweep_pos < b->p.sweep_pos ? -1 : 1;
  return a->seq - b->seq; /* scan-chromosome.c:218-225 under a stable sort */
}

static void stats_add(orc_stats_t *a, const orc_stats_t *b) {
  a->n_terms += b->n_terms; a->n_null += b->n_null; a->n_walks += b->n_walks;
  a->n_maxalpha += b->n_maxalpha; a->n_gp += b->n_gp; a->negj += b->negj;
}

/* scan-chromosome.c:228-265 (cells evaluated in any order; results identical) */
void orc_scan_chromosome(orc_scan_t *s, const orc_table_t *tab, const orc_opts_t *o, orc_stats_t *st) {
  int n, i;
  cell_t *c = scan_cells(s, o->large_grid_sp, &n);
  keyed_pt_t *kp = xmalloc(sizeof(keyed_pt_t) * (n ? n : 1));
  orc_stats_t tot = {0};
#pragma omp parallel num_threads(o->n_threads > 0 ? o->n_threads : 1)
  {
    orc_stats_t loc = {0};
#pragma omp for schedule(dynamic, 1)
    for (i = 0; i < n; i++) {
      kp[i].p = orc_search_maxpos(c[i].chr, c[i].start, c[i].end, s->snps, s->chr + c[i].chr,
                                  o->eval_range, o->bp_resl, tab, &loc);
      kp[i].seq = i;
    }
#pragma omp critical
    stats_add(&tot, &loc);
  }
  qsort(kp, n, sizeof(keyed_pt_t), pt_cmp);
  free(s->pts);
  s->pts = xmalloc(sizeof(orc_pt_t) * (n ? n : 1));
  for (i = 0; i < n; i++) s->pts[i] = kp[i].p;
  s->n_pts = n;
  free(kp);
  free(c);
  if (st) stats_add(st, &tot);
}

/* CPU-baseline sample (bench.py): n_sample scan cells spread evenly over the genome
   (every k-th cell of scan_chromosome's sequence; aligned: the G-aligned, unclipped cell
   a permutation trial evaluates for the same point, scan-chromosome.c:481-486) evaluated on
   snps with o->n_threads threads; returns the wall seconds and the cells evaluated */
double orc_sample_cells(orc_scan_t *s, const orc_table_t *tab, const orc_opts_t *o, const orc_snp_t *snps,
                        int n_sample, int aligned, int *n_done) {
  int n, i, m = 0;
  cell_t *c = scan_cells(s, o->large_grid_sp, &n);
  int *pick = xmalloc(sizeof(int) * (n_sample > 0 ? n_sample : 1));
  struct timespec t0, t1;
  for (i = 0; i < n_sample && n > 0; i++) {
    const int k = (int)(((long long)i * n) / n_sample);
    if (m == 0 || pick[m - 1] != k) pick[m++] = k;
  }
  if (aligned)
    for (i = 0; i < m; i++) {
      cell_t *x = c + pick[i];
      x->start -= x->start % o->large_grid_sp;
      x->end = x->start + o->large_grid_sp;
    }
  clock_gettime(CLOCK_MONOTONIC, &t0);
#pragma omp parallel for schedule(dynamic, 1) num_threads(o->n_threads > 0 ? o->n_threads : 1)
  for (i = 0; i < m; i++) {
    const cell_t *x = c + pick[i];
    orc_stats_t loc = {0};
    (void)orc_search_maxpos(x->chr, x->start, x->end, snps, s->chr + x->chr, o->eval_range, o->bp_resl, tab, &loc);
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(pick); free(c);
  if (n_done) *n_done = m;
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* scan-chromosome.c:336-389, with Q9 (negative j) repaired as j -= k - n */
void orc_block_permute(orc_snp_t *p, const orc_snp_t *snps, int n, double nbp, double width_mb,
                       orc_rand_t *g, orc_stats_t *st) {
  int i = 0, j, k;
  memcpy(p, snps, sizeof(orc_snp_t) * n);
  while (i < n) {
    int r1 = orc_rand(g), r2;
    j = r1 / (2147483647 + 1.0) * n;
    r2 = orc_rand(g);
    if (r2 == 0) k = n; /* Q10: log(0) guard */
    else k = j + (int)(-1.0 / nbp * log(r2 / (2147483647 + 1.0)));
    while (k < n && snps[k].chr == snps[j].chr && snps[k].pos - snps[j].pos < width_mb * 1e6) k++;
    if (i + (k - j) >= n) k = n;
    if (k > n) {
      if (st) st->negj++;
      j -= k - n;
      k = n;
    }
    while (j < k && i < n && j < n) {
      orc_snp_t t = p[i];
      p[i].obs_freq = p[j].obs_freq; p[i].depth_p = p[j].depth_p;
      p[i].folded = p[j].folded; p[i].null_logl = p[j].null_logl;
      p[j].obs_freq = t.obs_freq; p[j].depth_p = t.depth_p;
      p[j].folded = t.folded; p[j].null_logl = t.null_logl;
      i++;
      j++;
    }
  }
}

/* scan-chromosome.c:391-652 with --n-threads=1 semantics: lockstep trials,
   points evaluated (in parallel if n_threads > 1), then the prune pass in
   ascending point order so the rand() stream is exactly the 1-thread one. */
/* the rand() stream, seeded once per process as srand() in init_options (fscl.c:135): it
   continues across orc_scan_permute calls; orc_reseed restarts it */
static orc_rand_t g_rng;
static int g_rng_seeded = 0;
void orc_reseed(unsigned seed) { orc_srand(&g_rng, seed); g_rng_seeded = 1; }

/* The product's throughput mode (include/fscl_amd.h, fscl_amd_set_permute_mode; DESIGN.md
   §5.4) restated serially: the reference's trial loop and prune test above, with trial t's
   permutation drawn from the glibc stream seeded by orc_tp_trial_seed(seed, t) and point i's
   prune draw in trial t = orc_tp_prune_rand(seed, t, i).  Not the reference's stream, so this
   pins the product's own non-parity mode (its definition, not the reference's numbers). */
static uint64_t orc_mix64(uint64_t z) { /* splitmix64 output function */
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static unsigned orc_tp_trial_seed(uint64_t seed, long t) { return (unsigned)(orc_mix64(seed ^ orc_mix64((uint64_t)t + 1)) >> 32); }
static int orc_tp_prune_rand(uint64_t seed, long t, int i) {
  return (int)(orc_mix64(orc_mix64(seed ^ 0x632BE59BD9B4E019ull) ^ ((uint64_t)(uint32_t)t << 32 | (uint32_t)i)) >> 33);
}

void orc_scan_permute(orc_scan_t *s, const orc_table_t *tab, const orc_opts_t *o, orc_stats_t *st) {
  orc_rand_t *const gp = &g_rng;
  orc_snp_t *ps = xmalloc(sizeof(orc_snp_t) * s->n_snps);
  int *act = xmalloc(sizeof(int) * (s->n_pts ? s->n_pts : 1)), n_act = s->n_pts, i, k, trial = -1;
  double *clr = xmalloc(sizeof(double) * (s->n_pts ? s->n_pts : 1));
  const int save = CLR_NULL_DIST_SAVE; /* scan-chromosome.c:240,496 */
  orc_stats_t tot = {0};
  if (!g_rng_seeded) orc_reseed(0xFD821A6);
  if (!o->throughput) (void)orc_rand(gp); /* scan-chromosome.c:440: the usleep() draw of the one thread */
  for (i = 0; i < s->n_pts; i++) {
    act[i] = i;
    if (!s->pts[i].permute_clr) s->pts[i].permute_clr = xmalloc(sizeof(float) * CLR_NULL_DIST_SAVE);
  }
  for (;;) {
    if (o->throughput) { /* trial + 1's own stream (nothing else draws from it) */
      orc_rand_t tg;
      orc_srand(&tg, orc_tp_trial_seed(o->throughput_seed, trial + 1));
      orc_block_permute(ps, s->snps, s->n_snps, o->permute_nbp, o->scan_width_mb, &tg, &tot);
    } else {
      orc_block_permute(ps, s->snps, s->n_snps, o->permute_nbp, o->scan_width_mb, gp, &tot);
    }
    trial++;
    for (i = k = 0; i < n_act; i++)
      if (!s->pts[act[i]].permute_finished) act[k++] = act[i];
    n_act = k;
    if (n_act == 0 || trial > o->n_permute) break;
#pragma omp parallel num_threads(o->n_threads > 0 ? o->n_threads : 1)
    {
      orc_stats_t loc = {0};
#pragma omp for schedule(dynamic, 1)
      for (i = 0; i < n_act; i++) {
        const orc_pt_t *q = s->pts + act[i];
        int start = q->sweep_pos - (q->sweep_pos % o->large_grid_sp); /* Q5 */
        orc_pt_t mx = orc_search_maxpos(q->chr, start, start + o->large_grid_sp, ps, s->chr + q->chr,
                                        o->eval_range, o->bp_resl, tab, &loc);
        clr[i] = mx.clr;
      }
#pragma omp critical
      stats_add(&tot, &loc);
    }
    for (i = 0; i < n_act; i++) {
      orc_pt_t *q = s->pts + act[i];
      if (clr[i] >= q->clr) {
        q->permute_p++;
        if (q->permute_p >= 20 &&
            q->permute_p / (double)q->permute_n >=
                (o->throughput ? orc_tp_prune_rand(o->throughput_seed, trial, act[i]) : orc_rand(gp)) / (2147483647 + 1.0))
          q->permute_finished = 1; /* Q7 */
      }
      if (q->permute_n < save) q->permute_clr[q->permute_n] = (float)clr[i];
      q->permute_n++;
      if (clr[i] < 0 || clr[i] > 1000000 || isnan(clr[i]))
        fprintf(stderr, "%d\t%d\t%g\n", q->chr, q->sweep_pos - (q->sweep_pos % o->large_grid_sp), clr[i]);
    }
  }
  free(ps); free(act); free(clr);
  if (st) stats_add(st, &tot);
}

/* scan-chromosome.c:666-750 */
int orc_scan_output(const char *fname, orc_scan_t *s, int max_only, int n_permute, const char *label) {
  FILE *f = fname ? fopen(fname, "w") : stdout;
  int i;
  const orc_pt_t *best;
  double max_clr;
  if (!f) { fprintf(stderr, "Can't open output file \"%s\"\n", fname); return -1; }
  if (s->n_pts == 0) { if (fname) fclose(f); return 0; }
  best = s->pts;
  max_clr = s->pts[0].clr;
  for (i = 1; i < s->n_pts; i++)
    if (s->pts[i].clr > max_clr) { max_clr = s->pts[i].clr; best = s->pts + i; }
  if (max_only) {
    if (label) fprintf(f, "%s\t", label);
    fprintf(f, "%s\t%d\t%1.2f\t%1.3e\t%d\t%d\t%d\n", s->chr[best->chr].name, best->sweep_pos, max_clr,
            exp(best->lalpha), best->n_snps, s->snps[best->window_start].pos, s->snps[best->window_end].pos);
  } else if (n_permute > 0) {
    for (i = 0; i < s->n_pts; i++) {
      const orc_pt_t *q = s->pts + i;
      double pv = q->permute_p < 2 ? 1.0 / q->permute_n : (q->permute_p - 1.0) / (double)(q->permute_n - 1.0);
      if (label) fprintf(f, "%s\t", label);
      fprintf(f, "%s\t%d\t%1.2f\t%1.3e\t%d\t%d\t%1.3f\n", s->chr[q->chr].name, q->sweep_pos, q->clr,
              exp(q->lalpha), q->permute_p, q->permute_n, -log10(pv));
    }
  } else {
    for (i = 0; i < s->n_pts; i++) {
      const orc_pt_t *q = s->pts + i;
      if (label) fprintf(f, "%s\t", label);
      fprintf(f, "%s\t%d\t%1.2f\t%1.3e\t%d\t%d\t%d\n", s->chr[q->chr].name, q->sweep_pos, q->clr,
              exp(q->lalpha), q->n_snps, s->snps[q->window_start].pos, s->snps[q->window_end].pos);
    }
  }
  if (fname) fclose(f);
  return 0;
}

void orc_default_opts(orc_opts_t *o) {
  memset(o, 0, sizeof(*o));
  o->spline_pts = 200;      /* fscl.c:167 */
  o->minimum_depth = 5;     /* fscl.c:149, :188 */
  o->asc_min_freq = 1;      /* fscl.c:145 */
  o->permute_nbp = 0.1;     /* fscl.c:147 */
  o->scan_width_mb = 1.0;   /* fscl.c:160 */
  o->large_grid_sp = 100000;/* fscl.c:159 */
  o->eval_range = 81920;    /* fscl.c:175 */
  o->bp_resl = 128;         /* fscl.c:174 */
  o->n_threads = 1;
}

static void free_tables(orc_table_t *t, int nd) {
  int i, f;
  for (i = 0; i < nd; i++) {
    for (f = 0; f <= t[i].sample_size; f++) { free(t[i].spline[f].knots); free(t[i].spline[f].coef); }
    for (f = 0; f <= t[i].sample_size / 2; f++) { free(t[i].fspline[f].knots); free(t[i].fspline[f].coef); }
    free(t[i].spline); free(t[i].fspline);
  }
  free(t);
}

void orc_free_scan(orc_scan_t *s) {
  int i;
  if (!s) return;
  for (i = 0; i < s->n_pts; i++) free(s->pts[i].permute_clr);
  for (i = 0; i < s->n_chr; i++) free(s->chr[i].name);
  free(s->pts); free(s->chr); free(s->snps); free(s->sample_depths); free(s);
}

static int orc_float_compare(const void *va, const void *vb) { /* scan-chromosome.c:654-658 */
  const float a = *(const float *)va, b = *(const float *)vb;
  if (a < b) return -1;
  if (a > b) return 1;
  return 0;
}

/* scan-chromosome.c:753-796: <fname>-nulldist, each point's saved permutation CLRs sorted
   (the reference writes it from its SIGINT handler, :557-569; here at the end of the run) */
int orc_output_nulldist(const char *fname, orc_scan_t *s) {
  char *fn = xmalloc(strlen(fname) + 20);
  FILE *f;
  int i, j;
  sprintf(fn, "%s-nulldist", fname);
  f = fopen(fn, "w");
  free(fn);
  if (!f) return -1;
  fprintf(f, "chr\tpos\tCLR\talpha\tp\tn");
  for (j = 0; j < CLR_NULL_DIST_SAVE; j++) fprintf(f, "\t%1.4f", j / (double)CLR_NULL_DIST_SAVE);
  fprintf(f, "\n");
  for (i = 0; i < s->n_pts; i++) {
    orc_pt_t *q = s->pts + i;
    const int np = CLR_NULL_DIST_SAVE < q->permute_n ? CLR_NULL_DIST_SAVE : q->permute_n;
    if (q->permute_clr) qsort(q->permute_clr, np, sizeof(float), orc_float_compare);
    fprintf(f, "%s\t%d\t%1.3f\t%1.3e\t%d\t%d", s->chr[q->chr].name, q->sweep_pos, q->clr, exp(q->lalpha),
            q->permute_p, q->permute_n);
    for (j = 0; j < np && q->permute_clr; j++) fprintf(f, "\t%1.2f", (double)q->permute_clr[j]);
    fprintf(f, "\n");
  }
  fclose(f);
  return 0;
}

/* fscl.c:316-337 */
int orc_run_snpfile(const char *snp_fname, const char *out_fname, const orc_opts_t *o,
                    const char *label, orc_stats_t *st) {
  orc_scan_t *s;
  double **fsp;
  orc_table_t *tab;
  int i;
  orc_init_log_table();
  orc_reseed(0xFD821A6); /* init_options, fscl.c:135: a fresh process */
  s = orc_load_snp_input(snp_fname, o->include_invariant, o->minimum_depth);
  if (!s) return -1;
  fsp = orc_background_fsp(s, o->force_neutral, o->include_invariant);
  tab = orc_compute_tables(s, fsp, o);
  orc_null_model(s, fsp);
  orc_scan_chromosome(s, tab, o, st);
  if (o->n_permute > 0) orc_scan_permute(s, tab, o, st);
  orc_scan_output(out_fname, s, o->max_only, o->n_permute, label);
  if (getenv("ORC_DUMP_POINTS")) orc_dump_points(getenv("ORC_DUMP_POINTS"), s);
  if (getenv("ORC_NULLDIST")) orc_output_nulldist(out_fname, s);
  free_tables(tab, s->n_depths);
  for (i = 0; i < s->n_depths; i++) free(fsp[i]);
  free(fsp);
  orc_free_scan(s);
  return 0;
}

int orc_dump_points(const char *fname, const orc_scan_t *s) {
  FILE *f = fopen(fname, "w");
  int i;
  if (!f) return -1;
  for (i = 0; i < s->n_pts; i++) {
    const orc_pt_t *q = s->pts + i;
    fprintf(f, "%d\t%d\t%a\t%a\t%a\t%a\t%d\t%d\t%d\t%d\t%d\t%d\n", q->chr, q->sweep_pos, q->clr,
            q->lalpha, q->sm_logl, q->null_logl, q->nearest_snp, q->window_start, q->window_end,
            q->permute_p, q->permute_n, q->permute_finished);
  }
  fclose(f);
  return 0;
}
