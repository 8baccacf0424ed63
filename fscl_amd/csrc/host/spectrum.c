/* spectrum.c -- log-factorials, background site-frequency spectra and the
 * K-of-M ascertainment-bias correction (host setup of the scan path).
 *
 *   fh_log_fact / lchoose        sm-spline.c:18-46
 *   background_fsp               background-fsp.c:182-316 (+ neutral_spectra :19-51)
 *   output_background_fs         background-fsp.c:318-336
 *   ascbias_adjust_background    asc-bias.c:27-95
 *   ascbias_adjust_expect        asc-bias.c:97-109
 *
 * Floating-point expressions keep the reference's operation order; loops over
 * independent outputs run on OpenMP threads.
 */
#include <errno.h>
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fscl_host.h"

/* lf[i] = lf[i-1] + log(i) accumulated from lf[1] = 0: each entry depends only
   on i, so the table can be grown once up front and then read from threads */
static double *g_lf = NULL;
static int g_lf_n = 0; /* entries 0..g_lf_n valid */
static pthread_mutex_t g_lf_lock = PTHREAD_MUTEX_INITIALIZER;

void fh_log_fact_reserve(int n) {
  pthread_mutex_lock(&g_lf_lock);
  if (n > g_lf_n) {
    int i, from = g_lf_n < 1 ? 1 : g_lf_n;
    g_lf = fh_realloc(g_lf, sizeof(double) * (n + 1), "log_fact");
    g_lf[0] = 0.0;
    if (g_lf_n < 1) g_lf[1] = 0.0 + log(1);
    for (i = from + 1; i <= n; i++) g_lf[i] = g_lf[i - 1] + log(i);
    g_lf_n = n;
  }
  pthread_mutex_unlock(&g_lf_lock);
}

double fh_log_fact(int n) {
  if (n < 0) return -DBL_MAX;
  if (n == 0 || n == 1) return 0.;
  if (n > g_lf_n) fh_log_fact_reserve(n < 1024 ? 1024 : n);
  return g_lf[n];
}

double lchoose(int n, int k) {
  if (n == 0 && k == 0) return 0.;
  if (k > n || n == 0) return -DBL_MAX;
  return fh_log_fact(n) - fh_log_fact(k) - fh_log_fact(n - k);
}

/* background-fsp.c:19-51 */
static double **neutral_spectra(scan_t *s) {
  int n_inv = 0, n_fix = 0, i, k;
  double **fsp = fh_malloc(sizeof(double *) * s->n_depths, "neutral spectra");
  for (i = 0; i < s->n_snps; i++) {
    n_inv += s->snps[i].obs_freq == 0;
    n_fix += s->snps[i].obs_freq == s->sample_depths[s->snps[i].depth_p];
  }
  for (i = 0; i < s->n_depths; i++) {
    const int m = s->sample_depths[i];
    const int n_seg = s->n_snps - n_fix - n_inv;
    double seg_sum = 0.;
    fsp[i] = fh_malloc(sizeof(double) * (m + 1), "neutral spectra");
    fsp[i][0] = n_inv;
    fsp[i][m] = n_fix;
    for (k = 1; k < m; k++) seg_sum += 1 / (double)k;
    for (k = 1; k < m; k++) fsp[i][k] = (1. / (double)k) / seg_sum * n_seg;
    for (k = 0; k <= m; k++) fsp[i][k] /= (double)s->n_snps;
  }
  return fsp;
}

/* -b: reads the format output_background_fs writes ("depth f_0 ... f_depth");
   background-fsp.c:127-180 cannot read it (stale index, expects depth values) */
static double **load_spectra(scan_t *s, const char *fname) {
  FILE *f = fopen(fname, "r");
  double **fsp = fh_calloc(s->n_depths, sizeof(double *), "background spectra");
  char *line = NULL;
  size_t cap = 0;
  int i;
  if (!f) logmsg(MSG_FATAL, "\nCan't background frequency spectrum file \"%s\" (%s)", fname, strerror(errno));
  while (getline(&line, &cap, f) >= 0) {
    char *p = line, *e;
    long depth;
    int j, d;
    if (line[0] == '#' || line[0] == '\n' || line[0] == 0) continue;
    depth = strtol(p, &e, 10);
    if (e == p) continue;
    for (d = 0; d < s->n_depths && s->sample_depths[d] != depth; d++) {}
    if (d == s->n_depths) {
      logmsg(MSG_STATUS, "Frequency spectrum for %ld classes not required by snp data.", depth);
      continue;
    }
    fsp[d] = fh_realloc(fsp[d], sizeof(double) * (depth + 1), "background spectra");
    for (j = 0, p = e; j <= depth; j++, p = e) {
      fsp[d][j] = strtod(p, &e);
      if (e == p) logmsg(MSG_FATAL, "\nError: Frequency spectrum on line for depth %ld has %d classes, needs %ld.",
                         depth, j, depth + 1);
    }
  }
  free(line);
  fclose(f);
  for (i = 0; i < s->n_depths; i++)
    if (!fsp[i])
      logmsg(MSG_FATAL, "\nError: data requires background frequency spectrum for sample depth %d, not found %s",
             s->sample_depths[i], fname);
  return fsp;
}

double **background_fsp(scan_t *s, int force_neutral_spectrum, char *background_fsfname, int include_invariant) {
  int m, k, i, max_depth = -1000;
  double **fsp, *tmp, sum;
  if (force_neutral_spectrum) return neutral_spectra(s);
  if (background_fsfname) return load_spectra(s, background_fsfname);
  logmsg(MSG_STATUS, "Estimating background site frequency spectrum....   ");
  fsp = fh_malloc(sizeof(double *) * s->n_depths, "background spectra");
  for (m = 0; m < s->n_depths; m++) {
    fsp[m] = fh_calloc(s->sample_depths[m] + 1, sizeof(double), "background spectra");
    if (s->sample_depths[m] > max_depth) max_depth = s->sample_depths[m];
  }
  fh_log_fact_reserve(max_depth + 2);
  logmsg(MSG_STATUS, "%d distinct sample depths observed. Maximum sample depth is %d haplotypes.", s->n_depths,
         max_depth);
  /* sites at the maximum depth only; an unfolded site adds 1 to class n-f
     (Q1: the reference's mirrored polarity, background-fsp.c:226-233) */
  tmp = fh_calloc(max_depth + 1, sizeof(double), "background spectra");
  for (i = 0; i < s->n_snps; i++) {
    const snp_t *p = s->snps + i;
    const int depth = s->sample_depths[p->depth_p];
    double wa, wd;
    if (depth != max_depth) continue;
    if (p->folded) {
      if (p->obs_freq == 0) { wa = 1; wd = 0; }
      else if (p->obs_freq == depth) { wa = 0; wd = 1; }
      else { wa = 1. / (p->obs_freq); wd = 1. / (depth - p->obs_freq); }
    } else { wd = 1.; wa = 0.; }
    tmp[p->obs_freq] += wa / (wa + wd);
    tmp[depth - p->obs_freq] += wd / (wa + wd);
  }
  sum = 0.;
  for (k = 0; k <= max_depth; k++) sum += tmp[k];
  for (k = 0; k <= max_depth; k++) tmp[k] /= sum;
  logmsg(MSG_STATUS, "Total SNPs observed at max depth %d is %1.1f (%1.1f%%)", max_depth, sum,
         sum / (double)s->n_snps * 100.);
  /* hypergeometric down-sampling to every depth (background-fsp.c:72-88) */
#pragma omp parallel for schedule(dynamic, 1)
  for (m = 0; m < s->n_depths; m++) {
    const int n = s->sample_depths[m], N = max_depth;
    double *d = fsp[m], ssum = 0.;
    int a, b;
    for (a = include_invariant ? 0 : 1; a <= N; a++)
      for (b = include_invariant ? 0 : 1; b <= a && (include_invariant ? b <= n : b < n); b++)
        d[b] += exp(lchoose(a, b) + lchoose(N - a, n - b) - lchoose(N, n)) * tmp[a];
    for (b = 0; b <= n; b++) ssum += d[b];
    for (b = 0; b <= n; b++) d[b] /= ssum;
  }
  free(tmp);
  logmsg(MSG_STATUS, "\nDone estimating background frequency spectra.");
  return fsp;
}

void output_background_fs(char *fname, scan_t *s, double **fsp) {
  FILE *f = fopen(fname, "w");
  int i, j;
  if (!f)
    logmsg(MSG_FATAL, "\nCan't open background frequency spectrum file \"%s\" for output. (%s)", fname,
           strerror(errno));
  for (i = 0; i < s->n_depths; i++) {
    fprintf(f, "%d", s->sample_depths[i]);
    for (j = 0; j <= s->sample_depths[i]; j++) fprintf(f, "\t%1.6f", fsp[i][j]);
    fprintf(f, "\n");
  }
  fclose(f);
}

/* asc-bias.c:12-25: P(a site with k of n derived alleles is ascertained in a
   sub-sample of d with at least min_obs copies of each allele) */
static double ascprob_subsample(int k, int d, int min_obs, int n) {
  double no_asc = 0.;
  int i;
  for (i = 0; i < min_obs; i++)
    no_asc += exp(lchoose(k, d - i) + lchoose(n - k, i)) + exp(lchoose(n - k, d - i) + lchoose(k, i));
  no_asc /= exp(lchoose(n, d));
  return 1.0 - no_asc;
}

double *ascbias_adjust_background(double *bsf, int n, int asc_depth, int min_obs) {
  double *asc = fh_malloc(sizeof(double) * (n + 1), "asc"), *adj = fh_malloc(sizeof(double) * (n + 1), "asc");
  double asc_sum = 0., adj_sum = 0.;
  int i;
  asc[0] = asc[n] = 0.;
  for (i = 1; i < n; i++) {
    asc[i] = ascprob_subsample(i, asc_depth, min_obs, n);
    asc_sum += asc[i];
  }
  for (i = 1; i < n; i++) asc[i] /= asc_sum;
  adj[0] = adj[n] = 0.;
  for (i = 1; i < n; i++) {
    adj[i] = bsf[i] / asc[i];
    adj_sum += adj[i];
  }
  for (i = 1; i < n; i++) adj[i] /= adj_sum;
  free(asc);
  return adj;
}

void ascbias_adjust_expect(double *fsp, int n, int min_obs, int d) {
  double asc_sum = 0;
  int i;
  for (i = 0; i <= n; i++) asc_sum += fsp[i] * ascprob_subsample(i, d, min_obs, n);
  for (i = 0; i <= n; i++) fsp[i] = fsp[i] * ascprob_subsample(i, d, min_obs, n) / asc_sum;
}
