/* tables.c -- sweep-model likelihood tables: for every sample depth n and
 * every observed class f, a natural cubic spline of log P(f | log(alpha d))
 * over log(alpha d) in [-20, 4] (sm-spline.c:316-520).
 *
 * Bit-compatible with the reference: same expression order for every value,
 * and the reference's banded Gauss elimination (sm-spline.c:63-118) run on a
 * band image of the matrix instead of the dense 4(n+1)^2 array -- every entry
 * the dense solver reads lies in the band, entries it writes
 * outside the band are never read.  Independent outputs (pjh rows, knots,
 * splines) run on OpenMP threads.
 */
#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fscl_host.h"

__attribute__((weak)) int spline_pts = N_SPLINE_KNOTS; /* fscl.c:34 defines it when linked */
double log_ad_step = 24.0 / 201.0;                      /* sm-spline.c:16 */

double fh_log_ad_step(void) { return log_ad_step; }

double spline_interpolate(spline_t *spf, double x) {
  int i = (x - LOG_AD_MIN) / log_ad_step;
  if (i >= spf->n) i = spf->n - 1;
  if (i < 0) i = 0;
  return x * (spf->coef[i][0] * x * x + spf->coef[i][1] * x + spf->coef[i][2]) + spf->coef[i][3];
}

/* band image: row r keeps columns [r - BL, r - BL + BW) */
#define BL 8
#define BW 32
#define BAND(m, r, c) (m)[(size_t)(r) * BW + ((c) - (r) + BL)]
static inline double band_get(const double *m, int r, int c) {
  const int o = c - r + BL;
  return (o >= 0 && o < BW) ? m[(size_t)r * BW + o] : 0.0;
}

/* sm-spline.c:63-118 on the band image */
static void solve_band(double *b, double *m, double *v, int n) {
  int i, j, k;
  double f;
  for (i = 0; i < n; i++) {
    if (fabs(BAND(m, i, i)) < 1e-20) {
      int mx = i;
      for (j = i + 1; j < n && j <= i + BL; j++) {
        const double a = fabs(band_get(m, j, i));
        if (a > 0 && (mx == i || fabs(a - 1) < fabs(fabs(band_get(m, mx, i)) - 1))) mx = j;
      }
      if (mx == i)
        logmsg(MSG_FATAL, "Ill conditioned matrix while trying to estimate spline functions to approximate "
                          "sweep model likelihoods.");
      for (k = i - BL; k < i - BL + BW; k++)
        if (k >= 0 && k < n) BAND(m, i, k) += band_get(m, mx, k);
      v[i] += v[mx];
    }
    f = BAND(m, i, i);
    for (k = i; k < i + 8 && k < n; k++) BAND(m, i, k) /= f;
    v[i] /= f;
    for (j = i + 1; j < i + 8 && j < n; j++) {
      f = BAND(m, j, i);
      for (k = i; k < i + 8 && k < n; k++) BAND(m, j, k) = BAND(m, j, k) - BAND(m, i, k) * f;
      v[j] = v[j] - v[i] * f;
    }
  }
  for (i = n - 1; i >= 0;) {
    if (fabs(BAND(m, i, i)) < 1e-10) {
      logmsg(MSG_WARN, "Warning: setting a spline coefficient %d to zero", i);
      b[i--] = 0;
      continue;
    }
    b[i] = v[i];
    for (k = i + 1; k < i + 8 && k < n; k++) b[i] -= BAND(m, i, k) * b[k];
    i--;
  }
}

/* sm-spline.c:120-220: natural cubic spline through (x[0..n], y[0..n]),
   n intervals; second derivative 0 at both ends */
static spline_t *estimate_spline(const double *x, const double *y, int n, double *m, double *v, double *b) {
  const int dim = 4 * (n + 1);
  int i, j, k;
  spline_t *sp;
  memset(m, 0, sizeof(double) * (size_t)dim * BW);
  memset(v, 0, sizeof(double) * dim);
  memset(b, 0, sizeof(double) * dim);
  BAND(m, 0, 0) = 6 * x[0];
  BAND(m, 0, 1) = 2;
  for (i = 1, j = 0, k = 0; k < n - 1; i += 4, j += 4, k++) {
    /* value at both knots of interval k, C1 and C2 continuity at its right knot */
    BAND(m, i, j) = x[k] * x[k] * x[k];
    BAND(m, i, j + 1) = x[k] * x[k];
    BAND(m, i, j + 2) = x[k];
    BAND(m, i, j + 3) = 1.;
    v[i] = y[k];
    BAND(m, i + 1, j) = x[k + 1] * x[k + 1] * x[k + 1];
    BAND(m, i + 1, j + 1) = x[k + 1] * x[k + 1];
    BAND(m, i + 1, j + 2) = x[k + 1];
    BAND(m, i + 1, j + 3) = 1;
    v[i + 1] = y[k + 1];
    BAND(m, i + 2, j) = 3 * x[k + 1] * x[k + 1];
    BAND(m, i + 2, j + 1) = 2 * x[k + 1];
    BAND(m, i + 2, j + 2) = 1;
    BAND(m, i + 2, j + 4) = -3 * x[k + 1] * x[k + 1];
    BAND(m, i + 2, j + 5) = -2 * x[k + 1];
    BAND(m, i + 2, j + 6) = -1;
    BAND(m, i + 3, j) = 6 * x[k + 1];
    BAND(m, i + 3, j + 1) = 2;
    BAND(m, i + 3, j + 4) = -6 * x[k + 1];
    BAND(m, i + 3, j + 5) = -2;
  }
  BAND(m, i, j) = x[k] * x[k] * x[k];
  BAND(m, i, j + 1) = x[k] * x[k];
  BAND(m, i, j + 2) = x[k];
  BAND(m, i, j + 3) = 1;
  v[i] = y[k];
  BAND(m, i + 1, j) = x[n] * x[n] * x[n];
  BAND(m, i + 1, j + 1) = x[n] * x[n];
  BAND(m, i + 1, j + 2) = x[n];
  BAND(m, i + 1, j + 3) = 1;
  v[i + 1] = y[n];
  BAND(m, i + 2, j) = 6 * x[n];
  BAND(m, i + 2, j + 1) = 2;

  solve_band(b, m, v, 4 * n);

  sp = fh_malloc(sizeof(spline_t), "spline");
  sp->n = n;
  sp->knot_points = fh_malloc(sizeof(double) * (n + 1), "spline");
  sp->coef = fh_malloc(sizeof(double *) * n, "spline");
  sp->coef[0] = fh_malloc(sizeof(double) * 4 * n, "spline");
  for (i = 1; i < n; i++) sp->coef[i] = sp->coef[i - 1] + 4;
  for (i = 0; i < n; i++) {
    sp->knot_points[i] = x[i];
    for (k = 0; k < 4; k++) sp->coef[i][k] = b[i * 4 + k];
  }
  sp->knot_points[n] = x[n];
  return sp;
}

/* sm-spline.c:236-240: P(k of n lineages escape | alpha d) */
static double p_kescape(int k, int n, double ad) {
  if (k == 0) return exp(-n * ad);
  return exp(lchoose(n, k) + k * log(1.0 - exp(-ad)) - (n - k) * ad);
}

/* sm-spline.c:316-484 for one depth */
static sm_ptable_t sweep_model_fsp(double *fsp, int n, int asc_depth, int asc_min_freq, int bg_only,
                                   int include_invariant) {
  const int np = spline_pts, NN = n + 1;
  double *pjh = fh_malloc(sizeof(double) * NN * NN, "pjh");
  double *pbk0 = fh_malloc(sizeof(double) * NN * NN, "pbk");
  double **pbk = fh_malloc(sizeof(double *) * NN, "pbk");
  double *x = fh_malloc(sizeof(double) * (np + 1), "knots");
  double *y = fh_malloc(sizeof(double) * NN * (np + 1), "y");
  double *fy = fh_malloc(sizeof(double) * (n / 2 + 1) * (np + 1), "fy");
  sm_ptable_t t;
  int j, b, i, f;

  log_ad_step = (LOG_AD_MAX - LOG_AD_MIN) / (np + 1.);

  /* pjh[j][h]: P(j derived in a sub-sample of h) from the background fsp */
#pragma omp parallel for schedule(dynamic, 4)
  for (j = 0; j <= n; j++) {
    int h, a;
    for (h = 0; h <= n; h++) {
      double acc = 0.;
      for (a = j; a <= n; a++) acc += fsp[a] * exp(lchoose(a, j) + lchoose(n - a, h - j) - lchoose(n, h));
      pjh[j * NN + h] = acc;
    }
  }
  /* pbk[b][k]: P(b derived observed | k lineages escaped) */
  for (b = 0; b <= n; b++) {
    int k;
    pbk[b] = pbk0 + (size_t)b * NN;
    for (k = 0; k < n; k++) {
      double acc = 0.;
      const int q = b - (n - k) + 1;
      if (q > 0) acc += pjh[q * NN + k + 1] * (q / (double)(k + 1));
      if (b < k + 1) acc += pjh[b * NN + k + 1] * ((k + 1 - b) / (double)(k + 1));
      pbk[b][k] = acc;
    }
  }
  free(pjh);
  /* expected spectrum at each knot of log(alpha d) */
#pragma omp parallel for schedule(dynamic, 1)
  for (i = 0; i <= np; i++) {
    const double log_ad = LOG_AD_MIN + i * log_ad_step, ad = exp(log_ad);
    double *p = fh_malloc(sizeof(double) * NN, "p"), *pk = fh_malloc(sizeof(double) * NN, "pk");
    double p_sum = 0.;
    int ff, k;
    for (k = 0; k <= n; k++) pk[k] = p_kescape(k, n, ad);
    for (ff = 0; ff <= n; ff++) {
      p[ff] = pk[n] * fsp[ff];
      for (k = 0; k < n; k++) p[ff] += pk[k] * pbk[ff][k];
      p_sum += p[ff];
    }
    if (!include_invariant) {
      p_sum -= p[0] + p[n];
      p[0] = p[n] = 0.;
    }
    for (ff = 0; ff <= n; ff++) p[ff] /= p_sum;
    if (asc_depth > 0 && bg_only == 0) ascbias_adjust_expect(p, n, asc_min_freq, asc_depth);
    for (ff = 0; ff <= n; ff++) y[ff * (np + 1) + i] = p[ff] == 0. ? log(DBL_MIN) : log(p[ff]);
    for (ff = 0; ff < n - ff; ff++)
      fy[ff * (np + 1) + i] = p[ff] + p[n - ff] == 0. ? log(DBL_MIN) : log(p[ff] + p[n - ff]);
    if (ff == n - ff) fy[ff * (np + 1) + i] = p[ff] == 0. ? log(DBL_MIN) : log(p[ff]);
    x[i] = log_ad;
    free(p);
    free(pk);
  }
  t.sample_size = n;
  t.pbk = pbk;
  t.fsp = fsp;
  t.spline_func = fh_malloc(sizeof(spline_t *) * NN, "splines");
  t.fspline_func = fh_malloc(sizeof(spline_t *) * (n / 2 + 1), "splines");
#pragma omp parallel
  {
    const int dim = 4 * (np + 1);
    double *m = fh_malloc(sizeof(double) * (size_t)dim * BW, "band"), *v = fh_malloc(sizeof(double) * dim, "v");
    double *bb = fh_malloc(sizeof(double) * dim, "b");
#pragma omp for schedule(dynamic, 1)
    for (f = 0; f <= n + n / 2 + 1; f++) {
      if (f <= n) t.spline_func[f] = estimate_spline(x, y + f * (np + 1), np, m, v, bb);
      else t.fspline_func[f - n - 1] = estimate_spline(x, fy + (f - n - 1) * (np + 1), np, m, v, bb);
    }
    free(m); free(v); free(bb);
  }
  free(x); free(y); free(fy);
  return t;
}

sm_ptable_t *compute_sweep_model_tables(scan_t *s, double **fsp, int asc_depth, int asc_min_freq,
                                        int ascbias_background_only, int include_invariant) {
  sm_ptable_t *t = fh_malloc(sizeof(sm_ptable_t) * s->n_depths, "sm tables");
  int i, maxd = 0;
  for (i = 0; i < s->n_depths; i++) if (s->sample_depths[i] > maxd) maxd = s->sample_depths[i];
  fh_log_fact_reserve(maxd + 2);
  for (i = 0; i < s->n_depths; i++) {
    const int n = s->sample_depths[i];
    /* Q14: the adjusted background is per depth (the reference shares one pointer across OMP threads) */
    double *asc = asc_depth > 0 ? ascbias_adjust_background(fsp[i], n, asc_depth, asc_min_freq) : fsp[i];
    t[i] = sweep_model_fsp(asc, n, asc_depth, asc_min_freq, ascbias_background_only, include_invariant);
    cr_logmsg(MSG_STATUS, "Computing sweep models for all sample depths - %1.1f%% ",
              (i + 1) / (double)s->n_depths * 100.);
  }
  logmsg(MSG_STATUS, "");
  return t;
}
