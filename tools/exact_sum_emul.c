/*
 * exact_sum_emul.c -- CPU emulation of the GPU's order-free exact walk sum
 * (SURVEY Appendix B), checked against the sequential
 * reference order on every walk of a scan.  Development tool (links the
 * oracle, never the product).
 *
 *   exact_sum_emul <snpfile> [n_points]
 *
 * For every grid point's alpha candidates it computes the walk's terms in
 * reference order, the sequential fl-sum, and the integer-ulp sum with
 * ties resolved by prefix parity, and reports mismatches / unsafe walks /
 * tie counts.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../oracle/oracle.h"

static double term(const orc_snp_t *p, double la, int sweep, const orc_table_t *tab, double *x_out) {
  double x = orc_logt(abs(p->pos - sweep)) + la;
  const orc_table_t *t = tab + p->depth_p;
  double y = p->folded ? orc_spline_interpolate(t->fspline + p->obs_freq, x)
                       : orc_spline_interpolate(t->spline + p->obs_freq, x);
  *x_out = x;
  return y - p->null_logl;
}

int main(int argc, char **argv) {
  orc_opts_t o;
  orc_scan_t *s;
  double **fsp;
  orc_table_t *tab;
  long long walks = 0, mism = 0, unsafe = 0, ties = 0, tiewalks = 0, terms = 0, truly = 0, amb = 0, winner_unsafe = 0;
  int npts, pi;
  orc_default_opts(&o);
  orc_init_log_table();
  s = orc_load_snp_input(argv[1], 0, 5);
  fsp = orc_background_fsp(s, 0, 0);
  tab = orc_compute_tables(s, fsp, &o);
  orc_null_model(s, fsp);
  npts = argc > 2 ? atoi(argv[2]) : 50;
  double *t = malloc(sizeof(double) * s->n_snps);
  for (pi = 0; pi < npts; pi++) {
    orc_pt_t pt;
    int c = 0, a;
    int pos = s->chr[0].start_pos + (int)((double)(s->chr[0].bp_length - s->chr[0].start_pos) * pi / npts);
    orc_init_scan_result(&pt, c, s->snps, s->chr + c, o.eval_range, pos, NULL);
    double bestv = -DBL_MAX; int best_safe = 1; double appr[26], bnd[26]; int saf[26]; double sv[26]; int na = 0;
    for (a = 0; a < 26; a++) {
      double la = -20.0 + a * (24.0 / 25.0), x, seq;
      int len = 0, i, k;
      t[len] = term(s->snps + pt.nearest_snp, la, pt.sweep_pos, tab, &x);
      if (x > 4.0) { sv[na] = pt.null_logl; saf[na] = 1; appr[na] = sv[na]; bnd[na] = 0; na++; continue; }
      len++;
      for (i = pt.nearest_snp - 1; i >= pt.window_start; i--) {
        double v = term(s->snps + i, la, pt.sweep_pos, tab, &x);
        if (x > 4.0) break;
        t[len++] = v;
      }
      for (i = pt.nearest_snp + 1; i <= pt.window_end; i++) {
        double v = term(s->snps + i, la, pt.sweep_pos, tab, &x);
        if (x > 4.0) break;
        t[len++] = v;
      }
      seq = pt.null_logl;
      for (k = 0; k < len; k++) seq += t[k];
      /* integer scheme */
      {
        double N = pt.null_logl;
        int e;
        frexp(N, &e);                  /* |N| in [2^(e-1), 2^e) */
        double u = ldexp(1.0, e - 53), inv = ldexp(1.0, 53 - e);
        int64_t S0 = (int64_t)(N * inv), P = 0, Q = 0, adjs = 0, run = 0, mn = 0, mx = 0;
        int par = (int)(S0 & 1), T = 0;
        for (k = 0; k < len; k++) {
          double q = t[k] * inv, F = floor(q), fr = q - F;
          int64_t M = (int64_t)F + (fr > 0.5);
          if (fr == 0.5) {
            int adj = (par ^ (int)(M & 1)) & 1;
            T++;
            adjs += adj;
            par ^= adj;
          }
          if (M > 0) P += M; else Q += M;
          par ^= (int)(M & 1);
          run += M; if (run < mn) mn = run; if (run > mx) mx = run;
        }
        if (!(S0 + mn >= -(1LL << 53) && S0 + mx <= -((1LL << 52) + 1))) truly++;
        int safe = S0 < 0 && S0 + Q >= -(1LL << 53) && S0 + P + T <= -((1LL << 52) + 1);
        double v = (double)(S0 + P + Q + adjs) * u;
        walks++;
        terms += len;
        ties += T;
        tiewalks += T > 0;
        saf[na] = safe; sv[na] = seq; appr[na] = (double)(S0 + P + Q) * u;
        bnd[na] = len * u + len * ldexp(1.0, -51) * (fabs(N) + (double)(P - Q + len) * u);
        na++;
        if (!safe) unsafe++;
        else if (v != seq) {
          mism++;
          if (mism < 5) fprintf(stderr, "mismatch pt %d la %g len %d: %a vs %a\n", pi, la, len, v, seq);
        }
      }
    }
    { int q, bi = -1; double bv = -DBL_MAX; int am = 0;
      for (q = 0; q < na; q++) if (sv[q] > bv) { bv = sv[q]; bi = q; }
      if (!saf[bi]) winner_unsafe++;
      else for (q = 0; q < na; q++) if (!saf[q] && appr[q] + bnd[q] >= bv) am = 1;
      amb += am; (void)bestv; (void)best_safe; }
  }
  printf("truly_unsafe=%lld ambiguous_points=%lld winner_unsafe=%lld\n", truly, amb, winner_unsafe);
  printf("walks=%lld terms=%lld safe_mismatch=%lld unsafe=%lld ties=%lld walks_with_ties=%lld\n", walks, terms,
         mism, unsafe, ties, tiewalks);
  return mism != 0;
}
