/* ci_predict.c -- offline measurement for the split cells' alpha search (test tool, not
 * product): how often the coarse-phase winner of a bisection point equals a guess made from
 * the points evaluated before its round.  If the guess holds, the point's refine walks
 * (sm-search.c:283-295) can be evaluated in the same phase as its coarse walks.
 *
 * Built against the oracle's restatement (included whole, so its statics are visible):
 *   gcc -O2 -ffp-contract=off -fopenmp -o /tmp/ci_predict tools/ci_predict.c -lm
 *   /tmp/ci_predict file.snp n_cells [seed]
 * Cells are trial cells ([k G, (k+1) G], scan-chromosome.c:466-471) on one block permutation
 * of the input.  Rounds as the kernel runs them: {s, e}, then two bisection levels per round.
 */
#include "../oracle/oracle.c"

typedef struct { int ci, ri, pos; double clr; long long coarse_terms, list_terms[12]; } rec_t;
static rec_t g_rec[256];
static int g_nrec;
static const orc_table_t *g_tab;

static double coarse_la(int a) {  /* the accumulated loop of sm-search.c:274 */
  double la = LOG_AD_MIN, step = (LOG_AD_MAX - LOG_AD_MIN) / 10.0;
  int k;
  for (k = 0; k < a; k++) la += step;
  return la;
}

static long long list_terms(orc_pt_t *r, const orc_snp_t *snps, int ci) {
  orc_stats_t st = {0};
  double step = (LOG_AD_MAX - LOG_AD_MIN) / 10.0, best = ci < 11 ? coarse_la(ci) : LOG_AD_MAX, le, re, la;
  orc_pt_t t = *r;
  le = best - step; if (le < LOG_AD_MIN) le = LOG_AD_MIN;
  re = best + step; if (re > LOG_AD_MAX) re = LOG_AD_MAX;
  step = (re - le) / 15.;
  for (la = le + step; la < re; la += step) { t.lalpha = la; sm_likelihood(&t, snps, g_tab, &st); }
  return st.n_terms;
}

static void hook(orc_pt_t *r, const orc_snp_t *snps, void *ctx) {
  orc_pt_t t = *r;
  orc_stats_t st = {0};
  double best = -DBL_MAX;
  int a, ci = 11, k;
  rec_t *q = &g_rec[g_nrec < 255 ? g_nrec++ : 255];
  (void)ctx;
  for (a = 0; a < 11; a++) {
    t.lalpha = coarse_la(a);
    sm_likelihood(&t, snps, g_tab, &st);
    if (t.sm_logl > best) { best = t.sm_logl; ci = a; }
  }
  q->coarse_terms = st.n_terms;
  for (k = 0; k < 12; k++) q->list_terms[k] = getenv("CI_TERMS") ? list_terms(r, snps, k) : 0;
  orc_search_maxalpha(r, snps, g_tab, NULL);
  q->ci = ci;
  q->ri = 0;
  q->pos = r->sweep_pos;
  q->clr = r->clr;
}

int main(int argc, char **argv) {
  orc_opts_t o;
  orc_scan_t *s;
  double **fsp;
  orc_snp_t *p;
  orc_rand_t g;
  orc_stats_t st = {0};
  int n_cells = argc > 2 ? atoi(argv[2]) : 100, c, done = 0;
  long long n_pts = 0, hitA = 0, hitB = 0, hitC = 0, nB2 = 0, rounds = 0, rounds1 = 0;
  long long coarse_t = 0, refine_t = 0, extraA = 0, extraB = 0;
  if (argc < 2) return 2;
  orc_default_opts(&o);
  orc_init_log_table();
  s = orc_load_snp_input(argv[1], 0, 5);
  fsp = orc_background_fsp(s, 0, 0);
  g_tab = orc_compute_tables(s, fsp, &o);
  orc_null_model(s, fsp);
  p = xmalloc(sizeof(orc_snp_t) * s->n_snps);
  orc_srand(&g, argc > 3 ? atoi(argv[3]) : 7);
  orc_block_permute(p, s->snps, s->n_snps, o.permute_nbp, o.scan_width_mb, &g, &st);
  orc_set_maxalpha_hook(hook, NULL);
  for (c = 0; c < s->n_chr && done < n_cells; c++) {
    const orc_chr_t *lim = s->chr + c;
    int ncell = lim->bp_length / o.large_grid_sp, k, stride = ncell / (n_cells / s->n_chr + 1) + 1;
    for (k = 1; k < ncell && done < n_cells; k += stride) {
      int i, j;
      g_nrec = 0;
      orc_search_maxpos(c, k * o.large_grid_sp, (k + 1) * o.large_grid_sp, p, lim, o.eval_range, o.bp_resl, g_tab,
                        NULL);
      done++;
      /* replay the rounds: interval ends (ia, ib) into g_rec; rounds of two levels */
      {
        int ia = 0, ib = 1, nx = 2;
        while (nx < g_nrec) {
          const int m1 = nx, m2 = nx + 1 < g_nrec ? nx + 1 : -1;
          const rec_t *A = &g_rec[ia], *B = &g_rec[ib];
          const int guessA = A->clr >= B->clr ? A->ci : B->ci;
          int r1 = 1;
          for (j = 0; j < 2; j++) {
            const int m = j == 0 ? m1 : m2;
            if (m < 0) break;
            n_pts++;
            coarse_t += g_rec[m].coarse_terms;
            refine_t += g_rec[m].list_terms[g_rec[m].ci];
            hitA += g_rec[m].ci == guessA;
            hitB += g_rec[m].ci == A->ci || g_rec[m].ci == B->ci;
            nB2 += A->ci != B->ci;
            hitC += g_rec[m].ci == g_rec[m - 1].ci;
            if (g_rec[m].ci != guessA) { r1 = 0; extraA += g_rec[m].list_terms[guessA]; }
            extraB += g_rec[m].list_terms[A->ci] + (A->ci != B->ci ? g_rec[m].list_terms[B->ci] : 0);
          }
          rounds++;
          rounds1 += r1;
          /* advance two levels exactly as the reference does */
          for (j = 0; j < 2 && nx < g_nrec; j++, nx++) {
            if ((g_rec[ia].clr + g_rec[nx].clr) >= (g_rec[ib].clr + g_rec[nx].clr)) ib = nx; else ia = nx;
          }
        }
      }
      for (i = 0; i < g_nrec && getenv("CI_VERBOSE"); i++)
        fprintf(stderr, "%d %d ci=%d clr=%.3f\n", done, g_rec[i].pos, g_rec[i].ci, g_rec[i].clr);
    }
  }
  printf("cells %d, bisection points %lld, rounds %lld\n", done, n_pts, rounds);
  printf("guess A (coarse winner of the better interval end): %.3f of points, %.3f of rounds all right\n",
         (double)hitA / n_pts, (double)rounds1 / rounds);
  printf("guess B (either end's winner): %.3f (two lists in %.3f of points)\n", (double)hitB / n_pts,
         (double)nB2 / n_pts);
  printf("guess C (previous point's winner): %.3f\n", (double)hitC / n_pts);
  if (getenv("CI_TERMS"))
    printf("terms per point: coarse %.0f, own refine %.0f, wasted guess A %.0f, evaluated lists B %.0f\n",
           (double)coarse_t / n_pts, (double)refine_t / n_pts, (double)extraA / n_pts, (double)extraB / n_pts);
  return 0;
}
