/*
 * ref_harness.c -- drives the reference's OWN compiled sources (the subset
 * that builds in this image: sm-search.c, sm-spline.c, background-fsp.c,
 * asc-bias.c, snp-input.c, logmsg.c, cmdline-utils.c, compiled from
 * /root/reference into _ref/libfscl_refpart.so) to produce golden vectors.
 * TEST INFRASTRUCTURE ONLY.
 *
 *   ref_harness tables <snpfile> <out.bin> [opts]
 *       load_snp_input -> background_fsp -> compute_sweep_model_tables
 *       (all reference code) and dump fsp + every spline coefficient.
 *   ref_harness sample <snpfile> <n_cells> [opts]
 *       the CPU baseline's bounded sample (bench.py): n_cells evenly spread scan cells,
 *       one block permutation, and those cells' permutation-trial cells, timed.
 *   ref_harness scan <snpfile> <out.txt> <dump.txt> [opts]
 *       reference setup + the reference's search_maxalpha (sm-search.c:269)
 *       plugged into oracle.c's restatement of scan-chromosome.c (which cannot
 *       be compiled here: it includes GSL headers absent from the image).
 *
 * opts: --asc-depth=D --asc-minimum-freq=K --include-invariant --minimum-depth=M
 *       --splines=S --ascbias-background-only --force-neutral-spectrum
 *       --n-permute=N --permute-nbp=X --coarse-grid-spacing=G --sweep-width=W
 *       --n-threads=T (OpenMP threads over the grid cells; the reference's
 *       search_maxalpha is reentrant: fscl runs it from its own pthreads)
 * The scan mode prints the wall time of the initial scan alone (scan_s=) on
 * stderr: bench.py's cpu_baseline leg times the reference's hot code with it.
 */
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "fscl.h" /* the reference's own header, from -I/root/reference */
#include "oracle.h"

int spline_pts = N_SPLINE_KNOTS; /* defined in fscl.c:34, which cannot be built here */

_Static_assert(sizeof(snp_t) == sizeof(orc_snp_t), "snp_t layout");
_Static_assert(offsetof(snp_t, null_logl) == offsetof(orc_snp_t, null_logl), "snp_t layout");
_Static_assert(offsetof(snp_t, folded) == offsetof(orc_snp_t, folded), "snp_t layout");
_Static_assert(sizeof(scan_pt_t) == sizeof(orc_pt_t), "scan_pt_t layout");
_Static_assert(offsetof(scan_pt_t, clr) == offsetof(orc_pt_t, clr), "scan_pt_t layout");
_Static_assert(offsetof(scan_pt_t, permute_clr) == offsetof(orc_pt_t, permute_clr), "scan_pt_t layout");
_Static_assert(sizeof(scan_t) == sizeof(orc_scan_t), "scan_t layout");
_Static_assert(offsetof(scan_t, chr_limits) == offsetof(orc_scan_t, chr), "scan_t layout");
_Static_assert(sizeof(chr_limits_t) == sizeof(orc_chr_t), "chr_limits_t layout");

static void ref_maxalpha(orc_pt_t *pt, const orc_snp_t *snps, void *ctx) {
  search_maxalpha((scan_pt_t *)pt, (snp_t *)snps, (sm_ptable_t *)ctx);
}

static int arg_int(const char *a, const char *name, int *v) {
  size_t l = strlen(name);
  if (strncmp(a, name, l) == 0 && a[l] == '=') { *v = atoi(a + l + 1); return 1; }
  return 0;
}
static int arg_dbl(const char *a, const char *name, double *v) {
  size_t l = strlen(name);
  if (strncmp(a, name, l) == 0 && a[l] == '=') { *v = atof(a + l + 1); return 1; }
  return 0;
}

int main(int argc, char **argv) {
  orc_opts_t o;
  scan_t *s;
  double **fsp;
  sm_ptable_t *sm;
  int i;
  orc_stats_t st = {0};
  if (argc < 4) { fprintf(stderr, "usage: ref_harness tables|scan <snpfile> <out> [dump] [opts]\n"); return 2; }
  orc_default_opts(&o);
  for (i = 3; i < argc; i++) {
    const char *a = argv[i];
    if (arg_int(a, "--asc-depth", &o.asc_depth) || arg_int(a, "--asc-minimum-freq", &o.asc_min_freq) ||
        arg_int(a, "--minimum-depth", &o.minimum_depth) || arg_int(a, "--splines", &o.spline_pts) ||
        arg_int(a, "--n-permute", &o.n_permute) || arg_dbl(a, "--permute-nbp", &o.permute_nbp) ||
        arg_int(a, "--coarse-grid-spacing", &o.large_grid_sp) || arg_dbl(a, "--sweep-width", &o.scan_width_mb) ||
        arg_int(a, "--n-threads", &o.n_threads))
      continue;
    if (!strcmp(a, "--include-invariant")) o.include_invariant = 1;
    else if (!strcmp(a, "--ascbias-background-only")) o.ascbias_background_only = 1;
    else if (!strcmp(a, "--force-neutral-spectrum")) o.force_neutral = 1;
  }
  spline_pts = o.spline_pts;
  configure_logmsg(MSG_ERROR);
  init_log_table();
  orc_init_log_table();
  s = load_snp_input(argv[2], o.include_invariant, o.minimum_depth);
  fsp = background_fsp(s, o.force_neutral, NULL, o.include_invariant);
  sm = compute_sweep_model_tables(s, fsp, o.asc_depth, o.asc_min_freq, o.ascbias_background_only,
                                  o.include_invariant);
  if (!strcmp(argv[1], "tables")) {
    FILE *f = fopen(argv[3], "wb");
    int d, r;
    if (!f) return 1;
    fwrite(&s->n_depths, sizeof(int), 1, f);
    fwrite(&spline_pts, sizeof(int), 1, f);
    for (d = 0; d < s->n_depths; d++) {
      int n = s->sample_depths[d];
      fwrite(&n, sizeof(int), 1, f);
      fwrite(fsp[d], sizeof(double), n + 1, f);
      for (r = 0; r <= n; r++) fwrite(sm[d].spline_func[r]->coef[0], sizeof(double), 4 * spline_pts, f);
      for (r = 0; r <= n / 2; r++) fwrite(sm[d].fspline_func[r]->coef[0], sizeof(double), 4 * spline_pts, f);
    }
    fclose(f);
    return 0;
  }
  if (!strcmp(argv[1], "scan") && argc >= 5) {
    orc_scan_t *os = (orc_scan_t *)s;
    orc_null_model(os, fsp);
    orc_set_maxalpha_hook(ref_maxalpha, sm);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    orc_scan_chromosome(os, NULL, &o, &st);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    fprintf(stderr, "ref_harness: scan_s=%.6f threads=%d\n",
            (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec), o.n_threads);
    if (o.n_permute > 0) orc_scan_permute(os, NULL, &o, &st);
    orc_scan_output(argv[3], os, 0, o.n_permute, NULL);
    orc_dump_points(argv[4], os);
    fprintf(stderr, "ref_harness: gp=%lld maxalpha=%lld negj=%lld\n", st.n_gp, st.n_maxalpha, st.negj);
    return st.negj ? 3 : 0;
  }
  if (!strcmp(argv[1], "sample")) {
    /* ref_harness sample <snpfile> <n_cells> [opts]: the CPU baseline's bounded sample --
       n_cells evenly spread scan cells through the reference's own search_maxalpha (with
       --n-threads threads), then one block permutation (serial, as in the reference:
       scan-chromosome.c:441-456) and the same cells' permutation-trial cells on it */
    orc_scan_t *os = (orc_scan_t *)s;
    orc_snp_t *ps = malloc(sizeof(orc_snp_t) * (size_t)os->n_snps);
    orc_rand_t g;
    struct timespec t0, t1;
    int ns = atoi(argv[3]), done = 0, pdone = 0, r, reps = 3;
    double cell_s, pcell_s, perm_s;
    orc_null_model(os, fsp);
    orc_set_maxalpha_hook(ref_maxalpha, sm);
    cell_s = orc_sample_cells(os, NULL, &o, os->snps, ns, 0, &done);
    orc_srand(&g, 0xFD821A6);
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (r = 0; r < reps; r++) orc_block_permute(ps, os->snps, os->n_snps, o.permute_nbp, o.scan_width_mb, &g, &st);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    perm_s = ((double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec)) / reps;
    pcell_s = orc_sample_cells(os, NULL, &o, ps, ns, 1, &pdone);
    fprintf(stderr, "ref_harness: sample_cells=%d threads=%d cell_s=%.6f perm_gen_s=%.6f perm_cells=%d perm_cell_s=%.6f\n",
            done, o.n_threads, cell_s, perm_s, pdone, pcell_s);
    free(ps);
    return 0;
  }
  fprintf(stderr, "ref_harness: unknown mode %s\n", argv[1]);
  return 2;
}
