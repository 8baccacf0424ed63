/*
 * oracle_main.c -- command line front end of the CPU restatement (test
 * infrastructure only).  Mirrors fscl's option table (fscl.c:38-102),
 * defaults (fscl.c:127-178), validation (fscl.c:180-258) and the
 * "--long=value" / "-x value" parsing of cmdline-utils.c:28-100.
 * Supports the SNP-file path (fscl.c:316-337); -m (ms input) is routed by
 * the product CLI's converter, see DESIGN.md.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

enum { T_STR, T_INT, T_DBL, T_FLAG };
typedef struct { char s; const char *l; void *v; int t; } opt_t;

int main(int argc, char **argv) {
  orc_opts_t o;
  char *snp = NULL, *out = NULL, *label = NULL, *ms = NULL, *bs = NULL, *obs = NULL, *dump = NULL;
  int small_grid = 1000, verbosity = 3, no_scan = 0, dummy_i = 0, stop = 0, i, ms_folded = 0, nulldist = 0;
  char *tseed = NULL;
  double alpha_factor = 1.0;
  orc_stats_t st = {0};
  orc_default_opts(&o);
  {
    opt_t tab[] = {
        {'f', "snpfile", &snp, T_STR},
        {'d', "asc-depth", &o.asc_depth, T_INT},
        {0, "asc-minimum-freq", &o.asc_min_freq, T_INT},
        {'p', "n-permute", &o.n_permute, T_INT},
        {0, "permute-nbp", &o.permute_nbp, T_DBL},
        {0, "n-threads", &o.n_threads, T_INT},
        {'a', "alpha-factor", &alpha_factor, T_DBL},
        {'g', "fine-grid-spacing", &small_grid, T_INT},
        {'G', "coarse-grid-spacing", &o.large_grid_sp, T_INT},
        {'w', "sweep-width", &o.scan_width_mb, T_DBL},
        {0, "minimum-depth", &o.minimum_depth, T_INT},
        {'m', "msfile", &ms, T_STR},
        {0, "ms-segment-length", &dummy_i, T_INT},
        {0, "ms-folded", &ms_folded, T_FLAG},
        {0, "max-only", &o.max_only, T_FLAG},
        {0, "ms-sample-first", &dummy_i, T_INT},
        {0, "ms-sample-size", &dummy_i, T_INT},
        {0, "force-neutral-spectrum", &o.force_neutral, T_FLAG},
        {'b', "background-spectrum", &bs, T_STR},
        {0, "output-bs", &obs, T_STR},
        {0, "include-invariant", &o.include_invariant, T_FLAG},
        {0, "splines", &o.spline_pts, T_INT},
        {0, "prepend-label", &label, T_STR},
        {'v', "verbosity", &verbosity, T_INT},
        {'o', "output-file", &out, T_STR},
        {0, "no-scan", &no_scan, T_FLAG},
        {0, "ascbias-background-only", &o.ascbias_background_only, T_FLAG},
        {0, "dump-points", &dump, T_STR}, /* oracle only: hex-float dump of every point */
        {0, "nulldist", &nulldist, T_FLAG}, /* oracle only: write <output>-nulldist at the end */
        {0, "eval-range", &o.eval_range, T_INT}, /* oracle only: scan_chromosome's eval_range (fscl.c:175 fixes 81920) */
        {0, "throughput-seed", &tseed, T_STR}, /* oracle only: the product's throughput permutation mode */
        {0, NULL, NULL, 0}};
    i = 1;
    while (i < argc) {
      const char *a = argv[i], *arg = NULL;
      char name[256];
      int lng, j;
      if (a[0] != '-') { i++; continue; }
      if (a[1] == '-') {
        const char *eq = strchr(a + 2, '=');
        size_t ln = eq ? (size_t)(eq - (a + 2)) : strlen(a + 2);
        if (ln >= sizeof name) ln = sizeof name - 1;
        memcpy(name, a + 2, ln); name[ln] = 0;
        arg = eq ? eq + 1 : NULL;
        lng = 1;
      } else { name[0] = a[1]; name[1] = 0; arg = i + 1 < argc ? argv[i + 1] : NULL; lng = 0; }
      for (j = 0; tab[j].v; j++)
        if (lng ? strcmp(name, tab[j].l) == 0 : tab[j].s == name[0]) break;
      if (!tab[j].v) fprintf(stderr, "Unrecognized option \"%s\"\n", a);
      else if (tab[j].t == T_FLAG) *(int *)tab[j].v ^= 1;
      else if (!arg) { fprintf(stderr, "option \"%s\" needs a value (use --%s=value)\n", a, tab[j].l); return 255; }
      else if (tab[j].t == T_STR) *(char **)tab[j].v = strdup(arg);
      else if (tab[j].t == T_INT) *(int *)tab[j].v = atoi(arg);
      else *(double *)tab[j].v = atof(arg);
      i += (lng || (tab[j].v && tab[j].t == T_FLAG)) ? 1 : 2;
    }
  }
  (void)alpha_factor;
  if (o.minimum_depth < 5) o.minimum_depth = 5;
  if (o.spline_pts < 200) { fprintf(stderr, "Error: must use at least 200 spline functions\n"); stop = 1; }
  if (!snp && !ms) { fprintf(stderr, "Error: input snp frequency file or ms file not specified.\n"); stop = 1; }
  if (snp && ms) { fprintf(stderr, "Specify either a snp frequency file or an ms file, not both.\n"); stop = 1; }
  if (!out) { fprintf(stderr, "Specify an output file name with -o option\n"); stop = 1; }
  if (o.asc_depth == 1 || o.asc_depth < 0) { fprintf(stderr, "Error: asc depth must be at least 2.\n"); stop = 1; }
  if (o.asc_depth >= 2 && o.asc_min_freq > 2 * o.asc_depth) { fprintf(stderr, "Error: SNP ascertainment is impossible\n"); stop = 1; }
  if (o.asc_depth >= 2 && o.asc_min_freq == 0) o.asc_min_freq = 1;
  if (small_grid < 1 && !obs) { fprintf(stderr, "Error: specify sweep position grid spacing\n"); stop = 1; }
  if (!obs && small_grid > 0 && o.large_grid_sp % small_grid != 0) {
    fprintf(stderr, "Error: fine grid spacing must evenly divide coarse grid spacing.\n"); stop = 1;
  }
  if (ms || bs || obs || no_scan) { fprintf(stderr, "oracle: -m/-b/--output-bs/--no-scan not restated\n"); stop = 1; }
  if (stop) return 255;
  if (tseed) { o.throughput = 1; o.throughput_seed = strtoull(tseed, NULL, 0); }
  if (dump) setenv("ORC_DUMP_POINTS", dump, 1);
  if (nulldist) setenv("ORC_NULLDIST", "1", 1);
  if (orc_run_snpfile(snp, out, &o, label, &st) != 0) return 1;
  if (verbosity >= 4)
    fprintf(stderr, "oracle stats: gp=%lld maxalpha=%lld walks=%lld terms=%lld null=%lld negj=%lld\n",
            st.n_gp, st.n_maxalpha, st.n_walks, st.n_terms, st.n_null, st.negj);
  return 0;
}
