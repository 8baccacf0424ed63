/* fscl_main.c -- the `fscl` command line, drop-in for the reference's
 * (option table fscl.c:38-102, defaults :127-178, validation :180-258,
 * main :272-341, parsing cmdline-utils.c:28-100: "--long=value" or
 * "-x value", flags toggle).  The scan path runs on the GPU.
 *
 * Deliberate differences: "--long value" without '=' is an
 * error instead of a NULL dereference; -m reads ms output with defined
 * semantics (all blocks form one genome, one chromosome per block, --max-only
 * prints the maximum of each block); -b reads the format --output-bs writes.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "fscl_host.h"

enum { T_STR, T_INT, T_DBL, T_FLAG };
typedef struct { char s; const char *l; void *v; int t; const char *doc; } opt_t;

/* fscl.c:33-34 */
char *prepend_label, *output_fname;
int spline_pts, n_permute;

static void usage(const opt_t *o) {
  fprintf(stderr, "fscl (MI355X) -- composite-likelihood selective sweep scan\n");
  for (; o->v; o++) {
    if (o->s) fprintf(stderr, "  -%c, --%-28s %s\n", o->s, o->l, o->doc);
    else fprintf(stderr, "      --%-28s %s\n", o->l, o->doc);
  }
}

/* --max-only for ms input: one line per block (fscl.c:68-69, :307-308) */
static void output_block_maxima(const char *fname, scan_t *s, const char *label) {
  FILE *f = fname ? fopen(fname, "w") : stdout;
  int c, i;
  if (!f) { fprintf(stderr, "Can't open output file \"%s\"\n", fname); return; }
  for (c = 0; c < s->n_chromosomes; c++) {
    const scan_pt_t *b = NULL;
    for (i = 0; i < s->n_scan_pts; i++)
      if (s->scan_pts[i].chr == c && (!b || s->scan_pts[i].clr > b->clr)) b = s->scan_pts + i;
    if (!b) continue;
    if (label) fprintf(f, "%s\t", label);
    fprintf(f, "%s\t%d\t%1.2f\t%1.3e\t%d\t%d\t%d\n", s->chr_limits[c].name, b->sweep_pos, b->clr, exp(b->lalpha),
            b->n_snps, s->snps[b->window_start].pos, s->snps[b->window_end].pos);
  }
  if (fname) fclose(f);
}

int main(int argc, char **argv) {
  char *snp_fname = NULL, *ms_fname = NULL, *bs_fname = NULL, *output_bs_fname = NULL;
  int force_neutral = 0, ms_segment_length = 0, ms_folded = 0, ms_sample_first = 0, ms_sample_size = 0;
  int asc_depth = 0, asc_min_freq = 1, bg_only = 0, include_invariant = 0, maximum_only = 0;
  int small_grid_sp = 1000, large_grid_sp = 100000, dont_scan = 0, minimum_obs_depth = 5, n_threads = 1;
  int verbosity = MSG_STATUS, eval_range = 81920, bp_resl = 128, stop = 0, i, n_gpus = 0;
  double permute_nbp = 0.1, alpha_factor = 1.0, scan_width_mb = 1.0;
  char *permute_mode = NULL, *permute_seed = NULL;
  scan_t *s;
  double **fsp;
  opt_t opts[] = {
      {'f', "snpfile", &snp_fname, T_STR, "File name of file with SNP frequency data"},
      {'d', "asc-depth", &asc_depth, T_INT, "Depth of SNP ascertainment sample"},
      {0, "asc-minimum-freq", &asc_min_freq, T_INT, "minimum number of observations of both alleles for SNP ascertainment"},
      {'p', "n-permute", &n_permute, T_INT, "number of snp block permutations for p-value computations"},
      {0, "permute-nbp", &permute_nbp, T_DBL, "probability for switching to a new snp block for permutations"},
      {0, "n-threads", &n_threads, T_INT, "accepted for compatibility (the GPU evaluates all points at once)"},
      {'a', "alpha-factor", &alpha_factor, T_DBL, "multiply 1/alpha by this factor to determine single sweep window size"},
      {'g', "fine-grid-spacing", &small_grid_sp, T_INT, "Spacing of candidate sweep points along the chromosome (in bp)"},
      {'G', "coarse-grid-spacing", &large_grid_sp, T_INT, "Size of coarse grid in which CLR maxima will be selected"},
      {'w', "sweep-width", &scan_width_mb, T_DBL, "maximum width of sweep effect in scanning, in Mb"},
      {0, "minimum-depth", &minimum_obs_depth, T_INT, "minimum depth of sample (lower depth SNPs ignored)"},
      {'m', "msfile", &ms_fname, T_STR, "Name of an ms output file"},
      {0, "ms-segment-length", &ms_segment_length, T_INT, "Length in bp of simulated ms segments (use with -m option only)"},
      {0, "ms-folded", &ms_folded, T_FLAG, "For ms input, treat all sites as folded"},
      {0, "max-only", &maximum_only, T_FLAG, "for ms input, output only the maximum CLR for each input block"},
      {0, "ms-sample-first", &ms_sample_first, T_INT, "index of first chromosome in ms sample to analyze"},
      {0, "ms-sample-size", &ms_sample_size, T_INT, "number of consecutive chromosomes in ms output to take as the sample"},
      {0, "force-neutral-spectrum", &force_neutral, T_FLAG, "Do not estimate background spectrum from the data. Use sum(1/i)/i"},
      {'b', "background-spectrum", &bs_fname, T_STR, "Load the background frequency spectrum from a file"},
      {0, "output-bs", &output_bs_fname, T_STR, "write estimated background site-frequency spectra to file"},
      {0, "include-invariant", &include_invariant, T_FLAG, "Include invariant sites in analysis (default is to ignore them)"},
      {0, "splines", &spline_pts, T_INT, "Number of knot points to approximate sweep model w/ respect to alpha"},
      {0, "prepend-label", &prepend_label, T_STR, "optional token to prepend to each line of the sweep scan output"},
      {'v', "verbosity", &verbosity, T_INT, "verbosity level 0-5, default 3, debug 4 and above"},
      {'o', "output-file", &output_fname, T_STR, "output file for scan results"},
      {0, "no-scan", &dont_scan, T_FLAG, "do not scan chromosome, compute background frequency spectrum only"},
      {0, "ascbias-background-only", &bg_only, T_FLAG, "correct for ascertainment bias only in estimating the background site frequency spectrum"},
      {0, "n-gpus", &n_gpus, T_INT, "GPUs to use (default: every visible GPU, or $FSCL_AMD_DEVICE alone when set)"},
      {0, "permute-mode", &permute_mode, T_STR, "parity (default: the reference's rand() stream, identical results) or "
                                                "throughput (counter-based random numbers, trials independent; not identical)"},
      {0, "permute-seed", &permute_seed, T_STR, "seed of the throughput mode's random numbers (default 0xFD821A6)"},
      {0, NULL, NULL, 0, NULL}};

  spline_pts = N_SPLINE_KNOTS;
  n_permute = 0;
  init_log_table();
  if (argc == 1) { usage(opts); return 255; }
  for (i = 1; i < argc;) {
    const char *a = argv[i], *arg;
    char name[256];
    int lng, j;
    if (a[0] != '-') { i++; continue; }
    if (a[1] == '-') {
      const char *eq = strchr(a + 2, '=');
      size_t ln = eq ? (size_t)(eq - (a + 2)) : strlen(a + 2);
      if (ln >= sizeof name) ln = sizeof name - 1;
      memcpy(name, a + 2, ln);
      name[ln] = 0;
      arg = eq ? eq + 1 : NULL;
      lng = 1;
    } else {
      name[0] = a[1];
      name[1] = 0;
      arg = i + 1 < argc ? argv[i + 1] : NULL;
      lng = 0;
    }
    if (lng && !strcmp(name, "help")) { usage(opts); return 0; }
    for (j = 0; opts[j].v; j++)
      if (lng ? strcmp(name, opts[j].l) == 0 : opts[j].s == name[0]) break;
    if (!opts[j].v) fprintf(stderr, "Unrecognized option \"%s\"\n", a);
    else if (opts[j].t == T_FLAG) *(int *)opts[j].v ^= 1;
    else if (!arg) { fprintf(stderr, "Option \"%s\" needs a value (--%s=value or -x value)\n", a, opts[j].l); return 255; }
    else if (opts[j].t == T_STR) *(char **)opts[j].v = strdup(arg);
    else if (opts[j].t == T_INT) *(int *)opts[j].v = atoi(arg);
    else *(double *)opts[j].v = atof(arg);
    i += (lng || (opts[j].v && opts[j].t == T_FLAG)) ? 1 : 2;
  }

  /* fscl.c:180-258 */
  if (verbosity < 0) verbosity = 0;
  configure_logmsg(verbosity);
  if (bg_only) logmsg(MSG_STATUS, "ascertainment bias correction to background site frequency spectrum only\n");
  if (minimum_obs_depth < 5) minimum_obs_depth = 5;
  if (spline_pts < N_SPLINE_KNOTS) {
    logmsg(MSG_ERROR, "Error: must use at least %d spline functions to approximate sweep model\nlikelihood function.\n",
           N_SPLINE_KNOTS);
    stop = 1;
  }
  if (spline_pts > 500)
    logmsg(MSG_WARN, "Warning: estimating %d spline functions will significantly inflate execution\ntime with little "
                     "gain in accuracy...\n", spline_pts);
  if (!snp_fname && !ms_fname) {
    logmsg(MSG_ERROR, "Error: input snp frequency file or ms file not specified. Use -f option or -m option.\n");
    stop = 1;
  }
  if (snp_fname && ms_fname) { logmsg(MSG_ERROR, "Specify either a snp frequency file or an ms file, not both.\n"); stop = 1; }
  if (!output_fname) { logmsg(MSG_ERROR, "Specify an output file name with -o option\n"); stop = 1; }
  if (ms_segment_length && !ms_fname) {
    logmsg(MSG_WARN, "Warning: --ms-segment-length option ignored if -m option is not used.\n");
    ms_segment_length = 0;
  }
  if (asc_depth == 1 || asc_depth < 0) {
    logmsg(MSG_ERROR, "Error: if specified, ascertainment sample depth must be at least 2.\n");
    stop = 1;
  }
  if (asc_depth >= 2 && asc_min_freq > 2 * asc_depth) {
    logmsg(MSG_ERROR, "Error: SNP ascertainment is impossible with asc. sample depth and asc. minimum allele "
                      "frequency setting\n");
    stop = 1;
  }
  if (asc_depth >= 2 && asc_min_freq == 0) asc_min_freq = 1;
  if (small_grid_sp < 1 && !output_bs_fname) {
    logmsg(MSG_ERROR, "Error: specify sweep position grid spacing with -g option (in bp).\n");
    stop = 1;
  }
  if (!output_bs_fname && small_grid_sp > 0 && large_grid_sp % small_grid_sp != 0) {
    logmsg(MSG_ERROR, "Error: fine grid spacing must evenly divide coarse grid spacing.\n");
    stop = 1;
  }
  if (large_grid_sp < 1) { logmsg(MSG_ERROR, "Error: coarse grid spacing must be positive.\n"); stop = 1; }
  if (n_gpus < 0) { logmsg(MSG_ERROR, "Error: --n-gpus must be >= 0.\n"); stop = 1; }
  if (permute_mode && strcmp(permute_mode, "parity") && strcmp(permute_mode, "throughput")) {
    logmsg(MSG_ERROR, "Error: --permute-mode must be parity or throughput.\n");
    stop = 1;
  }
  if (permute_seed && !(permute_mode && !strcmp(permute_mode, "throughput")))
    logmsg(MSG_WARN, "Warning: --permute-seed is used only with --permute-mode=throughput.\n");
  if (stop) {
    if (verbosity <= MSG_FATAL) logmsg(MSG_FATAL, "Fatal errors have occurred, use -v 1 or greater to see them.\n");
    exit(-1);
  }

  s = ms_fname ? fh_load_ms(ms_fname, ms_segment_length, ms_folded, ms_sample_first, ms_sample_size)
               : load_snp_input(snp_fname, include_invariant, minimum_obs_depth);
  fsp = background_fsp(s, force_neutral, bs_fname, include_invariant);
  if (output_bs_fname) output_background_fs(output_bs_fname, s, fsp);
  if (!dont_scan) {
    sm_ptable_t *sm;
    const char *ws = getenv("WORLD_SIZE"), *rk = getenv("RANK");
    if (ws && rk && atoi(ws) > 1) {
      /* one process per GPU (e.g. under torch.distributed.run): GPU $LOCAL_RANK (or
         $FSCL_AMD_DEVICE), results exchanged through a shared-memory segment named by
         $FSCL_AMD_SHM_NAME, else the launcher's run id or port; rank 0 writes the output */
      const char *id = getenv("FSCL_AMD_SHM_NAME"), *run = getenv("TORCHELASTIC_RUN_ID"), *port = getenv("MASTER_PORT"),
                 *addr = getenv("MASTER_ADDR"), *sj = getenv("SLURM_JOB_ID"), *ss = getenv("SLURM_STEP_ID");
      char name[200];
      if (id) snprintf(name, sizeof name, "/fscl_amd_%s", id);
      else if (port || (run && strcmp(run, "none")) || sj)
        /* values a launcher gives every rank of one job alike, and two concurrent jobs on a node
           not: the rendezvous port (torch.distributed.run, mpirun wrappers), the launcher's run id
           (plain torchrun sets "none"), the Slurm job and step -- not the parent's pid, which
           differs between ranks started through a per-rank wrapper (a shell script, srun) */
        snprintf(name, sizeof name, "/fscl_amd_%s_%s_%s_%s_%s", run && strcmp(run, "none") ? run : "job",
                 addr ? addr : "-", port ? port : "0", sj ? sj : "-", ss ? ss : "-");
      else /* no launcher variables: the ranks of one launch are assumed to share their parent */
        snprintf(name, sizeof name, "/fscl_amd_job_%ld", (long)getppid());
      if (n_gpus > 1) logmsg(MSG_WARN, "Warning: --n-gpus is ignored with one process per GPU (WORLD_SIZE=%s).\n", ws);
      if (fscl_amd_set_ranks_shm(atoi(rk), atoi(ws), name) != 0)
        logmsg(MSG_FATAL, "fscl: rank %s of %s could not meet the other ranks (%s)", rk, ws, name);
    } else if ((n_gpus > 0 || !getenv("FSCL_AMD_DEVICE")) && fscl_amd_set_devices(NULL, n_gpus) != 0)
      logmsg(MSG_FATAL, "fscl: --n-gpus=%d: at most 16 GPUs per process", n_gpus);
    if (permute_mode && !strcmp(permute_mode, "throughput")) {
      fscl_amd_set_permute_mode(FSCL_AMD_PERMUTE_THROUGHPUT, permute_seed ? strtoull(permute_seed, NULL, 0) : 0xFD821A6ull);
      logmsg(MSG_STATUS, "permutation test in throughput mode (counter-based random numbers; not the reference's stream)\n");
    }
    sm = compute_sweep_model_tables(s, fsp, asc_depth, asc_min_freq, bg_only, include_invariant);
    compute_snp_null_model(s, fsp);
    scan_chromosome(s, sm, eval_range, bp_resl, large_grid_sp, n_threads);
    if (n_permute > 0)
      scan_permute(s, sm, n_permute, permute_nbp, alpha_factor, n_threads, eval_range, bp_resl, large_grid_sp,
                   scan_width_mb);
    if (ms_fname && maximum_only) output_block_maxima(output_fname, s, prepend_label);
    else scan_output(output_fname, s, maximum_only, n_permute, prepend_label);
    if (verbosity >= MSG_DEBUG1) {
      fscl_amd_stats_t st;
      fscl_amd_get_stats(&st);
      fprintf(stderr, "fscl_amd: scan %.3f s, permute %.3f s (host permutation %.3f s, %d trials), kernels %.3f s, "
                      "%llu grid-point evaluations, %llu terms, unsafe walks %llu, slow walks %llu, ties %llu, negj %llu\n",
              st.scan_s, st.permute_s, st.host_perm_s, st.trials, st.kernel_ms / 1e3, st.gp_evals, st.n_terms,
              st.n_unsafe, st.n_slow, st.n_ties, st.negj);
    }
    fscl_amd_shutdown();
  }
  return 0;
}
