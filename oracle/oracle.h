/*
 * oracle.h -- CPU restatement of slowkoni/fscl's CLR scan + permutation path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (fscl_amd/, include/)
 * includes, links or calls this.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, and only as the checker / CPU baseline.
 *
 * Every function restates one reference function (file:line in
 * /root/reference) with the same floating-point operation order, so that with
 * -ffp-contract=off it is bit-identical to the reference built the same way.
 * Parity pinning: the setup functions (tables, background, asc-bias, input)
 * and the alpha search are checked bit-for-bit against the reference's own
 * sources compiled under oracle/_ref (see oracle/Makefile);
 * scan-chromosome.c is unbuildable here (needs GSL headers absent from the
 * image), so the position search / permutation / output are restated from
 * its text and cross-checked against the harness that wraps the reference's
 * compiled search_maxalpha.
 */
#ifndef FSCL_ORACLE_H
#define FSCL_ORACLE_H

#include <stdint.h>

/* fscl.h:7-14 */
typedef struct {
  int chr;
  int pos;
  double null_logl;
  int obs_freq;
  int depth_p;
  int folded;
} orc_snp_t;

/* fscl.h:26-33 */
typedef struct {
  int chr;
  char *name;
  int start_index;
  int n_snps;
  int start_pos;
  int bp_length;
} orc_chr_t;

/* fscl.h:35-51 */
typedef struct {
  int chr;
  int nearest_snp;
  int sweep_pos;
  int n_snps;
  int window_start;
  int window_end;
  double lalpha;
  double null_logl;
  double sm_logl;
  double clr;
  int permute_n;
  int permute_p;
  int permute_finished;
  int scan_running;
  float *permute_clr;
} orc_pt_t;

/* fscl.h:53-62 */
typedef struct {
  int n_snps;
  orc_snp_t *snps;
  int n_depths;
  int *sample_depths;
  int n_pts;
  orc_pt_t *pts;
  orc_chr_t *chr;
  int n_chr;
} orc_scan_t;

/* one natural cubic spline: n intervals, coef[4*i + {0..3}] (sm-spline.c:196-211) */
typedef struct {
  int n;
  double *knots; /* n+1 */
  double *coef;  /* 4*n */
} orc_spline_t;

/* fscl.h:70-76, per sample depth */
typedef struct {
  orc_spline_t *spline;  /* sample_size+1 */
  orc_spline_t *fspline; /* sample_size/2+1 */
  int sample_size;
} orc_table_t;

typedef struct {
  int spline_pts;       /* --splines (fscl.c:84, default N_SPLINE_KNOTS at :167) */
  int include_invariant;
  int minimum_depth;
  int force_neutral;
  int asc_depth, asc_min_freq, ascbias_background_only;
  int n_permute;
  double permute_nbp;
  double scan_width_mb;
  int large_grid_sp;
  int eval_range;       /* fscl.c:175 */
  int bp_resl;          /* fscl.c:174 */
  int max_only;
  int n_threads;        /* OpenMP threads for the lockstep-parallel port (results identical) */
  int throughput;       /* the product's throughput mode (counter-based random numbers) */
  unsigned long long throughput_seed;
} orc_opts_t;

/* counters used for the algorithmic-bytes roofline */
typedef struct {
  long long n_terms;     /* snp_likelihood calls */
  long long n_null;      /* elements summed in init_scan_result */
  long long n_walks;     /* sm_likelihood calls */
  long long n_maxalpha;  /* search_maxalpha calls */
  long long n_gp;        /* search_maxpos calls */
  long long negj;        /* permutation blocks hitting the reference's negative-j bug */
} orc_stats_t;

/* glibc random_r TYPE_3 restatement, so the oracle owns its rand() stream */
typedef struct { int32_t r[31]; int f, b; } orc_rand_t;
void orc_srand(orc_rand_t *g, unsigned seed);
int orc_rand(orc_rand_t *g);
/* restart the process-wide permutation stream (srand, fscl.c:135) */
void orc_reseed(unsigned seed);

void orc_default_opts(orc_opts_t *o);
void orc_init_log_table(void);
const double *orc_log_table(void);
double orc_logt(int d);
double orc_log_fact(int n);
double orc_lchoose(int n, int k);
double orc_log_ad_step(void);
void orc_set_spline_pts(int spline_pts);

orc_scan_t *orc_load_snp_input(const char *fname, int include_invariant, int minimum_depth);
double **orc_background_fsp(orc_scan_t *s, int force_neutral, int include_invariant);
double *orc_ascbias_adjust_background(const double *bsf, int n, int asc_depth, int min_obs);
void orc_ascbias_adjust_expect(double *fsp, int n, int min_obs, int d);
orc_table_t *orc_compute_tables(orc_scan_t *s, double **fsp, const orc_opts_t *o);
double orc_spline_interpolate(const orc_spline_t *sp, double x);
void orc_null_model(orc_scan_t *s, double **fsp);

void orc_init_scan_result(orc_pt_t *pt, int chr, const orc_snp_t *snps, const orc_chr_t *lim,
                          int eval_range, int pos, orc_stats_t *st);
void orc_search_maxalpha(orc_pt_t *pt, const orc_snp_t *snps, const orc_table_t *tab, orc_stats_t *st);
orc_pt_t orc_search_maxpos(int chr, int start_pos, int end_pos, const orc_snp_t *snps,
                           const orc_chr_t *lim, int eval_range, int bp_resl,
                           const orc_table_t *tab, orc_stats_t *st);
void orc_scan_chromosome(orc_scan_t *s, const orc_table_t *tab, const orc_opts_t *o, orc_stats_t *st);
void orc_block_permute(orc_snp_t *p, const orc_snp_t *snps, int n, double nbp, double width_mb,
                       orc_rand_t *g, orc_stats_t *st);
void orc_scan_permute(orc_scan_t *s, const orc_table_t *tab, const orc_opts_t *o, orc_stats_t *st);
/* CPU-baseline sample: n_sample evenly spread scan cells (aligned: their permutation-trial
   cells) evaluated on snps; returns wall seconds, *n_done the cells evaluated */
double orc_sample_cells(orc_scan_t *s, const orc_table_t *tab, const orc_opts_t *o, const orc_snp_t *snps,
                        int n_sample, int aligned, int *n_done);
int orc_scan_output(const char *fname, orc_scan_t *s, int max_only, int n_permute, const char *label);

/* whole CLI pipeline on a SNP file (fscl.c:316-337); returns 0 on success */
int orc_run_snpfile(const char *snp_fname, const char *out_fname, const orc_opts_t *o,
                    const char *label, orc_stats_t *st);

void orc_free_scan(orc_scan_t *s);

/* high-precision dump of every scan point (hex floats), for parity tests */
int orc_dump_points(const char *fname, const orc_scan_t *s);
/* scan-chromosome.c:753-796: write <fname>-nulldist (sorts each point's saved CLRs) */
int orc_output_nulldist(const char *fname, orc_scan_t *s);

/* Optional replacement of orc_search_maxalpha inside the position search:
   ref_harness.c plugs the reference's own compiled search_maxalpha in here
   (orc_pt_t / orc_snp_t are layout-identical to scan_pt_t / snp_t). */
typedef void (*orc_maxalpha_hook_t)(orc_pt_t *pt, const orc_snp_t *snps, void *ctx);
void orc_set_maxalpha_hook(orc_maxalpha_hook_t hook, void *ctx);

#endif
