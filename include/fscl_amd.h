/*
 * fscl_amd.h -- drop-in C ABI for slowkoni/fscl's CLR scan + permutation path,
 * implemented on MI355X (gfx950).
 *
 * The data types are byte-compatible with the reference's fscl.h and the
 * entry points keep the reference's names, argument meaning and error
 * behaviour (fatal errors print and exit(1); OOM aborts).  A maintainer
 * replaces the reference objects scan-chromosome.o and sm-search.o (and, if
 * wanted, sm-spline.o background-fsp.o asc-bias.o snp-input.o logmsg.o) by
 * -lfscl_amd; fscl.c's main() links unchanged.  See INTEGRATION.md.
 *
 * Entry point -> reference interface it replaces (/root/reference):
 *   load_snp_input             fscl.h:87   snp-input.c:19-145
 *   background_fsp             fscl.h:91   background-fsp.c:182-316
 *   output_background_fs       fscl.h:93   background-fsp.c:318-336
 *   lchoose                    fscl.h:94   sm-spline.c:41-46
 *   compute_sweep_model_tables fscl.h:97   sm-spline.c:486-520
 *   spline_interpolate         fscl.h:101  sm-spline.c:48-60
 *   init_log_table             fscl.h:104  sm-search.c:14-26
 *   search_maxalpha            fscl.h:105  sm-search.c:269-300   (GPU)
 *   compute_snp_null_model     fscl.h:108  scan-chromosome.c:23-37
 *   scan_chromosome            fscl.h:109  scan-chromosome.c:228-329 (GPU)
 *   scan_permute               fscl.h:111  scan-chromosome.c:582-652 (GPU + host permutation)
 *   scan_output                fscl.h:115  scan-chromosome.c:666-750
 *   ms_openfile/ms_background/ms_next_block fscl.h:118-123 ms-input.c:11-151
 *   ascbias_adjust_background  fscl.h:126  asc-bias.c:27-95
 *   ascbias_adjust_expect      fscl.h:128  asc-bias.c:97-109
 *   configure_logmsg/logmsg/cr_logmsg fscl.h:134-136 logmsg.c:20-52
 */
#ifndef FSCL_AMD_H
#define FSCL_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- data model: same layout as fscl.h:7-76 -------------------------------- */
typedef struct {
  int chr;
  int pos;
  double null_logl;
  int obs_freq;
  int depth_p;
  int folded;
} snp_t;

typedef struct {
  int chr;
  char *name;
  int start_index;
  int n_snps;
  int start_pos;
  int bp_length;
} chr_limits_t;

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
} scan_pt_t;

typedef struct {
  int n_snps;
  snp_t *snps;
  int n_depths;
  int *sample_depths;
  int n_scan_pts;
  scan_pt_t *scan_pts;
  chr_limits_t *chr_limits;
  int n_chromosomes;
} scan_t;

typedef struct {
  int n;
  double *knot_points;
  double **coef;
} spline_t;

typedef struct {
  spline_t **spline_func;
  spline_t **fspline_func;
  int sample_size;
  double **pbk;
  double *fsp;
} sm_ptable_t;

#define LOG_AD_MIN (-20.0)
#define LOG_AD_MAX (4.0)
#define N_SPLINE_KNOTS (200)

enum { MSG_FATAL = 0, MSG_ERROR, MSG_WARN, MSG_STATUS, MSG_DEBUG1, MSG_DEBUG2 };

/* Globals the reference's fscl.c defines (fscl.c:33-34).  The library holds
   weak defaults so it also works without fscl.c; fscl.c's definitions win. */
extern int spline_pts;
extern int n_permute;
extern char *output_fname;
extern char *prepend_label;

/* ---- reference entry points -------------------------------------------------- */
scan_t *load_snp_input(char *snp_fname, int include_invariant, int minimum_obs_depth);
double **background_fsp(scan_t *scan_obj, int force_neutral_spectrum, char *background_fsfname,
                        int include_invariant);
void output_background_fs(char *fname, scan_t *scan_obj, double **fsp);
double lchoose(int n, int k);
sm_ptable_t *compute_sweep_model_tables(scan_t *scan_obj, double **fsp, int asc_depth, int asc_min_freq,
                                        int ascbias_background_only, int include_invariant);
double spline_interpolate(spline_t *spf, double x);
void init_log_table(void);
void search_maxalpha(scan_pt_t *scan_pt, snp_t *snps, sm_ptable_t *sm_p);
void compute_snp_null_model(scan_t *scan_obj, double **fsp);
void scan_chromosome(scan_t *scan_obj, sm_ptable_t *sm_p, int eval_range, int bp_resl, int large_grid_sp,
                     int n_threads);
void scan_permute(scan_t *scan_obj, sm_ptable_t *sm_p, int n_permute, double permute_nbp, double alpha_factor,
                  int n_threads, int eval_range, int bp_resl, int large_grid_sp, double scan_width_mb);
void scan_output(char *output_fname, scan_t *scan_obj, int maximum_only, int n_permute, char *prepend_label);
/* ms input block by block (fscl.h:118-123, ms-input.c; called at fscl.c:281-313),
   with fscl_amd_load_ms_input's semantics: ms_background = every block,
   ms_next_block = the next block as a one-chromosome scan_t, NULL at the end */
void ms_openfile(char *ms_fname);
scan_t *ms_background(char *ms_fname, int ms_segment_length, int ms_folded, int ms_sample_first,
                      int ms_sample_size);
scan_t *ms_next_block(int ms_segment_length, int ms_folded, int ms_sample_first, int ms_sample_size);
double *ascbias_adjust_background(double *bsf, int n, int asc_depth, int min_obs);
void ascbias_adjust_expect(double *fsp, int n, int min_obs, int d);
void configure_logmsg(int level);
void logmsg(int priority, volatile char *s, ...);
void cr_logmsg(int priority, volatile char *s, ...);

/* ---- MI355X extensions ------------------------------------------------------- */
/* ms input (defined semantics): every "//" block is one
   chromosome named by its 1-based block number, a site sits at
   (int)(x * segment_length), sites monomorphic in the chosen sample are
   dropped; returns the same scan_t as load_snp_input */
scan_t *fscl_amd_load_ms_input(const char *ms_fname, int segment_length, int ms_folded, int sample_first,
                               int sample_size);

/* the permutation rand() stream is process-wide and seeded once, as srand(0xFD821A6)
   in the reference's init_options (fscl.c:135): it continues across scan_permute calls.
   fscl_amd_srand restarts it (what a fresh process would see). */
void fscl_amd_srand(unsigned seed);

/* permutation mode of scan_permute.  FSCL_AMD_PERMUTE_PARITY (default): the reference's
   procedure on its rand() stream, results identical to the reference.
   FSCL_AMD_PERMUTE_THROUGHPUT (labelled non-parity): the same procedure with
   counter-based random numbers -- trial t's block permutation from the glibc stream seeded by a
   hash of (seed, t), point i's prune draw in trial t a hash of (seed, t, i) -- so trials run
   independently on every GPU and rank; results are a function of the seed alone (any number of
   GPUs), and match the oracle's --throughput-seed.  $FSCL_AMD_PERMUTE=throughput[:seed]
   overrides.  Returns 0, or -1 for an unknown mode. */
#define FSCL_AMD_PERMUTE_PARITY 0
#define FSCL_AMD_PERMUTE_THROUGHPUT 1
int fscl_amd_set_permute_mode(int mode, unsigned long long seed);

/* what a SIGINT during scan_permute writes (scan-chromosome.c:553-560): by default
   fscl.c's globals output_fname / prepend_label; a library caller sets them here */
void fscl_amd_set_dump_output(const char *fname, const char *label);

/* device selection.  Default: one device, $FSCL_AMD_DEVICE, else LOCAL_RANK, else 0.
   fscl_amd_set_devices(ids, n): this process drives n GPUs (ids NULL: 0 .. n-1; n = 0:
   every visible GPU) -- each batch of grid cells is split into cost-balanced contiguous
   shares, one per device, the host logic (permutation, pruning) runs once; results are
   identical to one device.  fscl_amd_n_devices: the devices opened (0 before the first scan). */
int fscl_amd_set_device(int device);
int fscl_amd_set_devices(const int *devices, int n);
int fscl_amd_n_devices(void);

/* Multi-process parity mode (one process per GPU).  Every rank runs the same
   host logic (rand() stream, block permutation, pruning) and evaluates a
   cost-balanced contiguous share of the grid cells / active points; the
   exchange callback must SUM-allreduce n int64 values across ranks (each slot
   is non-zero on exactly one rank, so the sum reproduces its 64-bit pattern
   exactly).  fn == NULL or world == 1: single process. */
typedef int (*fscl_amd_exchange_fn)(long long *buf, int n, void *ctx);
int fscl_amd_set_ranks(int rank, int world, fscl_amd_exchange_fn fn, void *ctx);

/* The same with the library's own exchange: the ranks share one node, and each batch's
   results are all-gathered through a POSIX shared-memory segment `name` (unique to the job,
   e.g. "/fscl_amd_<uuid>"; created by rank 0, unlinked once every rank has attached).
   Every rank calls it before its first scan; returns 0, or -1 if the ranks could not meet
   (within $FSCL_AMD_RANK_TIMEOUT seconds, default 600).  $FSCL_AMD_SHM_MB (default 64)
   bounds one exchange (64 B per grid cell of a batch). */
int fscl_amd_set_ranks_shm(int rank, int world, const char *name);

/* the cost-balanced contiguous split the ranks use: items [lo, hi) of n go to
   `rank` (costs: SNPs of the cell's chromosome, i.e. its window size) */
void fscl_amd_partition(const double *cost, int n, int rank, int world, int *lo, int *hi);

typedef struct {
  double scan_s;          /* wall seconds of scan_chromosome's evaluation */
  double permute_s;       /* wall seconds of scan_permute */
  double host_perm_s;     /* of which: host permutation generation */
  double kernel_ms;       /* summed GPU kernel time (HIP events) */
  unsigned long long gp_evals;   /* search_maxpos evaluations (grid points x trials) on this rank */
  unsigned long long n_terms, n_null, n_walks, n_maxalpha, n_unsafe, n_slow, n_ties, n_launches;
  unsigned long long negj; /* permutation blocks that hit the reference's negative-j bug (repaired) */
  int trials;             /* permutation trials run */
  int cache_iv0, cache_n_iv, cache_n_rows;  /* LDS coefficient window (fsclg_stats_t) */
  double cache_cover;
  double window_ms;       /* window null-sum kernels (chromosomes above 2*eval_range+1 SNPs) */
  double host_null_s;     /* scan_permute host phases: per-chromosome null sums */
  double host_upload_s;   /*   rows + null sums to the device */
  double search_s;        /*   cell evaluation (launch, kernel, results, rank exchange) */
  double prune_s;         /*   pruning and bookkeeping */
  unsigned long long n_dup_cells, n_ep_saved;  /* fsclg_stats_t: work shared between cells */
  double busy_ms;         /* fsclg_stats_t: union of the search kernels' intervals (overlap counted once) */
  double wait_s;          /* scan_permute: host time blocked on trial results */
  unsigned long long n_crit;  /* scan_permute: cells in the trials' blocking (near-critical) batches */
  unsigned long long n_drain; /* scan_permute: trials that had to wait for every bulk batch in flight */
  int n_devices;          /* local GPUs this process drives */
  int spec_threads;       /* scan_permute: permutation worker threads (0: no speculation) */
  unsigned long long spec_posted; /* trials whose next permutation was generated ahead, per draw count */
  unsigned long long spec_hits;   /*   of which the draw count was among the candidates */
  unsigned long long spec_cands;  /*   candidates generated */
  double spec_wait_s;     /* host time waiting for the chosen candidate to finish */
  unsigned long long spec_done; /* candidates completed (not cancelled) */
  double spec_gen_s;      /* worker seconds spent on the completed candidates */
  unsigned long long n_split_retry; /* fsclg_stats_t: split launches re-run unsplit */
  unsigned long long spec_claimed;  /* chosen candidates not started yet, built by the main thread instead */
  unsigned long long n_merged;      /* scan_permute: bulk cells evaluated in their trial's blocking batch */
  int perm_leader;        /* scan_permute: 1 if the node leader's shared permutation pool ran (one process
                             per GPU), 0 if this rank built its own permutations (single process, or the
                             pool's fallback when the shared segment could not be made) */
  int plan_mode;          /* scan_permute: 1 if the trials' permutations went to the devices as plans
                             (fsclg_slot_set_rows_plan), 0 as rows */
  unsigned long long plan_fallback; /* plan mode: trials whose plan did not fit its buffer (rows instead) */
  unsigned long long spec_rank[8];  /* speculation hits by the candidate's rank in the likeliest-first order
                                       (7: rank 7 or later): how many launched-ahead candidates would cover */
  unsigned long long prestaged;     /* plan mode, one process: trials whose likeliest candidate was applied to a
                                       spare device slot (with its window sums) while the trial before ran */
  unsigned long long prestage_hits; /*   of which it was the trial's permutation (its upload skipped) */
} fscl_amd_stats_t;
void fscl_amd_get_stats(fscl_amd_stats_t *st);
void fscl_amd_reset_stats(void);

/* release the device context (tables / snps) */
void fscl_amd_shutdown(void);

#ifdef __cplusplus
}
#endif
#endif
