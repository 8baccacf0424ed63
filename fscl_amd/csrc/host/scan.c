/* scan.c -- host driver of the CLR scan and block-permutation test
 * (scan-chromosome.c, sm-search.c entry points) over the gfx950 kernels.
 *
 * The host keeps what is inherently serial in the reference: the cell
 * sequence, the block permutation drawn from the glibc rand() stream, the
 * sequential window null sums, and the pruning pass in ascending point order
 * (each may draw rand()).  Every search_maxpos -- the 99.6 % of the
 * reference's time -- runs on the GPU, one workgroup per cell, in lockstep
 * trials: host permutes -> H2D rows -> GPU evaluates all active cells ->
 * D2H CLRs -> host prunes.  With several ranks (one process per GPU) every
 * rank replays the same host logic and evaluates a cost-balanced contiguous
 * share of the cells; one int64 sum-allreduce per trial assembles the CLRs.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <sched.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <unistd.h>

#include <omp.h>

#include "fscl_host.h"

#define CLR_NULL_DIST_SAVE 10000 /* scan-chromosome.c:227 */
#define PERM_SEED 0xFD821A6      /* fscl.c:135 */

/* fscl.c:33-34 define these; weak so the library links standalone */
__attribute__((weak)) int n_permute = 0;
__attribute__((weak)) char *output_fname = NULL;
__attribute__((weak)) char *prepend_label = NULL;

/* The permutation stream: glibc's rand() seeded once per process (srand(0xFD821A6) in
   init_options, fscl.c:135), so it continues across scan_permute calls as the reference's
   does (e.g. the per-block ms loop, fscl.c:296-305).  fscl_amd_srand() restarts it (what
   a fresh process would see). */
static fh_rand_t g_rng;
static int g_rng_seeded = 0;

void fscl_amd_srand(unsigned seed) {
  fh_srand(&g_rng, seed);
  g_rng_seeded = 1;
}

static fh_rand_t *perm_rng(void) {
  if (!g_rng_seeded) fscl_amd_srand(PERM_SEED);
  return &g_rng;
}

/* what the SIGINT dump writes (scan-chromosome.c:553-560 reads fscl.c's globals
   output_fname / prepend_label; a library caller without fscl.c sets them here) */
static const char *g_dump_fname = NULL, *g_dump_label = NULL;
static int g_dump_set = 0;

void fscl_amd_set_dump_output(const char *fname, const char *label) {
  g_dump_fname = fname; g_dump_label = label; g_dump_set = 1;
}

/* ----------------------------------------------------------------- log table */
static double *g_log_table = NULL;

void init_log_table(void) { /* sm-search.c:14-26 */
  int i;
  if (g_log_table) return;
  g_log_table = fh_malloc(sizeof(double) * 0x10000, "log_table");
  for (i = 1; i <= 0xFFFF; i++) g_log_table[i] = log(i);
  g_log_table[0] = 0.; /* a sweep on top of a SNP counts as 1 bp away */
}
const double *fh_log_table(void) { init_log_table(); return g_log_table; }

/* scan-chromosome.c:23-37 */
void compute_snp_null_model(scan_t *s, double **fsp) {
  int i;
  for (i = 0; i < s->n_snps; i++) {
    snp_t *p = s->snps + i;
    const int depth = s->sample_depths[p->depth_p];
    if (p->folded && p->obs_freq != depth - p->obs_freq)
      p->null_logl = log(fsp[p->depth_p][p->obs_freq] + fsp[p->depth_p][depth - p->obs_freq]);
    else
      p->null_logl = log(fsp[p->depth_p][p->obs_freq]);
  }
}

/* sm-search.c:269-295: the coarse grid is an accumulated for-loop, the refine
   grid depends only on the coarse winner, so all of them are tabulated here
   with the reference's own floating-point loops */
int fh_alpha_grid(double *coarse, int max_coarse, double *refine, int32_t *n_refine) {
  const double step = (LOG_AD_MAX - LOG_AD_MIN) / 10.0;
  double la;
  int nc = 0, c;
  for (la = LOG_AD_MIN; la <= LOG_AD_MAX; la += step) {
    if (nc == max_coarse) return -1;
    coarse[nc++] = la;
  }
  for (c = 0; c <= nc; c++) { /* row nc: the initial state lalpha = LOG_AD_MAX (sm-search.c:272) */
    const double best = c < nc ? coarse[c] : LOG_AD_MAX;
    double le = best - step, re = best + step, s2;
    int k = 0;
    if (le < LOG_AD_MIN) le = LOG_AD_MIN;
    if (re > LOG_AD_MAX) re = LOG_AD_MAX;
    s2 = (re - le) / 15.;
    for (la = le + s2; la < re; la += s2) {
      if (k == 16) return -2;
      refine[c * 16 + k++] = la;
    }
    n_refine[c] = k;
  }
  return nc;
}

/* ---------------------------------------------------------- device state
   One host process drives n_dev local GPUs (fscl_amd_set_devices; the fscl CLI's
   --n-gpus), and optionally takes part in a job of `world` such processes (one per GPU,
   fscl_amd_set_ranks / fscl_amd_set_ranks_shm).  The host logic -- cells, rand stream,
   block permutation, null sums, pruning -- runs once per process; every batch of cells is
   split into world * n_dev contiguous shares of equal estimated cost, share
   rank * n_dev + l evaluated by local device l; the local shares land in one host array,
   and with several processes one exchange per batch completes it on every rank. */
#define FH_MAX_DEV 16

typedef struct {
  fsclg_ctx *ctx[FH_MAX_DEV];
  int dev[FH_MAX_DEV];
  int n_dev;                       /* open contexts (0: not yet opened) */
  int want_n;                      /* requested local devices: 0 default (one), -1 all visible */
  int want_dev[FH_MAX_DEV];
  const sm_ptable_t *tab_key;
  const snp_t *snp_key;
  int n_snps_key;
  uint64_t key;
  fh_rowmap_t rm;
  uint32_t *row;  /* row of every site (unpermuted) */
  void *rowp;     /* the same at the staging width */
  int rb;         /* staging width: 1, 2 or 4 bytes per row (the narrowest that holds the device rows) */
  int *chr_list;  /* permutation trials: the chromosomes whose null sum is read (window = whole chromosome,
                     n <= 2 eval_range + 1, init_scan_result); NULL: every chromosome */
  int n_chr_list;
  int32_t *pos;
  double *nullrow;
  int32_t *chr_start, *chr_n;
  int n_chr;
  void *stage[FSCLG_N_SLOTS];  /* one trial's rows (rb bytes each), read by every local device (fsclg_host_alloc) */
  int stage_cap, stage_rb;
  /* ranks */
  int rank, world;
  fscl_amd_exchange_fn xfn;
  void *xctx;
  fh_shm_t *shm;
  FILE *sim;                       /* FSCL_AMD_SIM record / replay file (development: scaling rehearsal) */
  int sim_replay;
  fscl_amd_stats_t st;
} dev_t_;
static dev_t_ D = {.rank = 0, .world = 1};

static void dev_close_all(void) {
  int l, k;
  for (l = 0; l < D.n_dev; l++) fsclg_close(D.ctx[l]);
  for (k = 0; k < FSCLG_N_SLOTS; k++) { fsclg_host_free(D.stage[k]); D.stage[k] = NULL; }
  D.stage_cap = 0;
  D.n_dev = 0;
  D.tab_key = NULL; D.snp_key = NULL;
}

int fscl_amd_set_devices(const int *devices, int n) {
  int l;
  if (n > FH_MAX_DEV || n < -1) return -1;
  dev_close_all();
  if (n == 0 || n == -1) { D.want_n = -1; return 0; }  /* every visible device */
  D.want_n = n;
  for (l = 0; l < n; l++) D.want_dev[l] = devices ? devices[l] : l;
  return 0;
}

int fscl_amd_set_device(int device) { return fscl_amd_set_devices(&device, 1); }

int fscl_amd_n_devices(void) { return D.n_dev; }

static void pool_drop(void);

int fscl_amd_set_ranks(int rank, int world, fscl_amd_exchange_fn fn, void *ctx) {
  if (world < 1 || rank < 0 || rank >= world || (world > 1 && !fn)) return -1;
  pool_drop();  /* the pool belongs to the old exchange */
  fh_shm_close(D.shm); D.shm = NULL;
  D.rank = rank; D.world = world; D.xfn = fn; D.xctx = ctx;
  return 0;
}

int fscl_amd_set_ranks_shm(int rank, int world, const char *name) {
  const char *e = getenv("FSCL_AMD_SHM_MB");
  const size_t cap = (size_t)(e && atoi(e) > 0 ? atoi(e) : 64) << 20;
  if (world < 1 || rank < 0 || rank >= world || !name) return -1;
  pool_drop();  /* the pool belongs to the old exchange */
  fh_shm_close(D.shm); D.shm = NULL;
  D.rank = rank; D.world = world; D.xfn = NULL; D.xctx = NULL;
  if (world == 1) return 0;
  D.shm = fh_shm_open(rank, world, name, cap);
  return D.shm ? 0 : -1;
}

static int dbg(void) {
  static int v = -1;
  if (v < 0) v = getenv("FSCL_AMD_DEBUG") != NULL;
  return v;
}
#define DBG(...) do { if (dbg()) { fprintf(stderr, "[fscl_amd] " __VA_ARGS__); fflush(stderr); } } while (0)

static void dev_check(int r, const char *what) {
  if (r != FSCLG_OK) logmsg(MSG_FATAL, "fscl_amd: %s failed: %s (code %d)", what, fsclg_last_error(), r);
}

/* Scaling rehearsal (test build only: -DFSCL_AMD_REHEARSAL, fscl_amd/_build_rehearsal,
   tools/scale_sim.sh).  FSCL_AMD_SIM=record:<file> (one process, all shares) writes every
   batch's results; FSCL_AMD_SIM=replay:<file>:<world>[:<rank>] runs as one rank of a
   `world`-process job: it evaluates only its own share and takes the others from the recording
   (checking its own bit for bit) -- the time of a W-rank job's rank on one GPU.  The product
   library has no such hook: it refuses the variable. */
static void sim_init(void) {
  static int done = 0;
  const char *e = getenv("FSCL_AMD_SIM");
  if (done) return;
  done = 1;
  if (!e) return;
#ifdef FSCL_AMD_REHEARSAL
  {
    char path[1024];
    int w = 1, r = 0;
    if (sscanf(e, "record:%1023[^:]", path) == 1 && !strncmp(e, "record:", 7)) {
      D.sim = fopen(path, "wb");
      D.sim_replay = 0;
    } else if (!strncmp(e, "replay:", 7) && sscanf(e + 7, "%1023[^:]:%d:%d", path, &w, &r) >= 2) {
      D.sim = fopen(path, "rb");
      D.sim_replay = 1;
      D.world = w; D.rank = r; D.xfn = NULL; D.shm = NULL;
    }
    if (!D.sim) logmsg(MSG_FATAL, "fscl_amd: FSCL_AMD_SIM=%s: cannot open the file", e);
  }
#else
  logmsg(MSG_FATAL, "fscl_amd: FSCL_AMD_SIM is a scaling-rehearsal hook of the test build (fscl_amd/_build_rehearsal)");
#endif
}

#ifdef FSCL_AMD_REHEARSAL
/* the rehearsal's exchange: record the batch, or replay the other ranks' shares */
static void sim_exchange(fsclg_point_t *out, int n, int lo, int hi) {
  if (!D.sim_replay) {
    if (fwrite(&n, sizeof n, 1, D.sim) != 1 || fwrite(out, sizeof(fsclg_point_t), (size_t)n, D.sim) != (size_t)n)
      logmsg(MSG_FATAL, "fscl_amd: FSCL_AMD_SIM record write failed");
  } else {
    fsclg_point_t *rec = fh_malloc(sizeof(fsclg_point_t) * (n ? n : 1), "sim");
    int m = -1, i;
    if (fread(&m, sizeof m, 1, D.sim) != 1 || m != n || fread(rec, sizeof(fsclg_point_t), (size_t)n, D.sim) != (size_t)n)
      logmsg(MSG_FATAL, "fscl_amd: FSCL_AMD_SIM replay: batch of %d cells, recording has %d", n, m);
    for (i = lo; i < hi; i++)
      if (memcmp(&rec[i].lalpha, &out[i].lalpha, 4 * sizeof(double)) != 0)
        logmsg(MSG_FATAL, "fscl_amd: FSCL_AMD_SIM replay: cell %d of a batch differs from the recording", i);
    memcpy(out, rec, sizeof(fsclg_point_t) * (size_t)n);
    free(rec);
  }
}
#endif

static void dev_open(void) {
  int l, n;
  if (D.n_dev) return;
  sim_init();
  if (D.want_n == 0) {
    const char *e = getenv("FSCL_AMD_DEVICE");
    if (!e) e = getenv("LOCAL_RANK");
    D.want_dev[0] = e ? atoi(e) : 0;
    n = 1;
  } else if (D.want_n < 0) {
    n = fsclg_device_count();
    if (n > FH_MAX_DEV) n = FH_MAX_DEV;
    for (l = 0; l < n; l++) D.want_dev[l] = l;
  } else {
    n = D.want_n;
  }
  if (n < 1) logmsg(MSG_FATAL, "fscl_amd: no GPU visible (%s); the scan path runs only on the GPU", fsclg_last_error());
  for (l = 0; l < n; l++) {
    const int r = fsclg_open(D.want_dev[l], &D.ctx[l]);
    if (r != FSCLG_OK)
      logmsg(MSG_FATAL, "fscl_amd: cannot open GPU %d (%s); the scan path runs only on the GPU", D.want_dev[l],
             fsclg_last_error());
    D.dev[l] = D.want_dev[l];
    D.n_dev = l + 1;
    /* batch 0 -- the initial scan and the permutation pipeline's blocking batch: when it has
       few cells, each gets several workgroups (FSCL_AMD_SPLIT members, default 8; 1 = off) */
    {
      const char *e = getenv("FSCL_AMD_SPLIT");
      dev_check(fsclg_set_batch_split(D.ctx[l], 0, e ? (atoi(e) < 1 ? 1 : atoi(e)) : 8), "batch split");
    }
  }
  if (n > 1) logmsg(MSG_STATUS, "fscl_amd: %d GPUs in this process", n);
}

static void free_rowmap(fh_rowmap_t *m) {
  free(m->depth_n); free(m->row_base); free(m->dev_row);
  memset(m, 0, sizeof *m);
}

/* flatten the sm_ptable_t spline trees into [row][interval][4] and upload them to the
   given contexts; device rows are those some site of snps (idx) uses, ranked by site count
   (the device caches a window of every row in LDS), or every row when all_rows is set */
static double *flatten_tables(fh_rowmap_t *m, const sm_ptable_t *sm, int n_depths, const int *depth_n,
                              const snp_t *snps, const int *idx, int n_idx, int all_rows, double **nullrow_out,
                              const double *null_known, int n_known) {
  int d, r, i;
  double *coef, *nullrow;
  unsigned char *seen;
  free_rowmap(m);
  m->n_depths = n_depths;
  m->depth_n = fh_malloc(sizeof(int) * n_depths, "rowmap");
  m->row_base = fh_malloc(sizeof(int) * n_depths, "rowmap");
  m->n_rows = 0;
  for (d = 0; d < n_depths; d++) {
    if (sm[d].sample_size != depth_n[d])
      logmsg(MSG_FATAL, "fscl_amd: sweep-model table %d is for depth %d, data has %d", d, sm[d].sample_size,
             depth_n[d]);
    m->depth_n[d] = depth_n[d];
    m->row_base[d] = m->n_rows;
    m->n_rows += depth_n[d] + 1 + depth_n[d] / 2 + 1;
  }
  m->n_iv = sm[0].spline_func[0]->n;
  /* null_logl is a function of the row (scan-chromosome.c:23-37): take it from the sites */
  seen = fh_calloc(m->n_rows, 1, "null rows");
  m->dev_row = fh_malloc(sizeof(int) * m->n_rows, "rowmap");
  {
    double *full_null = fh_calloc(m->n_rows, sizeof(double), "null rows");
    if (null_known) memcpy(full_null, null_known, sizeof(double) * (size_t)(n_known < m->n_rows ? n_known : m->n_rows));
    for (i = 0; i < n_idx; i++) {
      const snp_t *p = snps + (idx ? idx[i] : i);
      const uint32_t rr = fh_full_row(m, p);
      if (!seen[rr]) { full_null[rr] = p->null_logl; seen[rr] = 1; }
      else if (memcmp(&full_null[rr], &p->null_logl, sizeof(double)) != 0)
        logmsg(MSG_FATAL, "fscl_amd: null_logl differs between sites of the same class (call "
                          "compute_snp_null_model first)");
    }
    if (all_rows) {
      for (r = 0; r < m->n_rows; r++) m->dev_row[r] = r;
      m->n_dev_rows = m->n_rows;
    } else {
      /* device rows in descending order of site count (ties by row) */
      long long *cnt = fh_calloc(m->n_rows, sizeof(long long), "row counts");
      int *ord = fh_malloc(sizeof(int) * m->n_rows, "row order");
      int nu = 0, a, b;
      for (i = 0; i < n_idx; i++) cnt[fh_full_row(m, snps + (idx ? idx[i] : i))]++;
      for (r = 0; r < m->n_rows; r++) if (seen[r]) ord[nu++] = r;
      for (a = 1; a < nu; a++) {  /* insertion sort: a few hundred rows */
        const int v = ord[a];
        for (b = a; b > 0 && (cnt[ord[b - 1]] < cnt[v] || (cnt[ord[b - 1]] == cnt[v] && ord[b - 1] > v)); b--)
          ord[b] = ord[b - 1];
        ord[b] = v;
      }
      for (r = 0; r < m->n_rows; r++) m->dev_row[r] = -1;
      for (a = 0; a < nu; a++) m->dev_row[ord[a]] = a;
      m->n_dev_rows = nu;
      free(cnt);
      free(ord);
    }
    if (m->n_dev_rows == 0) m->n_dev_rows = 1;  /* no sites: one zero row keeps the tables well-formed */
    nullrow = fh_calloc(m->n_dev_rows, sizeof(double), "null rows");
    for (r = 0; r < m->n_rows; r++) if (m->dev_row[r] >= 0) nullrow[m->dev_row[r]] = full_null[r];
    free(full_null);
  }
  coef = fh_calloc((size_t)m->n_dev_rows * m->n_iv * 4, sizeof(double), "flat tables");
  for (d = 0; d < n_depths; d++) {
    const int n = depth_n[d];
    for (r = 0; r <= n + n / 2 + 1; r++) {
      const spline_t *sp = r <= n ? sm[d].spline_func[r] : sm[d].fspline_func[r - n - 1];
      const int dr = m->dev_row[m->row_base[d] + r];
      if (sp->n != m->n_iv) logmsg(MSG_FATAL, "fscl_amd: splines with different knot counts");
      if (dr < 0) continue;
      for (i = 0; i < sp->n; i++) memcpy(coef + ((size_t)dr * m->n_iv + i) * 4, sp->coef[i], sizeof(double) * 4);
    }
  }
  free(seen);
  *nullrow_out = nullrow;
  return coef;
}

static void upload_flat(fsclg_ctx *const *ctx, int n_ctx, const fh_rowmap_t *m, const double *coef,
                        const double *nullrow) {
  double coarse[16], refine[17 * 16];
  int32_t nref[17];
  const int nc = fh_alpha_grid(coarse, 16, refine, nref);
  int l;
  if (nc <= 0) logmsg(MSG_FATAL, "fscl_amd: alpha grid");
  for (l = 0; l < n_ctx; l++) {
    /* log_ad_step of the tables' knot grid (sm-spline.c:325) */
    dev_check(fsclg_upload_tables(ctx[l], fh_log_table(), coef, m->n_dev_rows, m->n_iv, nullrow,
                                  (LOG_AD_MAX - LOG_AD_MIN) / (m->n_iv + 1.)),
              "upload tables");
    dev_check(fsclg_set_alpha_grid(ctx[l], coarse, nc, refine, nref), "alpha grid");
  }
}

static void check_site(const scan_t *s, const snp_t *p) {
  const int n = s->sample_depths[p->depth_p];
  if (p->obs_freq < 0 || p->obs_freq > n || (p->folded && p->obs_freq > n / 2))
    logmsg(MSG_FATAL, "fscl_amd: site class %d out of range for depth %d (folded=%d)", p->obs_freq, n, p->folded);
}

/* content hash (64-bit words, multiply-xorshift), for the device caches' keys */
static uint64_t hash_words(const void *p, size_t n, uint64_t h) {
  const unsigned char *b = p;
  size_t i;
  for (i = 0; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, b + i, 8);
    h = (h ^ w) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
  }
  for (; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

/* make every local device hold this scan's sites and these tables; the cache key is a hash
   of the content (a freed and re-allocated scan may reuse addresses) */
static void prepare(scan_t *s, sm_ptable_t *sm) {
  int i, d, l;
  uint64_t key = 1469598103934665603ull;
  double *coef, *nullrow;
  init_log_table();
  dev_open();
  key = hash_words(&s->n_snps, sizeof s->n_snps, key);
  key = hash_words(s->snps, sizeof(snp_t) * (size_t)s->n_snps, key);
  key = hash_words(s->sample_depths, sizeof(int) * (size_t)s->n_depths, key);
  for (i = 0; i < s->n_chromosomes; i++) key = hash_words(&s->chr_limits[i].start_index, 4 * sizeof(int), key);
  for (d = 0; d < s->n_depths; d++) {
    const int n = sm[d].sample_size;
    key = hash_words(&n, sizeof n, key);
    for (i = 0; i <= n + n / 2 + 1; i++) {
      const spline_t *sp = i <= n ? sm[d].spline_func[i] : sm[d].fspline_func[i - n - 1];
      key = hash_words(sp->coef[0], sizeof(double) * 4 * (size_t)sp->n, key);
    }
  }
  if (D.snp_key && key == D.key) return;
  DBG("prepare: uploading %d sites, %d depths to %d device(s)\n", s->n_snps, s->n_depths, D.n_dev);
  for (i = 0; i < s->n_snps; i++) check_site(s, s->snps + i);
  coef = flatten_tables(&D.rm, sm, s->n_depths, s->sample_depths, s->snps, NULL, s->n_snps, 0, &nullrow, NULL, 0);
  upload_flat(D.ctx, D.n_dev, &D.rm, coef, nullrow);
  free(coef);
  free(D.nullrow);
  D.nullrow = nullrow;
  free(D.row); free(D.pos); free(D.chr_start); free(D.chr_n);
  D.row = fh_malloc(sizeof(uint32_t) * s->n_snps, "rows");
  D.pos = fh_malloc(sizeof(int32_t) * s->n_snps, "positions");
  for (i = 0; i < s->n_snps; i++) {
    D.row[i] = fh_row_of(&D.rm, s->snps + i);
    D.pos[i] = s->snps[i].pos;
  }
  D.rb = D.rm.n_dev_rows <= 0x100 ? 1 : D.rm.n_dev_rows <= 0x10000 ? 2 : 4;
  free(D.rowp);
  D.rowp = fh_malloc((size_t)D.rb * (s->n_snps ? s->n_snps : 1), "rows");
  for (i = 0; i < s->n_snps; i++) {
    if (D.rb == 1) ((uint8_t *)D.rowp)[i] = (uint8_t)D.row[i];
    else if (D.rb == 2) ((uint16_t *)D.rowp)[i] = (uint16_t)D.row[i];
    else ((uint32_t *)D.rowp)[i] = D.row[i];
  }
  D.n_chr = s->n_chromosomes;
  D.chr_start = fh_malloc(sizeof(int32_t) * D.n_chr, "chr");
  D.chr_n = fh_malloc(sizeof(int32_t) * D.n_chr, "chr");
  for (i = 0; i < D.n_chr; i++) {
    D.chr_start[i] = s->chr_limits[i].start_index;
    D.chr_n[i] = s->chr_limits[i].n_snps;
  }
  for (l = 0; l < D.n_dev; l++)
    dev_check(fsclg_upload_snps(D.ctx[l], D.pos, D.row, s->n_snps, D.chr_start, D.chr_n, D.n_chr), "upload snps");
  if (D.stage_cap < s->n_snps || D.stage_rb != D.rb) {
    int k;
    for (k = 0; k < FSCLG_N_SLOTS; k++) {
      fsclg_host_free(D.stage[k]);
      D.stage[k] = fsclg_host_alloc((size_t)D.rb * s->n_snps);
      if (!D.stage[k]) logmsg(MSG_FATAL, "fscl_amd: row staging: %s", fsclg_last_error());
    }
    D.stage_cap = s->n_snps;
    D.stage_rb = D.rb;
  }
  D.tab_key = sm; D.snp_key = s->snps; D.n_snps_key = s->n_snps; D.key = key;
}

/* OpenMP threads of the main thread's whole-chromosome null sums (a speculation miss): with the
   node leader's permutations the other ranks' main threads hold W - 1 of the usable CPUs, and
   an OpenMP team larger than what is left spins in its barriers */
static int g_null_nt = 0;
static int null_threads(void) { return g_null_nt > 0 ? g_null_nt : omp_get_max_threads(); }

/* The block permutation's geometry (perm.c: the 1 Mb extension's end of every site, for the
   scan's sites and scan_width_mb) and the device plan mode: when no trial reads
   a whole-chromosome null sum -- every chromosome longer than its window, C5 -- the host needs
   no permuted rows, and each trial's permutation goes to the devices as its plan
   (fsclg_slot_set_rows_plan): ~16 B per block instead of rb bytes per site, and the host's part
   is drawing the blocks (~50 ns each) instead of an O(n) copy and swap pass. */
typedef struct { int32_t n_ent, n_grp, ok, pad; } plan_hdr_t;
static struct {
  int32_t *ext;        /* fh_ext_table of D's sites for ext_width */
  double ext_width;
  int ext_n;
  uint64_t ext_key;    /* D.key (the sites' content hash) the table was built for */
  fh_perm_geom_t G;
  int on;              /* plan mode in the current permute_pipelined call */
  int ecap, gcap;      /* a plan buffer's capacity: entries, groups */
  size_t bytes;        /* a plan buffer's size */
} PM;

static void perm_geom(double width_mb) {
  if (!PM.ext || PM.ext_n != D.n_snps_key || PM.ext_width != width_mb || PM.ext_key != D.key) {
    free(PM.ext);
    PM.ext = fh_malloc(sizeof(int32_t) * (size_t)(D.n_snps_key ? D.n_snps_key : 1), "extension table");
    fh_ext_table(PM.ext, D.pos, D.chr_start, D.chr_n, D.n_chr, width_mb);
    PM.ext_n = D.n_snps_key; PM.ext_width = width_mb; PM.ext_key = D.key;
  }
  PM.G.n = D.n_snps_key; PM.G.n_chr = D.n_chr; PM.G.chr_start = D.chr_start; PM.G.chr_n = D.chr_n;
  PM.G.pos = D.pos; PM.G.ext = PM.ext;
}

static int32_t *plan_grp(void *buf) { return (int32_t *)((char *)buf + sizeof(plan_hdr_t)); }
static fsclg_swap_t *plan_ent(void *buf) {
  return (fsclg_swap_t *)((char *)buf + sizeof(plan_hdr_t) + ((sizeof(int32_t) * (size_t)(PM.gcap + 1) + 15) & ~(size_t)15));
}

/* one trial's plan into a plan buffer from rand() state *g (advanced); 0, -1 cancelled, -2 it did
   not fit (hdr->ok = 0: the trial's rows are built on the host instead) */
static int plan_into(void *buf, fh_plan_t *P, double nbp, double width_mb, fh_rand_t *g, unsigned long long *negj,
                     const volatile unsigned *gen, unsigned my_gen) {
  plan_hdr_t *h = buf;
  const int r = fh_plan_build(P, &PM.G, nbp, width_mb, g, negj, plan_ent(buf), PM.ecap, plan_grp(buf), PM.gcap,
                              &h->n_ent, &h->n_grp, gen, my_gen);
  h->ok = r == 0;
  return r;
}

/* the row-array routines at each staging width (rows_impl.h), and their dispatch on D.rb */
#define ROW_T uint8_t
#define ROW_SFX 8
#include "rows_impl.h"
#undef ROW_T
#undef ROW_SFX
#define ROW_T uint16_t
#define ROW_SFX 16
#include "rows_impl.h"
#undef ROW_T
#undef ROW_SFX
#define ROW_T uint32_t
#define ROW_SFX 32
#include "rows_impl.h"
#undef ROW_T
#undef ROW_SFX

static void chr_null_sums(const void *row, double *out) {
  if (D.rb == 1) chr_null_sums_8(row, out);
  else if (D.rb == 2) chr_null_sums_16(row, out);
  else chr_null_sums_32(row, out);
}

static int block_permute(void *prow, const void *row, int n, double nbp, double width_mb, fh_rand_t *g,
                         unsigned long long *negj, const volatile unsigned *gen, unsigned my_gen) {
  if (D.rb == 1) return block_permute_8(prow, row, n, nbp, width_mb, g, negj, gen, my_gen);
  if (D.rb == 2) return block_permute_16(prow, row, n, nbp, width_mb, g, negj, gen, my_gen);
  return block_permute_32(prow, row, n, nbp, width_mb, g, negj, gen, my_gen);
}

static int chr_null_sums_1t(const void *row, double *out, const volatile unsigned *gen, unsigned my_gen) {
  if (D.rb == 1) return chr_null_sums_1t_8(row, out, gen, my_gen);
  if (D.rb == 2) return chr_null_sums_1t_16(row, out, gen, my_gen);
  return chr_null_sums_1t_32(row, out, gen, my_gen);
}

/* contiguous share [lo, hi) of n items for one share index: item i belongs to the
   share whose slice of the total cost holds the cost accumulated before i */
void fscl_amd_partition(const double *cost, int n, int rank, int world, int *lo, int *hi) {
  double tot = 0., acc = 0.;
  int i;
  *lo = *hi = n;
  if (world <= 1) { *lo = 0; return; }
  for (i = 0; i < n; i++) tot += cost[i];
  for (i = 0; i < n; i++) {
    int owner = tot > 0 ? (int)(acc / tot * world) : (int)((long long)i * world / n);
    if (owner >= world) owner = world - 1;
    if (owner >= rank && *lo == n) *lo = i;
    if (owner > rank) { *hi = i; break; }
    acc += cost[i];
  }
}

/* the local devices' shares of n items: lo[l], hi[l] (consecutive; this process's range is
   [lo[0], hi[n_dev - 1])) */
static void dev_shares(const double *cost, int n, int *lo, int *hi) {
  const int T = D.world * D.n_dev;
  int l;
  for (l = 0; l < D.n_dev; l++) {
    if (T <= 1) { lo[l] = 0; hi[l] = n; continue; }
    fscl_amd_partition(cost, n, D.rank * D.n_dev + l, T, &lo[l], &hi[l]);
  }
}

/* complete a batch's results on every rank: this process holds [lo, hi) of out[n].  With
   `flags` (this rank's flag word on entry, the OR over the ranks on return) the exchange is
   made even for an empty batch, and out[] must have room for n + 1 items (the torch
   exchange carries the word in item n). */
static void exchange_points_flags(fsclg_point_t *out, int n, int lo, int hi, unsigned *flags) {
#ifdef FSCL_AMD_REHEARSAL
  if (D.sim) { sim_exchange(out, n, lo, hi); return; }
#endif
  if (D.world <= 1 || (n == 0 && !flags)) return;
  if (D.shm) {
    if (fh_shm_allgather_flags(D.shm, out, sizeof(fsclg_point_t), n, lo, hi, flags) != 0)
      logmsg(MSG_FATAL, "fscl_amd: rank exchange failed");
    return;
  }
  memset(out, 0, sizeof(fsclg_point_t) * (size_t)lo);
  memset(out + hi, 0, sizeof(fsclg_point_t) * (size_t)(n - hi));
  if (flags) {
    memset(out + n, 0, sizeof(fsclg_point_t));
    ((long long *)(out + n))[0] = *flags;
  }
  if (D.xfn((long long *)out, (int)((n + (flags ? 1 : 0)) * (sizeof(fsclg_point_t) / sizeof(long long))), D.xctx) != 0)
    logmsg(MSG_FATAL, "fscl_amd: rank exchange failed");
  if (flags) *flags = ((long long *)(out + n))[0] != 0;
}

static void exchange_points(fsclg_point_t *out, int n, int lo, int hi) { exchange_points_flags(out, n, lo, hi, NULL); }

/* every rank's `word` must be the same (collective; not in a rehearsal replay, whose exchanges
   are the recorded batches) */
static void ranks_agree(const char *what, uint64_t word) {
  fsclg_point_t *a;
  int r;
  if (D.world <= 1 || D.sim) return;
  a = fh_calloc((size_t)D.world + 1, sizeof(fsclg_point_t), "agree");
  memcpy(&a[D.rank].lalpha, &word, sizeof word);
  a[D.rank].flags = 1;
  exchange_points(a, D.world, D.rank, D.rank + 1);
  for (r = 0; r < D.world; r++)
    if (a[r].flags != 1 || memcmp(&a[r].lalpha, &word, sizeof word) != 0)
      logmsg(MSG_FATAL, "fscl_amd: ranks disagree on %s (rank %d vs rank %d)", what, D.rank, r);
  free(a);
}

/* the cost of a cell: its window size (snp_likelihood terms scale with it) */
static double window_cost(int chr, int eval_range) {
  return (double)(D.chr_n[chr] < 2 * eval_range + 1 ? D.chr_n[chr] : 2 * eval_range + 1);
}

/* evaluate cells, each local device its share, then complete the results on every rank */
static void eval_cells(const fsclg_cell_t *cells, int n, int eval_range, int bp_resl, fsclg_point_t *out) {
  double *cost = NULL;
  int lo[FH_MAX_DEV], hi[FH_MAX_DEV], l, i;
  if (D.world * D.n_dev > 1) {
    cost = fh_malloc(sizeof(double) * (n ? n : 1), "cost");
    for (i = 0; i < n; i++) cost[i] = window_cost(cells[i].chr, eval_range);
  }
  dev_shares(cost, n, lo, hi);
  free(cost);
  for (l = 0; l < D.n_dev; l++) {
    DBG("search_maxpos: device %d, cells [%d, %d)\n", D.dev[l], lo[l], hi[l]);
    dev_check(fsclg_search_submit(D.ctx[l], 0, 0, cells + lo[l], hi[l] - lo[l], eval_range, bp_resl),
              "search submit");
    D.st.gp_evals += (unsigned long long)(hi[l] - lo[l]);
  }
  for (l = 0; l < D.n_dev; l++) dev_check(fsclg_search_wait(D.ctx[l], 0, out + lo[l]), "search wait");
  exchange_points(out, n, lo[0], hi[D.n_dev - 1]);
}

static void to_scan_pt(scan_pt_t *p, const fsclg_point_t *o) {
  memset(p, 0, sizeof *p);
  p->chr = o->chr; p->nearest_snp = o->nearest_snp; p->sweep_pos = o->sweep_pos; p->n_snps = o->n_snps;
  p->window_start = o->window_start; p->window_end = o->window_end;
  p->lalpha = o->lalpha; p->null_logl = o->null_logl; p->sm_logl = o->sm_logl; p->clr = o->clr;
}

typedef struct { scan_pt_t p; int seq; } keyed_pt_t;
static int pt_cmp(const void *va, const void *vb) {
  const keyed_pt_t *a = va, *b = vb;
  if (a->p.chr != b->p.chr) return a->p.chr < b->p.chr ? -1 : 1;
  if (a->p.sweep_pos != b->p.sweep_pos) return a->p.sweep_pos < b->p.sweep_pos ? -1 : 1;
  return a->seq - b->seq; /* scan-chromosome.c:218-225 under glibc's stable merge sort */
}

/* the unpermuted rows and whole-chromosome null sums into slot 0 of every device */
static void set_original_rows(void) {
  double *nul = fh_malloc(sizeof(double) * (D.n_chr ? D.n_chr : 1), "null sums");
  int l;
  chr_null_sums(D.rowp, nul);
  for (l = 0; l < D.n_dev; l++) {
    dev_check(fsclg_set_rows(D.ctx[l], NULL), "set rows");
    dev_check(fsclg_set_chr_null(D.ctx[l], nul), "set null sums");
  }
  free(nul);
}

/* scan-chromosome.c:228-265 */
void scan_chromosome(scan_t *s, sm_ptable_t *sm, int eval_range, int bp_resl, int large_grid_sp, int n_threads) {
  fsclg_cell_t *cells;
  fsclg_point_t *out;
  keyed_pt_t *kp;
  int n = 0, cap = 1024, chm = 0, pos, i;
  double t0 = fh_now();
  (void)n_threads; /* the GPUs evaluate every cell concurrently */
  prepare(s, sm);
  /* the cell sequence one scan_thread walks (scan-chromosome.c:176-212) */
  cells = fh_malloc(sizeof(fsclg_cell_t) * cap, "cells");
  if (s->n_chromosomes > 0) {
    pos = s->chr_limits[0].start_pos;
    for (;;) {
      if (pos >= s->chr_limits[chm].bp_length) {
        if (++chm == s->n_chromosomes) break;
        pos = s->chr_limits[chm].start_pos;
      }
      if (n == cap) cells = fh_realloc(cells, sizeof(fsclg_cell_t) * (cap *= 2), "cells");
      cells[n].chr = chm;
      cells[n].start_pos = pos;
      cells[n].end_pos = pos + large_grid_sp > s->chr_limits[chm].bp_length ? s->chr_limits[chm].bp_length
                                                                             : pos + large_grid_sp;
      cells[n].pad = 0;
      n++;
      pos += large_grid_sp;
    }
  }
  set_original_rows();
  out = fh_malloc(sizeof(fsclg_point_t) * (n ? n : 1), "points");
  eval_cells(cells, n, eval_range, bp_resl, out);
  kp = fh_malloc(sizeof(keyed_pt_t) * (n ? n : 1), "points");
  for (i = 0; i < n; i++) { to_scan_pt(&kp[i].p, out + i); kp[i].seq = i; }
  qsort(kp, n, sizeof(keyed_pt_t), pt_cmp);
  if (s->scan_pts)
    for (i = 0; i < s->n_scan_pts; i++) free(s->scan_pts[i].permute_clr);
  free(s->scan_pts);
  s->scan_pts = fh_malloc(sizeof(scan_pt_t) * (n ? n : 1), "scan points");
  for (i = 0; i < n; i++) { /* scan-chromosome.c:239-241: a null-distribution buffer per point */
    s->scan_pts[i] = kp[i].p;
    s->scan_pts[i].permute_clr = fh_malloc(sizeof(float) * CLR_NULL_DIST_SAVE, "permute_clr");
  }
  s->n_scan_pts = n;
  free(kp); free(out); free(cells);
  D.st.scan_s += fh_now() - t0;
  logmsg(MSG_STATUS, "\nInitial scan finished.\n");
}

/* ------------------------------------------------------------ permutation */
/* block_permute and chr_null_sums_1t: rows_impl.h (scan-chromosome.c:336-389, 92-94) */

/* one trial's rows (in D.stage[slot]) and null sums to the slot on every local device;
   waits until the slot's previous upload has read the staging before it is rewritten */
static void *slot_stage(int slot) {
  int l;
  for (l = 0; l < D.n_dev; l++) dev_check(fsclg_slot_wait(D.ctx[l], slot), "slot wait");
  return D.stage[slot];
}

static void slot_upload_buf(int slot, const void *rows, const double *nul) {
  int l;
  for (l = 0; l < D.n_dev; l++) dev_check(fsclg_slot_set_rows_packed(D.ctx[l], slot, rows, D.rb, nul), "set rows");
}

static void slot_upload(int slot, const double *nul) { slot_upload_buf(slot, D.stage[slot], nul); }

/* plan mode: the trial's plan (a plan buffer) to the slot on every local device */
static void slot_upload_plan(int slot, void *buf, const double *nul) {
  const plan_hdr_t *h = buf;
  int l;
  for (l = 0; l < D.n_dev; l++)
    dev_check(fsclg_slot_set_rows_plan(D.ctx[l], slot, plan_ent(buf), plan_grp(buf), h->n_grp, nul), "set rows (plan)");
}

static volatile sig_atomic_t g_sigint = 0;
static struct timeval g_last_dump;
static double g_sigint_window = 10.;  /* seconds; FSCL_AMD_SIGINT_WINDOW_MS (tests) shortens it */
static void on_sigint(int sig) { /* scan-chromosome.c:557-569 */
  struct timeval now;
  (void)sig;
  gettimeofday(&now, NULL);
  if ((now.tv_sec - g_last_dump.tv_sec) + (now.tv_usec - g_last_dump.tv_usec) / 1e6 < g_sigint_window) {
    static const char msg[] = "\nanother interrupt signal received, aborting permutation\n";
    if (write(2, msg, sizeof msg - 1) < 0) {}
    _exit(255);
  }
  g_sigint = 1;
}

static void output_clr_null_distribution(const char *fname, scan_t *s);

/* whether to dump now: with several ranks the dump is collective -- every rank drains its
   bulk batches and dumps at the same trial, so they keep making the same exchanges.  Each
   rank's flag goes into one exchange made at the same point of every trial (round); all ranks
   act on the OR.  A signal that arrives after this trial's exchange counts at the next. */
static int sigint_agreed(void) {
  unsigned f = g_sigint ? 1u : 0u;
  if (D.world <= 1 || D.sim) return (int)f;
  if (D.shm) {
    char dummy = 0;
    if (fh_shm_allgather_flags(D.shm, &dummy, 1, 0, 0, 0, &f) != 0) logmsg(MSG_FATAL, "fscl_amd: rank exchange failed");
    return f != 0;
  }
  {
    long long v = f;
    if (D.xfn(&v, 1, D.xctx) != 0) logmsg(MSG_FATAL, "fscl_amd: rank exchange failed");
    return v != 0;
  }
}

/* scan-chromosome.c:553-560, taken between trials: the current table and null distributions
   (one writer: rank 0); every rank restarts its 10-second window, so a second interrupt
   ends all ranks alike */
static void sigint_dump(scan_t *s, int n_perm) {
  const char *fn = g_dump_set ? g_dump_fname : output_fname;
  const char *lb = g_dump_set ? g_dump_label : prepend_label;
  g_sigint = 0;
  if (D.rank == 0) {
    scan_output((char *)fn, s, 0, n_perm, (char *)lb);
    if (fn) output_clr_null_distribution(fn, s);
  }
  gettimeofday(&g_last_dump, NULL);
}

/* ------------------------------------------------ speculative permutations
   (SURVEY §8(f) row 1).  The reference builds each trial's permutation serially from the
   rand() stream after the previous trial's prune draws (scan-chromosome.c:441-456, 488-498),
   and so does this host: trial t+1's permutation starts at the state S left by trial t's own
   permutation, advanced by d_t draws -- one per hit of a point whose permute_p is already
   >= 19.  d_t is known only when trial t's results are in, but its distribution is
   predictable from those points' hit rates.  So while the GPUs evaluate trial t, worker
   threads build the permutations (and whole-chromosome null sums) for the most likely d_t,
   each from its own copy of S; when d_t is known the matching candidate is taken (its end
   state becomes the stream's) and the others are cancelled; a miss builds it on the main
   thread as before.  The stream, and so every result, is unchanged.  Before any point can
   draw (the first 19 trials) d_t = 0 is certain: one candidate, never a miss. */
#define SPEC_MAX 32
#define PB_FREE (-1)
#define PB_CAND (-2)
#define PB_HELD (-3)
#define PB_PRE (-4)   /* a candidate a spare device slot is being prepared from (pre-staging) */

typedef struct {
  void *buf;       /* one trial's rows (D.rb bytes each), pinned: every local device's upload reads it */
  double *nul;     /* its whole-chromosome null sums */
  int owner;       /* the row slot whose upload reads it, or PB_FREE / PB_CAND / PB_HELD */
} pbuf_t;

static struct {
  pthread_t th[SPEC_MAX];
  int n_th;
  pthread_mutex_t mu;
  pthread_cond_t cv, done;
  volatile unsigned gen;  /* bumped to cancel the posted candidates */
  int stop;
  fh_rand_t base;         /* the posted job: S, and the draw counts to build */
  int n_job, next, running;
  int n_keep;             /* workers with an index >= n_keep exit (spec_start shrinking the team) */
  int d[SPEC_MAX], bi[SPEC_MAX], state[SPEC_MAX];  /* 0 queued, 1 running, 2 done, 3 cancelled */
  fh_rand_t end[SPEC_MAX];
  unsigned long long negj[SPEC_MAX];
  const snp_t *snps;      /* the permutation's inputs (fixed while a job is posted) */
  int n;
  double nbp, width_mb;
  pbuf_t pb[FSCLG_N_SLOTS + 3 * SPEC_MAX + 1];
  int n_pb, pb_cap, pb_nchr, pb_rb;
  size_t pb_bytes;        /* one buffer: a trial's rows (rb bytes per site) or, in plan mode, its plan */
  fh_plan_t plan[SPEC_MAX + 1];  /* each worker's plan scratch; [SPEC_MAX]: the main thread's */
  int pb_in_pool;         /* the buffers are the leader's pool's (not owned here) */
} SP = {.mu = PTHREAD_MUTEX_INITIALIZER, .cv = PTHREAD_COND_INITIALIZER, .done = PTHREAD_COND_INITIALIZER,
        .n_keep = SPEC_MAX};

static void *spec_worker(void *arg) {
  const int w = (int)(intptr_t)arg;
  pthread_mutex_lock(&SP.mu);
  for (;;) {
    while (!SP.stop && w < SP.n_keep && SP.next >= SP.n_job) pthread_cond_wait(&SP.cv, &SP.mu);
    if (SP.stop || w >= SP.n_keep) break;
    {
      const int c = SP.next++;
      const unsigned my = SP.gen;
      const int d = SP.d[c];
      pbuf_t *b = SP.pb + SP.bi[c];
      fh_rand_t r = SP.base;
      unsigned long long negj = 0;
      int t, ok;
      SP.state[c] = 1;
      SP.running++;
      pthread_mutex_unlock(&SP.mu);
      const double t0 = fh_now();
      for (t = 0; t < d; t++) (void)fh_rand(&r);
      if (PM.on) { /* the plan only (no whole-chromosome null sums are read in plan mode) */
        ok = plan_into(b->buf, SP.plan + w, SP.nbp, SP.width_mb, &r, &negj, &SP.gen, my) == 0;
        memset(b->nul, 0, sizeof(double) * (size_t)(D.n_chr ? D.n_chr : 1));
      } else
        ok = block_permute(b->buf, D.rowp, SP.n, SP.nbp, SP.width_mb, &r, &negj, &SP.gen, my) == 0 &&
             chr_null_sums_1t(b->buf, b->nul, &SP.gen, my) == 0;
      pthread_mutex_lock(&SP.mu);
      SP.running--;
      if (ok && SP.gen == my) {
        SP.state[c] = 2; SP.end[c] = r; SP.negj[c] = negj;
        D.st.spec_gen_s += fh_now() - t0;
        D.st.spec_done++;
      }
      else { /* cancelled: its buffer is free again (index c may already belong to a newer job) */
        if (SP.gen == my) SP.state[c] = 3;
        b->owner = PB_FREE;
      }
      pthread_cond_broadcast(&SP.done);
    }
  }
  pthread_mutex_unlock(&SP.mu);
  return NULL;
}

/* CPUs this process may use (affinity, capped by the cgroup v2 quota) */
static int usable_cpus(void) {
  cpu_set_t cs;
  int n = 1;
  FILE *f;
  if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = CPU_COUNT(&cs);
  if ((f = fopen("/sys/fs/cgroup/cpu.max", "r"))) {
    char q[32];
    long per = 0;
    if (fscanf(f, "%31s %ld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0) {
      const long c = atol(q) / per;
      if (c >= 1 && c < n) n = (int)c;
    }
    fclose(f);
  }
  return n;
}

/* The node leader's permutations (one process per GPU, parity mode): rank 0 builds every
   trial's permutation once, with speculation on the node's spare CPUs, into a shared pool
   that every rank's devices read (ranks.c, fh_pool_*); the other ranks take each trial's
   rows and rand() state from it instead of replaying the permutation and its speculation.
   FSCL_AMD_PERM_LEADER=0 turns it off (every rank builds its own, as before). */
static struct {
  int on;            /* in the current permute_pipelined call */
  int sizing;        /* the leader's CPU sizing (on, or rank 0 of a rehearsal replay, FSCL_AMD_SIM) */
  fh_pool_t *pool;
  int registered;    /* this rank's devices read the pool directly (else: a copy into D.stage) */
} PL;

static int perm_leader_wanted(void) {
  const char *e = getenv("FSCL_AMD_PERM_LEADER");
  return D.world > 1 && D.shm && !D.sim && (!e || atoi(e) != 0);
}

/* the rehearsal (FSCL_AMD_SIM replay as rank 0 of world) sizes its threads as the leader would */
static int perm_leader_sizing(void) {
  const char *e = getenv("FSCL_AMD_PERM_LEADER");
  return perm_leader_wanted() || (D.sim && D.sim_replay && D.world > 1 && D.rank == 0 && (!e || atoi(e) != 0));
}

/* worker threads: FSCL_AMD_SPEC, else this process's share of the usable CPUs (one process
   per GPU shares the node: LOCAL_WORLD_SIZE) less the main thread.  With the node leader's
   permutations: the leader takes every CPU the ranks' main threads leave, the others none */
static int spec_threads_wanted(void) {
  const char *e = getenv("FSCL_AMD_SPEC"), *lw = getenv("LOCAL_WORLD_SIZE");
  const int local = lw && atoi(lw) > 0 ? atoi(lw) : PL.sizing ? D.world : 1;
  int n;
  if (PL.on && D.rank != 0) return 0;
  n = e ? atoi(e) : PL.sizing ? usable_cpus() - local : usable_cpus() / local - 1;
  return n < 0 ? 0 : n > SPEC_MAX ? SPEC_MAX : n;
}

static void spec_start(void) {
  const int want = spec_threads_wanted();
  if (SP.n_th > want) {  /* a layout with fewer workers than the last call's (no job is posted here) */
    int t;
    pthread_mutex_lock(&SP.mu);
    SP.n_keep = want;
    pthread_cond_broadcast(&SP.cv);
    pthread_mutex_unlock(&SP.mu);
    for (t = want; t < SP.n_th; t++) {
      pthread_join(SP.th[t], NULL);
      fh_plan_free(SP.plan + t);  /* the joined worker's plan scratch */
    }
    SP.n_th = want;
    SP.n_keep = SPEC_MAX;
  }
  while (SP.n_th < want) {
    if (pthread_create(&SP.th[SP.n_th], NULL, spec_worker, (void *)(intptr_t)SP.n_th) != 0) break;
    SP.n_th++;
  }
}

static void spec_stop(void) {
  int t;
  pthread_mutex_lock(&SP.mu);
  SP.stop = 1;
  SP.gen++;
  pthread_cond_broadcast(&SP.cv);
  pthread_mutex_unlock(&SP.mu);
  for (t = 0; t < SP.n_th; t++) pthread_join(SP.th[t], NULL);
  for (t = 0; t <= SPEC_MAX; t++) fh_plan_free(SP.plan + t);  /* workers' and the main thread's plan scratch */
  SP.n_th = 0;
  SP.stop = 0;
  if (!SP.pb_in_pool)
    for (t = 0; t < SP.n_pb; t++) { fsclg_host_free(SP.pb[t].buf); free(SP.pb[t].nul); }
  SP.n_pb = SP.pb_cap = SP.pb_nchr = SP.pb_rb = SP.pb_in_pool = 0;
  SP.pb_bytes = 0;
}

/* candidates posted per trial: two per worker thread (a C4 candidate takes ~0.7 ms of one
   thread, a tail trial at 8 GPUs ~1.5-2.5 ms, so each thread builds two or three; the most
   likely are posted first), at most SPEC_MAX */
static int spec_ncand(void) { return SP.n_th * 2 < SPEC_MAX ? SP.n_th * 2 : SPEC_MAX; }

/* buffers: K slots, the posted candidates, the cancelled ones still running (one per thread)
   and the main thread's own (no job posted) */
static int pb_count(int K) { return K + spec_ncand() + SP.n_th + 1; }

/* one buffer's bytes: a trial's rows, or its plan in plan mode */
static size_t pb_item_bytes(int n_snps) { return PM.on ? PM.bytes : (size_t)D.rb * (size_t)(n_snps ? n_snps : 1); }

/* buffers for K slots, the candidates and the main thread's own (no job posted) */
static void pb_reserve(int n_snps, int K) {
  const int want = pb_count(K);
  const size_t item = pb_item_bytes(n_snps);
  int b;
  if (SP.pb_in_pool) { SP.n_pb = 0; SP.pb_in_pool = 0; SP.pb_cap = 0; }
  if (SP.pb_cap < n_snps || SP.pb_nchr < D.n_chr || SP.pb_rb != D.rb || SP.pb_bytes != item) {
    for (b = 0; b < SP.n_pb; b++) { fsclg_host_free(SP.pb[b].buf); free(SP.pb[b].nul); }
    SP.n_pb = 0;
    SP.pb_cap = n_snps;
    SP.pb_nchr = D.n_chr;
    SP.pb_rb = D.rb;
    SP.pb_bytes = item;
  }
  for (; SP.n_pb < want; SP.n_pb++) {
    pbuf_t *p = SP.pb + SP.n_pb;
    p->buf = fsclg_host_alloc(item);
    if (!p->buf) logmsg(MSG_FATAL, "fscl_amd: row staging: %s", fsclg_last_error());
    p->nul = fh_malloc(sizeof(double) * (SP.pb_nchr ? SP.pb_nchr : 1), "null sums");
  }
  for (b = 0; b < SP.n_pb; b++) SP.pb[b].owner = PB_FREE;
}

static int pb_get(void) {
  int b;
  for (b = 0; b < SP.n_pb; b++)
    if (SP.pb[b].owner == PB_FREE) { SP.pb[b].owner = PB_HELD; return b; }
  logmsg(MSG_FATAL, "fscl_amd: no free permutation buffer");
  return -1;
}

/* the slot's last upload has read its buffer on every local device: free it (the leader's
   pool: once every rank has released the slot too; the releases are counted per rank, and
   every rank makes the same sequence of them) */
static void slot_release(int slot) {
  int l, b;
  for (l = 0; l < D.n_dev; l++) dev_check(fsclg_slot_wait(D.ctx[l], slot), "slot wait");
  if (PL.on) {
    fh_pool_release(PL.pool);
    if (D.rank == 0 && fh_pool_wait_released(PL.pool) != 0)
      logmsg(MSG_FATAL, "fscl_amd: permutation pool: a rank stopped releasing its row slots");
  }
  for (b = 0; b < SP.n_pb; b++) if (SP.pb[b].owner == slot) SP.pb[b].owner = PB_FREE;
}

/* collective: a pool large enough for the leader's buffers (K slots, two per worker thread, one
   for the main thread), then (leader) the buffers carved from it */
static void pool_setup(int n_snps, int K) {
  const size_t rows = (pb_item_bytes(n_snps) + 4095) & ~(size_t)4095;  /* rows, or a plan */
  const size_t nulb = ((sizeof(double) * (size_t)(D.n_chr ? D.n_chr : 1)) + 255) & ~(size_t)255;
  const int nbuf = pb_count(K);
  const size_t want = (size_t)nbuf * (rows + nulb);
  unsigned f = D.rank == 0 && (!PL.pool || fh_pool_bytes(PL.pool) < want) ? 1u : 0u;
  char dummy = 0;
  int b;
  if (fh_shm_allgather_flags(D.shm, &dummy, 1, 0, 0, 0, &f) != 0) logmsg(MSG_FATAL, "fscl_amd: rank exchange failed");
  if (f) {  /* the leader needs a new pool: every rank drops the old one and maps the new one */
    if (PL.pool) {
      if (PL.registered) fsclg_host_unregister(fh_pool_data(PL.pool));
      fh_pool_close(PL.pool);
    }
    PL.pool = fh_pool_open(D.shm, want);
    PL.registered = 0;
    if (!PL.pool) {  /* collective: every rank builds its own permutations this time */
      PL.on = 0;
      PL.sizing = 0;
      g_null_nt = 0;
      spec_start();
      D.st.spec_threads = SP.n_th;
      pb_reserve(n_snps, K);
      return;
    }
    /* FSCL_AMD_POOL_COPY=1 (tests): the fallback taken when page-locking fails, on purpose */
    PL.registered = !getenv("FSCL_AMD_POOL_COPY") &&
                    fsclg_host_register(fh_pool_data(PL.pool), fh_pool_bytes(PL.pool)) == FSCLG_OK;
    if (!PL.registered && !getenv("FSCL_AMD_POOL_COPY"))
      logmsg(MSG_WARN, "fscl_amd: the permutation pool could not be page-locked (%s): rows are copied to the "
                       "device staging\n", fsclg_last_error());
  }
  if (D.rank != 0) return;
  if (!SP.pb_in_pool)
    for (b = 0; b < SP.n_pb; b++) { fsclg_host_free(SP.pb[b].buf); free(SP.pb[b].nul); }
  for (b = 0; b < nbuf; b++) {
    char *base = fh_pool_data(PL.pool) + (size_t)b * (rows + nulb);
    SP.pb[b].buf = base;
    SP.pb[b].nul = (double *)(base + rows);
    SP.pb[b].owner = PB_FREE;
  }
  SP.n_pb = nbuf;
  SP.pb_in_pool = 1;
  SP.pb_cap = n_snps; SP.pb_nchr = D.n_chr; SP.pb_rb = D.rb; SP.pb_bytes = pb_item_bytes(n_snps);
}

static void pool_drop(void) {
  if (!PL.pool) return;
  if (SP.pb_in_pool) { SP.n_pb = 0; SP.pb_in_pool = 0; SP.pb_cap = 0; }
  if (PL.registered) fsclg_host_unregister(fh_pool_data(PL.pool));
  fh_pool_close(PL.pool);
  PL.pool = NULL;
  PL.registered = 0;
}

/* no candidate running (cancelled ones included): the buffers are the caller's again */
static void spec_quiesce(void) {
  pthread_mutex_lock(&SP.mu);
  SP.gen++;
  SP.n_job = SP.next = 0;
  while (SP.running) pthread_cond_wait(&SP.done, &SP.mu);
  pthread_mutex_unlock(&SP.mu);
}

/* build candidates for the draw counts dl[0..nd) from stream state *g */
static void spec_post(const fh_rand_t *g, const int *dl, int nd) {
  int c;
  pthread_mutex_lock(&SP.mu);
  SP.base = *g;
  for (c = 0; c < nd; c++) {
    int b;
    for (b = 0; b < SP.n_pb && SP.pb[b].owner != PB_FREE; b++) {}
    if (b == SP.n_pb) break;
    SP.pb[b].owner = PB_CAND;
    SP.d[c] = dl[c]; SP.bi[c] = b; SP.state[c] = 0;
  }
  SP.next = 0;
  SP.n_job = c;
  SP.gen++;
  pthread_cond_broadcast(&SP.cv);
  pthread_mutex_unlock(&SP.mu);
  D.st.spec_posted++;
  D.st.spec_cands += (unsigned long long)c;
}

/* the candidate for d draws (its end state into *g), or -1; the others are cancelled and
   their buffers freed */
static int spec_take(int d, fh_rand_t *g) {
  int c, hit = -1, bi = -1;
  pthread_mutex_lock(&SP.mu);
  for (c = 0; c < SP.n_job; c++) if (SP.d[c] == d) hit = c;
  if (hit >= 0) D.st.spec_rank[hit < 7 ? hit : 7]++;  /* the draw count's rank among the candidates posted */
  if (hit >= 0 && SP.state[hit] == 0) {
    /* not started (the workers are still on likelier ones): building it here is faster than
       waiting for a worker to get to it; the caller builds it (its buffer is freed below) */
    D.st.spec_claimed++;
    hit = -1;
  }
  if (hit >= 0) {
    const double t0 = fh_now();
    while (SP.state[hit] < 2) pthread_cond_wait(&SP.done, &SP.mu);
    D.st.spec_wait_s += fh_now() - t0;
    if (SP.state[hit] == 2) {
      *g = SP.end[hit];
      D.st.negj += SP.negj[hit];
      bi = SP.bi[hit];
      SP.pb[bi].owner = PB_HELD;
      D.st.spec_hits++;
    }
  }
  /* cancel the rest without waiting: a running one frees its buffer when it stops */
  for (c = 0; c < SP.n_job; c++)
    if (c != hit && SP.state[c] != 1 && SP.pb[SP.bi[c]].owner == PB_CAND) SP.pb[SP.bi[c]].owner = PB_FREE;
  SP.gen++;
  SP.n_job = SP.next = 0;
  pthread_mutex_unlock(&SP.mu);
  return bi;
}

/* ------------------------------------------------ pipelined permutation trials
   scan-chromosome.c:582-652 with --n-threads=1 pruning semantics, K trials in flight
   (FSCL_AMD_DEPTH, default 4, at most FSCLG_N_SLOTS).  What orders the trials is the rand() stream: trial t+1's permutation depends on
   the draws of trial t, and a point draws only on a hit that takes its permute_p to >= 20
   (scan-chromosome.c:488-498); only those points can be pruned.  Each point keeps a queue of
   its results by trial, applied strictly in trial order; u = permute_p + queued results is an
   upper bound of permute_p before the next trial.
     * points with u >= 20 - K ("near-critical") form the trial's blocking batch, on the
       high-priority stream; the next permutation is built once it has been applied;
     * the rest form a bulk batch on a normal stream, waited only when its row slot comes
       round again (K trials later).
   A point with u <= 19 cannot draw in any queued trial (its permute_p stays <= 19 through
   them), so results may be applied late without changing a draw.  A point enters the
   near-critical class at u = 20 - K and can draw no earlier than K - 1 trials later, by when
   its bulk results have been waited for: each trial's draws happen in point order after its
   own permutation, as in the lockstep loop (a violation is caught and the pending batches
   are drained first; never seen, counted in stats).  Results are identical to the lockstep
   order (FSCL_AMD_LOCKSTEP=1). */
#define PQ (FSCLG_N_SLOTS + 2)
typedef struct {
  int trial;
  int have;
  double clr, lalpha;
  int start_pos;
} pres_t;
typedef struct {
  pres_t e[PQ];
  int head, n;
} pqueue_t;

typedef struct {
  int batch;              /* device batch */
  int trial;
  int n, cap;
  int *pt;                /* scan point of each cell, ascending */
  fsclg_cell_t *cells;
  fsclg_point_t *out;
  int submitted;
  int lo[FH_MAX_DEV], hi[FH_MAX_DEV];  /* the local devices' shares, fixed at submission */
} trial_batch_t;

/* per scan point: its permutation cell's cost in the last trial that evaluated it
   (snp_likelihood terms / 1024, from the completed results, so identical on every rank);
   0 = not yet measured */
static double *g_pcost;

static void tb_reserve(trial_batch_t *b, int n) {
  if (n <= b->cap) return;
  b->cap = n;
  b->pt = fh_realloc(b->pt, sizeof(int) * n, "batch");
  b->cells = fh_realloc(b->cells, sizeof(fsclg_cell_t) * n, "batch");
  b->out = fh_realloc(b->out, sizeof(fsclg_point_t) * (n + 1), "batch");  /* + the exchange's flag word */
}

static void tb_free(trial_batch_t *b) { free(b->pt); free(b->cells); free(b->out); memset(b, 0, sizeof *b); }

/* the most cells any device (of every rank) would get if batch B joined batch A: the devices'
   shares are the cost-balanced contiguous split of tb_plan, over the merged ascending point list */
static int merged_max_share(const scan_t *s, const trial_batch_t *A, const trial_batch_t *B, int eval_range) {
  const int T = D.world * D.n_dev, n = A->n + B->n;
  double *cost;
  int ia = 0, ib = 0, k, g, mx = 0;
  if (T <= 1) return n;
  cost = fh_malloc(sizeof(double) * (size_t)n, "cost");
  for (k = 0; k < n; k++) {
    const int pt = (ib >= B->n || (ia < A->n && A->pt[ia] < B->pt[ib])) ? A->pt[ia++] : B->pt[ib++];
    cost[k] = g_pcost && g_pcost[pt] > 0 ? g_pcost[pt] : window_cost(s->scan_pts[pt].chr, eval_range) / 32.0;
  }
  for (g = 0; g < T; g++) {
    int lo, hi;
    fscl_amd_partition(cost, n, g, T, &lo, &hi);
    if (hi - lo > mx) mx = hi - lo;
  }
  free(cost);
  return mx;
}

/* the local devices' shares of a batch, fixed at planning */
static void tb_plan(trial_batch_t *b, int eval_range) {
  double *cost = NULL;
  int i;
  if (D.world * D.n_dev > 1) {
    /* a point's measured cell cost from its last trial, else its window size (~32 terms /
       1024 per window site) */
    cost = fh_malloc(sizeof(double) * (b->n ? b->n : 1), "cost");
    for (i = 0; i < b->n; i++)
      cost[i] = g_pcost && g_pcost[b->pt[i]] > 0 ? g_pcost[b->pt[i]] : window_cost(b->cells[i].chr, eval_range) / 32.0;
  }
  dev_shares(cost, b->n, b->lo, b->hi);
  free(cost);
}

/* each local device's window null sums for its shares of a trial's two batches, before their
   submits (the pruned tail: only the few active cells' windows) */
static void trial_windows(int slot, const trial_batch_t *a, const trial_batch_t *b, int eval_range) {
  fsclg_cell_t *tmp = NULL;
  int l;
  for (l = 0; l < D.n_dev; l++) {
    const int na = a->hi[l] - a->lo[l], nb = b->hi[l] - b->lo[l];
    tmp = fh_realloc(tmp, sizeof(fsclg_cell_t) * (na + nb ? na + nb : 1), "cells");
    memcpy(tmp, a->cells + a->lo[l], sizeof(fsclg_cell_t) * (size_t)na);
    memcpy(tmp + na, b->cells + b->lo[l], sizeof(fsclg_cell_t) * (size_t)nb);
    dev_check(fsclg_slot_windows(D.ctx[l], slot, tmp, na + nb, eval_range), "window sums");
  }
  free(tmp);
}

static void tb_submit(trial_batch_t *b, int slot, int eval_range, int bp_resl) {
  int l;
  for (l = 0; l < D.n_dev; l++) {
    dev_check(fsclg_search_submit(D.ctx[l], b->batch, slot, b->cells + b->lo[l], b->hi[l] - b->lo[l], eval_range,
                                  bp_resl),
              "search submit");
    D.st.gp_evals += (unsigned long long)(b->hi[l] - b->lo[l]);
  }
  b->submitted = 1;
}

/* wait for a batch and file each result in its point's queue; `flags`: see exchange_points_flags */
static void tb_wait_flags(trial_batch_t *b, pqueue_t *pq, unsigned *flags) {
  int k, l;
  double tw = fh_now();
  if (!b->submitted) return;
  for (l = 0; l < D.n_dev; l++) dev_check(fsclg_search_wait(D.ctx[l], b->batch, b->out + b->lo[l]), "search wait");
  b->submitted = 0;
  D.st.wait_s += fh_now() - tw;
  exchange_points_flags(b->out, b->n, b->lo[0], b->hi[D.n_dev - 1], flags);
  if (g_pcost)
    for (k = 0; k < b->n; k++) g_pcost[b->pt[k]] = (double)b->out[k].cost;
  for (k = 0; k < b->n; k++) {
    pqueue_t *q = pq + b->pt[k];
    int j;
    for (j = 0; j < q->n; j++) {
      pres_t *e = q->e + (q->head + j) % PQ;
      if (e->trial == b->trial) {
        e->have = 1; e->clr = b->out[k].clr; e->lalpha = b->out[k].lalpha; e->start_pos = b->cells[k].start_pos;
        break;
      }
    }
    if (j == q->n) logmsg(MSG_FATAL, "fscl_amd: permutation pipeline lost a result");
  }
}

static void tb_wait(trial_batch_t *b, pqueue_t *pq) { tb_wait_flags(b, pq, NULL); }

/* apply point i's queued results in trial order, up to trial `upto`; only trial `draw`
   may draw rand() (scan-chromosome.c:488-502) */
static unsigned long long g_draws;  /* rand() draws of the pruning pass so far */

static void pq_flush(scan_t *s, pqueue_t *pq, int i, int upto, int draw, fh_rand_t *g, int save) {
  pqueue_t *q = pq + i;
  scan_pt_t *p = s->scan_pts + i;
  while (q->n > 0) {
    pres_t *e = q->e + q->head;
    if (!e->have || e->trial > upto) break;
    if (e->clr >= p->clr) {
      p->permute_p++;
      if (p->permute_p >= 20) {
        if (e->trial != draw) logmsg(MSG_FATAL, "fscl_amd: permutation pipeline: out-of-order rand draw");
        g_draws++;
        if (p->permute_p / (double)p->permute_n >= fh_rand(g) / (2147483647 + 1.0))
          p->permute_finished = 1; /* Q7: ratio uses the pre-increment count */
      }
    }
    if (p->permute_n < save) p->permute_clr[p->permute_n] = (float)e->clr;
    p->permute_n++;
    if (e->clr < 0 || e->clr > 1000000 || isnan(e->clr))
      fprintf(stderr, "%d\t%d\t%g\t%1.3e\n", p->chr, e->start_pos, e->clr, exp(e->lalpha));
    q->head = (q->head + 1) % PQ;
    q->n--;
  }
}

/* the most likely draw counts of the trial whose blocking batch is A (into dl, at most nmax):
   every point that may draw hits with probability ~ its hit rate so far; d is their sum, taken
   as normal -- a window of integers around the mean, 3.3 sigma each side */
static int spec_candidates(const scan_t *s, const pqueue_t *pq, const trial_batch_t *A, int nmax, int *dl) {
  double mu = 0., var = 0.;
  int m = 0, k, lo, nd;
  for (k = 0; k < A->n; k++) {
    const scan_pt_t *q = s->scan_pts + A->pt[k];
    if (q->permute_p + pq[A->pt[k]].n >= 20) {
      const double h = (q->permute_p + 1.0) / (q->permute_n + 2.0);
      mu += h;
      var += h * (1. - h);
      m++;
    }
  }
  if (m == 0) { dl[0] = 0; return 1; }
  nd = 2 * (int)ceil(3.3 * sqrt(var)) + 1;
  if (nd > nmax) nd = nmax;
  if (nd > m + 1) nd = m + 1;
  lo = (int)floor(mu + 0.5) - nd / 2;
  if (lo + nd - 1 > m) lo = m - nd + 1;
  if (lo < 0) lo = 0;
  for (k = 0; k < nd; k++) dl[k] = lo + k;
  for (k = 1; k < nd; k++) { /* most likely first: free workers take them in this order */
    const int v = dl[k];
    int b = k;
    for (; b > 0 && fabs(dl[b - 1] - mu) > fabs(v - mu); b--) dl[b] = dl[b - 1];
    dl[b] = v;
  }
  return nd;
}

/* plan mode for this permute_pipelined call (PM.on): only when no chromosome's whole-chromosome
   null sum is read (the host never needs the permuted rows);
   the buffers are sized from one plan drawn from a copy of the stream (every rank draws the same).
   FSCL_AMD_PLAN=0: never; FSCL_AMD_PLAN_ECAP=m (tests): buffers of m entries, so that a plan can
   fail to fit and the trial falls back to rows built on the host */
static int plan_mode_setup(double nbp, double width_mb, const fh_rand_t *g) {
  const char *e = getenv("FSCL_AMD_PLAN"), *ec = getenv("FSCL_AMD_PLAN_ECAP");
  const int n = D.n_snps_key, ecap0 = n + n / 4096 + 16, gcap0 = 1 << 16;
  fh_rand_t r = *g;
  unsigned long long nj = 0;
  fsclg_swap_t *ent;
  int32_t *grp;
  int ne = 0, ng = 0, st;
  if ((e && atoi(e) == 0) || !D.chr_list || D.n_chr_list > 0 || n <= 0) return 0;
  ent = fh_malloc(sizeof(fsclg_swap_t) * (size_t)ecap0, "plan");
  grp = fh_malloc(sizeof(int32_t) * (size_t)(gcap0 + 1), "plan");
  st = fh_plan_build(SP.plan + SPEC_MAX, &PM.G, nbp, width_mb, &r, &nj, ent, ecap0, grp, gcap0, &ne, &ng, NULL, 0);
  free(ent); free(grp);
  if (st != 0) return 0;
  PM.ecap = 2 * ne + 4096 < ecap0 ? 2 * ne + 4096 : ecap0;
  PM.gcap = 2 * ng + 1024;
  if (ec) PM.ecap = atoi(ec) > 0 ? atoi(ec) : 1;
  PM.bytes = sizeof(plan_hdr_t) + ((sizeof(int32_t) * (size_t)(PM.gcap + 1) + 15) & ~(size_t)15) +
             sizeof(fsclg_swap_t) * (size_t)PM.ecap;
  if (PM.bytes > (size_t)D.rb * (size_t)D.stage_cap) {  /* small genomes: the slots' staging holds a plan too */
    const int cap = (int)((PM.bytes + (size_t)D.rb - 1) / (size_t)D.rb);
    int k;
    for (k = 0; k < FSCLG_N_SLOTS; k++) {
      fsclg_host_free(D.stage[k]);
      D.stage[k] = fsclg_host_alloc((size_t)D.rb * (size_t)cap);
      if (!D.stage[k]) logmsg(MSG_FATAL, "fscl_amd: row staging: %s", fsclg_last_error());
    }
    D.stage_cap = cap;
  }
  return 1;
}

static void permute_pipelined(scan_t *s, int n_perm, double permute_nbp, int eval_range, int bp_resl,
                              int large_grid_sp, double scan_width_mb, fh_rand_t *g, int save) {
  const char *env = getenv("FSCL_AMD_DEPTH");
  const int K = env ? (atoi(env) < 2 ? 2 : (atoi(env) > FSCLG_N_SLOTS ? FSCLG_N_SLOTS : atoi(env))) : 4;
  /* row slots (and bulk batches): S >= K trials' rows on the devices (FSCL_AMD_SLOTS, at most FSCLG_N_SLOTS).
     The blocking class keeps the margin K; a bulk batch is waited only when its slot comes round, S
     trials later, and a point that may draw before its bulk results are in drains them first. */
  const char *senv = getenv("FSCL_AMD_SLOTS");
  const int S = senv ? (atoi(senv) < K ? K : (atoi(senv) > FSCLG_N_SLOTS ? FSCLG_N_SLOTS : atoi(senv))) : K;
  /* the bulk batches' cells get up to FSCL_AMD_BULK_SPLIT workgroups each when they are few (the
     pruned tail), so that a bulk batch is done before its slot comes round again */
  const char *bsenv = getenv("FSCL_AMD_BULK_SPLIT");
  const int bulk_split = bsenv ? (atoi(bsenv) < 1 ? 1 : atoi(bsenv)) : 4;
  const int no_merge = getenv("FSCL_AMD_NO_MERGE") != NULL;  /* read once: every rank must decide alike */
  int *act, n_act = s->n_scan_pts, i, k, trial = -1, done = -1;
  pqueue_t *pq;
  double *nul[FSCLG_N_SLOTS];
  trial_batch_t A, Bt[FSCLG_N_SLOTS];
  memset(&A, 0, sizeof A);
  memset(Bt, 0, sizeof Bt);
  A.batch = 0; /* high-priority stream */
  for (k = 0; k < S; k++) {
    int l;
    Bt[k].batch = 2 + k;
    nul[k] = fh_malloc(sizeof(double) * (D.n_chr ? D.n_chr : 1), "null sums");
    for (l = 0; l < D.n_dev; l++) dev_check(fsclg_set_batch_split(D.ctx[l], Bt[k].batch, bulk_split), "batch split");
  }
  act = fh_malloc(sizeof(int) * (n_act ? n_act : 1), "active points");
  pq = fh_calloc(n_act ? n_act : 1, sizeof(pqueue_t), "result queues");
  if (D.world * D.n_dev > 1) g_pcost = fh_calloc(n_act ? n_act : 1, sizeof(double), "point costs");
  tb_reserve(&A, n_act ? n_act : 1);
  for (k = 0; k < S; k++) tb_reserve(&Bt[k], n_act ? n_act : 1);
  for (i = 0; i < n_act; i++) act[i] = i;
  FILE *tt = getenv("FSCL_AMD_TRIAL_TRACE") ? fopen(getenv("FSCL_AMD_TRIAL_TRACE"), "w") : NULL;  /* development aid */
  double tr[8];
  unsigned long long draw_mark = 0;
  int posted = 0, from_spec, bi;
  unsigned sig = 0;
  double *pnul;
  PL.on = perm_leader_wanted();
  PL.sizing = perm_leader_sizing();
  if (PL.sizing) {
    const char *lw = getenv("LOCAL_WORLD_SIZE");
    const int local = lw && atoi(lw) > 0 ? atoi(lw) : D.world;
    g_null_nt = usable_cpus() - local + 1;
    if (g_null_nt < 1) g_null_nt = 1;
  }
  PM.on = plan_mode_setup(permute_nbp, scan_width_mb, g);
  D.st.plan_mode = PM.on;
  /* the switches every rank's batches and collectives follow must agree (an environment variable
     set on one rank only would otherwise diverge the exchanges) */
  ranks_agree("FSCL_AMD_DEPTH / FSCL_AMD_SLOTS / FSCL_AMD_NO_MERGE / FSCL_AMD_PERM_LEADER / FSCL_AMD_PLAN*",
              (uint64_t)K | (uint64_t)S << 4 | (uint64_t)no_merge << 8 | (uint64_t)PL.on << 9 | (uint64_t)PM.on << 10 |
              (uint64_t)(PM.on ? PM.ecap : 0) << 11 | (uint64_t)(PM.on ? PM.gcap : 0) << 40);
  spec_start();
  D.st.spec_threads = SP.n_th;
  if (PL.on) pool_setup(s->n_snps, S);
  else pb_reserve(s->n_snps, S);
  D.st.perm_leader = PL.on;
  SP.snps = s->snps; SP.n = s->n_snps; SP.nbp = permute_nbp; SP.width_mb = scan_width_mb;
  /* pre-staging (plan mode, one process of one rank): while trial t's blocking batch runs, each of
     the likeliest candidates for trial t + 1 that a worker has finished by then is applied to a
     spare device slot with its window sums; when one is taken, its slot is swapped in and the
     trial's upload chain (plan kernels, window sums) is off its critical path.  Not with several
     ranks (the leader's candidates are not the other ranks').  FSCL_AMD_PRESTAGE=n: the n
     likeliest, in spare slots S .. S + n - 1 (0: off) */
  const char *pse = getenv("FSCL_AMD_PRESTAGE");
  int n_pre = pse ? atoi(pse) : 2;  /* 2: C5 one chromosome 15.1 s against 15.4 s with 1, 15.3 s with 3 */
  if (n_pre > FSCLG_N_SLOTS - S) n_pre = FSCLG_N_SLOTS - S;
  if (!(PM.on && D.world == 1 && !PL.on && SP.n_th > 0)) n_pre = 0;
  if (n_pre < 0) n_pre = 0;
  const int pre_on = n_pre > 0;
  int pre_bi[FSCLG_N_SLOTS];  /* the candidate buffer spare slot S + i was prepared from (owner PB_PRE), or -1 */
  for (k = 0; k < FSCLG_N_SLOTS; k++) pre_bi[k] = -1;
  for (;;) {
    const int slot = (trial + 1) % S;
    trial_batch_t *B = &Bt[slot];
    double tp = fh_now();
    void *prow;
    int rows_here = 0;  /* plan mode: this trial's rows were built on the host into D.stage[slot] */
    int use_pre = 0;    /* this trial's permutation was pre-staged in spare slot use_pre (>= S), swapped in */
    tr[0] = tp;
    /* the slot's previous trial: its bulk results (no draws among them) */
    if (B->submitted) {
      tb_wait(B, pq);
      for (k = 0; k < B->n; k++) pq_flush(s, pq, B->pt[k], done, -1, g, save);
    }
    D.st.search_s += fh_now() - tp;
    tp = fh_now();
    tr[1] = tp;
    slot_release(slot);
    if (PL.on && D.rank != 0) {
      /* the leader's permutation of this trial: its rows, its null sums, and the rand() state
         after it (the prune draws that follow are this rank's own, the same as the leader's) */
      size_t ro, no;
      unsigned long long nj;
      fh_rand_t g0 = *g;
      if (fh_pool_take(PL.pool, &ro, &no, g, &nj) != 0) logmsg(MSG_FATAL, "fscl_amd: permutation pool: no leader");
      prow = fh_pool_data(PL.pool) + ro;
      pnul = (double *)(fh_pool_data(PL.pool) + no);
      from_spec = 1;  /* the null sums come with it */
      if (PM.on && !((plan_hdr_t *)prow)->ok) {  /* a plan that did not fit: the rows, from this rank's own stream */
        unsigned long long nj2 = 0;
        block_permute(D.stage[slot], D.rowp, s->n_snps, permute_nbp, scan_width_mb, &g0, &nj2, NULL, 0);
        if (memcmp(&g0, g, sizeof g0) != 0 || nj2 != nj) logmsg(MSG_FATAL, "fscl_amd: permutation pool: stream mismatch");
        rows_here = 1;
        D.st.plan_fallback++;
      }
      D.st.negj += nj;
    } else {
      const unsigned long long negj0 = D.st.negj;
      /* this trial's permutation: the candidate for the previous trial's draw count, else built here */
      bi = posted ? spec_take((int)(g_draws - draw_mark), g) : -1;
      from_spec = bi >= 0;
      for (k = 0; k < n_pre; k++) {
        if (pre_bi[k] < 0) continue;
        if (bi == pre_bi[k]) use_pre = S + k;  /* this spare slot holds the trial */
        else {  /* not taken: free its buffer once the spare's upload has read it */
          int l;
          for (l = 0; l < D.n_dev; l++) dev_check(fsclg_slot_wait(D.ctx[l], S + k), "slot wait");
          if (SP.pb[pre_bi[k]].owner == PB_PRE) SP.pb[pre_bi[k]].owner = PB_FREE;
        }
        pre_bi[k] = -1;
      }
      if (bi < 0) {
        bi = pb_get();
        if (PM.on) {
          const fh_rand_t g0 = *g;
          unsigned long long nj = 0;
          if (plan_into(SP.pb[bi].buf, SP.plan + SPEC_MAX, permute_nbp, scan_width_mb, g, &nj, NULL, 0) == 0)
            D.st.negj += nj;
          else {  /* the plan did not fit its buffer: this trial's rows on the host (hdr.ok = 0 tells the ranks) */
            *g = g0;
            block_permute(D.stage[slot], D.rowp, s->n_snps, permute_nbp, scan_width_mb, g, &D.st.negj, NULL, 0);
            rows_here = 1;
            D.st.plan_fallback++;
          }
        } else
          block_permute(SP.pb[bi].buf, D.rowp, s->n_snps, permute_nbp, scan_width_mb, g, &D.st.negj, NULL, 0);
      }
      SP.pb[bi].owner = slot;
      prow = SP.pb[bi].buf;
      pnul = SP.pb[bi].nul;
      if (PL.on) {  /* the leader: complete and publish it */
        if (!from_spec) {
          if (PM.on) memset(pnul, 0, sizeof(double) * (D.n_chr ? D.n_chr : 1));
          else chr_null_sums(prow, pnul);
        }
        from_spec = 1;
        if (fh_pool_publish(PL.pool, (size_t)((char *)prow - fh_pool_data(PL.pool)),
                            (size_t)((char *)pnul - fh_pool_data(PL.pool)), g, D.st.negj - negj0) != 0)
          logmsg(MSG_FATAL, "fscl_amd: permutation pool: a rank stopped taking permutations");
      }
    }
    D.st.host_perm_s += fh_now() - tp;
    trial++;
    for (i = k = 0; i < n_act; i++)
      if (!s->scan_pts[act[i]].permute_finished) act[k++] = act[i];
    n_act = k;
    cr_logmsg(MSG_STATUS, "Scanning snp block permutations... %7d (%d scan pts remaining)        ", trial, n_act);
    if (n_act == 0 || trial > n_perm) break;
    tp = fh_now();
    tr[2] = tp;
    if (!from_spec && !PM.on) chr_null_sums(prow, pnul);  /* a candidate carries its own; plan mode reads none */
    if (!from_spec && PM.on) memset(pnul, 0, sizeof(double) * (D.n_chr ? D.n_chr : 1));
    D.st.host_null_s += fh_now() - tp;
    memcpy(nul[slot], pnul, sizeof(double) * (D.n_chr ? D.n_chr : 1));
    tp = fh_now();
    if (rows_here) slot_upload_buf(slot, D.stage[slot], nul[slot]);
    else if (use_pre) {
      int l;
      for (l = 0; l < D.n_dev; l++) dev_check(fsclg_slot_swap(D.ctx[l], slot, use_pre), "slot swap");
      D.st.prestage_hits++;
    } else {
      if (PL.on && !PL.registered) {  /* the pool is not page-locked here: through the slot's own staging */
        memcpy(D.stage[slot], prow, PM.on ? PM.bytes : (size_t)D.rb * (size_t)s->n_snps);
        prow = D.stage[slot];
      }
      if (PM.on) slot_upload_plan(slot, prow, nul[slot]);
      else slot_upload_buf(slot, prow, nul[slot]);
    }
    D.st.host_upload_s += fh_now() - tp;
    tp = fh_now();
    A.n = B->n = 0;
    A.trial = B->trial = trial;
    for (i = 0; i < n_act; i++) {
      const int a = act[i];
      const scan_pt_t *q = s->scan_pts + a;
      trial_batch_t *b = q->permute_p + pq[a].n >= 20 - K ? &A : B;
      fsclg_cell_t *cl = b->cells + b->n;
      pres_t *e = pq[a].e + (pq[a].head + pq[a].n) % PQ;
      if (pq[a].n == PQ) logmsg(MSG_FATAL, "fscl_amd: permutation pipeline queue overflow");
      cl->chr = q->chr;
      cl->start_pos = q->sweep_pos - (q->sweep_pos % large_grid_sp); /* Q5: G-aligned, unclipped */
      cl->end_pos = cl->start_pos + large_grid_sp;
      cl->pad = 0;
      b->pt[b->n++] = a;
      e->trial = trial; e->have = 0;
      pq[a].n++;
    }
    /* a small bulk batch joins the blocking batch when the blocking batch's cells keep their full
       split (8 members within 256 workgroups, half the launch budget, HISTORY.md §11.11): the
       early-prune tail's few bulk cells -- the most significant points, which never reach the
       blocking class -- would otherwise run one workgroup per cell and hold up the host K trials
       later.  Merged in ascending point order (the blocking batch's draws go in that order; the
       merged points cannot draw).  The decision depends only on the counts: the same on every
       rank.  FSCL_AMD_NO_MERGE=1: never. */
    if (B->n > 0 && A.n + B->n <= 32 * D.world * D.n_dev && !no_merge &&
        merged_max_share(s, &A, B, eval_range) <= 32) {
      int ia = A.n - 1, ib = B->n - 1, o = A.n + B->n - 1;
      while (ib >= 0) {  /* merge from the back, in place in A (its capacity holds every active point) */
        if (ia >= 0 && A.pt[ia] > B->pt[ib]) { A.pt[o] = A.pt[ia]; A.cells[o] = A.cells[ia]; ia--; }
        else { A.pt[o] = B->pt[ib]; A.cells[o] = B->cells[ib]; ib--; }
        o--;
      }
      D.st.n_merged += (unsigned long long)B->n;
      A.n += B->n;
      B->n = 0;
    }
    D.st.n_crit += (unsigned long long)A.n;
    /* both batches always go through submit / wait (an empty share is a no-op), so that
       every rank takes part in the same exchanges */
    tr[3] = fh_now();
    tb_plan(&A, eval_range);
    tb_plan(B, eval_range);
    trial_windows(slot, &A, B, eval_range);
    tb_submit(&A, slot, eval_range, bp_resl);
    tb_submit(B, slot, eval_range, bp_resl);
    /* while the GPUs work: the next trial's permutation for this trial's likely draw counts */
    posted = SP.n_th > 0 && !(PL.on && D.rank != 0);  /* with the leader's permutations only the leader speculates */
    if (posted) {
      int dl[SPEC_MAX];
      spec_post(g, dl, spec_candidates(s, pq, &A, spec_ncand(), dl));
    }
    draw_mark = g_draws;
    for (k = 0; pre_on && posted && A.n > 0 && k < n_pre; k++) {
      /* the k-th likeliest candidate, if a worker finishes it before the blocking batch is done */
      int st0 = 0, b0 = -1, done = 0;
      for (;;) {
        int l;
        pthread_mutex_lock(&SP.mu);
        if (SP.n_job > k) { st0 = SP.state[k]; b0 = SP.bi[k]; } else st0 = 3;
        if (st0 == 2) SP.pb[b0].owner = PB_PRE;  /* spec_take's cancelling leaves it alone */
        pthread_mutex_unlock(&SP.mu);
        if (st0 >= 2) break;
        for (done = 1, l = 0; l < D.n_dev && done; l++) done = fsclg_search_done(D.ctx[l], A.batch) > 0;
        if (done) break;
        sched_yield();
      }
      if (st0 != 2) break;
      slot_upload_plan(S + k, SP.pb[b0].buf, SP.pb[b0].nul);
      trial_windows(S + k, &A, B, eval_range);
      pre_bi[k] = b0;
      D.st.prestaged++;
    }
    {
      int drain = 0, m = 0;
      for (k = 0; k < A.n; k++) m += s->scan_pts[A.pt[k]].permute_p + pq[A.pt[k]].n >= 20;
      tr[4] = fh_now();
      /* the blocking batch's exchange (made every trial, even for no cells) carries each rank's
         SIGINT flag: every rank gets the OR, so all dump at the same trial (no extra collective) */
      sig = g_sigint ? 1u : 0u;
      tb_wait_flags(&A, pq, &sig);
      if (D.world <= 1 || D.sim) sig = g_sigint ? 1u : 0u;
      tr[5] = fh_now();
      /* a point that may draw in this trial needs every earlier result applied first */
      for (k = 0; k < A.n && !drain; k++) {
        const int a = A.pt[k];
        if (s->scan_pts[a].permute_p + pq[a].n >= 20)
          for (i = 0; i < pq[a].n; i++)
            if (!pq[a].e[(pq[a].head + i) % PQ].have) drain = 1;
      }
      if (drain) { /* never expected: wait the bulk batches in trial order */
        D.st.n_drain++;
        for (;;) {
          trial_batch_t *old = NULL;
          for (k = 0; k < S; k++)
            if (Bt[k].submitted && Bt[k].trial < trial && (!old || Bt[k].trial < old->trial)) old = &Bt[k];
          if (!old) break;
          tb_wait(old, pq);
          for (k = 0; k < old->n; k++) pq_flush(s, pq, old->pt[k], trial - 1, -1, g, save);
        }
      }
      for (k = 0; k < A.n; k++) pq_flush(s, pq, A.pt[k], trial, trial, g, save); /* ascending point order */
      tr[6] = m; tr[7] = (double)(g_draws - draw_mark);
    }
    done = trial;
    D.st.search_s += fh_now() - tp;
    D.st.trials++;
    if (tt) /* trial, active, blocking cells, bulk cells; us: bulk wait, permute, null sums + upload + build,
               submit, blocking wait, flush; points that could draw, draws */
      fprintf(tt, "%d %d %d %d %.0f %.0f %.0f %.0f %.0f %.0f %.0f %.0f\n", trial, n_act, A.n, B->n,
              (tr[1] - tr[0]) * 1e6, (tr[2] - tr[1]) * 1e6, (tr[3] - tr[2]) * 1e6, (tr[4] - tr[3]) * 1e6,
              (tr[5] - tr[4]) * 1e6, (fh_now() - tr[5]) * 1e6, tr[6], tr[7]);
    if (sig) {
      /* the dump shows every trial up to this one: the bulk results still in flight first
         (no draws among them) */
      for (;;) {
        trial_batch_t *old = NULL;
        for (k = 0; k < S; k++)
          if (Bt[k].submitted && (!old || Bt[k].trial < old->trial)) old = &Bt[k];
        if (!old) break;
        tb_wait(old, pq);
        for (k = 0; k < old->n; k++) pq_flush(s, pq, old->pt[k], trial, -1, g, save);
      }
      sigint_dump(s, n_perm);
    }
  }
  /* the bulk batches still in flight, oldest first */
  for (;;) {
    trial_batch_t *old = NULL;
    double tp = fh_now();
    for (k = 0; k < S; k++)
      if (Bt[k].submitted && (!old || Bt[k].trial < old->trial)) old = &Bt[k];
    if (!old) break;
    tb_wait(old, pq);
    for (k = 0; k < old->n; k++) pq_flush(s, pq, old->pt[k], done, -1, g, save);
    D.st.search_s += fh_now() - tp;
  }
  for (i = 0; i < s->n_scan_pts; i++)
    if (pq[i].n) logmsg(MSG_FATAL, "fscl_amd: permutation pipeline: unapplied results");
  for (k = 0; k < n_pre; k++) {  /* the spare slots' last uploads have read their buffers (a trial that did
                                    not come, or one taken just before the last trial ended the loop) */
    int l;
    for (l = 0; l < D.n_dev; l++) dev_check(fsclg_slot_wait(D.ctx[l], S + k), "slot wait");
    if (pre_bi[k] >= 0 && SP.pb[pre_bi[k]].owner == PB_PRE) SP.pb[pre_bi[k]].owner = PB_FREE;
  }
  for (k = 0; k < S; k++) slot_release(k);  /* every upload has read its buffer */
  spec_quiesce();
  PL.on = 0;
  PL.sizing = 0;
  PM.on = 0;
  g_null_nt = 0;
  if (tt) fclose(tt);
  tb_free(&A);
  for (k = 0; k < S; k++) {
    int l;
    for (l = 0; l < D.n_dev; l++) dev_check(fsclg_set_batch_split(D.ctx[l], Bt[k].batch, 1), "batch split");
    tb_free(&Bt[k]);
    free(nul[k]);
  }
  free(act); free(pq);
  free(g_pcost); g_pcost = NULL;
}

/* ------------------------------------------------ throughput mode (non-parity)
   The reference's trials are serial because one rand() stream feeds every permutation and
   every prune draw (scan-chromosome.c:441-456, 488-498).  In throughput mode the randomness
   is counter-based instead, so no trial depends on another:
     * trial t's permutation is block_permute driven by its own generator, the glibc TYPE_3
       stream seeded with tp_trial_seed(seed, t);
     * point i's prune draw in trial t is tp_prune_rand(seed, t, i);
     * a point's results are applied in trial order (hits, the p >= 20 prune test with the
       pre-increment count, the saved null CLRs) and it stops at its first prune, exactly as
       in the reference; results of later trials that were already evaluated are dropped.
   Each point's outcome is then a function of (seed, point) alone: identical for any number
   of GPUs, ranks, trials in flight or worker threads, and restated by the oracle
   (--throughput-seed).  Not bit-identical to the reference (different random numbers), but
   the same procedure: every trial is an independent block permutation, so the p-values have
   the reference's distribution.
   Schedule: rounds of Q = world * n_dev trials, trial r*Q + rank*n_dev + l on local device l;
   up to K rounds in flight (one row slot and one batch per round and device); round r
   evaluates the points still active after every round <= r - K is applied.  Worker threads
   build the permutations (and whole-chromosome null sums) of the next trials ahead, in any
   order, into a ring of pinned buffers. */
static int g_pmode = FSCL_AMD_PERMUTE_PARITY;
static unsigned long long g_pseed = 0xFD821A6ull;

int fscl_amd_set_permute_mode(int mode, unsigned long long seed) {
  if (mode != FSCL_AMD_PERMUTE_PARITY && mode != FSCL_AMD_PERMUTE_THROUGHPUT) return -1;
  g_pmode = mode;
  g_pseed = seed;
  return 0;
}

static uint64_t mix64(uint64_t z) { /* splitmix64's output function */
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static unsigned tp_trial_seed(uint64_t seed, long t) { return (unsigned)(mix64(seed ^ mix64((uint64_t)t + 1)) >> 32); }
static int tp_prune_rand(uint64_t seed, long t, int i) { /* 31 bits, as rand() */
  return (int)(mix64(mix64(seed ^ 0x632BE59BD9B4E019ull) ^ ((uint64_t)(uint32_t)t << 32 | (uint32_t)i)) >> 33);
}

static struct {
  pthread_t th[SPEC_MAX];
  int n_th;
  pthread_mutex_t mu;
  pthread_cond_t cv, done;
  int stop;
  long next, limit, total;  /* local trials j: the next to build; build only j < limit, j < total */
  int nb;                   /* ring of buffers: trial j in buf[j % nb] */
  void **buf;
  double **nul;
  long *built;              /* the trial each buffer holds, -1 none */
  long q, rank_off, n_perm; /* local trial j -> global trial (j / n_dev) * q + rank_off + j % n_dev */
  int n_dev;
  const snp_t *snps;
  int n;
  double nbp, width_mb;
  unsigned long long negj;
  double gen_s;
} TB = {.mu = PTHREAD_MUTEX_INITIALIZER, .cv = PTHREAD_COND_INITIALIZER, .done = PTHREAD_COND_INITIALIZER};

static long tb_trial(long j) { return j / TB.n_dev * TB.q + TB.rank_off + j % TB.n_dev; }

static void tb_build(long j) {
  static const unsigned zero = 0;
  const int b = (int)(j % TB.nb);
  const long t = tb_trial(j);
  unsigned long long negj = 0;
  if (t <= TB.n_perm) {
    fh_rand_t g;
    fh_srand(&g, tp_trial_seed(g_pseed, t));
    block_permute(TB.buf[b], D.rowp, TB.n, TB.nbp, TB.width_mb, &g, &negj, NULL, 0);
    chr_null_sums_1t(TB.buf[b], TB.nul[b], &zero, 0);
  }
  pthread_mutex_lock(&TB.mu);
  TB.negj += negj;
  TB.built[b] = j;
  pthread_cond_broadcast(&TB.done);
  pthread_mutex_unlock(&TB.mu);
}

static void *tb_worker(void *arg) {
  (void)arg;
  pthread_mutex_lock(&TB.mu);
  for (;;) {
    while (!TB.stop && !(TB.next < TB.limit && TB.next < TB.total)) pthread_cond_wait(&TB.cv, &TB.mu);
    if (TB.stop) break;
    {
      const long j = TB.next++;
      double t0;
      pthread_mutex_unlock(&TB.mu);
      t0 = fh_now();
      tb_build(j);
      pthread_mutex_lock(&TB.mu);
      TB.gen_s += fh_now() - t0;
    }
  }
  pthread_mutex_unlock(&TB.mu);
  return NULL;
}

/* trial j's buffer index, once it is built (by the main thread when there are no workers) */
static int tb_get(long j) {
  const int b = (int)(j % TB.nb);
  if (TB.n_th == 0) {
    if (TB.built[b] != j) tb_build(j);
    return b;
  }
  pthread_mutex_lock(&TB.mu);
  while (TB.built[b] != j) pthread_cond_wait(&TB.done, &TB.mu);
  pthread_mutex_unlock(&TB.mu);
  return b;
}

/* every trial below j has been read by its upload: their buffers may take later trials */
static void tb_release(long j) {
  pthread_mutex_lock(&TB.mu);
  if (j + TB.nb > TB.limit) TB.limit = j + TB.nb;
  pthread_cond_broadcast(&TB.cv);
  pthread_mutex_unlock(&TB.mu);
}

static void tb_stop(void) {
  int t;
  pthread_mutex_lock(&TB.mu);
  TB.stop = 1;
  pthread_cond_broadcast(&TB.cv);
  pthread_mutex_unlock(&TB.mu);
  for (t = 0; t < TB.n_th; t++) pthread_join(TB.th[t], NULL);
  for (t = 0; t < TB.nb; t++) { fsclg_host_free(TB.buf[t]); free(TB.nul[t]); }
  free(TB.buf); free(TB.nul); free(TB.built);
  TB.buf = NULL; TB.nul = NULL; TB.built = NULL;
  TB.n_th = TB.nb = 0;
  TB.stop = 0;
}

typedef struct {
  long r;
  int n, cap;
  int *pt;               /* the round's active points, ascending */
  fsclg_cell_t *cells;   /* their G-aligned cells (Q5), the same for every trial of the round */
  fsclg_point_t *out;    /* [Q][n]: trial q of the round at out + q * n */
  size_t out_cap;
  int live[FH_MAX_DEV];  /* local device l submitted its trial */
} tp_round_t;

static void permute_throughput(scan_t *s, int n_perm, double permute_nbp, int eval_range, int bp_resl,
                               int large_grid_sp, double scan_width_mb, int save) {
  /* rounds in flight: about 8 trials in all (at least 2 rounds), so that a pruned point's
     evaluations past its prune stay few; FSCL_AMD_DEPTH overrides */
  const char *env = getenv("FSCL_AMD_DEPTH");
  const int nd = D.n_dev, Q = D.world * nd;
  const int K = env ? (atoi(env) < 1 ? 1 : (atoi(env) > FSCLG_N_SLOTS ? FSCLG_N_SLOTS : atoi(env)))
                    : (Q >= 4 ? 2 : FSCLG_N_SLOTS / Q);
  const long R = ((long)n_perm + Q) / Q; /* rounds holding trials 0 .. n_perm */
  tp_round_t rd[FSCLG_N_SLOTS];
  long r_sub = 0, r_done = 0;
  int stop_sub = 0, i, k, l;
  memset(rd, 0, sizeof rd);
  /* the builders: one ring buffer per trial in flight and per worker, plus a round ahead */
  TB.n_dev = nd; TB.q = Q; TB.rank_off = (long)D.rank * nd; TB.n_perm = n_perm;
  TB.snps = s->snps; TB.n = s->n_snps; TB.nbp = permute_nbp; TB.width_mb = scan_width_mb;
  TB.total = R * nd; TB.next = 0; TB.negj = 0; TB.gen_s = 0.;
  {
    const int want = spec_threads_wanted();
    TB.nb = (K + 1) * nd + want;
    TB.limit = TB.nb;
    TB.buf = fh_calloc((size_t)TB.nb, sizeof(void *), "permutation ring");
    TB.nul = fh_calloc((size_t)TB.nb, sizeof(double *), "permutation ring");
    TB.built = fh_malloc(sizeof(long) * (size_t)TB.nb, "permutation ring");
    for (i = 0; i < TB.nb; i++) {
      TB.buf[i] = fsclg_host_alloc((size_t)D.rb * (s->n_snps ? s->n_snps : 1));
      if (!TB.buf[i]) logmsg(MSG_FATAL, "fscl_amd: row staging: %s", fsclg_last_error());
      TB.nul[i] = fh_malloc(sizeof(double) * (D.n_chr ? D.n_chr : 1), "null sums");
      TB.built[i] = -1;
    }
    for (TB.n_th = 0; TB.n_th < want; TB.n_th++)
      if (pthread_create(&TB.th[TB.n_th], NULL, tb_worker, NULL) != 0) break;
    D.st.spec_threads = TB.n_th;
  }
  while (r_done < r_sub || (!stop_sub && r_sub < R)) {
    if (!stop_sub && r_sub < R && r_sub - r_done < K) {
      tp_round_t *b = rd + r_sub % K;
      const int slot = (int)(r_sub % K);
      double tp = fh_now();
      b->n = 0;
      if (b->cap < s->n_scan_pts) {
        b->cap = s->n_scan_pts;
        b->pt = fh_realloc(b->pt, sizeof(int) * (size_t)(b->cap ? b->cap : 1), "round");
        b->cells = fh_realloc(b->cells, sizeof(fsclg_cell_t) * (size_t)(b->cap ? b->cap : 1), "round");
      }
      for (i = 0; i < s->n_scan_pts; i++) {
        const scan_pt_t *q = s->scan_pts + i;
        fsclg_cell_t *cl = b->cells + b->n;
        if (q->permute_finished) continue;
        cl->chr = q->chr;
        cl->start_pos = q->sweep_pos - (q->sweep_pos % large_grid_sp); /* Q5: G-aligned, unclipped */
        cl->end_pos = cl->start_pos + large_grid_sp;
        cl->pad = 0;
        b->pt[b->n++] = i;
      }
      if (b->n == 0) { stop_sub = 1; continue; }
      if (b->out_cap < (size_t)Q * b->n) {
        b->out_cap = (size_t)Q * b->n;
        b->out = fh_realloc(b->out, sizeof(fsclg_point_t) * b->out_cap, "round");
      }
      b->r = r_sub;
      cr_logmsg(MSG_STATUS, "Scanning snp block permutations... %7ld (%d scan pts remaining)        ", r_sub * Q, b->n);
      for (l = 0; l < nd; l++) {
        const long j = r_sub * nd + l;
        int bi;
        b->live[l] = tb_trial(j) <= n_perm;
        if (!b->live[l]) continue;
        tp = fh_now();
        bi = tb_get(j);
        D.st.host_perm_s += fh_now() - tp;
        tp = fh_now();
        dev_check(fsclg_slot_set_rows_packed(D.ctx[l], slot, TB.buf[bi], D.rb, TB.nul[bi]), "set rows");
        D.st.host_upload_s += fh_now() - tp;
        dev_check(fsclg_slot_windows(D.ctx[l], slot, b->cells, b->n, eval_range), "window sums");
        dev_check(fsclg_search_submit(D.ctx[l], 2 + slot, slot, b->cells, b->n, eval_range, bp_resl), "search submit");
        D.st.gp_evals += (unsigned long long)b->n;
      }
      r_sub++;
    } else {
      tp_round_t *b = rd + r_done % K;
      const int lo = D.rank * nd;
      double tw = fh_now();
      for (l = 0; l < nd; l++)
        if (b->live[l])
          dev_check(fsclg_search_wait(D.ctx[l], 2 + (int)(r_done % K), b->out + (size_t)(lo + l) * b->n), "search wait");
        else
          memset(b->out + (size_t)(lo + l) * b->n, 0, sizeof(fsclg_point_t) * (size_t)b->n);
      D.st.wait_s += fh_now() - tw;
      exchange_points(b->out, Q * b->n, lo * b->n, (lo + nd) * b->n);
      tb_release((r_done + 1) * nd); /* the round's uploads ran before its searches */
      tw = fh_now();
      for (k = 0; k < Q; k++) { /* the round's trials in order, each point in ascending order */
        const long t = r_done * Q + k;
        const fsclg_point_t *o = b->out + (size_t)k * b->n;
        int any = 0;
        if (t > n_perm) break;
        for (i = 0; i < b->n; i++) {
          scan_pt_t *p = s->scan_pts + b->pt[i];
          const double clr = o[i].clr;
          if (p->permute_finished) continue; /* pruned in an earlier trial: later results dropped */
          any = 1;
          if (clr >= p->clr) {
            p->permute_p++;
            if (p->permute_p >= 20 && p->permute_p / (double)p->permute_n >= tp_prune_rand(g_pseed, t, b->pt[i]) / (2147483647 + 1.0))
              p->permute_finished = 1; /* Q7: ratio uses the pre-increment count */
          }
          if (p->permute_n < save) p->permute_clr[p->permute_n] = (float)clr;
          p->permute_n++;
          if (clr < 0 || clr > 1000000 || isnan(clr))
            fprintf(stderr, "%d\t%d\t%g\t%1.3e\n", p->chr, b->cells[i].start_pos, clr, exp(o[i].lalpha));
        }
        D.st.trials += any;
      }
      D.st.prune_s += fh_now() - tw;
      r_done++;
      if (sigint_agreed()) sigint_dump(s, n_perm); /* every trial applied so far */
    }
  }
  D.st.negj += TB.negj;
  D.st.spec_gen_s += TB.gen_s;
  tb_stop();
  for (k = 0; k < FSCLG_N_SLOTS; k++) { free(rd[k].pt); free(rd[k].cells); free(rd[k].out); }
}

/* scan-chromosome.c:582-652 (with --n-threads=1 pruning semantics) */
void scan_permute(scan_t *s, sm_ptable_t *sm, int n_perm, double permute_nbp, double alpha_factor, int n_threads,
                  int eval_range, int bp_resl, int large_grid_sp, double scan_width_mb) {
  fh_rand_t *g = perm_rng();
  void *prow;
  int *act, n_act = s->n_scan_pts, i, k, trial = -1;
  const int save = CLR_NULL_DIST_SAVE; /* scan-chromosome.c:496 */
  fsclg_cell_t *cells;
  fsclg_point_t *out;
  double *nul, t0 = fh_now();
  struct sigaction sa;
  (void)alpha_factor; (void)n_threads; /* -a is inert in the reference too (scan-chromosome.c:584) */
  prepare(s, sm);
  {
    const char *e = getenv("FSCL_AMD_SIGINT_WINDOW_MS");
    g_sigint_window = e ? atof(e) / 1e3 : 10.;
  }
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_sigint;
  sigemptyset(&sa.sa_mask);
  gettimeofday(&g_last_dump, NULL);
  sigaction(SIGINT, &sa, NULL);
  for (i = 0; i < s->n_scan_pts; i++) /* points a caller built without scan_chromosome */
    if (!s->scan_pts[i].permute_clr) s->scan_pts[i].permute_clr = fh_malloc(sizeof(float) * save, "permute_clr");
  {
    const char *e = getenv("FSCL_AMD_PERMUTE"); /* throughput[:seed] overrides the mode set by the API */
    if (e && !strncmp(e, "throughput", 10)) fscl_amd_set_permute_mode(FSCL_AMD_PERMUTE_THROUGHPUT,
                                                                       e[10] == ':' ? strtoull(e + 11, NULL, 0) : g_pseed);
  }
  /* a trial's whole-chromosome null sums are read only where the window is the whole chromosome
     (scan-chromosome.c:75-94): the other chromosomes' sums are not computed */
  D.chr_list = fh_malloc(sizeof(int) * (D.n_chr ? D.n_chr : 1), "chromosomes");
  D.n_chr_list = 0;
  for (i = 0; i < D.n_chr; i++)
    if ((long long)D.chr_n[i] <= 2ll * eval_range + 1) D.chr_list[D.n_chr_list++] = i;
  perm_geom(scan_width_mb);
  if (g_pmode == FSCL_AMD_PERMUTE_THROUGHPUT) { /* the rand() stream is not used */
    permute_throughput(s, n_perm, permute_nbp, eval_range, bp_resl, large_grid_sp, scan_width_mb, save);
    goto done;
  }
  (void)fh_rand(g); /* scan-chromosome.c:440: the single thread's usleep() draw */
  if (!getenv("FSCL_AMD_LOCKSTEP")) {
    permute_pipelined(s, n_perm, permute_nbp, eval_range, bp_resl, large_grid_sp, scan_width_mb, g, save);
    goto done;
  }
  /* lockstep: permute -> rows to the devices -> every active cell -> prune */
  act = fh_malloc(sizeof(int) * (n_act ? n_act : 1), "active points");
  cells = fh_malloc(sizeof(fsclg_cell_t) * (n_act ? n_act : 1), "cells");
  out = fh_malloc(sizeof(fsclg_point_t) * (n_act ? n_act : 1), "points");
  nul = fh_malloc(sizeof(double) * (D.n_chr ? D.n_chr : 1), "null sums");
  for (i = 0; i < s->n_scan_pts; i++) act[i] = i;
  for (;;) {
    double tp = fh_now();
    prow = slot_stage(0);
    block_permute(prow, D.rowp, s->n_snps, permute_nbp, scan_width_mb, g, &D.st.negj, NULL, 0);
    D.st.host_perm_s += fh_now() - tp;
    trial++;
    for (i = k = 0; i < n_act; i++)
      if (!s->scan_pts[act[i]].permute_finished) act[k++] = act[i];
    n_act = k;
    cr_logmsg(MSG_STATUS, "Scanning snp block permutations... %7d (%d scan pts remaining)        ", trial, n_act);
    if (n_act == 0 || trial > n_perm) break;
    tp = fh_now();
    chr_null_sums(prow, nul);
    D.st.host_null_s += fh_now() - tp;
    tp = fh_now();
    slot_upload(0, nul);
    D.st.host_upload_s += fh_now() - tp;
    for (i = 0; i < n_act; i++) {
      const scan_pt_t *q = s->scan_pts + act[i];
      cells[i].chr = q->chr;
      cells[i].start_pos = q->sweep_pos - (q->sweep_pos % large_grid_sp); /* Q5: G-aligned, unclipped */
      cells[i].end_pos = cells[i].start_pos + large_grid_sp;
      cells[i].pad = 0;
    }
    tp = fh_now();
    eval_cells(cells, n_act, eval_range, bp_resl, out);
    D.st.search_s += fh_now() - tp;
    tp = fh_now();
    D.st.trials++;
    for (i = 0; i < n_act; i++) { /* scan-chromosome.c:488-502, ascending point order */
      scan_pt_t *q = s->scan_pts + act[i];
      const double clr = out[i].clr;
      if (clr >= q->clr) {
        q->permute_p++;
        if (q->permute_p >= 20 && q->permute_p / (double)q->permute_n >= fh_rand(g) / (2147483647 + 1.0))
          q->permute_finished = 1; /* Q7: ratio uses the pre-increment count */
      }
      if (q->permute_n < save) q->permute_clr[q->permute_n] = (float)clr;
      q->permute_n++;
      if (clr < 0 || clr > 1000000 || isnan(clr))
        fprintf(stderr, "%d\t%d\t%g\t%1.3e\n", q->chr, cells[i].start_pos, clr, exp(out[i].lalpha));
    }
    D.st.prune_s += fh_now() - tp;
    if (sigint_agreed()) sigint_dump(s, n_perm);
  }
  free(act); free(cells); free(out); free(nul);
done:
  cr_logmsg(MSG_STATUS, "Scanning snp block permutations... finished.\n");
  signal(SIGINT, SIG_DFL);
  free(D.chr_list);
  D.chr_list = NULL;
  D.n_chr_list = 0;
  set_original_rows();
  D.st.permute_s += fh_now() - t0;
}

/* --------------------------------------------------- search_maxalpha drop-in
   sm-search.c:269-300 for one caller-initialised point.  The reference calls it once per
   point from its own scan loop (scan-chromosome.c:126-135), so the drop-in keeps a context
   of its own on the first device, with state that survives between calls:
     * the tables, keyed by the sm_ptable_t pointer, the depths in use and a hash of the
       coefficients (every row of those depths on the device; a row's null_logl, known only
       from the sites, is added when a window first shows it);
     * the sites of the last window uploaded, as (position, row) pairs: the next call reuses
       them when its window lies inside and its sites compare equal (the caller's scan
       loop evaluates many points of one window; a permuted array differs and is uploaded).
   The scan path's own contexts are not touched. */
static struct {
  fsclg_ctx *ctx;
  const sm_ptable_t *sm;
  int n_depths;
  uint64_t tab_hash;
  fh_rowmap_t rm;
  double *null_full;       /* [rm.n_rows] null_logl of each row, as seen so far */
  unsigned char *null_seen;
  int32_t *pos;            /* uploaded window [lo, lo + n) */
  uint32_t *row;
  int lo, n, cap;
  int32_t *tpos;
  uint32_t *trow;
  int tcap;
} DI;

/* the first and last coefficient blocks of every row (tables are built once and never
   changed by the reference; this catches a caller that rebuilds them in place) */
static uint64_t tables_hash(const sm_ptable_t *sm, int n_depths) {
  uint64_t h = 88172645463325252ull;
  int d, i;
  for (d = 0; d < n_depths; d++) {
    const int n = sm[d].sample_size;
    h = hash_words(&n, sizeof n, h);
    for (i = 0; i <= n + n / 2 + 1; i++) {
      const spline_t *sp = i <= n ? sm[d].spline_func[i] : sm[d].fspline_func[i - n - 1];
      h = hash_words(sp->coef[0], sizeof(double) * 4, h);
      h = hash_words(sp->coef[sp->n - 1], sizeof(double) * 4, h);
    }
  }
  return h;
}

/* every row of depths [0, n_depths) on the drop-in context; the null values known so far
   (rows of earlier depths keep their numbers when depths are added) plus this window's */
static void dropin_tables(const sm_ptable_t *sm, int n_depths, const snp_t *snps, int ws, int n, int keep) {
  int *dn = fh_malloc(sizeof(int) * n_depths, "depths"), *idx = fh_malloc(sizeof(int) * (n ? n : 1), "window");
  const int n_known = keep ? DI.rm.n_rows : 0;
  unsigned char *seen;
  double *coef, *nullrow;
  int d, i;
  for (d = 0; d < n_depths; d++) dn[d] = sm[d].sample_size;
  for (i = 0; i < n; i++) idx[i] = ws + i;
  coef = flatten_tables(&DI.rm, sm, n_depths, dn, snps, idx, n, 1, &nullrow, DI.null_full, n_known);
  seen = fh_calloc(DI.rm.n_rows, 1, "null rows");
  if (n_known) memcpy(seen, DI.null_seen, (size_t)(n_known < DI.rm.n_rows ? n_known : DI.rm.n_rows));
  for (i = 0; i < n; i++) seen[fh_full_row(&DI.rm, snps + ws + i)] = 1;
  free(DI.null_full); free(DI.null_seen);
  DI.null_full = nullrow;  /* every row: device row = row */
  DI.null_seen = seen;
  upload_flat(&DI.ctx, 1, &DI.rm, coef, nullrow);
  free(coef); free(dn); free(idx);
  DI.n = 0;  /* the tables were replaced: the sites go up again */
}

static void search_maxalpha_locked(scan_pt_t *pt, snp_t *snps, sm_ptable_t *sm) {
  const int ws = pt->window_start, we = pt->window_end, n = we - ws + 1;
  int i, maxd = 0, need_tables, reuse;
  fsclg_point_t p;
  init_log_table();
  dev_open();
  if (!DI.ctx) dev_check(fsclg_open(D.dev[0], &DI.ctx), "open the search_maxalpha context");
  if (n <= 0) logmsg(MSG_FATAL, "fscl_amd: search_maxalpha: empty window");
  for (i = ws; i <= we; i++) if (snps[i].depth_p > maxd) maxd = snps[i].depth_p;
  need_tables = DI.sm != sm || DI.n_depths < maxd + 1 || tables_hash(sm, DI.n_depths) != DI.tab_hash;
  if (!need_tables) /* a row class this window shows for the first time: its null value */
    for (i = ws; i <= we && !need_tables; i++) {
      const uint32_t r = fh_full_row(&DI.rm, snps + i);
      if (!DI.null_seen[r]) need_tables = 1;
      else if (memcmp(&DI.null_full[r], &snps[i].null_logl, sizeof(double)) != 0)
        logmsg(MSG_FATAL, "fscl_amd: null_logl differs between sites of the same class (call "
                          "compute_snp_null_model first)");
    }
  if (need_tables) {
    const int same = DI.sm == sm && DI.null_full != NULL;
    const int nd = !same || maxd + 1 > DI.n_depths ? maxd + 1 : DI.n_depths;
    dropin_tables(sm, nd, snps, ws, n, same);
    DI.sm = sm; DI.n_depths = nd; DI.tab_hash = tables_hash(sm, nd);
  }
  /* the window's sites as the device holds them */
  if (DI.tcap < n) {
    DI.tcap = n;
    DI.tpos = fh_realloc(DI.tpos, sizeof(int32_t) * n, "window");
    DI.trow = fh_realloc(DI.trow, sizeof(uint32_t) * n, "window");
  }
  for (i = 0; i < n; i++) { DI.tpos[i] = snps[ws + i].pos; DI.trow[i] = fh_row_of(&DI.rm, snps + ws + i); }
  reuse = DI.n > 0 && ws >= DI.lo && we < DI.lo + DI.n &&
          !memcmp(DI.pos + (ws - DI.lo), DI.tpos, sizeof(int32_t) * n) &&
          !memcmp(DI.row + (ws - DI.lo), DI.trow, sizeof(uint32_t) * n);
  if (!reuse) {
    int32_t cs = 0, cn = n;
    if (DI.cap < n) {
      DI.cap = n;
      DI.pos = fh_realloc(DI.pos, sizeof(int32_t) * n, "window");
      DI.row = fh_realloc(DI.row, sizeof(uint32_t) * n, "window");
    }
    memcpy(DI.pos, DI.tpos, sizeof(int32_t) * n);
    memcpy(DI.row, DI.trow, sizeof(uint32_t) * n);
    DI.lo = ws; DI.n = n;
    dev_check(fsclg_upload_snps(DI.ctx, DI.pos, DI.row, n, &cs, &cn, 1), "upload window");
  }
  memset(&p, 0, sizeof p);
  p.chr = 0; p.nearest_snp = pt->nearest_snp - DI.lo; p.sweep_pos = pt->sweep_pos; p.n_snps = pt->n_snps;
  p.window_start = ws - DI.lo; p.window_end = we - DI.lo; p.null_logl = pt->null_logl;
  dev_check(fsclg_search_points(DI.ctx, &p, 1), "search_maxalpha");
  pt->lalpha = p.lalpha; pt->sm_logl = p.sm_logl; pt->clr = p.clr;
}

/* the reference calls search_maxalpha from its --n-threads workers (scan-chromosome.c:258,
   514, 531): the drop-in's state (DI: context, tables, the resident window) is shared, so
   calls are serialised; each is one short device launch */
static pthread_mutex_t g_dropin_mu = PTHREAD_MUTEX_INITIALIZER;

void search_maxalpha(scan_pt_t *pt, snp_t *snps, sm_ptable_t *sm) {
  pthread_mutex_lock(&g_dropin_mu);
  search_maxalpha_locked(pt, snps, sm);
  pthread_mutex_unlock(&g_dropin_mu);
}

/* ---------------------------------------------------------------- output */
void scan_output(char *fname, scan_t *s, int maximum_only, int n_perm, char *label) {
  FILE *f = stdout;
  const scan_pt_t *best;
  double max_clr;
  char pos_str[64];
  int i;
  if (D.world > 1 && D.rank != 0) return; /* one writer */
  if (fname) {
    f = fopen(fname, "w");
    if (!f) { fprintf(stderr, "Can't open output file \"%s\" (%s)", fname, strerror(errno)); return; }
  }
  if (s->n_scan_pts == 0) { if (fname) fclose(f); return; }
  best = s->scan_pts;
  max_clr = s->scan_pts[0].clr;
  for (i = 1; i < s->n_scan_pts; i++)
    if (s->scan_pts[i].clr > max_clr) { max_clr = s->scan_pts[i].clr; best = s->scan_pts + i; }
  if (best->sweep_pos > 1000000)
    snprintf(pos_str, sizeof pos_str, "chromosome %s %1.2f Mb", s->chr_limits[best->chr].name, best->sweep_pos / 1e6);
  else if (best->sweep_pos > 2000)
    snprintf(pos_str, sizeof pos_str, "chromosome %s %1.2f Kb", s->chr_limits[best->chr].name, best->sweep_pos / 1e3);
  else
    snprintf(pos_str, sizeof pos_str, "chromosome %s %d bp", s->chr_limits[best->chr].name, best->sweep_pos);
  logmsg(MSG_STATUS, "\rOutput complete -- maximum CLR of %g at %s (alpha = %g)\n", max_clr, pos_str,
         exp(best->lalpha));
  if (maximum_only) {
    if (label) fprintf(f, "%s\t", label);
    fprintf(f, "%s\t%d\t%1.2f\t%1.3e\t%d\t%d\t%d\n", s->chr_limits[best->chr].name, best->sweep_pos, max_clr,
            exp(best->lalpha), best->n_snps, s->snps[best->window_start].pos, s->snps[best->window_end].pos);
    if (fname) fclose(f); /* the reference leaks the handle here (scan-chromosome.c:715) */
    return;
  }
  for (i = 0; i < s->n_scan_pts; i++) {
    const scan_pt_t *q = s->scan_pts + i;
    if (label) fprintf(f, "%s\t", label);
    if (n_perm > 0) {
      /* Q8: an empirical ratio, no chi-square projection */
      const double pv = q->permute_p < 2 ? 1.0 / q->permute_n : (q->permute_p - 1.0) / (double)(q->permute_n - 1.0);
      fprintf(f, "%s\t%d\t%1.2f\t%1.3e\t%d\t%d\t%1.3f\n", s->chr_limits[q->chr].name, q->sweep_pos, q->clr,
              exp(q->lalpha), q->permute_p, q->permute_n, -log10(pv));
    } else {
      fprintf(f, "%s\t%d\t%1.2f\t%1.3e\t%d\t%d\t%d\n", s->chr_limits[q->chr].name, q->sweep_pos, q->clr,
              exp(q->lalpha), q->n_snps, s->snps[q->window_start].pos, s->snps[q->window_end].pos);
    }
  }
  if (fname) fclose(f);
}

static int float_cmp(const void *a, const void *b) {
  const float x = *(const float *)a, y = *(const float *)b;
  return (x > y) - (x < y);
}

/* scan-chromosome.c:753-796 */
static void output_clr_null_distribution(const char *fname, scan_t *s) {
  char *fn = fh_malloc(strlen(fname) + 20, "fname");
  FILE *f;
  int i, j;
  sprintf(fn, "%s-nulldist", fname);
  f = fopen(fn, "w");
  free(fn);
  if (!f) { fprintf(stderr, "Can't open output file for CLR null distribution (%s)\n", strerror(errno)); return; }
  fprintf(f, "chr\tpos\tCLR\talpha\tp\tn");
  for (j = 0; j < CLR_NULL_DIST_SAVE; j++) fprintf(f, "\t%1.4f", j / (double)CLR_NULL_DIST_SAVE);
  fprintf(f, "\n");
  for (i = 0; i < s->n_scan_pts; i++) {
    scan_pt_t *q = s->scan_pts + i;
    const int np = q->permute_n < CLR_NULL_DIST_SAVE ? q->permute_n : CLR_NULL_DIST_SAVE;
    if (q->permute_clr) qsort(q->permute_clr, np, sizeof(float), float_cmp);
    fprintf(f, "%s\t%d\t%1.3f\t%1.3e\t%d\t%d", s->chr_limits[q->chr].name, q->sweep_pos, q->clr, exp(q->lalpha),
            q->permute_p, q->permute_n);
    for (j = 0; j < np && q->permute_clr; j++) fprintf(f, "\t%1.2f", (double)q->permute_clr[j]);
    fprintf(f, "\n");
  }
  fclose(f);
}

/* ----------------------------------------------------------------- stats */
/* this process's counters; device counters summed over its devices (busy_ms: the sum of
   each device's busy time, i.e. device-seconds) */
void fscl_amd_get_stats(fscl_amd_stats_t *st) {
  int l;
  *st = D.st;
  st->kernel_ms = 0; st->n_terms = st->n_null = st->n_walks = st->n_maxalpha = 0;
  st->n_unsafe = st->n_slow = st->n_ties = st->n_launches = 0;
  st->window_ms = 0; st->n_dup_cells = st->n_ep_saved = 0; st->busy_ms = 0; st->n_split_retry = 0;
  for (l = 0; l < D.n_dev; l++) {
    fsclg_stats_t g;
    if (fsclg_get_stats(D.ctx[l], &g) != FSCLG_OK) continue;
    st->kernel_ms += g.kernel_ms;
    st->n_terms += g.n_terms; st->n_null += g.n_null; st->n_walks += g.n_walks; st->n_maxalpha += g.n_maxalpha;
    st->n_unsafe += g.n_unsafe; st->n_slow += g.n_slow; st->n_ties += g.n_ties; st->n_launches += g.n_launches;
    st->window_ms += g.window_ms;
    st->n_dup_cells += g.n_dup_cells; st->n_ep_saved += g.n_ep_saved;
    st->busy_ms += g.busy_ms;
    st->n_split_retry += g.n_split_retry;
    if (l == 0) {
      st->cache_iv0 = g.cache_iv0; st->cache_n_iv = g.cache_n_iv; st->cache_n_rows = g.cache_n_rows;
      st->cache_cover = g.cache_cover;
    }
  }
  if (DI.ctx) {  /* the drop-in search_maxalpha's own context */
    fsclg_stats_t g;
    if (fsclg_get_stats(DI.ctx, &g) == FSCLG_OK) {
      st->kernel_ms += g.kernel_ms;
      st->n_terms += g.n_terms; st->n_walks += g.n_walks; st->n_maxalpha += g.n_maxalpha;
      st->n_launches += g.n_launches;
      st->busy_ms += g.busy_ms;
    }
  }
  st->n_devices = D.n_dev;
}

void fscl_amd_reset_stats(void) {
  int l;
  memset(&D.st, 0, sizeof D.st);
  for (l = 0; l < D.n_dev; l++) fsclg_reset_stats(D.ctx[l]);
  if (DI.ctx) fsclg_reset_stats(DI.ctx);
}

void fscl_amd_shutdown(void) {
  pool_drop();
  spec_stop();
  dev_close_all();
  if (DI.ctx) fsclg_close(DI.ctx);
  free(DI.null_full); free(DI.null_seen); free(DI.pos); free(DI.row); free(DI.tpos); free(DI.trow);
  free_rowmap(&DI.rm);
  memset(&DI, 0, sizeof DI);
  free(D.row); free(D.pos); free(D.chr_start); free(D.chr_n); free(D.nullrow); free(D.rowp);
  D.rowp = NULL;
  D.row = NULL; D.pos = NULL; D.chr_start = NULL; D.chr_n = NULL; D.nullrow = NULL;
  free_rowmap(&D.rm);
  if (D.sim) { fclose(D.sim); D.sim = NULL; }
}
