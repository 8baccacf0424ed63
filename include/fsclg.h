/*
 * fsclg.h -- device shim C-ABI of the MI355X (gfx950) CLR scan kernels.
 *
 * Plain C, plain pointers and sizes, int status returns, no exceptions and no
 * torch types cross this boundary.  One context per process per GPU.  It sits
 * below the fscl.h-compatible host library (include/fscl_amd.h): the host C
 * code (scan_chromosome / scan_permute) calls these; a maintainer can also
 * bind them directly (ctypes stub in INTEGRATION.md).
 *
 * Reference interfaces each entry replaces (all in /root/reference):
 *   fsclg_search_maxpos  -> search_maxpos() batch, scan-chromosome.c:126-139
 *                           (with init_scan_result :58-101, search_maxalpha
 *                           sm-search.c:269-300, sm_likelihood :105-150)
 *   fsclg_search_points  -> search_maxalpha() on caller-initialised points,
 *                           sm-search.c:269-300 (fscl.h:105)
 *   fsclg_set_rows       -> the permuted snp array of one trial,
 *                           scan-chromosome.c:443 (snp_block_permute output)
 *   fsclg_slot_set_rows  -> the same for one of FSCLG_N_SLOTS trials in flight
 *   fsclg_slot_set_rows_plan -> snp_block_permute itself (scan-chromosome.c:336-389)
 *                           applied on the device from the host's block plan
 *   fsclg_search_submit/ -> the per-trial search_maxpos calls of
 *   fsclg_search_wait       scan_permute_thread (scan-chromosome.c:478-487),
 *                           split so that consecutive trials overlap on the GPU
 *   fsclg_upload_tables  -> sm_ptable_t spline tables (fscl.h:64-76) and
 *                           log_table (sm-search.c:14-26)
 *   fsclg_upload_snps    -> snp_t positions + chr_limits_t (fscl.h:7-33)
 */
#ifndef FSCLG_H
#define FSCLG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  FSCLG_OK = 0,
  FSCLG_E_ARG = -1,        /* bad argument / shape */
  FSCLG_E_HIP = -2,        /* HIP runtime error (message in fsclg_last_error) */
  FSCLG_E_STATE = -3,      /* tables / snps not uploaded */
  FSCLG_E_UNSUPPORTED = -4,/* a window narrower than its chromosome (chromosome > 2*eval_range+1 SNPs) */
  FSCLG_E_KERNEL = -5      /* device-side failure flag (e.g. position bisection did not converge) */
};

typedef struct fsclg_ctx fsclg_ctx;

/* one coarse grid cell: search_maxpos(chr, start_pos, end_pos) */
typedef struct {
  int32_t chr, start_pos, end_pos, pad;
} fsclg_cell_t;

/* one evaluated scan point (the fields of scan_pt_t the path produces) */
typedef struct {
  int32_t chr, nearest_snp, sweep_pos, n_snps, window_start, window_end, flags;
  uint32_t cost;  /* out: snp_likelihood terms / 1024 spent on this point's cell (scheduling hint) */
  double lalpha, null_logl, sm_logl, clr;
} fsclg_point_t;

/* cumulative device counters (reset by fsclg_reset_stats) */
typedef struct {
  unsigned long long n_terms;      /* snp_likelihood evaluations */
  unsigned long long n_null;       /* window null-sum elements (reference-equivalent count) */
  unsigned long long n_walks;      /* sm_likelihood walks */
  unsigned long long n_maxalpha;   /* search_maxalpha evaluations */
  unsigned long long n_unsafe;     /* walks whose integer-ulp sum left its binade */
  unsigned long long n_slow;       /* walks re-summed sequentially to settle an argmax */
  unsigned long long n_ties;       /* round-half-even ties resolved by prefix parity */
  unsigned long long n_cells;      /* search_maxpos evaluations */
  double kernel_ms;                /* summed duration of the search kernels (HIP events) */
  unsigned long long n_launches;
  int cache_iv0, cache_n_iv, cache_n_rows;  /* LDS coefficient window: intervals, device rows */
  double cache_cover;              /* its planned share of the terms */
  double window_ms;                /* summed duration of the window null-sum kernels (HIP events) */
  unsigned long long n_dup_cells;  /* cells answered by an identical cell of the same launch */
  unsigned long long n_ep_saved;   /* endpoint evaluations saved by sharing between neighbouring cells */
  double busy_ms;                  /* union of the search batches' kernel intervals (overlapping batches
                                      counted once): the GPU time the search kernels occupied */
  unsigned long long n_split_retry; /* split launches whose members were not resident together (a
                                       member waited > ~1 s), re-run with one workgroup per cell */
} fsclg_stats_t;

/* trials in flight: row slots (one permuted row array + null sums each) and launch batches
   (cells and outputs each).  Batches 0 and 1 run on one high-priority stream, batches
   2 .. FSCLG_N_BATCHES-1 on two normal-priority streams (even / odd batch): with the upload
   stream, four streams, one per hardware queue (GPU_MAX_HW_QUEUES = 4) */
#define FSCLG_N_SLOTS 8
#define FSCLG_N_BATCHES 10

int fsclg_open(int device, fsclg_ctx **out);
int fsclg_close(fsclg_ctx *c);
const char *fsclg_last_error(void);
int fsclg_device_count(void);

/* log_table: 65536 doubles (log_table[0] = 0, log_table[i] = log(i));
   coef: n_rows * n_iv * 4 doubles, row-major [row][interval][c0..c3];
   nullrow: n_rows doubles (null_logl of a site with that row);
   log_ad_step = (LOG_AD_MAX - LOG_AD_MIN) / (spline_pts + 1) */
int fsclg_upload_tables(fsclg_ctx *c, const double *log_table, const double *coef, int n_rows, int n_iv,
                        const double *nullrow, double log_ad_step);

/* pos: n_snps int32 sorted within each chromosome; row: n_snps uint32 (spline row of each site);
   chr_start/chr_n: first index and SNP count of each chromosome */
int fsclg_upload_snps(fsclg_ctx *c, const int32_t *pos, const uint32_t *row, int n_snps,
                      const int32_t *chr_start, const int32_t *chr_n, int n_chr);

/* replace the per-site rows (one permutation trial); NULL restores the uploaded rows */
/* a pinned host buffer of n_snps rows owned by the context (valid until the next
   fsclg_upload_snps / fsclg_close): a caller that permutes into it saves one copy in
   fsclg_set_rows (the buffer may be rewritten once fsclg_set_rows's search has returned) */
uint32_t *fsclg_row_buffer(fsclg_ctx *c);
int fsclg_set_rows(fsclg_ctx *c, const uint32_t *row);

/* asynchronous trials.  A row slot holds one trial's rows on the device; a batch is one
   search_maxpos launch over the rows of one slot.  fsclg_slot_row_buffer returns the slot's
   pinned staging buffer (NULL while a batch submitted on the slot is not waited for);
   fsclg_slot_set_rows uploads it (or row, or the uploaded rows when row is NULL) and, when
   chr_null is not NULL, the slot's whole-chromosome null sums; both are asynchronous and
   fail with FSCLG_E_STATE while the slot is in use.  fsclg_search_submit queues a batch
   (cells are copied; the batch must be idle) and returns at once; fsclg_search_wait blocks
   until its points are in out[n_cells] (input order).  Slot 0 and batch 0 are also what the
   synchronous calls (fsclg_set_rows, fsclg_search_maxpos) use. */
uint32_t *fsclg_slot_row_buffer(fsclg_ctx *c, int slot);
int fsclg_slot_set_rows(fsclg_ctx *c, int slot, const uint32_t *row, const double *chr_null);
/* the window null sums (chromosomes above 2*eval_range+1 SNPs) for the cells that the slot's
   next batches will evaluate, given before the slot's first submit of a trial: only those
   windows when they are few, every window otherwise.  A submit checks its cells against what
   was summed and sums any window still missing (also without this call), so a batch may
   submit other cells too, at the cost of a second window launch. */
int fsclg_slot_windows(fsclg_ctx *c, int slot, const fsclg_cell_t *cells, int n_cells, int eval_range);
int fsclg_search_submit(fsclg_ctx *c, int batch, int slot, const fsclg_cell_t *cells, int n_cells, int eval_range,
                        int bp_resl);
int fsclg_search_wait(fsclg_ctx *c, int batch, fsclg_point_t *out);

/* Several devices fed from one host buffer.  fsclg_host_alloc returns pinned host memory that
   every device's kernels read directly (portable, mapped, coherent); fsclg_slot_set_rows_host
   uploads a slot's rows straight from such a buffer (no copy into the context's own staging,
   no range check: every row must be < the n_rows of fsclg_upload_tables) and returns at once;
   the caller keeps the buffer unchanged until fsclg_slot_wait(c, slot) has returned on every
   context it was handed to (the slot's last upload has read it). */
void *fsclg_host_alloc(size_t bytes);
void fsclg_host_free(void *p);
/* The same for memory the caller mapped itself (a POSIX shared-memory segment that several
   processes map: one node leader builds each trial's rows once, every rank's devices read
   them): page-locks [p, p + bytes) for every device (portable, mapped).  Returns FSCLG_OK only
   if the devices address the memory by the same pointer (the pointer can go to
   fsclg_slot_set_rows_packed as it is); fsclg_host_unregister undoes it. */
int fsclg_host_register(void *p, size_t bytes);
int fsclg_host_unregister(void *p);
int fsclg_slot_wait(fsclg_ctx *c, int slot);
/* exchange two slots' device state (rows, window sums, their upload events): a trial prepared in
   a spare slot ahead of time becomes slot a.  Neither slot may have a batch not waited for. */
int fsclg_slot_swap(fsclg_ctx *c, int a, int b);
/* 1 if the batch's last submit has completed (or none is pending), 0 if it is still running:
   fsclg_search_wait would not block */
int fsclg_search_done(fsclg_ctx *c, int batch);
int fsclg_slot_set_rows_host(fsclg_ctx *c, int slot, const uint32_t *row, const double *chr_null);
/* the same with rows of row_bytes = 1, 2 or 4 bytes each (1: n_rows <= 256, 2: n_rows <= 65536):
   a narrower staging is fewer PCIe bytes for every device's upload of every trial */
int fsclg_slot_set_rows_packed(fsclg_ctx *c, int slot, const void *row, int row_bytes, const double *chr_null);

/* A trial's block permutation as a plan, applied on the device (scan-chromosome.c:336-389:
   snp_block_permute's swaps, from the rand() stream, on the uploaded rows).  The host draws the
   blocks and groups them (fh_plan_build, fscl_amd/csrc/host/perm.c); the device copies the
   uploaded rows into the slot and applies the groups in order.  Within a group the entries touch
   disjoint sites, so they run in any order.  kind 0: rows[i + t] <-> rows[j + t] for t < len, the
   two ranges disjoint (a block, or a piece of one).  kind 1: a block whose ranges overlap,
   |i - j| < len, the reference's sequential element swaps (a rotation of [min(i,j), min(i,j) +
   len + |i - j|)), alone in its group.  ent and grp (n_grp + 1 offsets into ent) are host
   memory the devices read directly (fsclg_host_alloc or fsclg_host_register) and must stay
   unchanged until fsclg_slot_wait(c, slot) returns; only the chr_null values are copied.
   Validation is at call time only, on the buffers as they are then: every range is checked
   against n_snps, and a kind-0 entry's own two ranges for disjointness.  That the entries of one
   group touch disjoint sites is the CALLER's contract (fh_plan_build guarantees it by
   construction); entries that overlap across a group race on those sites without an error,
   though never outside [0, n_snps). */
typedef struct {
  int32_t i, j, len, kind;
} fsclg_swap_t;
int fsclg_slot_set_rows_plan(fsclg_ctx *c, int slot, const fsclg_swap_t *ent, const int32_t *grp, int n_grp,
                             const double *chr_null);

/* sequential window null sums (init_scan_result's sum from 0.0) for each chromosome's
   whole-chromosome window, for the rows currently set */
int fsclg_set_chr_null(fsclg_ctx *c, const double *chr_null);

/* alpha grids: coarse (11 values of the for-loop at sm-search.c:277) and, for each
   coarse argmax index c in [0, n_coarse), the refine values of sm-search.c:283-295
   (max 16 each, row-major [c][16]); row n_coarse holds the refine values around
   LOG_AD_MAX, used when no candidate beats the initial -DBL_MAX (sm-search.c:272) */
int fsclg_set_alpha_grid(fsclg_ctx *c, const double *coarse, int n_coarse, const double *refine,
                         const int32_t *n_refine);

/* Split cells: a launch of batch `batch` with few cells gives each cell up to max_members
   (<= 8) workgroups that share its walks' segments (default 1).  For latency, not throughput:
   the pipeline's blocking batch, whose result orders the next trial.  A launch takes at most
   512 workgroups ($FSCLG_SPLIT_BUDGET), the device's resident slots, so the members of a cell
   run together once the workgroups ahead of them finish; a cell whose members were not all
   resident within ~1 s is re-run with one workgroup (counted, n_split_retry). */
int fsclg_set_batch_split(fsclg_ctx *c, int batch, int max_members);

/* batched search_maxpos over n_cells cells; blocks until out[] is written */
int fsclg_search_maxpos(fsclg_ctx *c, const fsclg_cell_t *cells, int n_cells, int eval_range, int bp_resl,
                        fsclg_point_t *out);

/* search_maxalpha on points whose chr/nearest_snp/sweep_pos/window/null_logl are
   already set (init_scan_result done by the caller); fills lalpha/sm_logl/clr */
int fsclg_search_points(fsclg_ctx *c, fsclg_point_t *pts, int n_pts);

/* the exact interval thresholds the kernel uses in place of spline_interpolate's
   division (sm-spline.c:52): thr[j] = least double x with
   (int)((x - LOG_AD_MIN) / log_ad_step) >= j, for j = 1..n_iv (thr has n_iv+1 slots) */
int fsclg_interval_thresholds(double log_ad_step, int n_iv, double *thr);

int fsclg_get_stats(fsclg_ctx *c, fsclg_stats_t *st);
int fsclg_reset_stats(fsclg_ctx *c);

#ifdef __cplusplus
}
#endif
#endif
