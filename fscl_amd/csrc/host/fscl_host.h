/* fscl_host.h -- internal declarations of the host side of fscl_amd. */
#ifndef FSCL_HOST_H
#define FSCL_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "../../../include/fscl_amd.h"
#include "../../../include/fsclg.h"

void *fh_malloc(size_t n, const char *where);
void *fh_calloc(size_t n, size_t m, const char *where);
void *fh_realloc(void *p, size_t n, const char *where);
double fh_now(void);

/* glibc random_r TYPE_3 stream (the reference draws glibc rand(), seeded by
   srand(0xFD821A6) at fscl.c:135); own state so ranks and speculation can
   replay it exactly */
typedef struct { int32_t r[31]; int f, b; } fh_rand_t;
void fh_srand(fh_rand_t *g, unsigned seed);
int fh_rand(fh_rand_t *g);

/* the block permutation as a device plan (perm.c; scan-chromosome.c:336-389) */
typedef struct {
  int n, n_chr;
  const int32_t *chr_start, *chr_n, *pos;
  const int32_t *ext;  /* fh_ext_table */
} fh_perm_geom_t;
typedef struct {     /* per-thread scratch of fh_plan_build */
  fsclg_swap_t *blk;
  int bcap;
  uint16_t *gran;
  int gcap;
  int *lvl;
  int lcap;
} fh_plan_t;
void fh_ext_table(int32_t *ext, const int32_t *pos, const int32_t *chr_start, const int32_t *chr_n, int n_chr,
                  double width_mb);
int fh_block_draw(const fh_perm_geom_t *G, double nbp, double width_mb, fh_rand_t *g, int i, int *jo,
                  unsigned long long *negj);
int fh_plan_build(fh_plan_t *P, const fh_perm_geom_t *G, double nbp, double width_mb, fh_rand_t *g,
                  unsigned long long *negj, fsclg_swap_t *ent, int ecap, int32_t *grp, int gcap, int *n_ent,
                  int *n_grp, const volatile unsigned *gen, unsigned my_gen);
void fh_plan_free(fh_plan_t *P);
void fh_plan_apply_u32(uint32_t *rows, int n, const fsclg_swap_t *ent, const int32_t *grp, int n_grp);

/* log_fact table shared by lchoose (sm-spline.c:18-39) */
double fh_log_fact(int n);
void fh_log_fact_reserve(int n);

/* spline row layout: per depth, (n+1) unfolded then (n/2+1) folded rows; the device holds
   only the rows some site uses, renumbered in that order */
typedef struct {
  int n_depths;
  int *depth_n;      /* sample size of each depth index */
  int *row_base;     /* first row of each depth */
  int n_rows;        /* all rows */
  int n_iv;          /* spline intervals (spline_pts) */
  int *dev_row;      /* [n_rows] device row of each row, -1 if no site uses it */
  int n_dev_rows;
} fh_rowmap_t;

static inline uint32_t fh_full_row(const fh_rowmap_t *m, const snp_t *s) {
  return (uint32_t)(m->row_base[s->depth_p] + (s->folded ? m->depth_n[s->depth_p] + 1 + s->obs_freq : s->obs_freq));
}

static inline uint32_t fh_row_of(const fh_rowmap_t *m, const snp_t *s) {
  return (uint32_t)m->dev_row[fh_full_row(m, s)];
}

/* current global log_ad_step (sm-spline.c:16,325) */
double fh_log_ad_step(void);
const double *fh_log_table(void);

/* the alpha grids of search_maxalpha (sm-search.c:277-295), computed with the
   reference's own floating-point loop */
int fh_alpha_grid(double *coarse, int max_coarse, double *refine /* [max_coarse][16] */, int32_t *n_refine);

/* multi-process exchange through POSIX shared memory (ranks.c) */
typedef struct fh_shm fh_shm_t;
fh_shm_t *fh_shm_open(int rank, int world, const char *name, size_t cap);
void fh_shm_close(fh_shm_t *m);
int fh_shm_allgather(fh_shm_t *m, void *buf, size_t item, int n, int lo, int hi);
int fh_shm_allgather_flags(fh_shm_t *m, void *buf, size_t item, int n, int lo, int hi, unsigned *flags);
int fh_shm_barrier(fh_shm_t *m);
int fh_shm_rank(const fh_shm_t *m);
int fh_shm_world(const fh_shm_t *m);

/* the node leader's permutation pool: a second shared segment holding every trial's rows,
   built once by rank 0 and read by every rank's devices (ranks.c) */
typedef struct fh_pool fh_pool_t;
fh_pool_t *fh_pool_open(fh_shm_t *m, size_t data_bytes);  /* collective */
void fh_pool_close(fh_pool_t *p);
char *fh_pool_data(fh_pool_t *p);
size_t fh_pool_bytes(const fh_pool_t *p);
int fh_pool_publish(fh_pool_t *p, size_t rows_off, size_t nul_off, const fh_rand_t *end, unsigned long long negj);
int fh_pool_take(fh_pool_t *p, size_t *rows_off, size_t *nul_off, fh_rand_t *end, unsigned long long *negj);
void fh_pool_release(fh_pool_t *p);
int fh_pool_wait_released(fh_pool_t *p);

/* ms reader */
scan_t *fh_load_ms(const char *fname, int segment_length, int folded, int sample_first, int sample_size);

#endif
