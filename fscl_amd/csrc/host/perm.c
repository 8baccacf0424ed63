/* perm.c -- the permutation trials' block permutation (scan-chromosome.c:336-389,
   snp_block_permute) as a plan that the device applies.

   The reference copies the sites and then, while the cursor i < n, draws a block from the
   rand() stream -- a source j, a length ~ 1 + Exp(nbp) extended to at least scan_width_mb on
   j's chromosome -- and swaps the rows of [i, i + len) with those of [j, j + len) element by
   element, i advancing by len.  Which blocks are drawn depends only on the rand() stream and the
   positions, never on the rows, so the block list (phase 1) is the sequential part and costs
   ~50 ns a block here (the extension is one lookup: fh_ext_table).  Applying it (phase 2) is
   O(n) memory traffic: on the device.  A block must follow every earlier block whose sites it
   meets; the plan gives each block a level one above the highest such block, and the blocks of
   one level touch disjoint sites, so the device applies a level in any order and the levels in
   turn (about 15 levels for 5 000 blocks at C5).  The result is the sequential one, element for
   element (tests/test_host.py: against the oracle's orc_block_permute). */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "fscl_host.h"

#define PLAN_GRAN 64      /* sites per granule of the level map */
#define PLAN_CHUNK 4096   /* a disjoint swap longer than this is split into pieces (one device workgroup each) */
#define PLAN_MAX_LEVEL 65000

/* ext[j]: the first index of j's chromosome at or after j with (double)(pos - pos[j]) >= width,
   else the chromosome's end.  The reference's extension `while (k < n && chr[k] == chr[j] &&
   pos[k] - pos[j] < width) k++` (scan-chromosome.c:355-357), started at k >= j, stops at
   max(k, ext[j]): positions ascend within a chromosome. */
void fh_ext_table(int32_t *ext, const int32_t *pos, const int32_t *chr_start, const int32_t *chr_n, int n_chr,
                  double width_mb) {
  const double width = width_mb * 1e6;
  int c;
  for (c = 0; c < n_chr; c++) {
    const int cs = chr_start[c], ce = cs + chr_n[c];
    int j, e = cs;
    for (j = cs; j < ce; j++) {
      if (e < j) e = j;
      while (e < ce && (double)(pos[e] - pos[j]) < width) e++;
      ext[j] = e;
    }
  }
}

static int chr_of(const fh_perm_geom_t *G, int j) { /* j's chromosome */
  int lo = 0, hi = G->n_chr - 1;
  while (lo < hi) {
    const int m = (lo + hi + 1) / 2;
    if (G->chr_start[m] <= j) lo = m; else hi = m - 1;
  }
  return lo;
}

/* one block at cursor i (scan-chromosome.c:349-363): its source j and length; Q9 (k > n: the
   reference reads p[-m]) repaired as j -= k - n and counted; Q10 (rand() == 0: log(0)) runs the
   block to the end */
int fh_block_draw(const fh_perm_geom_t *G, double nbp, double width_mb, fh_rand_t *g, int i, int *jo,
                  unsigned long long *negj) {
  const int n = G->n;
  const int r1 = fh_rand(g), r2 = fh_rand(g);
  int j = r1 / (2147483647 + 1.0) * n, k;
  if (r2 == 0) k = n;
  else k = j + (int)(-1.0 / nbp * log(r2 / (2147483647 + 1.0)));
  if (k >= 0 && k < n) {
    if (k >= j) {
      if (G->ext[j] > k) k = G->ext[j];
    } else { /* a backward k (nbp < 0): the reference's loop as written */
      const int c = chr_of(G, j), cs = G->chr_start[c], ce = cs + G->chr_n[c];
      const double width = width_mb * 1e6;
      if (k >= cs)
        while (k < ce && (double)(G->pos[k] - G->pos[j]) < width) k++;
    }
  }
  if (i + (k - j) >= n) k = n;
  if (k > n) { (*negj)++; j -= k - n; k = n; }
  *jo = j;
  return k - j < n - i ? k - j : n - i;
}

void fh_plan_free(fh_plan_t *P) {
  free(P->blk); free(P->gran); free(P->lvl);
  memset(P, 0, sizeof *P);
}

/* phase 1: the blocks from rand() state *g (advanced past them), leveled and grouped into
   out (ent[0..ecap), grp[0..gcap]); 0, -1 cancelled (*gen != my_gen), -2 the plan does not fit
   (the caller permutes the rows itself) */
int fh_plan_build(fh_plan_t *P, const fh_perm_geom_t *G, double nbp, double width_mb, fh_rand_t *g,
                  unsigned long long *negj, fsclg_swap_t *ent, int ecap, int32_t *grp, int gcap, int *n_ent,
                  int *n_grp, const volatile unsigned *gen, unsigned my_gen) {
  const int n = G->n, ng = n / PLAN_GRAN + 2;
  int i = 0, nb = 0, b, maxl = 0, l, e, q;
  if (P->gcap < ng) {
    P->gran = fh_realloc(P->gran, sizeof(uint16_t) * (size_t)ng, "plan");
    P->gcap = ng;
  }
  /* blocks in draw order (.kind: level) */
  while (i < n) {
    int j, len;
    if (nb == P->bcap) {
      P->bcap = P->bcap ? 2 * P->bcap : 8192;
      P->blk = fh_realloc(P->blk, sizeof(fsclg_swap_t) * (size_t)P->bcap, "plan");
      if (gen && __atomic_load_n(gen, __ATOMIC_RELAXED) != my_gen) return -1;
    }
    len = fh_block_draw(G, nbp, width_mb, g, i, &j, negj);
    P->blk[nb].i = i; P->blk[nb].j = j; P->blk[nb].len = len; P->blk[nb].kind = 0;
    nb++;
    if (len > 0) i += len;
  }
  if (gen && __atomic_load_n(gen, __ATOMIC_RELAXED) != my_gen) return -1;
  /* levels: a block follows every earlier block whose sites it meets.  Earlier targets
     [i_a, i_a + len_a) tile [0, i_b) in order (a binary search finds those a source meets);
     earlier sources are recorded per granule (conservative: a shared granule counts as a
     meeting) */
  memset(P->gran, 0, sizeof(uint16_t) * (size_t)ng);
  for (b = 0; b < nb; b++) {
    fsclg_swap_t *x = P->blk + b;
    const int bi = x->i, bj = x->j, L = x->len;
    int lv = 0, a, u;
    if (L <= 0) continue;
    if (bj < bi) {
      int lo = 0, hi = b - 1;
      while (lo < hi) {
        const int m = (lo + hi + 1) / 2;
        if (P->blk[m].i <= bj) lo = m; else hi = m - 1;
      }
      for (a = lo; a < b && P->blk[a].i < bj + L; a++)
        if (P->blk[a].len > 0 && P->blk[a].i + P->blk[a].len > bj && P->blk[a].kind > lv) lv = P->blk[a].kind;
    }
    for (u = bj / PLAN_GRAN; u <= (bj + L - 1) / PLAN_GRAN; u++) if (P->gran[u] > lv) lv = P->gran[u];
    for (u = bi / PLAN_GRAN; u <= (bi + L - 1) / PLAN_GRAN; u++) if (P->gran[u] > lv) lv = P->gran[u];
    if (++lv > PLAN_MAX_LEVEL) return -2;
    x->kind = lv;
    for (u = bj / PLAN_GRAN; u <= (bj + L - 1) / PLAN_GRAN; u++) P->gran[u] = (uint16_t)lv;
    if (lv > maxl) maxl = lv;
  }
  /* group by level: each level's disjoint swaps (long ones in pieces), then each of its
     overlapping blocks alone */
  if (P->lcap < maxl + 2) {
    P->lcap = maxl + 2;
    P->lvl = fh_realloc(P->lvl, sizeof(int) * (size_t)P->lcap * 2, "plan");
  }
  {
    int *cnt = P->lvl, *rot = P->lvl + P->lcap;  /* entries (pieces) and overlapping blocks per level */
    memset(cnt, 0, sizeof(int) * (size_t)P->lcap * 2);
    for (b = 0; b < nb; b++) {
      const fsclg_swap_t *x = P->blk + b;
      if (x->len <= 0) continue;
      if (abs(x->i - x->j) < x->len) rot[x->kind]++;
      else cnt[x->kind] += (x->len + PLAN_CHUNK - 1) / PLAN_CHUNK;
    }
    {
      int ne = 0, gg = 0;
      for (l = 1; l <= maxl; l++) {
        gg += (cnt[l] > 0) + rot[l];
        ne += cnt[l] + rot[l];
      }
      if (ne > ecap || gg > gcap) return -2;
      *n_ent = ne; *n_grp = gg;
    }
    /* offsets: level l's swaps at [cnt[l], ...), its overlapping blocks right after */
    for (l = 1, e = 0, q = 0; l <= maxl; l++) {
      const int c = cnt[l], r = rot[l];
      if (c > 0) grp[q++] = e;
      cnt[l] = e;
      e += c;
      for (b = 0; b < r; b++) grp[q++] = e + b;
      rot[l] = e;
      e += r;
    }
    grp[q] = e;
    for (b = 0; b < nb; b++) {
      const fsclg_swap_t *x = P->blk + b;
      if (x->len <= 0) continue;
      if (abs(x->i - x->j) < x->len) {
        fsclg_swap_t *o = ent + rot[x->kind]++;
        *o = *x;
        o->kind = 1;
      } else {
        int t;
        for (t = 0; t < x->len; t += PLAN_CHUNK) {
          fsclg_swap_t *o = ent + cnt[x->kind]++;
          o->i = x->i + t; o->j = x->j + t; o->len = x->len - t < PLAN_CHUNK ? x->len - t : PLAN_CHUNK; o->kind = 0;
        }
      }
    }
  }
  return 0;
}

/* the device's semantics on the host (fsclg_slot_set_rows_plan): the groups in order; a kind-1
   entry is the reference's sequential swaps of an overlapping block, i.e. the rotation
   out[lo + t] = in[lo + d + t] (t < len), out[lo + t] = in[lo + t % d] (len <= t < len + d) */
void fh_plan_apply_u32(uint32_t *rows, int n, const fsclg_swap_t *ent, const int32_t *grp, int n_grp) {
  int q, e, t;
  uint32_t *tmp = NULL;
  (void)n;
  for (q = 0; q < n_grp; q++)
    for (e = grp[q]; e < grp[q + 1]; e++) {
      const fsclg_swap_t *x = ent + e;
      if (x->kind == 0) {
        for (t = 0; t < x->len; t++) {
          const uint32_t v = rows[x->i + t];
          rows[x->i + t] = rows[x->j + t];
          rows[x->j + t] = v;
        }
      } else {
        const int lo = x->i < x->j ? x->i : x->j, d = abs(x->i - x->j), R = x->len + d;
        tmp = fh_realloc(tmp, sizeof(uint32_t) * (size_t)R, "plan");
        memcpy(tmp, rows + lo, sizeof(uint32_t) * (size_t)R);
        for (t = 0; t < R; t++) rows[lo + t] = tmp[t < x->len ? d + t : t % d];
      }
    }
  free(tmp);
}

/* test hook (tests/test_host.py): one trial's permutation of rows[0..n) (in place) through the
   plan, from rand() state `state` (fh_rand_t, advanced); out: [blocks' negative-j repairs,
   entries, groups, overlapping blocks]; returns fh_plan_build's status */
int fscl_amd_plan_permute_test(int n, const int32_t *pos, const int32_t *chr_start, const int32_t *chr_n,
                               int n_chr, double nbp, double width_mb, void *state, uint32_t *rows,
                               long long *out) {
  fh_plan_t P;
  fh_perm_geom_t G;
  int32_t *ext = fh_malloc(sizeof(int32_t) * (size_t)(n ? n : 1), "plan");
  const int ecap = n + n / PLAN_CHUNK + 16, gcap = 4 * n + 16;
  fsclg_swap_t *ent = fh_malloc(sizeof(fsclg_swap_t) * (size_t)ecap, "plan");
  int32_t *grp = fh_malloc(sizeof(int32_t) * (size_t)(gcap + 1), "plan");
  unsigned long long negj = 0;
  int ne = 0, ngr = 0, r;
  memset(&P, 0, sizeof P);
  fh_ext_table(ext, pos, chr_start, chr_n, n_chr, width_mb);
  G.n = n; G.n_chr = n_chr; G.chr_start = chr_start; G.chr_n = chr_n; G.pos = pos; G.ext = ext;
  r = fh_plan_build(&P, &G, nbp, width_mb, (fh_rand_t *)state, &negj, ent, ecap, grp, gcap, &ne, &ngr, NULL, 0);
  if (r == 0) fh_plan_apply_u32(rows, n, ent, grp, ngr);
  out[0] = (long long)negj; out[1] = ne; out[2] = ngr; out[3] = 0;
  for (int k = 0; r == 0 && k < ne; k++) out[3] += ent[k].kind == 1;
  fh_plan_free(&P);
  free(ext); free(ent); free(grp);
  return r;
}
