/* The row-array routines of the permutation trials, for one staging width: included by scan.c
   once per width with ROW_T (uint8_t, uint16_t or uint32_t) and ROW_SFX defined.  The trials'
   rows are staged at the narrowest width that holds the device table's rows (D.rb bytes), so
   that a candidate permutation moves fewer bytes on the host and every device's upload reads
   fewer over PCIe; the values, and so every result, are the same at any width. */
#define ROW_CAT2(a, b) a##_##b
#define ROW_CAT(a, b) ROW_CAT2(a, b)

/* init_scan_result's window sum (scan-chromosome.c:92-94): sequential from 0.0 over the
   whole chromosome for the given rows, for the chromosomes whose window is the whole
   chromosome (D.chr_list; the others' entries are never read and are set to 0) */
static void ROW_CAT(chr_null_sums, ROW_SFX)(const ROW_T *row, double *out) {
  const int nl = D.chr_list ? D.n_chr_list : D.n_chr;
  int q, i;
  if (D.chr_list) for (q = 0; q < D.n_chr; q++) out[q] = 0.;
#pragma omp parallel for schedule(dynamic, 1) private(i) if (nl > 1) num_threads(null_threads())
  for (q = 0; q < nl; q++) {
    const int c = D.chr_list ? D.chr_list[q] : q;
    double acc = 0.;
    for (i = D.chr_start[c]; i < D.chr_start[c] + D.chr_n[c]; i++) acc += D.nullrow[row[i]];
    out[c] = acc;
  }
}

/* scan-chromosome.c:336-389 on the row array: blocks of consecutive sites (length ~ 1 +
   Exp(nbp), extended to at least scan_width_mb on the same chromosome; fh_block_draw, shared
   with the device plan of perm.c) are swapped into place; positions never move.  Q9: a block
   running past the end is shifted left (j -= k - n) instead of indexing p[-m] as the reference
   does; such events are counted. */
static int ROW_CAT(block_permute, ROW_SFX)(ROW_T *prow, const ROW_T *row, int n, double nbp, double width_mb,
                                           fh_rand_t *g, unsigned long long *negj, const volatile unsigned *gen,
                                           unsigned my_gen) {
  int i = 0, j, nb = 0;
  const int piece = (1 << 20) / (int)sizeof(ROW_T);
  for (i = 0; i < n; i += piece) { /* in 1 MB pieces: a cancelled candidate stops soon */
    if (gen && __atomic_load_n(gen, __ATOMIC_RELAXED) != my_gen) return -1;
    memcpy(prow + i, row + i, sizeof(ROW_T) * (size_t)(n - i < piece ? n - i : piece));
  }
  i = 0;
  while (i < n) {
    const int len = fh_block_draw(&PM.G, nbp, width_mb, g, i, &j, negj);
    if ((++nb & 255) == 0 && gen && __atomic_load_n(gen, __ATOMIC_RELAXED) != my_gen) return -1; /* cancelled */
    /* scan-chromosome.c:365-372: swap p[i++] with p[j++] while j < k and i < n; disjoint
       ranges in one vectorisable pass, overlapping ones element by element as written */
    if (len > 0 && (j >= i + len || i >= j + len)) {
      ROW_T *__restrict a = prow + i, *__restrict b = prow + j;
      int t;
      for (t = 0; t < len; t++) {
        const ROW_T x = a[t];
        a[t] = b[t];
        b[t] = x;
      }
    } else {
      int t;
      for (t = 0; t < len; t++) {
        const ROW_T x = prow[i + t];
        prow[i + t] = prow[j + t];
        prow[j + t] = x;
      }
    }
    if (len > 0) i += len;
  }
  return 0;
}

/* chr_null_sums on one thread: four chromosomes' sequential sums interleaved (independent
   chains, each in the reference's order; four accumulators hide the add latency) */
static int ROW_CAT(chr_null_sums_1t, ROW_SFX)(const ROW_T *row, double *out, const volatile unsigned *gen,
                                              unsigned my_gen) {
  const double *nr = D.nullrow;
  const int nl = D.chr_list ? D.n_chr_list : D.n_chr;
  int q = 0, t, t1, k, cc[4];
  if (D.chr_list) for (k = 0; k < D.n_chr; k++) out[k] = 0.;
  for (; q < nl; q += 4) {
    const int nc = nl - q < 4 ? nl - q : 4;
    const ROW_T *r[4];
    double a[4] = {0., 0., 0., 0.};
    int m = 1 << 30;
    for (k = 0; k < 4; k++) {
      cc[k] = D.chr_list ? D.chr_list[q + (k < nc ? k : 0)] : q + (k < nc ? k : 0);
      r[k] = row + D.chr_start[cc[k]];
      if (k < nc && D.chr_n[cc[k]] < m) m = D.chr_n[cc[k]];
    }
    for (t1 = 0; t1 < m; t1 += 8192) {
      const int te = m - t1 < 8192 ? m : t1 + 8192;
      double a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
      const ROW_T *r0 = r[0], *r1 = r[1], *r2 = r[2], *r3 = r[3];
      if (__atomic_load_n(gen, __ATOMIC_RELAXED) != my_gen) return -1; /* cancelled */
      for (t = t1; t < te; t++) { /* chains k >= nc repeat chain 0 and are dropped */
        a0 += nr[r0[t]];
        a1 += nr[r1[t]];
        a2 += nr[r2[t]];
        a3 += nr[r3[t]];
      }
      a[0] = a0; a[1] = a1; a[2] = a2; a[3] = a3;
    }
    for (k = 0; k < nc; k++) {
      for (t = m; t < D.chr_n[cc[k]]; t++) a[k] += nr[r[k][t]];
      out[cc[k]] = a[k];
    }
  }
  return 0;
}

#undef ROW_CAT
#undef ROW_CAT2
