// Host-side ordering of a batch's cells for fsclg_search_submit and fsclg_slot_windows
// (fsclg.hip): identical cells evaluated once, endpoints shared by neighbouring cells evaluated
// once, and the site ranges of a trial's cells' windows.  Exact comparisons in (chromosome, position)
// order, no hashing: the host submits its points in that order (one ascending run per class of
// cells), so ordering is a linear check or a merge of the runs, and equal cells and shared
// endpoints are neighbours.  Plain C++ (templated on the cell and int-pair types) so that
// tests/test_host.py compiles it on the CPU against a hash-map restatement.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace cellorder {

template <class Cell>
inline bool same_cell(const Cell& a, const Cell& b) {
  return a.chr == b.chr && a.start_pos == b.start_pos && a.end_pos == b.end_pos;
}

// sort idx by less: a linear pass when it is already in order, a merge when it is two
// ascending runs (the host's classes of cells), a stable sort otherwise
template <class Less>
inline void sort_runs(std::vector<int>& idx, Less less) {
  const size_t n = idx.size();
  size_t k = 1;
  while (k < n && !less(idx[k], idx[k - 1])) k++;
  if (k >= n) return;
  size_t m = k + 1;
  while (m < n && !less(idx[m], idx[m - 1])) m++;
  if (m >= n) std::inplace_merge(idx.begin(), idx.begin() + k, idx.end(), less);
  else std::stable_sort(idx.begin(), idx.end(), less);
}

// lower_bound(pos + 1, pos + n, x) - pos for every chromosome's ascending positions, through a
// table of the answers at every 2^16 bp from the chromosome's first site: a query searches one
// bucket's sites (a few cache lines) instead of the whole array (C5: 227k sites, 0.9 MB per
// chromosome, a miss per probe)
struct SiteIndex {
  static constexpr int SH = 16;
  std::vector<int> idx, off, nb;
  std::vector<long long> base;
  void build(const int32_t* all_pos, const int32_t* chr_start, const int* chr_n, int n_chr) {
    idx.clear(); off.assign(n_chr, 0); nb.assign(n_chr, 0); base.assign(n_chr, 0);
    for (int ch = 0; ch < n_chr; ch++) {
      const int n = (int)chr_n[ch];
      off[ch] = (int)idx.size();
      if (n <= 1) continue;
      const int32_t* pos = all_pos + chr_start[ch];
      base[ch] = pos[0];
      nb[ch] = (int)(((long long)pos[n - 1] - base[ch]) >> SH) + 1;
      int j = 1;
      for (int b = 0; b <= nb[ch]; b++) {
        const long long x = base[ch] + ((long long)b << SH);
        while (j < n && pos[j] < x) j++;
        idx.push_back(j);
      }
    }
  }
  int find(const int32_t* pos, int ch, int n, int x) const {
    if (n <= 1) return 1;
    const long long d = (long long)x - base[ch];
    if (d < 0) return 1;
    const long long b = d >> SH;
    if (b >= nb[ch]) return n;
    const int* t = idx.data() + off[ch] + b;
    return (int)(std::lower_bound(pos + t[0], pos + t[1], x) - pos);
  }
};

// Each cell's site range [lo, hi) of window starts (fsclg.hip's window_ranges), remembered from
// the previous call: a permutation trial's cells are mostly the previous trial's, so a merge of
// the two ordered lists finds them with sequential reads, and only new cells search the sites
// (a search is a few cache misses in a 20-MB site array).  ranges(): the cells' ranges in
// (chromosome, start, end) order.
template <class Cell, class I2>
struct RangeMemo {
  struct Ent { Cell c; I2 r; };
  std::vector<Ent> prev, next;
  std::vector<int> sidx;
  long long key = -1;  // the window length and site upload the entries belong to
  template <class Compute>
  void ranges(const Cell* cells, int n, long long k, std::vector<I2>& out, Compute compute) {
    auto cless = [](const Cell& x, const Cell& y) {
      return x.chr != y.chr ? x.chr < y.chr : x.start_pos != y.start_pos ? x.start_pos < y.start_pos : x.end_pos < y.end_pos;
    };
    if (k != key) { prev.clear(); key = k; }
    sidx.resize(n);
    for (int i = 0; i < n; i++) sidx[i] = i;
    sort_runs(sidx, [cells, &cless](int a, int b) { return cless(cells[a], cells[b]); });
    next.clear();
    out.clear();
    size_t j = 0;
    for (int t = 0; t < n; t++) {
      const Cell& x = cells[sidx[t]];
      if (!next.empty() && same_cell(next.back().c, x)) continue;
      while (j < prev.size() && cless(prev[j].c, x)) j++;
      I2 r;
      if (j < prev.size() && same_cell(prev[j].c, x)) r = prev[j].r;
      else if (!compute(x, r)) continue;  // no range (a chromosome within one window)
      next.push_back(Ent{x, r});
      out.push_back(r);
    }
    prev.swap(next);
  }
};

// distinct cells in (chromosome, start, end) order; uidx[i]: cells[i]'s index among them.
// sidx is scratch.
template <class Cell>
inline void dedup_cells(const Cell* cells, int n, std::vector<int>& sidx, std::vector<Cell>& ucells,
                        std::vector<int>& uidx) {
  auto less = [cells](int a, int b) {
    const Cell &x = cells[a], &y = cells[b];
    return x.chr != y.chr ? x.chr < y.chr : x.start_pos != y.start_pos ? x.start_pos < y.start_pos : x.end_pos < y.end_pos;
  };
  sidx.resize(n);
  for (int i = 0; i < n; i++) sidx[i] = i;
  sort_runs(sidx, less);
  ucells.clear();
  uidx.resize(n);
  for (int k = 0; k < n; k++) {
    const Cell& x = cells[sidx[k]];
    if (ucells.empty() || !same_cell(ucells.back(), x)) ucells.push_back(x);
    uidx[sidx[k]] = (int)ucells.size() - 1;
  }
}

// distinct endpoints (chromosome, position) of the distinct cells, in that order; ucell_ep[u]:
// the indices of cell u's start and end among them.  ekeys and sidx are scratch.
template <class Cell, class I2>
inline void dedup_endpoints(const std::vector<Cell>& ucells, std::vector<unsigned long long>& ekeys,
                            std::vector<int>& sidx, std::vector<I2>& epos, std::vector<I2>& ucell_ep) {
  const int nu = (int)ucells.size();
  auto ekey = [](int chr, int pos) {  // order-preserving for signed positions
    return ((unsigned long long)(uint32_t)chr << 32) | (uint32_t)(pos ^ (int)0x80000000);
  };
  // endpoint 2u is cell u's start, 2u + 1 its end; the starts are in order, the ends too unless cells nest
  ekeys.resize(2 * (size_t)nu);
  for (int u = 0; u < nu; u++) {
    ekeys[2 * u] = ekey(ucells[u].chr, ucells[u].start_pos);
    ekeys[2 * u + 1] = ekey(ucells[u].chr, ucells[u].end_pos);
  }
  sidx.resize(2 * (size_t)nu);
  bool ends_sorted = true;
  for (int u = 1; u < nu && ends_sorted; u++) ends_sorted = ekeys[2 * u + 1] >= ekeys[2 * u - 1];
  auto less = [&ekeys](int a, int b) { return ekeys[a] < ekeys[b] || (ekeys[a] == ekeys[b] && a < b); };
  if (ends_sorted) {  // merge the two ascending sequences
    int i = 0, j = 0, k = 0;
    while (i < nu || j < nu) {
      if (j >= nu || (i < nu && !less(2 * j + 1, 2 * i))) sidx[k++] = 2 * i++;
      else sidx[k++] = 2 * j++ + 1;
    }
  } else {
    for (int e = 0; e < 2 * nu; e++) sidx[e] = e;
    std::sort(sidx.begin(), sidx.end(), less);
  }
  epos.clear();
  ucell_ep.resize(nu);
  unsigned long long last = 0;
  for (int k = 0; k < 2 * nu; k++) {
    const int e = sidx[k], u = e >> 1;
    if (epos.empty() || ekeys[e] != last) {
      epos.push_back(I2{ucells[u].chr, (e & 1) ? ucells[u].end_pos : ucells[u].start_pos});
      last = ekeys[e];
    }
    if (e & 1) ucell_ep[u].y = (int)epos.size() - 1;
    else ucell_ep[u].x = (int)epos.size() - 1;
  }
}

}  // namespace cellorder
