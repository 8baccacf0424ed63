// CPU check of fscl_amd/csrc/device/cell_order.h (built and run by tests/test_host.py): the
// ordered dedup of cells and endpoints against std::map restatements, over cell lists in the
// host's order (ascending), two ascending runs, shuffled, with duplicates, nested cells and
// negative positions; the bucketed site index against std::lower_bound.  Prints "ok <cases>".
#include <stdio.h>

#include <map>
#include <random>
#include <tuple>

#include "../../fscl_amd/csrc/device/cell_order.h"

struct Cell { int chr, start_pos, end_pos; };
struct I2 { int x, y; };

static int fail(const char* what, int it) { printf("FAIL %s (case %d)\n", what, it); return 1; }

int main() {
  std::mt19937 g(12345);
  int cases = 0;
  for (int it = 0; it < 4000; it++, cases++) {
    const int n = (int)(g() % 200);
    const int grid = 1 + (int)(g() % 50), span = 1 + (int)(g() % 4);
    std::vector<Cell> cells(n);
    for (auto& c : cells) {
      c.chr = (int)(g() % 4);
      c.start_pos = ((int)(g() % 40) - 5) * grid;  // some negative
      c.end_pos = c.start_pos + grid * ((g() % 8) ? 1 : span);  // some longer cells nest others
    }
    const int mode = it % 4;
    auto key = [](const Cell& c) { return std::make_tuple(c.chr, c.start_pos, c.end_pos); };
    auto lt = [&](const Cell& a, const Cell& b) { return key(a) < key(b); };
    if (mode == 0) std::sort(cells.begin(), cells.end(), lt);
    if (mode == 1 && n > 1) {
      const int k = (int)(g() % n);
      std::sort(cells.begin(), cells.begin() + k, lt);
      std::sort(cells.begin() + k, cells.end(), lt);
    }
    std::vector<int> sidx, uidx;
    std::vector<Cell> ucells;
    cellorder::dedup_cells(cells.data(), n, sidx, ucells, uidx);
    std::map<std::tuple<int, int, int>, int> want;
    for (auto& c : cells) want[key(c)] = 0;
    if (ucells.size() != want.size()) return fail("distinct cells", it);
    for (size_t u = 1; u < ucells.size(); u++)
      if (!lt(ucells[u - 1], ucells[u])) return fail("cell order", it);
    for (int i = 0; i < n; i++)
      if (key(ucells[uidx[i]]) != key(cells[i])) return fail("cell index", it);
    std::vector<unsigned long long> ekeys;
    std::vector<I2> epos, uep;
    cellorder::dedup_endpoints(ucells, ekeys, sidx, epos, uep);
    std::map<std::pair<int, int>, int> ew;
    for (auto& c : ucells) { ew[{c.chr, c.start_pos}] = 0; ew[{c.chr, c.end_pos}] = 0; }
    if (epos.size() != ew.size()) return fail("distinct endpoints", it);
    for (size_t e = 1; e < epos.size(); e++)
      if (std::make_pair(epos[e - 1].x, epos[e - 1].y) >= std::make_pair(epos[e].x, epos[e].y)) return fail("endpoint order", it);
    for (size_t u = 0; u < ucells.size(); u++) {
      const I2 a = epos[uep[u].x], b = epos[uep[u].y];
      if (a.x != ucells[u].chr || a.y != ucells[u].start_pos || b.x != ucells[u].chr || b.y != ucells[u].end_pos)
        return fail("endpoint index", it);
    }
    // the range memo over a run of calls (cells dropping out, new ones, another key): the
    // computed range of every distinct cell, in cell order
    {
      cellorder::RangeMemo<Cell, I2> memo;
      std::vector<Cell> cur = cells;
      for (int call = 0; call < 6; call++) {
        const long long mk = call < 4 ? 7 : 9;
        auto f = [mk](const Cell& x, I2& r) {
          if (x.chr == 3) return false;  // no range
          r = I2{x.start_pos * 3 + (int)mk, x.end_pos - x.chr};
          return true;
        };
        std::vector<I2> got;
        memo.ranges(cur.data(), (int)cur.size(), mk, got, f);
        std::map<std::tuple<int, int, int>, I2> w;
        for (auto& x : cur) { I2 r; if (f(x, r)) w[key(x)] = r; }
        if (got.size() != w.size()) return fail("memo count", it);
        size_t q = 0;
        for (auto& kv : w) {
          if (got[q].x != kv.second.x || got[q].y != kv.second.y) return fail("memo range", it);
          q++;
        }
        std::vector<Cell> nx;  // the next trial: most cells stay, a few new
        for (auto& x : cur) if (g() % 5) nx.push_back(x);
        for (int a = 0; a < 3; a++) nx.push_back(Cell{(int)(g() % 4), (int)(g() % 40) * grid, (int)(g() % 40) * grid + grid});
        cur.swap(nx);
      }
    }
    // the site index: every chromosome's lower_bound(pos + 1, pos + n, x)
    const int nchr = 1 + (int)(g() % 4);
    std::vector<int32_t> all;
    std::vector<int32_t> cst(nchr);
    std::vector<int> cn(nchr);
    for (int ch = 0; ch < nchr; ch++) {
      cst[ch] = (int32_t)all.size();
      cn[ch] = (int)(g() % 300);  // some empty or one-site chromosomes
      int v = (int)(g() % 200000) - 100000;
      const int step = 1 << (g() % 18);  // sparse to dense against the 2^16-bp buckets
      for (int i = 0; i < cn[ch]; i++) { v += (int)(g() % (unsigned)step) * (g() % 5 ? 1 : 0); all.push_back(v); }
    }
    cellorder::SiteIndex si;
    si.build(all.data(), cst.data(), cn.data(), nchr);
    for (int ch = 0; ch < nchr; ch++) {
      const int32_t* pos = all.data() + cst[ch];
      const int m = cn[ch];
      if (m < 1) continue;
      for (int q = 0; q < 40; q++) {
        const long long span = (long long)pos[m - 1] - pos[0] + 4;
        const int x = (int)(pos[0] - 2 + (long long)(g() % (unsigned)(span + 4)) - 2);
        const int got = si.find(pos, ch, m, x);
        const int ref = (int)(std::lower_bound(pos + 1, pos + m, x) - pos);
        if (got != ref) return fail("site index", it);
      }
    }
  }
  printf("ok %d\n", cases);
  return 0;
}
