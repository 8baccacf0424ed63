// CPU check of fscl_amd/csrc/device/cell_order.h (built and run by tests/test_host.py): the
// ordered dedup of cells and endpoints against std::map restatements, over cell lists in the
// host's order (ascending), two ascending runs, shuffled, with duplicates, nested cells and
// negative positions; the galloping search against std::lower_bound.  Prints "ok <cases>".
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
    // the galloping search
    const int m = 1 + (int)(g() % 300);
    std::vector<int32_t> pos(m);
    int v = (int)(g() % 5) - 2;
    for (auto& p : pos) { v += (int)(g() % 4); p = v; }
    for (int q = 0; q < 30; q++) {
      const int h = 1 + (int)(g() % m), x = (int)(g() % (v + 12)) - 4;
      const int got = cellorder::lower_bound_from(pos.data(), m, std::min(h, m), x);
      const int ref = (int)(std::lower_bound(pos.begin() + std::min(1, m), pos.end(), x) - pos.begin());
      if (got != std::max(ref, 1)) return fail("lower_bound_from", it);
    }
  }
  printf("ok %d\n", cases);
  return 0;
}
