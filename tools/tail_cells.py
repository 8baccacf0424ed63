"""Blocking-batch launches of a FSCLG_CELL_TRACE file (split launches, header split > 1): per
launch the span, the longest cell and the median cell, and what a perfectly balanced member
allocation could reach.  python tools/tail_cells.py <file>"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64)
i = 0
rows = []
while i < raw.size:
    h = int(raw[i]); i += 1
    n, batch, split = h & 0xFFFFFFFFFF, (h >> 40) & 0xFF, h >> 48
    a = raw[i:i + 8 * n].reshape(n, 8).astype(np.int64); i += 8 * n
    a = a[a[:, 0] > 0]
    if split <= 1 or len(a) == 0:
        continue
    t0 = a[:, 0].min()
    dur = (a[:, 1] - a[:, 0]) / 100.0  # us (100 MHz wall clock)
    span = (a[:, 1].max() - t0) / 100.0
    rows.append((len(a), split, span, dur.max(), np.median(dur), dur.mean(), a[:, 3].sum(), a[:, 3].max()))
r = np.array(rows)
print(f"split launches: {len(r)}")
for q in (10, 50, 90):
    print(f"p{q}: cells {np.percentile(r[:, 0], q):.0f} split {np.percentile(r[:, 1], q):.0f} span {np.percentile(r[:, 2], q):.0f} us "
          f"max cell {np.percentile(r[:, 3], q):.0f} us median cell {np.percentile(r[:, 4], q):.0f} us")
print(f"sum span {r[:, 2].sum() / 1e3:.0f} ms, sum max-cell {r[:, 3].sum() / 1e3:.0f} ms, sum median-cell {r[:, 4].sum() / 1e3:.0f} ms, "
      f"sum mean-cell {r[:, 5].sum() / 1e3:.0f} ms")
print(f"longest cell's terms / mean cell's terms (p50): {np.median(r[:, 7] / (r[:, 6] / r[:, 0])):.2f}")
# FSCLG_PHASE_TIMING builds: slots 4..7 of member 0 = ticks in bounds + layout, wave 0's own
# segments, the wait for the workgroup's other waves, the members' combine + resolve
ph, nph = [], []
i = 0
while i < raw.size:
    h = int(raw[i]); i += 1
    n, split = h & 0xFFFFFFFFFF, h >> 48
    a = raw[i:i + 8 * n].reshape(n, 8).astype(np.int64); i += 8 * n
    a = a[a[:, 0] > 0]
    if split <= 1 or len(a) == 0:
        continue
    j = np.argmax(a[:, 1] - a[:, 0])
    ph.append(np.concatenate([[a[j, 1] - a[j, 0]], a[j, 4:8], [a[j, 2] & 0xFFFFFFFFFFFF]]) / 100.0)
    nph.append(np.median(a[:, 2] >> 48))
ph = np.array(ph)
if ph[:, 1:].sum() > 0:
    s = ph.sum(axis=0)
    print(f"longest cells, summed over launches (ms): total {s[0] / 1e3:.0f}, bounds+layout {s[1] / 1e3:.0f}, "
          f"own segments {s[2] / 1e3:.0f}, wait {s[3] / 1e3:.0f}, combine+resolve {s[4] / 1e3:.0f} "
          f"(of it the members' arrival {s[5] / 1e3:.0f}), rest {(s[0] - s[1:5].sum()) / 1e3:.0f}")
    print(f"phases (eval_walks instances) per cell, median over launches of the per-launch median: {np.median(nph):.0f}")
