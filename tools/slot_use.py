"""Workgroup-slot use of a permutation job from an FSCLG_CELL_TRACE file (records appended per
waited launch: header n | batch << 40 | split << 48, then n x [start, end, cu, terms, 4 phase
ticks]).  Prints, over the last `frac` of the job's span (default: all of it), the share of time
with k cells running (k binned against the device's resident slots), and per batch class
(high-priority blocking batches 0-1, bulk batches 2..) the mean launch: cells, span, mean and
longest cell, and sum of cell time / (span x slots).
python tools/slot_use.py <file> [slots=512] [frac=1.0]"""
import sys

import numpy as np

path = sys.argv[1]
slots = int(sys.argv[2]) if len(sys.argv) > 2 else 512
frac = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
raw = np.fromfile(path, dtype=np.uint64)
i, recs = 0, []
while i < raw.size:
    h = int(raw[i]); i += 1
    n, batch, split = h & ((1 << 40) - 1), (h >> 40) & 0xFF, h >> 48
    a = raw[i:i + 8 * n].reshape(n, 8).astype(np.int64); i += 8 * n
    a = a[a[:, 1] > 0]  # idle blocks of the XCD placement never start
    if len(a):
        recs.append((batch, split, a[:, 0], a[:, 1], a[:, 3]))
t0 = min(r[2].min() for r in recs)
t1 = max(r[3].max() for r in recs)
lo = t1 - frac * (t1 - t0)
s = np.concatenate([r[2] for r in recs]); e = np.concatenate([r[3] for r in recs])
sp = np.concatenate([np.full(len(r[2]), max(r[1], 1)) for r in recs])  # members per cell
t = np.concatenate([s, e]); d = np.concatenate([sp, -sp])
o = np.argsort(t, kind="stable"); t = t[o]; run = np.cumsum(d[o])
dt = np.diff(t); run = run[:-1]; mid = t[:-1]
m = mid >= lo
dt, run = dt[m], run[m]
tot = dt.sum()
print(f"span {(t1 - lo) / 1e8:.2f} s (100 MHz ticks), {len(recs)} launches")
edges = [0, 1, slots // 4, slots // 2, 3 * slots // 4, slots, 10 ** 9]
for a, b in zip(edges[:-1], edges[1:]):
    sel = (run >= a) & (run < b)
    print(f"  workgroups running in [{a}, {b}): {dt[sel].sum() / tot:.3f} of the time")
print(f"  mean workgroups running {np.sum(dt * run) / tot:.1f} of {slots}")
for name, cls in (("blocking (batches 0-1)", lambda b: b < 2), ("bulk (batches 2..)", lambda b: b >= 2)):
    rr = [r for r in recs if cls(r[0]) and r[2].min() >= lo]
    if not rr:
        continue
    span = np.array([r[3].max() - r[2].min() for r in rr]) / 1e2  # us
    ncell = np.array([len(r[2]) for r in rr]); spl = np.array([max(r[1], 1) for r in rr])
    mean_c = np.array([(r[3] - r[2]).mean() for r in rr]) / 1e2
    max_c = np.array([(r[3] - r[2]).max() for r in rr]) / 1e2
    fill = np.array([((r[3] - r[2]).sum() * max(r[1], 1)) for r in rr]) / 1e2 / (span * slots)
    print(f"{name}: {len(rr)} launches, mean {ncell.mean():.0f} cells x {spl.mean():.1f} members, span {span.mean():.0f} us,"
          f" cell mean {mean_c.mean():.0f} us, longest {max_c.mean():.0f} us, slot fill {fill.mean():.3f}")
