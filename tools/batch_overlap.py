"""Concurrency of search batches from an FSCLG_CELL_TRACE file (one record per batch, in
wait order): share of the span with cells of two or more batches running, and slot use.
python tools/batch_overlap.py <file>"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64)
i, recs = 0, []
while i < raw.size:
    n = int(raw[i]) & ((1 << 40) - 1); i += 1  # header: n | batch << 40 | split << 48
    recs.append(raw[i:i + 8 * n].reshape(n, 8).astype(np.int64)); i += 8 * n
t0 = min(a[:, 0].min() for a in recs)
ev = []
for b, a in enumerate(recs):
    for s, e in zip(a[:, 0] - t0, a[:, 1] - t0):
        ev.append((s, 1, b)); ev.append((e, -1, b))
ev.sort()
run = {}
last, multi, busy, slot = 0, 0, 0, 0.0
for t, d, b in ev:
    dt = t - last
    if run:
        busy += dt
        if len(run) > 1:
            multi += dt
        slot += dt * sum(run.values())
    run[b] = run.get(b, 0) + d
    if run[b] == 0:
        del run[b]
    last = t
span = last
print(f"batches {len(recs)}  span {span / 100:.0f} us  cells running {busy / span:.3f} of it, "
      f"two+ batches at once {multi / span:.3f}, mean cells running {slot / span:.0f} (512 slots)")
