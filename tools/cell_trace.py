"""Summarise FSCLG_CELL_TRACE output: per launch, busy fraction of the workgroup slots
over the kernel span, tail length, cell duration spread.  python tools/cell_trace.py <file>"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64)
i, k = 0, 0
while i < raw.size:
    n = int(raw[i]); i += 1
    a = raw[i:i + 4 * n].reshape(n, 4).astype(np.int64); i += 4 * n
    t0, t1 = a[:, 0] - a[:, 0].min(), a[:, 1] - a[:, 0].min()
    span = t1.max()
    dur = t1 - t0
    slots = 512  # 256 CUs x 2 workgroups
    busy = dur.sum() / (span * slots)
    # time after which fewer than half the slots are busy
    ends = np.sort(t1)
    half = ends[max(0, n - slots // 2)] if n > slots // 2 else 0
    if k < 3 or k % 5 == 0:
        print(f"launch {k}: cells {n} span {span / 100:.0f} us  slot-busy {busy:.2f}  "
              f"dur p50 {np.median(dur) / 100:.0f} us max {dur.max() / 100:.0f} us  "
              f"tail(<half busy) {(span - half) / 100:.0f} us  terms/us p50 {np.median(a[:, 3] / np.maximum(dur, 1) * 100):.0f}")
    k += 1
