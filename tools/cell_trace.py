"""Summarise FSCLG_CELL_TRACE output: per launch, busy fraction of the workgroup slots
over the kernel span, tail length, cell duration spread, and (builds with
-DFSCLG_PHASE_TIMING) the share of cell time in each eval_walks phase.
python tools/cell_trace.py <file>"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64)
i, k = 0, 0
while i < raw.size:
    n = int(raw[i]) & 0xFFFFFFFFFF; i += 1  # header: n | batch << 40 | split << 48
    a = raw[i:i + 8 * n].reshape(n, 8).astype(np.int64); i += 8 * n
    a = a[a[:, 0] > 0]  # idle blocks of the XCD placement
    n = len(a)
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
        ph = a[:, 4:8].sum(axis=0)
        if ph.sum():
            print("   phases (share of cell time): " + "  ".join(
                f"{nm} {v / dur.sum():.3f}" for nm, v in zip(("bounds", "layout", "segments", "resolve"), ph)))
    k += 1
